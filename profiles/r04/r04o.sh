#!/bin/bash
# op e_step (block-partitioned op_xi) tests + bench + trace, then the profile
# collection of configs 2, 3, 5 at HEAD (profiles/collect.sh r04o ...).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04o; mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_opchain_estep.py \
  > $O/tests_op.log 2>&1; rc=$?; echo "tests rc=$rc" >> $O/tests_op.log; [ $rc -eq 0 ] || exit 1
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_op -o run --output-format csv -- \
  python3 $GRAFT_REPO_ROOT/bench.py --workload estep_opchain --steps 3 --warmup 1 --no-cpu-baseline --no-secondary \
  > $GRAFT_REPO_ROOT/$O/prof_op.log 2>&1 || exit 1
cd "$GRAFT_REPO_ROOT"
bash profiles/collect.sh r04o fb config3 config5
echo done
