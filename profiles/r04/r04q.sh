#!/bin/bash
# op e_step with the counting-sort op_xi: its tests and kernel trace first,
# then the whole GPU suite, smoke() and the default bench line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04q; mkdir -p $O
timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread -m gpu tests/test_gpu_opchain_estep.py \
  > $O/tests_op.log 2>&1; rc=$?; echo "tests rc=$rc" >> $O/tests_op.log; [ $rc -eq 0 ] || exit 1
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_op -o run --output-format csv -- \
  python3 $GRAFT_REPO_ROOT/bench.py --workload estep_opchain --steps 3 --warmup 1 --no-cpu-baseline --no-secondary \
  > $GRAFT_REPO_ROOT/$O/prof_op.log 2>&1 || exit 1
cd "$GRAFT_REPO_ROOT"
bash profiles/r04/full_pass.sh r04q
