#!/bin/bash
# A/B of configs 5, 3-e_step and 4-e_step against HEAD~1's build (ab/base.so),
# the operator-chain e_step bench and its general-engine comparator, the
# op e_step tests.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04k; mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_opchain_estep.py \
  > $O/tests_op.log 2>&1; rc=$?; echo "tests rc=$rc" >> $O/tests_op.log; [ $rc -le 1 ] || exit 1
bash profiles/r04/ab_tests.sh r04k/c5 config5 "" nip_amd/_lib/ab/base.so || exit 1
bash profiles/r04/ab_tests.sh r04k/e3 estep_config3 "" nip_amd/_lib/ab/base.so || exit 1
bash profiles/r04/ab_tests.sh r04k/e4 estep "" nip_amd/_lib/ab/base.so || exit 1
for w in estep_opchain estep_opchain_jt; do
  timeout -k 10 300 python bench.py --workload $w --no-secondary --no-cpu-baseline > $O/$w.jsonl 2>$O/$w.err || exit 1
done
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_e3 -o run --output-format csv -- \
  python3 $GRAFT_REPO_ROOT/bench.py --workload estep_config3 --steps 5 --warmup 2 --no-cpu-baseline --no-secondary \
  > $GRAFT_REPO_ROOT/$O/prof_e3.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_op -o run --output-format csv -- \
  python3 $GRAFT_REPO_ROOT/bench.py --workload estep_opchain --steps 3 --warmup 1 --no-cpu-baseline --no-secondary \
  > $GRAFT_REPO_ROOT/$O/prof_op.log 2>&1
echo done
