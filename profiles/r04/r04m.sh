#!/bin/bash
# Relative-block row64 (hazard-padded swaps): wide/fold tests and config-5 A/B;
# op e_step (prefetched op_xi) tests, bench and kernel trace; microbenchmark.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04m; mkdir -p $O
timeout -k 10 60 ./profiles/r04/mb_r64 > $O/mb_r64.txt 2>&1 || exit 1
timeout -k 10 400 env NIPAMD_LIB=$PWD/nip_amd/_lib/ab/r64rel.so python -u -m pytest -q --timeout 120 --timeout-method thread \
  -m gpu tests/test_gpu_wide.py tests/test_gpu_fold.py tests/test_gpu_filter.py > $O/tests_rel.log 2>&1; rc=$?; echo "tests rc=$rc" >> $O/tests_rel.log; [ $rc -le 1 ] || exit 1
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_opchain_estep.py \
  > $O/tests_op.log 2>&1; rc=$?; echo "tests rc=$rc" >> $O/tests_op.log; [ $rc -le 1 ] || exit 1
bash profiles/r04/ab_tests.sh r04m/c5 config5 "" nip_amd/_lib/ab/r64rel.so || exit 1
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_op -o run --output-format csv -- \
  python3 $GRAFT_REPO_ROOT/bench.py --workload estep_opchain --steps 3 --warmup 1 --no-cpu-baseline --no-secondary \
  > $GRAFT_REPO_ROOT/$O/prof_op.log 2>&1
echo done
