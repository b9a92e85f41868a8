#!/bin/bash
# row64 with 16-step chunks: wide/fold/filter tests, stamps, A/B vs HEAD~ (ab/prev.so).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04n; mkdir -p $O
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_wide.py tests/test_gpu_fold.py tests/test_gpu_filter.py tests/test_gpu_opchain_estep.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/tests.log; [ $rc -le 1 ] || exit 1
timeout -k 10 120 env NIPAMD_LIB=$PWD/nip_amd/_lib/diag/libnip_amd_diag.so NIPAMD_PHASE_TIMES=1 python bench.py --workload config5 \
  --no-secondary --no-cpu-baseline --steps 1 --warmup 1 --no-check > $O/stamps.txt 2>&1 || exit 1
bash profiles/r04/ab_tests.sh r04n/c5 config5 "" nip_amd/_lib/ab/prev.so
