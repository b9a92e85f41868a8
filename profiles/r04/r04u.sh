#!/bin/bash
# 64-bit operand copies in the lane-swap sums (ab/b64b.so): wide / e_step
# tests on the variant, A/B of configs 5 and 3-e_step against HEAD's product.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04u; mkdir -p $O
timeout -k 10 400 env NIPAMD_LIB=$PWD/nip_amd/_lib/ab/b64b.so python -u -m pytest -q --timeout 120 --timeout-method thread \
  -m gpu tests/test_gpu_wide.py tests/test_gpu_fold.py tests/test_gpu_estep_wide.py tests/test_gpu_filter.py \
  > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc" >> $O/tests.log; [ $rc -le 1 ] || exit 1
bash profiles/r04/ab_tests.sh r04u/c5 config5 "" nip_amd/_lib/ab/b64b.so || exit 1
bash profiles/r04/ab_tests.sh r04u/e3 estep_config3 "" nip_amd/_lib/ab/b64b.so
