#!/bin/bash
# 64-bit operand copies in configs 2 and 3's lane sums too (ab/b64c.so):
# chain-kernel tests on the variant, A/B of configs 2 and 3.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04v; mkdir -p $O
timeout -k 10 500 env NIPAMD_LIB=$PWD/nip_amd/_lib/ab/b64c.so python -u -m pytest -q --timeout 200 --timeout-method thread \
  -m gpu tests/test_gpu_ckpt.py tests/test_gpu_parity.py tests/test_gpu_wide.py tests/test_gpu_joint.py \
  > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc" >> $O/tests.log; [ $rc -le 1 ] || exit 1
bash profiles/r04/ab_tests.sh r04v/c2 fb "" nip_amd/_lib/ab/b64c.so || exit 1
bash profiles/r04/ab_tests.sh r04v/c3 config3 "" nip_amd/_lib/ab/b64c.so
