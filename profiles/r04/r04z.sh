#!/bin/bash
# Nontemporal posterior stores (ab/nt.so: NIPAMD_POST_NT=1 in chain_fb_ckpt_kernel
# and chain_mfma_wide_kernel) and config 3's partner priority (ab/prioA.so),
# interleaved A/B against the product library, two rounds each.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04z
bash profiles/r04/ab_tests.sh r04z/fb fb "" nip_amd/_lib/ab/nt.so || exit 1
bash profiles/r04/ab_tests.sh r04z/config3 config3 "" nip_amd/_lib/ab/nt.so nip_amd/_lib/ab/prioA.so || exit 1
bash profiles/r04/ab_tests.sh r04z/config3b config3 "" nip_amd/_lib/ab/nt.so nip_amd/_lib/ab/prioA.so || exit 1
timeout -k 10 240 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_em_dist.py \
  -k rccl > gpurun_out/r04z/rccl_test.txt 2>&1 || { tail -30 gpurun_out/r04z/rccl_test.txt; exit 1; }
echo done
