#!/bin/bash
# Nontemporal posterior stores now the product default (store_pol.h): the
# affected kernels' GPU tests, then interleaved A/B against the previous
# policy (ab/post0.so) and against nontemporal scratch rows too (ab/scrnt.so).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04za
L=nip_amd/_lib/ab
bash profiles/r04/ab_tests.sh r04za/fb fb "tests/test_gpu_ckpt.py tests/test_gpu_parity.py tests/test_gpu_wide.py tests/test_gpu_fold.py tests/test_gpu_estep.py" $L/post0.so $L/scrnt.so || exit 1
grep -q "tests rc=0" gpurun_out/r04za/fb_tests.log || exit 1
for wl in config3 config5 estep; do
  bash profiles/r04/ab_tests.sh r04za/$wl $wl "" $L/post0.so $L/scrnt.so || exit 1
done
echo done
