#!/bin/bash
# Product: nontemporal posterior stores everywhere, nontemporal scratch rows in
# the wide kernels (store_pol.h).  GPU tests of the wide kernels, then
# interleaved A/B against the round's earlier policy (ab/post0.so) and
# against nontemporal scratch loads on top (ab/ntld.so).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04zb
L=nip_amd/_lib/ab
bash profiles/r04/ab_tests.sh r04zb/config3 config3 "tests/test_gpu_wide.py tests/test_gpu_fold.py tests/test_gpu_filter.py tests/test_gpu_joint.py" $L/post0.so $L/ntld.so || exit 1
grep -q "tests rc=0" gpurun_out/r04zb/config3_tests.log || exit 1
for wl in config5 fb estep; do
  bash profiles/r04/ab_tests.sh r04zb/$wl $wl "" $L/post0.so $L/ntld.so || exit 1
done
echo done
