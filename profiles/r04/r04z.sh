#!/bin/bash
# Nontemporal posterior stores (ab/nt.so: NIPAMD_POST_NT=1 in chain_fb_ckpt_kernel
# and chain_mfma_wide_kernel), interleaved A/B against the product library.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for wl in fb config3; do
  bash profiles/r04/ab_tests.sh r04z/$wl $wl "" nip_amd/_lib/ab/nt.so || exit 1
done
echo done
