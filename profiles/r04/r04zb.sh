#!/bin/bash
# Scratch rows read back with nontemporal loads (ab/ntld.so: NIPAMD_SCR_NTLD=1,
# their last use), interleaved A/B against the product library.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04zb
for wl in fb config3 estep; do
  bash profiles/r04/ab_tests.sh r04zb/$wl $wl "" nip_amd/_lib/ab/ntld.so || exit 1
done
echo done
