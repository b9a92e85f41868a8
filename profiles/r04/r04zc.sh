#!/bin/bash
# The e_step message kernels' rows with nontemporal stores (ab/msgnt.so:
# NIPAMD_MSG_NT=1 in chain_msgs_kernel / op_wide_msgs_kernel), interleaved A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04zc
for wl in estep_config3 opchain_wide; do
  bash profiles/r04/ab_tests.sh r04zc/$wl $wl "" nip_amd/_lib/ab/msgnt.so || exit 1
done
echo done
