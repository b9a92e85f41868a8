#!/bin/bash
# Nontemporal posterior stores (ab/nt.so: NIPAMD_POST_NT=1 in chain_fb_ckpt_kernel
# and chain_mfma_wide_kernel) and config 3's partner priority (ab/prioA.so),
# interleaved A/B against the product library, two rounds each.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash profiles/r04/ab_tests.sh r04z/fb fb "" nip_amd/_lib/ab/nt.so || exit 1
bash profiles/r04/ab_tests.sh r04z/config3 config3 "" nip_amd/_lib/ab/nt.so nip_amd/_lib/ab/prioA.so || exit 1
bash profiles/r04/ab_tests.sh r04z/config3b config3 "" nip_amd/_lib/ab/nt.so nip_amd/_lib/ab/prioA.so || exit 1
echo done
