#!/bin/bash
# The e_step's backward rows (the block's bound, r04f5 stamps) at wave
# priority 1 (ab/eprio1.so: NIPAMD_ESTEP_PRIO=1), interleaved A/B on em, twice.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04zs
bash profiles/r04/ab_tests.sh r04zs/em em "" nip_amd/_lib/ab/eprio1.so || exit 1
bash profiles/r04/ab_tests.sh r04zs/emb em "" nip_amd/_lib/ab/eprio1.so || exit 1
echo done
