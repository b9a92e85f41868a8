#!/bin/bash
# per-wave cycle stamps of the checkpoint kernels (stamps build: python -c "from nip_amd import build as b;
# b.build(defines=['NIPAMD_DIAGNOSTICS', 'NIPAMD_WAIT_TIMES=1'], out='nip_amd/_lib/diag/libnip_amd_stamps.so')").  $1 = tag
set -o pipefail
tag=${1:-r03c}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 env NIPAMD_LIB=$PWD/nip_amd/_lib/diag/libnip_amd_stamps.so NIPAMD_PHASE_TIMES=1 python bench.py --no-secondary --no-cpu-baseline --steps 1 --warmup 1 --no-check > gpurun_out/${tag}_diag.txt 2>&1 || exit 1
