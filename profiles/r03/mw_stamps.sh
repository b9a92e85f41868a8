#!/bin/bash
# per-wave cycle stamps of chain_mfma_wide_kernel (config 3; stamps build).  $1 = tag
set -o pipefail
tag=${1:-r03i}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 env NIPAMD_LIB=$PWD/nip_amd/_lib/diag/libnip_amd_stamps.so NIPAMD_PHASE_TIMES=1 python bench.py --workload config3 --no-cpu-baseline --steps 1 --warmup 1 --no-check > gpurun_out/${tag}_mw_stamps.txt 2>&1 || exit 1
