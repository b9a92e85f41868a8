#!/bin/bash
# per-wave phase stamps of chain_estep16_kernel (stamps build), config 4 shard.  $1 = tag
set -o pipefail
tag=${1:-r03s}
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 120 env NIPAMD_LIB=$PWD/nip_amd/_lib/diag/libnip_amd_stamps.so NIPAMD_PHASE_TIMES=1 python bench.py --workload estep --no-secondary --no-cpu-baseline --steps 1 --warmup 1 > gpurun_out/${tag}_estep_stamps.txt 2>&1 || exit 1
