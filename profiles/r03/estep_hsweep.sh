#!/bin/bash
# chain_estep16_kernel phase split sweep (stamps build): block cycles per H, config 4 shard.  $1 = tag
set -o pipefail
tag=${1:-r03s}
mkdir -p gpurun_out
export PYTHONPATH=$PWD
out=gpurun_out/${tag}_estep_hsweep.txt
: > $out
for h in 50 46 42 38 54; do
  echo "H=$h%" >> $out
  timeout -k 10 120 env NIPAMD_LIB=$PWD/nip_amd/_lib/diag/libnip_amd_stamps.so NIPAMD_PHASE_TIMES=1 NIPAMD_ESTEP_H=$h python bench.py --workload estep --no-secondary --no-cpu-baseline --steps 1 --warmup 1 2>&1 | grep "estep16" | tail -2 >> $out || exit 1
done
