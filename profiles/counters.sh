#!/bin/bash
# PMC passes (each in its own rocprofv3 run, kernel-trace only) for one library build.
# Usage on the GPU box: bash profiles/counters.sh <tag> [lib.so]
set -euo pipefail
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/cnt_$TAG
mkdir -p $OUT
if [ $# -ge 2 ]; then case $2 in /*) export NIPAMD_LIB=$2;; *) export NIPAMD_LIB=$R/$2;; esac; fi
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 5 --warmup 1 --no-cpu-baseline"
i=0
for set in \
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM" \
  "SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA" \
  "SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS" \
  "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $set --kernel-trace -d $OUT/p$i -o run --output-format csv -- python3 $B > $OUT/p$i.log 2>&1
done
echo done
