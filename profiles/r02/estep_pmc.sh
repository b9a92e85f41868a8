#!/bin/bash
# SQ counters (one pass) of the DPP e_step kernel (config 4 shard).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/pmc_estep -o run --output-format csv -- python3 bench.py --workload estep --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_estep.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVES -d gpurun_out/pmc_estep2 -o run --output-format csv -- python3 bench.py --workload estep --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_estep2.log 2>&1 || exit 1
