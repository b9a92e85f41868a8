#!/bin/bash
# SQ counters (one pass) of the checkpoint and scratch fb kernels.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES"
export NIPAMD_FB_KERNEL=ckpt
timeout -s KILL 90 rocprofv3 --pmc $C -d gpurun_out/pmc_ckpt -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_ckpt.log 2>&1 || exit 1
export NIPAMD_FB_KERNEL=scratch
timeout -s KILL 90 rocprofv3 --pmc $C -d gpurun_out/pmc_scratch -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_scratch.log 2>&1 || exit 1
