#!/bin/bash
# SQ counters (separate passes) of the e_step kernel, config 4 shard: the
# default (chain_estep16_kernel) and, with $2 = dpp8, the round-2 kernel
# (diagnostics build).  Summaries: profiles/summarize_pmc.py-style csv.
set -o pipefail
tag=${1:-r03q}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
if [ "$2" = dpp8 ]; then export NIPAMD_LIB=$PWD/nip_amd/_lib/diag/libnip_amd_diag.so NIPAMD_ESTEP_KERNEL=dpp8; fi
C1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
C2="SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C1 -d gpurun_out/${tag}_pmc1 -o run --output-format csv -- python3 bench.py --workload estep --steps 2 --warmup 1 --no-secondary --no-cpu-baseline > gpurun_out/${tag}_pmc1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C2 -d gpurun_out/${tag}_pmc2 -o run --output-format csv -- python3 bench.py --workload estep --steps 2 --warmup 1 --no-secondary --no-cpu-baseline > gpurun_out/${tag}_pmc2.log 2>&1 || exit 1
