#!/bin/bash
# e_step timing diagnostics: per-block phase stamps of the matrix-core e_step
# (diagnostics build) and kernel-trace stats of the estep workload.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
NIPAMD_LIB=$PWD/nip_amd/_lib/variants/libnip_amd_diag.so NIPAMD_PHASE_TIMES=1 timeout -k 10 200 python bench.py --workload estep --steps 1 --warmup 1 --no-check > gpurun_out/estep_diag.txt 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_estep -o run --output-format csv -- python3 bench.py --workload estep --steps 2 --warmup 1 > gpurun_out/prof_estep.log 2>&1 || exit 1
