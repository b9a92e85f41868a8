#!/bin/bash
# Per-wave cycle stamps of the checkpoint fb kernel (diagnostics build).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
NIPAMD_FB_KERNEL=ckpt NIPAMD_LIB=$PWD/nip_amd/_lib/diag/libnip_amd_diag.so NIPAMD_PHASE_TIMES=1 timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/ckpt_diag.txt 2>&1 || exit 1
