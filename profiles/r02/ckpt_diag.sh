#!/bin/bash
# Per-wave cycle stamps of the checkpoint fb kernel (diagnostics builds; the
# "fake" build reads its checkpoints from LDS: timing only), then bench lines.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
NIPAMD_FB_KERNEL=ckpt NIPAMD_LIB=$PWD/nip_amd/_lib/diag/libnip_amd_diag.so NIPAMD_PHASE_TIMES=1 timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/ckpt_diag.txt 2>&1 || exit 1
NIPAMD_FB_KERNEL=ckpt NIPAMD_LIB=$PWD/nip_amd/_lib/diag/libnip_amd_fake.so NIPAMD_PHASE_TIMES=1 timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-check > gpurun_out/ckpt_diag_fake.txt 2>&1 || exit 1
NIPAMD_FB_KERNEL=ckpt timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ckpt_bench2.jsonl 2>&1 || exit 1
