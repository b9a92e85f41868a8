#!/bin/bash
# Checkpoint + recompute fb kernel (chain_ckpt.hip): agreement with the
# scratch kernel and the oracle, the parity suite under NIPAMD_FB_KERNEL=scratch,
# interleaved bench lines of both kernels, per-wave stamps (diagnostics build).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_ckpt.py -q --timeout 200 --timeout-method thread > gpurun_out/ckpt_bitid.log 2>&1; [ $? -le 1 ] || exit 1
NIPAMD_FB_KERNEL=scratch timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/ckpt_parity.log 2>&1 || exit 1
for rep in 1 2; do
  NIPAMD_FB_KERNEL=scratch timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline >> gpurun_out/ckpt_bench.jsonl 2>> gpurun_out/ckpt_bench.err || exit 1
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline >> gpurun_out/ckpt_bench.jsonl 2>> gpurun_out/ckpt_bench.err || exit 1
done
NIPAMD_LIB=$PWD/nip_amd/_lib/diag/libnip_amd_diag.so NIPAMD_PHASE_TIMES=1 timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/ckpt_diag.txt 2>&1 || exit 1
