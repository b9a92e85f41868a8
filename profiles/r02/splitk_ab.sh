#!/bin/bash
# SPLITK (two 2-MFMA accumulation chains per mat-vec) for the checkpoint fb
# kernel: parity of the variant, stamps, interleaved bench lines.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
V=$PWD/nip_amd/_lib/diag/libnip_amd_splitk.so
NIPAMD_LIB=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/splitk_parity.log 2>&1 || exit 1
NIPAMD_LIB=$PWD/nip_amd/_lib/diag/libnip_amd_splitk_diag.so NIPAMD_PHASE_TIMES=1 timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/splitk_diag.txt 2>&1 || exit 1
for rep in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline >> gpurun_out/splitk_bench.jsonl 2>> gpurun_out/splitk_bench.err || exit 1
  NIPAMD_LIB=$V timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline >> gpurun_out/splitk_bench.jsonl 2>> gpurun_out/splitk_bench.err || exit 1
done
