#!/bin/bash
# Matrix-core e_step with the M1 counts as one-hot MFMAs (no atomics): the
# e_step suite (its mfma tests run the kernel explicitly), then interleaved
# estep bench lines of the DPP and matrix-core kernels.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_estep.py -x -q --timeout 200 --timeout-method thread > gpurun_out/esm_parity.log 2>&1 || exit 1
NIPAMD_ESTEP_KERNEL=mfma timeout -k 10 300 python -u -m pytest tests/test_gpu_estep.py tests/test_gpu_train.py -x -q --timeout 200 --timeout-method thread > gpurun_out/esm_parity_mfma.log 2>&1 || exit 1
for rep in 1 2; do
  echo dpp >> gpurun_out/esm_bench.txt
  timeout -k 10 200 python bench.py --workload estep --steps 5 --warmup 1 --no-cpu-baseline >> gpurun_out/esm_bench.txt 2>&1 || exit 1
  echo mfma >> gpurun_out/esm_bench.txt
  NIPAMD_ESTEP_KERNEL=mfma timeout -k 10 200 python bench.py --workload estep --steps 5 --warmup 1 --no-cpu-baseline >> gpurun_out/esm_bench.txt 2>&1 || exit 1
done
