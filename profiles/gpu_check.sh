#!/bin/bash
# One GPU-box pass used while iterating on the kernels: the GPU test suite,
# phase timestamps of the built library, phase/bench lines of every variant
# under nip_amd/_lib/variants, and a bench line of the built library.
# Each GPU step has its own time limit; a failing step ends the script.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/gpu_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/gpu_tests.log
NIPAMD_PHASE_TIMES=1 timeout -k 10 120 python bench.py --no-cpu-baseline --no-check --steps 2 --warmup 1 \
  > gpurun_out/phase_base.txt 2>&1 || exit 1
bash profiles/phase_times.sh > gpurun_out/phase_var.txt 2>&1 || exit 1
timeout -k 10 120 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 || exit 1
timeout -k 10 300 python profiles/variants.py bench > gpurun_out/var_bench.txt 2>&1
