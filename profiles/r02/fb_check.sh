#!/bin/bash
# fb kernel change check: parity suites touching the matrix-core kernel, phase
# stamps (diagnostics build) and three bench lines of the headline config.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_estep.py tests/test_gpu_derived.py tests/test_gpu_filter.py \
  -x -q --timeout 120 --timeout-method thread > gpurun_out/fb_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/fb_tests.log
NIPAMD_LIB=$PWD/nip_amd/_lib/variants/libnip_amd_diag.so NIPAMD_PHASE_TIMES=1 timeout -k 10 120 python bench.py --no-cpu-baseline --no-check --steps 2 --warmup 1 > gpurun_out/fb_phase.txt 2>&1 || exit 1
for i in 1 2 3; do timeout -k 10 120 python bench.py --no-cpu-baseline > gpurun_out/fb_bench_$i.jsonl 2>/dev/null || exit 1; done
