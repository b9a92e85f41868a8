#!/bin/bash
# four-wave wide kernel: parity (wide, fold, filter, derived), phase stamps
# (diagnostics build), config5 bench lines of both kernels, kernel-trace stats.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_fold.py tests/test_gpu_filter.py tests/test_gpu_derived.py tests/test_gpu_likelihood.py tests/test_gpu_compat.py \
  -x -q --timeout 300 --timeout-method thread > gpurun_out/wide4_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/wide4_tests.log
NIPAMD_LIB=$PWD/nip_amd/_lib/variants/libnip_amd_diag.so NIPAMD_PHASE_TIMES=1 timeout -k 10 200 python bench.py --workload config5 --steps 2 --warmup 1 --no-check --no-cpu-baseline > gpurun_out/w4_diag.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload config5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c5_w4.jsonl 2> gpurun_out/bench_c5.err || exit 1
NIPAMD_WIDE_KERNEL=wave1 timeout -k 10 300 python bench.py --workload config5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c5_w1.jsonl 2>> gpurun_out/bench_c5.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o run --output-format csv -- python3 bench.py --workload config5 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_c5.log 2>&1 || exit 1
