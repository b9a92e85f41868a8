#!/bin/bash
# e_step on the matrix cores: parity (e_step / em / train / dist tests and the
# fb parity suite, whose ll shares the code), then bench lines of the estep
# workload for the MFMA kernel and the DPP kernel, and the fb headline.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_estep.py tests/test_gpu_em_dist.py tests/test_gpu_train.py \
  tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/estep_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/estep_tests.log
timeout -k 10 200 python bench.py --workload estep --steps 3 --warmup 1 > gpurun_out/bench_estep.jsonl 2> gpurun_out/bench_estep.err || exit 1
NIPAMD_FB_KERNEL=dpp timeout -k 10 200 python bench.py --workload estep --steps 3 --warmup 1 > gpurun_out/bench_estep_dpp.jsonl 2>> gpurun_out/bench_estep.err || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/bench_fb.jsonl 2>> gpurun_out/bench_estep.err || exit 1
