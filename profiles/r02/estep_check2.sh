#!/bin/bash
# e_step kernels after the switch: parity of both (DPP default, matrix-core by
# NIPAMD_ESTEP_KERNEL=mfma), the fb parity suite (shared ll code), phase
# breakdown of the matrix-core e_step (diagnostics build), bench lines.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_estep.py tests/test_gpu_em_dist.py tests/test_gpu_train.py \
  tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/estep_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/estep_tests.log
NIPAMD_ESTEP_KERNEL=mfma NIPAMD_LIB=$PWD/nip_amd/_lib/variants/libnip_amd_diag.so NIPAMD_PHASE_TIMES=1 \
  timeout -k 10 200 python bench.py --workload estep --steps 1 --warmup 1 --no-check > gpurun_out/estep_diag.txt 2>&1 || exit 1
timeout -k 10 200 python bench.py --workload estep --steps 3 --warmup 1 > gpurun_out/bench_estep.jsonl 2> gpurun_out/bench_estep.err || exit 1
NIPAMD_ESTEP_KERNEL=mfma timeout -k 10 200 python bench.py --workload estep --steps 3 --warmup 1 > gpurun_out/bench_estep_mfma.jsonl 2>> gpurun_out/bench_estep.err || exit 1
