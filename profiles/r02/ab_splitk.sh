#!/bin/bash
# A/B of the split-K MFMA matvec (NIPAMD_MFMA_SPLITK) on config 2: parity of
# the variant, then interleaved bench lines and phase timestamps.
set -o pipefail
mkdir -p gpurun_out
NIPAMD_LIB=$PWD/nip_amd/_lib/variants/libnip_amd_splitk.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_parity.log 2>&1 || exit 1
for rep in 1 2 3; do
  for so in nip_amd/_lib/libnip_amd.so nip_amd/_lib/variants/libnip_amd_splitk.so; do
    echo "== $(basename $so) rep $rep"
    NIPAMD_LIB=$PWD/$so timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 --warmup 3 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().splitlines()[-1]); print(d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])" || exit 1
  done
done > gpurun_out/ab_bench.txt 2>&1
for so in nip_amd/_lib/variants/libnip_amd_diag.so nip_amd/_lib/variants/libnip_amd_diagsplit.so; do
  echo "== $(basename $so)"
  NIPAMD_LIB=$PWD/$so NIPAMD_PHASE_TIMES=1 timeout -k 10 120 python bench.py --no-cpu-baseline --no-check --steps 1 --warmup 1 2>&1 | grep 'nipamd' | tail -2
done > gpurun_out/ab_phase.txt 2>&1
