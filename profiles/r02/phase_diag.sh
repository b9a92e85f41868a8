#!/bin/bash
# Phase timestamps / barrier waits of every diagnostics variant (config 2).
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
for so in nip_amd/_lib/variants/libnip_amd_diag*.so; do
  echo "== $(basename $so) rep $rep"
  NIPAMD_LIB=$PWD/$so NIPAMD_PHASE_TIMES=1 timeout -k 10 120 python bench.py --no-cpu-baseline --no-check --steps 1 --warmup 1 2>&1 | grep 'nipamd' | tail -4
done
done > gpurun_out/phase_diag.txt 2>&1
