#!/bin/bash
# Phase timestamps (NIPAMD_PHASE_TIMES) and bench value of every built variant.
for so in nip_amd/_lib/variants/*.so; do
  echo "== $(basename $so)"
  NIPAMD_LIB=$PWD/$so NIPAMD_PHASE_TIMES=1 timeout -k 10 120 python bench.py --no-cpu-baseline --no-check --steps 2 --warmup 1 2>&1 | grep 'nipamd' | tail -3
done
