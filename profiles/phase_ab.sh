#!/bin/bash
# A/B phase timestamps on one box: the main library and every variant, three
# single launches each, interleaved.
for rep in 1 2 3; do
  for so in nip_amd/_lib/libnip_amd.so nip_amd/_lib/variants/*.so; do
    echo "== $(basename $so) rep $rep"
    NIPAMD_LIB=$PWD/$so NIPAMD_PHASE_TIMES=1 timeout -k 10 120 python bench.py --no-cpu-baseline --no-check --steps 1 --warmup 1 2>&1 | grep 'nipamd' | tail -2
  done
done
