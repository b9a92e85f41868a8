#!/bin/bash
# Config-2 model, throughput vs sequences per GPU (256 blocks = one per CU at
# B=4096): how much of the gap to the HBM roofline is the single block wave.
set -o pipefail
mkdir -p gpurun_out
for b in 2048 4096 8192 16384 32768; do
  timeout -k 10 120 python bench.py --batch $b --steps 20 --warmup 3 --no-cpu-baseline \
    >> gpurun_out/batch_sweep.jsonl 2>> gpurun_out/batch_sweep.err || exit 1
done
