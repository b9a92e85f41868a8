#!/bin/bash
# Split filters for 32-state chains (chain_mfma_wide_kernel<2, false, true>):
# the wide-kernel parity suite with the split (default) and without, then
# interleaved config 3 bench lines.  (The split variant was measured slower
# and removed; this script now runs the unsplit kernel both times.)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_derived.py tests/test_gpu_filter.py -x -q --timeout 200 --timeout-method thread > gpurun_out/split_parity.log 2>&1 || exit 1
for rep in 1 2; do
  NIPAMD_WIDE_SPLIT=0 timeout -k 10 200 python bench.py --workload config3 --steps 5 --warmup 1 --no-cpu-baseline >> gpurun_out/split_bench.jsonl 2>> gpurun_out/split_bench.err || exit 1
  timeout -k 10 200 python bench.py --workload config3 --steps 5 --warmup 1 --no-cpu-baseline >> gpurun_out/split_bench.jsonl 2>> gpurun_out/split_bench.err || exit 1
done
