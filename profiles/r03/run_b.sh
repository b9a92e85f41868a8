#!/bin/bash
# Round 3 pass b: the tests touched by the diagnostics-build move, the default
# bench line (headline + secondary configs + CPU baselines), the latency
# microbenchmark, then rocprofv3 kernel-trace / PMC passes of every config.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "tests"
timeout -k 10 600 python -u -m pytest tests/test_gpu_ckpt.py tests/test_gpu_wide.py tests/test_gpu_estep.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/r03b_tests.log 2>&1 || exit 1
echo "mb_lat"
timeout -k 10 60 ./profiles/r03/mb_lat > gpurun_out/r03_mb_lat.txt 2>&1 || exit 1
echo "bench"
timeout -k 10 600 python bench.py > gpurun_out/r03b_bench.jsonl 2> gpurun_out/r03b_bench.err || exit 1
echo "collect"
timeout -k 10 900 bash profiles/collect.sh r03b fb config3 config5 em || exit 1
echo done
