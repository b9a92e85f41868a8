#!/bin/bash
# config 3 kernel (chain_mfma_wide): parity tests, then bench lines.  $1 = tag
set -o pipefail
tag=${1:-r03e}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_parity.py tests/test_gpu_joint.py tests/test_gpu_filter.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 300 python bench.py --workload config3 --no-cpu-baseline >> gpurun_out/${tag}_bench.jsonl 2>> gpurun_out/${tag}_bench.err || exit 1
done
