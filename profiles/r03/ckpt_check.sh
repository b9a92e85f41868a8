#!/bin/bash
# checkpoint fb kernel: parity tests, then bench lines (headline only) and kernel stats.  $1 = tag
set -o pipefail
tag=${1:-r03c}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_ckpt.py tests/test_gpu_parity.py tests/test_gpu_joint.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || exit 1
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --no-secondary --no-cpu-baseline >> gpurun_out/${tag}_bench.jsonl 2>> gpurun_out/${tag}_bench.err || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o run --output-format csv -- python3 bench.py --no-secondary --no-cpu-baseline --steps 20 > gpurun_out/${tag}_prof.log 2>&1 || exit 1
timeout -k 10 120 env NIPAMD_LIB=$PWD/nip_amd/_lib/diag/libnip_amd_stamps.so NIPAMD_PHASE_TIMES=1 python bench.py --no-secondary --no-cpu-baseline --steps 1 --warmup 1 > gpurun_out/${tag}_diag.txt 2>&1 || exit 1
