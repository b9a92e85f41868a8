#!/bin/bash
# GPU pass for generate_data: its parity tests, the compat tests, the whole
# GPU suite, a bench line of the generate workload and a rocprofv3 kernel
# trace of it.  Each GPU step has its own time limit; a failing step ends it.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_generate.py tests/test_gpu_compat.py -x -v --timeout 120 \
  --timeout-method thread > gpurun_out/generate.log 2>&1 || exit 1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/gpu_all.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --workload generate --steps 10 --warmup 2 > gpurun_out/bench_generate.jsonl \
  2> gpurun_out/bench_generate.err || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gen -o gen -- \
  python bench.py --workload generate --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_gen.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_fb.jsonl 2>&1
