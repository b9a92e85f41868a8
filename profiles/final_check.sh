#!/bin/bash
# End-of-session GPU pass: the whole GPU suite, smoke(), the default bench
# line (config 2 headline) and a rocprofv3 kernel-trace summary of it.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/gpu_all.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench_default.jsonl 2> gpurun_out/bench_default.err || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fb -o run --output-format csv -- \
  python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof_fb.log 2>&1
