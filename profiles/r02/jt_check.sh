#!/bin/bash
# General join-tree engine: its GPU parity suite, the "jtree" bench line
# (factorial HMM) and its rocprof kernel stats.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_jtree.py tests/test_gpu_fold.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/jt_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload jtree --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_jtree.jsonl 2> gpurun_out/bench_jtree.err || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_jt -o run --output-format csv -- \
  python3 bench.py --workload jtree --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_jt.log 2>&1 || exit 1
