#!/bin/bash
# Joint-interface chains: their parity suite (vs the general engine and the
# oracle), the general-engine suite (golden fixtures through both engines),
# the chain-kernel suites they share code with, then bench lines of the
# factorial HMM on both paths and the joint path's rocprof kernel stats.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="--timeout 150 --timeout-method thread"
timeout -k 10 600 python -u -m pytest tests/test_gpu_joint.py tests/test_gpu_jtree.py tests/test_gpu_derived.py tests/test_gpu_parity.py -x -q $T > gpurun_out/o_tests.log 2>&1 || exit 1
for w in joint jtree joint; do
  timeout -k 10 300 python bench.py --workload $w --steps 5 --warmup 1 --no-cpu-baseline >> gpurun_out/o_bench.jsonl 2>> gpurun_out/o_bench.err || exit 1
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/o_prof_joint -o run --output-format csv -- \
  python3 bench.py --workload joint --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/o_prof_joint.log 2>&1 || exit 1
