#!/bin/bash
# GPU fold of the wide in-clique: parity tests, config5 bench line (fold
# roofline, PCIe-inclusive figure), kernel-trace stats of the config5 run.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest tests/test_gpu_fold.py tests/test_gpu_wide.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/fold_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/fold_tests.log
timeout -k 10 300 python bench.py --workload config5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_config5.jsonl 2> gpurun_out/bench_config5.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o run --output-format csv -- python3 bench.py --workload config5 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_c5.log 2>&1 || exit 1
