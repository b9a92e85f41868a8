#!/bin/bash
# Round-2 GPU pass (HEAD after the r02m/r02n A/B passes): the whole GPU suite, smoke(), default bench (config 2
# headline) with its rocprof kernel stats, the other workloads' bench lines.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_all.log 2>&1
echo "rc=$?" >> gpurun_out/gpu_all.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench_default.jsonl 2> gpurun_out/bench_default.err || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fb_l -o run --output-format csv -- \
  python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof_fb_l.log 2>&1 || exit 1
for w in config3 config5 estep em generate jtree; do
  timeout -k 10 300 python bench.py --workload $w --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_$w.jsonl 2>> gpurun_out/bench_default.err || exit 1
done
bash profiles/collect.sh r02n fb > gpurun_out/collect_r02n.log 2>&1 || exit 1
