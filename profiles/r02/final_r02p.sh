#!/bin/bash
# Round-2 GPU pass p (joint-interface chains in): the whole GPU suite, smoke(),
# default bench (config 2 headline) with its rocprof kernel stats, every other
# workload's bench line (joint and jtree: the factorial HMM on both paths),
# the joint path's rocprof kernel stats.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/p_gpu_all.log 2>&1
echo "rc=$?" >> gpurun_out/p_gpu_all.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/p_smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/p_bench_default.jsonl 2> gpurun_out/p_bench.err || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/p_prof_fb -o run --output-format csv -- \
  python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/p_prof_fb.log 2>&1 || exit 1
for w in joint jtree config3 config5 estep em generate; do
  timeout -k 10 300 python bench.py --workload $w --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/p_bench_$w.jsonl 2>> gpurun_out/p_bench.err || exit 1
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/p_prof_joint -o run --output-format csv -- \
  python3 bench.py --workload joint --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/p_prof_joint.log 2>&1 || exit 1
