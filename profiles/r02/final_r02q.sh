#!/bin/bash
# Round-2 pass q (HEAD, joint-interface e_step in): the whole GPU suite,
# smoke(), the default bench line and the joint / jtree lines.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/q_gpu_all.log 2>&1
echo "rc=$?" >> gpurun_out/q_gpu_all.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/q_smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/q_bench_default.jsonl 2> gpurun_out/q_bench.err || exit 1
for w in joint jtree; do
  timeout -k 10 300 python bench.py --workload $w --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/q_bench_$w.jsonl 2>> gpurun_out/q_bench.err || exit 1
done
