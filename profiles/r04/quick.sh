#!/bin/bash
# Iteration pass on the GPU box: selected GPU tests (args), the default bench
# line without CPU baselines, and a kernel-trace summary of the headline.
# Usage: bash profiles/r04/quick.sh TAG [pytest targets...]
set -o pipefail
TAG=${1:-q}; shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$R"
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest "$@" -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
  rc=$?; echo "tests rc=$rc" >> $O/tests.log; [ $rc -eq 0 ] || exit 1
fi
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.jsonl 2> $O/bench.err || exit 1
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_fb -o run --output-format csv -- \
  python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-secondary > $O/prof_fb.log 2>&1 || exit 1
echo done
