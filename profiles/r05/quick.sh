#!/bin/bash
# Iteration pass: selected GPU tests, then bench lines of named workloads
# (headline only, no CPU baseline) and their kernel traces.
# Usage: bash profiles/r05/quick.sh TAG "WORKLOAD..." [pytest targets...]
set -o pipefail
TAG=${1:-q}; WLS=$2; shift 2 || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$R"
if [ $# -gt 0 ]; then
  timeout -k 10 900 python -u -m pytest "$@" -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
  rc=$?; echo "tests rc=$rc" >> $O/tests.log; [ $rc -eq 0 ] || exit 1
fi
for w in $WLS; do
  timeout -k 10 300 python bench.py --workload $w --no-secondary --no-cpu-baseline --min-warm 0.5 --detail "" \
    > $O/bench_$w.jsonl 2> $O/bench_$w.err || exit 1
done
cd /tmp
for w in $WLS; do
  mkdir -p $O/prof_$w
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$w -o run --output-format csv -- \
    python3 $R/bench.py --workload $w --no-secondary --no-cpu-baseline --min-warm 0.5 --detail "" > $O/prof_$w/trace.log 2>&1 || exit 1
done
echo done
