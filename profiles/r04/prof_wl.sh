#!/bin/bash
# Kernel-trace summaries of named bench workloads (headline only, no CPU
# baseline), after optional GPU tests.
# Usage: bash profiles/r04/prof_wl.sh TAG "WORKLOAD..." [pytest targets...]
set -o pipefail
TAG=${1:-q}; WLS=$2; shift 2 || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$R"
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest "$@" -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
  rc=$?; echo "tests rc=$rc" >> $O/tests.log; [ $rc -eq 0 ] || exit 1
fi
cd /tmp
for w in $WLS; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_$w -o run --output-format csv -- \
    python3 $R/bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline --no-secondary > $O/prof_$w.log 2>&1 || exit 1
done
echo done
