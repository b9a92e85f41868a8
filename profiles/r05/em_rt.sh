#!/bin/bash
# HIP runtime + kernel trace of a short em run (the iteration's host gaps),
# and the deterministic-row BAD_LUCK tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r05e}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_gpu_estep.py -k "deterministic or bad_luck" -m gpu -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
echo "tests rc=$?" >> $O/tests.log
cd /tmp
timeout -k 10 300 rocprofv3 --runtime-trace --kernel-trace --memory-copy-trace -d $O/rt -o run --output-format csv -- \
  python3 $R/bench.py --workload em --steps 4 --warmup 2 --no-secondary --no-cpu-baseline --detail "" > $O/rt.log 2>&1 || exit 1
echo done
