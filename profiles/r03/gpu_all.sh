#!/bin/bash
# Round 3: the whole GPU suite, smoke(), the default bench line (tag = $1).
set -o pipefail
tag=${1:-r03}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/${tag}_gpu_all.log 2>&1
rc=$?
echo "rc=$rc" >> gpurun_out/${tag}_gpu_all.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/${tag}_bench_default.jsonl 2> gpurun_out/${tag}_bench.err || exit 1
