#!/bin/bash
# The whole GPU suite, smoke() and the default bench line at HEAD.
# Usage: bash profiles/r05/full_pass.sh TAG
set -o pipefail
tag=${1:-r05}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  > $O/gpu_all.txt 2>&1
echo "tests rc=$?" >> $O/gpu_all.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 1
timeout -k 10 400 python bench.py --detail $O/bench_detail.json > $O/bench_default.jsonl 2> $O/bench_default.err || exit 1
echo done
