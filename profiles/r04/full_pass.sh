#!/bin/bash
# The whole GPU suite, smoke() and the default bench line at HEAD.
# Usage: full_pass.sh TAG
set -o pipefail
tag=${1:-r04}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  > gpurun_out/${tag}_gpu_all.txt 2>&1
echo "tests rc=$?" >> gpurun_out/${tag}_gpu_all.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.txt 2>&1 || exit 1
timeout -k 10 400 python bench.py > gpurun_out/${tag}_bench_default.jsonl 2> gpurun_out/${tag}_bench_default.err || exit 1
echo done
