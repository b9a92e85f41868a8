#!/bin/bash
# Interleaved A/B of the product library against variant builds on one box.
#   ab_bench.sh TAG WORKLOAD VARIANT.so... [-- pytest targets]
# Each library runs the workload's bench line twice, alternating; pytest
# targets (product library) run first.
set -o pipefail
tag=$1; wl=$2; shift 2
libs=(); tests=()
while [ $# -gt 0 ]; do
  if [ "$1" = "--" ]; then shift; tests=("$@"); break; fi
  libs+=("$1"); shift
done
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${tag}_ab.txt
: > $out
if [ ${#tests[@]} -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu "${tests[@]}" \
    > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
  tail -1 gpurun_out/${tag}_tests.log >> $out
fi
for rep in 1 2; do
  for lib in product "${libs[@]}"; do
    if [ "$lib" = product ]; then env=(); else env=(NIPAMD_LIB=$PWD/$lib); fi
    r=$(env "${env[@]}" timeout -k 10 120 python bench.py --workload $wl --no-secondary --no-cpu-baseline --steps 20 2>gpurun_out/${tag}_err.txt | tail -1) || { cat gpurun_out/${tag}_err.txt; exit 1; }
    echo "$lib $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.4f ms  kernel %.4f ms  %s" % (d["ms_per_step"], d["roofline"]["kernel_ms"], d["roofline"]["kernel"]))')" >> $out
  done
done
cat $out
