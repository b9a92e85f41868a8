#!/bin/bash
# Interleaved A/B of the product library against variant builds on one box.
#   ab.sh TAG WORKLOAD REPS VARIANT.so... [-- pytest targets]
# pytest targets (product library) first; then REPS rounds of every library's
# bench line of the workload (headline only, 0.5 s warmup).
set -o pipefail
tag=$1; wl=$2; reps=$3; shift 3
libs=(); tests=()
while [ $# -gt 0 ]; do
  if [ "$1" = "--" ]; then shift; tests=("$@"); break; fi
  libs+=("$1"); shift
done
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$R"
out=$O/ab_$wl.txt
: > $out
if [ ${#tests[@]} -gt 0 ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu "${tests[@]}" \
    > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -1 $O/tests.log >> $out
fi
for rep in $(seq $reps); do
  for lib in product "${libs[@]}"; do
    if [ "$lib" = product ]; then env=(); else env=(NIPAMD_LIB=$R/$lib); fi
    r=$(env "${env[@]}" timeout -k 10 200 python bench.py --workload $wl --no-secondary --no-cpu-baseline --min-warm 0.5 --detail "" 2>$O/err.txt | tail -1) || { cat $O/err.txt; exit 1; }
    echo "$lib $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.4f ms  kernel %.4f ms  %s" % (d["ms_per_step"], d["roofline"]["kernel_ms"], d["roofline"]["kernel"]))')" >> $out
  done
done
cat $out
