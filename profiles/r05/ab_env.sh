#!/bin/bash
# Interleaved A/B of environment settings on one box (same library):
#   ab_env.sh TAG WORKLOAD REPS "VAR=a" "VAR=b" ...
set -o pipefail
tag=$1; wl=$2; reps=$3; shift 3
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$R"
out=$O/abenv_$wl.txt
: > $out
for rep in $(seq $reps); do
  for e in "$@"; do
    r=$(env $e timeout -k 10 200 python bench.py --workload $wl --no-secondary --no-cpu-baseline --min-warm 0.5 --detail "" 2>$O/err.txt | tail -1) || { cat $O/err.txt; exit 1; }
    echo "$e $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.4f ms  kernel %.4f ms  %s" % (d["ms_per_step"], d["roofline"]["kernel_ms"], d["roofline"]["kernel"]))')" >> $out
  done
done
cat $out
