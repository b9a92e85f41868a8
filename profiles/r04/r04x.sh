#!/bin/bash
# Kernel traces (no counters) of the headline and configs 3 and 5 at HEAD,
# with the bench's own warmup, for the committed kernel averages.
# Usage: r04x.sh [TAG]   (default r04x; output gpurun_out/prof_TAG)
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r04x}
cd /tmp && export TMPDIR=/tmp
for W in fb config3 config5; do
  mkdir -p $R/gpurun_out/prof_$TAG/$W
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG/$W/trace -o run --output-format csv -- \
    python3 $R/bench.py --workload $W --no-secondary --no-cpu-baseline > $R/gpurun_out/prof_$TAG/$W/trace.log 2>&1 || exit 1
done
echo done
