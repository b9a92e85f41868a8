#!/bin/bash
# Kernel traces (no counters) of every workload of the default bench line at
# HEAD, each run as the headline of its own bench process (the secondary ones
# with the line's 0.5 s warmup), then the timed-region check against the line
# printed by the same run (profiles/timed_region.py).
# Usage: bash profiles/r05/traces.sh TAG [WORKLOAD...]
set -o pipefail
TAG=${1:-r05t}; shift || true
WLS=${@:-fb config3 em config5 estep_config3}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/prof_$TAG
cd /tmp && export TMPDIR=/tmp
for W in $WLS; do
  mkdir -p $O/$W
  warm=""; [ "$W" != fb ] && warm="--min-warm 0.5"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$W/trace -o run --output-format csv -- \
    python3 $R/bench.py --workload $W --no-secondary --no-cpu-baseline --detail "" $warm > $O/$W/trace.log 2>&1 || exit 1
done
cd $R && python3 profiles/timed_region.py $TAG $O $WLS > $O/timed_region.out 2>&1
cp profiles/${TAG}_timed_region.txt $O/ 2>/dev/null
echo done
