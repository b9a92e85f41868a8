#!/bin/bash
# config 5: diagnostics-build stamps and a kernel trace.   c5.sh TAG
set -o pipefail
tag=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$R"
NIPAMD_LIB=$R/nip_amd/_lib/diag/libnip_amd_diag.so NIPAMD_PHASE_TIMES=1 timeout -k 10 200 python bench.py --workload config5 --steps 3 --warmup 2 --min-warm 0.3 --no-cpu-baseline --no-secondary --detail "" > $O/c5_stamps.jsonl 2> $O/c5_stamps.err || { tail -5 $O/c5_stamps.err; exit 1; }
grep "wide4" $O/c5_stamps.err | tail -4
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --workload config5 --no-secondary --no-cpu-baseline --min-warm 0.5 --detail "" > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp $f $O/kernel_stats.csv; head -4 $O/kernel_stats.csv | cut -c1-200
