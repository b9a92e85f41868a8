#!/bin/bash
# rocprofv3 collection for the bench workloads: kernel-trace stats passes plus
# separate PMC passes (counters never combined with sys/runtime traces).
# Usage (on the GPU box, from the repo root):  bash profiles/collect.sh <tag>
# then, back in the build container:  python profiles/summarize.py <tag>
set -euo pipefail
TAG=${1:-run}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
BENCH="$R/bench.py --steps 5 --warmup 1 --no-cpu-baseline"
EST="$R/bench.py --workload estep --batch 131072 --steps 3 --warmup 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $BENCH > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_estep -o run --output-format csv -- python3 $EST > $OUT/trace_estep.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc2 -o run --output-format csv -- python3 $BENCH > $OUT/pmc2.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/pmc3 -o run --output-format csv -- python3 $BENCH > $OUT/pmc3.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-trace -d $OUT/pmc1 -o run --output-format csv -- python3 $BENCH > $OUT/pmc1.log 2>&1
echo done
