#!/bin/bash
# rocprofv3 collection for the bench workloads: kernel-trace stats passes plus
# separate PMC passes (counters never combined with sys/runtime traces).
# Usage (on the GPU box, from the repo root):  bash profiles/collect.sh <tag> [workloads...]
# then, back in the build container:  python profiles/summarize.py <tag>
# Workloads: fb (config 2, the headline), config3, config5, em (config 4: one
# em_learn iteration over the 131072 x 1024 shard), estep (its e_step alone).
set -euo pipefail
TAG=${1:-run}
shift || true
WLS=${*:-fb config3 config5 em estep_config3}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT; for W in $WLS; do mkdir -p $OUT/$W; done
cd /tmp && export TMPDIR=/tmp
for W in $WLS; do
  case $W in
    estep|em|estep_config3) ARGS="--workload $W --steps 3 --warmup 1 --no-cpu-baseline" ;;
    *) ARGS="--workload $W --no-secondary --steps 5 --warmup 1 --no-cpu-baseline" ;;
  esac
  B="$R/bench.py $ARGS"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$W/trace -o run --output-format csv -- python3 $B > $OUT/$W/trace.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/$W/pmc2 -o run --output-format csv -- python3 $B > $OUT/$W/pmc2.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/$W/pmc3 -o run --output-format csv -- python3 $B > $OUT/$W/pmc3.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-trace -d $OUT/$W/pmc1 -o run --output-format csv -- python3 $B > $OUT/$W/pmc1.log 2>&1
  # the matrix pipes' busy cycles and the effective clock (GRBM_GUI_ACTIVE / 8 XCDs / wall)
  timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $OUT/$W/pmc4 -o run --output-format csv -- python3 $B > $OUT/$W/pmc4.log 2>&1 || true
  echo "$W done"
done
