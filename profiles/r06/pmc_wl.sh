#!/bin/bash
# PMC passes over one bench workload, each its own rocprofv3 run (kernel
# trace only, <= 8 SQ counters a pass).   pmc_wl.sh TAG WORKLOAD [sq|all]
set -o pipefail
tag=$1; wl=$2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$R"
sets=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
      "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC SQ_INSTS_SALU GRBM_GUI_ACTIVE")
if [ "$3" = all ]; then sets+=("FETCH_SIZE" "WRITE_SIZE"); fi
i=0
for set in "${sets[@]}"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $set --kernel-trace -d $O/pmc$i -o run --output-format csv -- python3 $R/bench.py --workload $wl --steps 2 --warmup 1 --min-warm 0 --no-cpu-baseline --no-secondary --detail "" > $O/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $O/pmc$i.log; exit 1; }
done
echo pmc done
