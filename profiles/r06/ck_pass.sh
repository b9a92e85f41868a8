#!/bin/bash
# ck e_step pass: its GPU tests, the em and estep bench lines, a kernel
# trace of em (csv stats) and PMC passes over the em workload, each its own
# rocprofv3 run (kernel trace only).   ck_pass.sh TAG [pmc]
set -o pipefail
tag=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 600 python -u -m pytest -x -q --timeout 180 --timeout-method thread -m gpu tests/test_gpu_estep_ck.py > $O/ck_tests.log 2>&1 || { tail -40 $O/ck_tests.log; exit 1; }
tail -1 $O/ck_tests.log
for wl in em estep; do
  timeout -k 10 300 python bench.py --workload $wl --no-secondary --no-cpu-baseline --min-warm 0.5 --detail "" > $O/bench_$wl.jsonl 2>$O/bench_$wl.err || { tail -20 $O/bench_$wl.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/bench_$wl.jsonl').read().strip().splitlines()[-1]); print('$wl', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['kernel'], d['roofline']['frac'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_em -o run --output-format csv -- python3 bench.py --workload em --no-secondary --no-cpu-baseline --min-warm 0.5 --detail "" > $O/prof_em.log 2>&1 || { tail -20 $O/prof_em.log; exit 1; }
f=$(find $O/prof_em -name "*kernel_stats.csv" | head -1); cp $f $O/em_kernel_stats.csv; head -4 $O/em_kernel_stats.csv | cut -c1-220
if [ "$2" = pmc ]; then
  B="$R/bench.py --workload em --steps 2 --warmup 1 --min-warm 0 --no-cpu-baseline --no-secondary --detail ''"
  i=0
  for set in \
    "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM" \
    "SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA" \
    "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" \
    "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 200 rocprofv3 --pmc $set --kernel-trace -d $O/pmc$i -o run --output-format csv -- python3 $R/bench.py --workload em --steps 2 --warmup 1 --min-warm 0 --no-cpu-baseline --no-secondary --detail "" > $O/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $O/pmc$i.log; exit 1; }
  done
  echo pmc done
fi
