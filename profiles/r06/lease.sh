#!/bin/bash
# Round 6's GPU lease commands in one place (run on the GPU box from the repo
# root; outputs under gpurun_out/TAG, the records kept are copied into
# profiles/r06/gpu/).  Every GPU step runs under its own time limit and the
# steps are chained: the first failure ends the call.
#
#   lease.sh tests  TAG FILE...                 pytest -m gpu on the files
#   lease.sh ab     TAG WORKLOAD REPS LIB.so... [-- TEST...]
#                                               interleaved A/B of the workload's
#                                               line: the product library against
#                                               variant builds (profiles/r05/ab.sh)
#   lease.sh bench  TAG WORKLOAD...             one line per workload (0.5 s warm-up)
#   lease.sh trace  TAG WORKLOAD                rocprofv3 kernel trace + stats
#   lease.sh pmc    TAG WORKLOAD [all]          SQ counter passes (+ FETCH/WRITE_SIZE)
#   lease.sh stamps TAG WORKLOAD                diagnostics build with NIPAMD_PHASE_TIMES=1
#                                               (estep: chain_estep_ck_kernel's groups,
#                                               config5: chain_row64_kernel's blocks)
#   lease.sh jtl    TAG                         the general engine's lanes per unit
#   lease.sh obscal TAG                         FETCH_SIZE calibration (mb_obsread.hip)
#   lease.sh mb     TAG                         mb_lat6 and mb_pipe6 (microbenchmarks)
set -o pipefail
cmd=$1; tag=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag
DIAG=$R/nip_amd/_lib/diag/libnip_amd_diag.so
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$R"

line() {   # WORKLOAD LOG: the line's headline numbers
  python -c "import json,sys; d=json.loads(open('$2').read().strip().splitlines()[-1]); print('$1', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['kernel'], round(d['roofline']['frac'], 4))"
}

case $cmd in
  tests)
    timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu "$@" \
      > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
    tail -1 $O/tests.log ;;
  ab)
    bash $R/profiles/r05/ab.sh $tag "$@" ;;
  bench)
    for wl in "$@"; do
      timeout -k 10 300 python bench.py --workload $wl --no-secondary --no-cpu-baseline --min-warm 0.5 --detail "" \
        > $O/bench_$wl.jsonl 2> $O/bench_$wl.err || { tail -20 $O/bench_$wl.err; exit 1; }
      line $wl $O/bench_$wl.jsonl
    done ;;
  trace)
    wl=$1
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_$wl -o run --output-format csv -- \
      python3 $R/bench.py --workload $wl --no-secondary --no-cpu-baseline --min-warm 0.5 --detail "" \
      > $O/trace_$wl.log 2>&1 || { tail -20 $O/trace_$wl.log; exit 1; }
    f=$(find $O/trace_$wl -name "*kernel_stats.csv" | head -1); cp $f $O/${wl}_kernel_stats.csv
    head -5 $O/${wl}_kernel_stats.csv | cut -c1-200 ;;
  pmc)
    wl=$1
    sets=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
          "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC SQ_INSTS_SALU GRBM_GUI_ACTIVE")
    if [ "$2" = all ]; then sets+=("FETCH_SIZE" "WRITE_SIZE"); fi
    i=0
    for set in "${sets[@]}"; do
      i=$((i+1))
      timeout -s KILL 200 rocprofv3 --pmc $set --kernel-trace -d $O/pmc$i -o run --output-format csv -- \
        python3 $R/bench.py --workload $wl --steps 2 --warmup 1 --min-warm 0 --no-cpu-baseline --no-secondary --detail "" \
        > $O/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $O/pmc$i.log; exit 1; }
    done
    echo "pmc done (python3 profiles/pmc_kernel.py $tag KERNEL)" ;;
  stamps)
    wl=$1
    NIPAMD_LIB=$DIAG NIPAMD_PHASE_TIMES=1 timeout -k 10 300 python bench.py --workload $wl --steps 3 --warmup 2 \
      --min-warm 0.3 --no-secondary --no-cpu-baseline --detail "" > $O/stamps_$wl.jsonl 2> $O/stamps_$wl.err \
      || { tail -20 $O/stamps_$wl.err; exit 1; }
    grep "\[nipamd\]" $O/stamps_$wl.err | tail -6 ;;
  jtl)
    for rep in 1 2; do
      for L in 64 32 16; do
        NIPAMD_LIB=$DIAG NIPAMD_JT_L=$L timeout -k 10 300 python bench.py --workload jtree --no-secondary \
          --no-cpu-baseline --min-warm 0.3 --detail "" > $O/jt_$L.jsonl 2> $O/err.txt || { tail -5 $O/err.txt; exit 1; }
        line "L=$L" $O/jt_$L.jsonl | tee -a $O/ab_jt_l.txt
      done
    done ;;
  obscal)
    cd /tmp
    timeout -k 10 120 $R/profiles/r06/mb_obsread > $O/plain.txt 2>&1 || { cat $O/plain.txt; exit 1; }
    cat $O/plain.txt
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc -o run --output-format csv -- \
      $R/profiles/r06/mb_obsread > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
    echo "FETCH_SIZE per dispatch: python3 profiles/pmc_kernel.py $tag obs_read" ;;
  mb)
    cd /tmp
    for m in mb_lat6 mb_pipe6; do
      timeout -k 10 120 $R/profiles/r06/$m > $O/$m.txt 2>&1 || { tail -5 $O/$m.txt; exit 1; }
      cat $O/$m.txt
    done ;;
  *)
    sed -n 2,25p $0; exit 2 ;;
esac
