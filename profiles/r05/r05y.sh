set -o pipefail
# LDS bank-conflict survey: one PMC pass per workload (SQ block only)
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/prof_r05y
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_opchain_estep_wide.py tests/test_gpu_opchain.py tests/test_gpu_opchain_estep.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
cd /tmp
for w in fb config3 estep_config3 config5 estep estep_opchain_wide opchain_wide; do
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES --kernel-trace -d $O/$w -o run --output-format csv -- python3 $R/bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline --no-secondary --detail "" > $O/$w.log 2>&1 || exit 1
  echo "$w done"
done
