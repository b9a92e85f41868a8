set -o pipefail
# the general join-tree engine (bench jtree): kernel trace + two PMC passes
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/prof_r05ab
mkdir -p $O
A="$R/bench.py --workload jtree --steps 2 --warmup 1 --no-cpu-baseline --no-secondary --detail ''"
timeout -k 10 200 python3 $R/bench.py --workload jtree --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --detail "" > $O/bench.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SMEM --kernel-trace -d $O/pmc1 -o run --output-format csv -- python3 $R/bench.py --workload jtree --steps 2 --warmup 1 --no-cpu-baseline --no-secondary --detail "" > $O/pmc1.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH --kernel-trace -d $O/pmc2 -o run --output-format csv -- python3 $R/bench.py --workload jtree --steps 2 --warmup 1 --no-cpu-baseline --no-secondary --detail "" > $O/pmc2.log 2>&1 || exit 1
echo done
