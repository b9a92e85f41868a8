set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/prof_r05s/opw
mkdir -p $O
B="$R/bench.py --workload estep_opchain_wide --steps 2 --warmup 1 --no-cpu-baseline --no-secondary --detail ''"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-trace -d $O/pmc1 -o run --output-format csv -- python3 $R/bench.py --workload estep_opchain_wide --steps 2 --warmup 1 --no-cpu-baseline --no-secondary --detail "" > $O/pmc1.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_MFMA --kernel-trace -d $O/pmc2 -o run --output-format csv -- python3 $R/bench.py --workload estep_opchain_wide --steps 2 --warmup 1 --no-cpu-baseline --no-secondary --detail "" > $O/pmc2.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $O/pmc3 -o run --output-format csv -- python3 $R/bench.py --workload estep_opchain_wide --steps 2 --warmup 1 --no-cpu-baseline --no-secondary --detail "" > $O/pmc3.log 2>&1 || exit 1
echo done
