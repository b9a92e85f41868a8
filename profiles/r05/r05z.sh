set -o pipefail
# tests + A/B against HEAD + the LDS counters of the opchain workloads
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_r05z
mkdir -p $O
bash $R/profiles/r05/ab.sh r05z estep_opchain_wide 2 nip_amd/_lib/ab/head.so -- tests/test_gpu_opchain_estep_wide.py tests/test_gpu_opchain.py tests/test_gpu_opchain_estep.py || exit 1
bash $R/profiles/r05/ab.sh r05z opchain_wide 2 nip_amd/_lib/ab/head.so || exit 1
cd /tmp && export TMPDIR=/tmp
for w in estep_opchain_wide; do
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES --kernel-trace -d $O/$w -o run --output-format csv -- python3 $R/bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline --no-secondary --detail "" > $O/$w.log 2>&1 || exit 1
done
