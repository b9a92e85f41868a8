set -o pipefail
R=$GRAFT_REPO_ROOT
bash $R/profiles/r05/ab.sh r05o fb 4 nip_amd/_lib/ab/ckprio3.so || exit 1
cd /tmp && export TMPDIR=/tmp && cd $R
mkdir -p gpurun_out/r05o
timeout -k 10 120 env NIPAMD_LIB=$R/nip_amd/_lib/diag/libnip_amd_stamps.so NIPAMD_PHASE_TIMES=1 python bench.py --no-secondary --no-cpu-baseline --steps 1 --warmup 1 --no-check --detail "" > gpurun_out/r05o/stamps_fb.txt 2>&1 || exit 1
grep "nipamd" gpurun_out/r05o/stamps_fb.txt | tail -12
