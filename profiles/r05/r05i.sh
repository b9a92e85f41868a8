set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r05i
bash $R/profiles/r05/ab_env.sh r05i em 3 NIPAMD_EM_PACKED=1 NIPAMD_EM_PACKED=0 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r05i/opw -o run --output-format csv -- \
  python3 $R/bench.py --workload estep_opchain_wide --steps 3 --warmup 1 --no-secondary --no-cpu-baseline --detail "" > $R/gpurun_out/r05i/opw.log 2>&1 || exit 1
echo done
