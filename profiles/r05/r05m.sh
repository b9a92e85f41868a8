set -o pipefail
R=$GRAFT_REPO_ROOT
bash $R/profiles/r05/full_pass.sh r05m || exit 1
tail -3 $R/gpurun_out/r05m/gpu_all.txt
bash $R/profiles/r05/traces.sh r05m || exit 1
cat $R/gpurun_out/prof_r05m/timed_region.out | tail -12
