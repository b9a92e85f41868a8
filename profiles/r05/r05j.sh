set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05j
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_opchain_estep_wide.py tests/test_gpu_opchain_estep.py tests/test_gpu_em_dist.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash $R/profiles/r05/ab_env.sh r05j em 3 NIPAMD_EM_PACKED=1 NIPAMD_EM_PACKED=0 || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/opw -o run --output-format csv -- \
  python3 $R/bench.py --workload estep_opchain_wide --steps 3 --warmup 1 --no-secondary --no-cpu-baseline --detail "" > $O/opw.log 2>&1 || exit 1
tail -1 $O/opw.log | cut -c1-200
echo done
