#!/bin/bash
# 16-state e_step: its tests, em A/B against variants, one FETCH/WRITE pass of em.
set -o pipefail
tag=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$R"
bash $R/profiles/r05/ab.sh $tag em 3 "$@" -- tests/test_gpu_estep_ck.py tests/test_gpu_estep.py || exit 1
B="$R/bench.py --workload em --steps 3 --warmup 1 --no-cpu-baseline"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --kernel-trace -d $O/pmc_$c -o run --output-format csv -- python3 $B > $O/pmc_$c.log 2>&1 || { tail -5 $O/pmc_$c.log; exit 1; }
done
python3 $R/profiles/pmc_kernel.py $tag chain_estep_ck_kernel 2>/dev/null || true
