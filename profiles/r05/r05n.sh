set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05n
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_opchain.py tests/test_gpu_opchain_estep_wide.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for w in opchain_wide estep_opchain_wide; do
  timeout -k 10 300 python bench.py --workload $w --steps 5 --warmup 2 --no-secondary --no-cpu-baseline --min-warm 0.5 --detail "" > $O/b_$w.txt 2>&1 || { tail -20 $O/b_$w.txt; exit 1; }
  tail -1 $O/b_$w.txt | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"], d["roofline"]["kernel"])'
done
