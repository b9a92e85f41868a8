set -o pipefail
mkdir -p gpurun_out/r05h
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_opchain_estep_wide.py tests/test_gpu_opchain.py tests/test_gpu_opchain_estep.py tests/test_gpu_em_dist.py tests/test_gpu_train.py tests/test_gpu_estep.py > gpurun_out/r05h/tests.log 2>&1 || { tail -40 gpurun_out/r05h/tests.log; exit 1; }
tail -1 gpurun_out/r05h/tests.log
for w in estep_opchain_wide opchain_wide em; do
  timeout -k 10 300 python bench.py --workload $w --steps 5 --warmup 2 --no-secondary --no-cpu-baseline --min-warm 0.5 --detail "" > gpurun_out/r05h/b_$w.txt 2>&1 || { tail -20 gpurun_out/r05h/b_$w.txt; exit 1; }
  tail -1 gpurun_out/r05h/b_$w.txt | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["config"]["workload"][:60], d["ms_per_step"], d["roofline"]["kernel_ms"], d["roofline"]["kernel"])'
done
