#!/bin/bash
# 32-state ck e_step pass: its GPU tests and the wide e_step tests, the
# estep_config3 bench line, a kernel trace of it (csv stats).   ckw_pass.sh TAG
set -o pipefail
tag=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 600 python -u -m pytest -x -q --timeout 180 --timeout-method thread -m gpu tests/test_gpu_estep_ckw.py > $O/ckw_tests.log 2>&1 || { tail -60 $O/ckw_tests.log; exit 1; }
tail -1 $O/ckw_tests.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 180 --timeout-method thread -m gpu tests/test_gpu_estep_wide.py > $O/wide_tests.log 2>&1 || { tail -60 $O/wide_tests.log; exit 1; }
tail -1 $O/wide_tests.log
for wl in estep_config3; do
  timeout -k 10 300 python bench.py --workload $wl --no-secondary --no-cpu-baseline --min-warm 0.5 --detail "" > $O/bench_$wl.jsonl 2>$O/bench_$wl.err || { tail -20 $O/bench_$wl.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/bench_$wl.jsonl').read().strip().splitlines()[-1]); print('$wl', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['kernel'], d['roofline']['frac'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --workload estep_config3 --no-secondary --no-cpu-baseline --min-warm 0.5 --detail "" > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp $f $O/kernel_stats.csv; head -4 $O/kernel_stats.csv | cut -c1-220
