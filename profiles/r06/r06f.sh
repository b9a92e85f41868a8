#!/bin/bash
# ck e_step: its GPU tests, then the em and estep bench lines (product
# library) and a kernel trace of the em workload.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06f
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 600 python -u -m pytest -x -v --timeout 180 --timeout-method thread -m gpu tests/test_gpu_estep_ck.py > $O/ck_tests.log 2>&1 || { tail -40 $O/ck_tests.log; exit 1; }
tail -3 $O/ck_tests.log
for wl in em estep; do
  timeout -k 10 300 python bench.py --workload $wl --no-secondary --no-cpu-baseline --min-warm 0.5 --detail "" > $O/bench_$wl.jsonl 2>$O/bench_$wl.err || { tail -20 $O/bench_$wl.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/bench_$wl.jsonl').read().strip().splitlines()[-1]); print('$wl', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['kernel'], d['roofline']['frac'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_em -o em -- python bench.py --workload em --no-secondary --no-cpu-baseline --min-warm 0.5 --detail "" > $O/prof_em.log 2>&1 || { tail -20 $O/prof_em.log; exit 1; }
find $O/prof_em -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/em_kernel_stats.csv
head -6 $O/em_kernel_stats.csv | cut -c1-200
