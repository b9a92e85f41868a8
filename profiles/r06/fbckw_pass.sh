#!/bin/bash
# fb ckw pass: its tests and the wide fb tests, the config3 (fb) and
# estep_config3 lines, an A/B of the e_step against variant libraries.
#   fbckw_pass.sh TAG [VARIANT.so...]
set -o pipefail
tag=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$R"
for t in test_gpu_fb_ckw test_gpu_wide test_gpu_estep_ckw; do
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/$t.py > $O/$t.log 2>&1 || { tail -60 $O/$t.log; exit 1; }
  echo "$t: $(tail -1 $O/$t.log)"
done
for wl in config3 estep_config3; do
  timeout -k 10 300 python bench.py --workload $wl --no-secondary --no-cpu-baseline --min-warm 0.5 --detail "" > $O/bench_$wl.jsonl 2>$O/bench_$wl.err || { tail -20 $O/bench_$wl.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/bench_$wl.jsonl').read().strip().splitlines()[-1]); print('$wl', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['kernel'], d['roofline']['frac'])"
done
if [ $# -gt 0 ]; then bash $R/profiles/r05/ab.sh $tag estep_config3 3 "$@"; fi
