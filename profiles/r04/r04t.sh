#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04t; mkdir -p $O
for w in opchain_wide opchain_wide_jt opchain; do
  timeout -k 10 400 python bench.py --workload $w --no-secondary --no-cpu-baseline > $O/$w.jsonl 2>$O/$w.err || exit 1
done
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_w -o run --output-format csv -- \
  python3 $GRAFT_REPO_ROOT/bench.py --workload opchain_wide --steps 3 --warmup 1 --no-cpu-baseline --no-secondary \
  > $GRAFT_REPO_ROOT/$O/prof_w.log 2>&1
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 env NIPAMD_LIB=$PWD/nip_amd/_lib/ab/b64.so python -u -m pytest -q --timeout 120 --timeout-method thread \
  -m gpu tests/test_gpu_wide.py tests/test_gpu_fold.py > $O/tests_b64.log 2>&1; rc=$?; echo "tests rc=$rc" >> $O/tests_b64.log; [ $rc -le 1 ] || exit 1
bash profiles/r04/ab_tests.sh r04t/c5 config5 "" nip_amd/_lib/ab/b64.so
echo done
