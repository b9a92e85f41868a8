#!/bin/bash
# GPU tests (product library) then an interleaved A/B bench of one workload
# against variant libraries.  Usage: ab_tests.sh TAG WORKLOAD "pytest targets" LIB.so...
set -o pipefail
tag=$1; wl=$2; tests=$3; shift 3
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${tag}_ab.txt
: > $out
if [ -n "$tests" ]; then
  timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu $tests \
    > gpurun_out/${tag}_tests.log 2>&1
  echo "tests rc=$?" >> gpurun_out/${tag}_tests.log
  tail -3 gpurun_out/${tag}_tests.log >> $out
fi
for rep in 1 2; do
  for lib in product "$@"; do
    if [ "$lib" = product ]; then env=(); else env=(NIPAMD_LIB=$PWD/$lib); fi
    r=$(env "${env[@]}" timeout -k 10 180 python bench.py --workload $wl --no-secondary --no-cpu-baseline 2>gpurun_out/${tag}_err.txt | tail -1) || { cat gpurun_out/${tag}_err.txt; exit 1; }
    echo "$lib $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.4f ms  kernel %.4f ms  %s" % (d["ms_per_step"], d["roofline"]["kernel_ms"], d["roofline"]["kernel"]))')" >> $out
  done
done
cat $out
