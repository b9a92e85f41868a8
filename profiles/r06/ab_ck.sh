#!/bin/bash
# ck e_step A/B: the ck tests on the product library and on each variant
# (NIPAMD_LIB), then REPS interleaved rounds of the em line.   ab_ck.sh TAG REPS VARIANT.so...
set -o pipefail
tag=$1; reps=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$R"
for lib in product "$@"; do
  if [ "$lib" = product ]; then env=(); else env=(NIPAMD_LIB=$R/$lib); fi
  env "${env[@]}" timeout -k 10 600 python -u -m pytest -x -q --timeout 180 --timeout-method thread -m gpu tests/test_gpu_estep_ck.py > $O/tests_$(basename $lib).log 2>&1 || { echo "tests failed: $lib"; tail -30 $O/tests_$(basename $lib).log; exit 1; }
  echo "$lib: $(tail -1 $O/tests_$(basename $lib).log)"
done
bash $R/profiles/r05/ab.sh $tag em $reps "$@"
