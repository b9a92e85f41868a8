#!/bin/bash
# ckw tests (product), A/B of estep_config3 and config3 against variants,
# config-5 filter stamps on the diagnostics build.   ab2.sh TAG VARIANT.so...
set -o pipefail
tag=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_estep_ckw.py tests/test_gpu_fb_ckw.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash $R/profiles/r05/ab.sh $tag estep_config3 3 "$@" || exit 1
bash $R/profiles/r05/ab.sh $tag config3 3 "$@" || exit 1
NIPAMD_LIB=$R/nip_amd/_lib/diag/libnip_amd_diag.so NIPAMD_PHASE_TIMES=1 timeout -k 10 200 python bench.py --workload config5 --steps 3 --warmup 2 --min-warm 0 --no-cpu-baseline --no-secondary --detail "" > $O/c5_stamps.jsonl 2> $O/c5_stamps.err || { tail -5 $O/c5_stamps.err; exit 1; }
grep "wide4 cycles" $O/c5_stamps.err | tail -3
