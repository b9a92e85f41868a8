#!/bin/bash
# config-5 A/B: the wide tests on the product, interleaved config5 lines
# against variants, and the product's diagnostics stamps.   ab_c5.sh TAG VARIANT.so...
set -o pipefail
tag=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$R"
bash $R/profiles/r05/ab.sh $tag config5 4 "$@" -- tests/test_gpu_wide.py || exit 1
NIPAMD_LIB=$R/nip_amd/_lib/diag/libnip_amd_diag.so NIPAMD_PHASE_TIMES=1 timeout -k 10 200 python bench.py --workload config5 --steps 3 --warmup 2 --min-warm 0.3 --no-cpu-baseline --no-secondary --detail "" > $O/c5_stamps.jsonl 2> $O/c5_stamps.err || { tail -5 $O/c5_stamps.err; exit 1; }
grep "wide4" $O/c5_stamps.err | tail -4
