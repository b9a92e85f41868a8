#!/bin/bash
# per-group stamps of chain_estep_ck_kernel (diagnostics library, NIPAMD_PHASE_TIMES)
set -o pipefail
tag=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$R"
NIPAMD_LIB=$R/nip_amd/_lib/diag/libnip_amd_diag.so NIPAMD_PHASE_TIMES=1 timeout -k 10 300 python bench.py --workload estep --steps 3 --warmup 1 --min-warm 0 --no-secondary --no-cpu-baseline --detail "" > $O/stamps.jsonl 2> $O/stamps.err || { tail -20 $O/stamps.err; exit 1; }
grep estep_ck $O/stamps.err | tail -4
