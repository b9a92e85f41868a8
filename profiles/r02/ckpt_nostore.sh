#!/bin/bash
# Timing-only build of the checkpoint fb kernel without the posterior stores
# (NIPAMD_CKPT_NO_STORES=1): is phase B bound by the HBM writes?
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
NIPAMD_LIB=$PWD/nip_amd/_lib/diag/libnip_amd_nostore_diag.so NIPAMD_PHASE_TIMES=1 timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-check > gpurun_out/nostore_diag.txt 2>&1 || exit 1
for rep in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline >> gpurun_out/nostore_bench.jsonl 2>&1 || exit 1
  NIPAMD_LIB=$PWD/nip_amd/_lib/diag/libnip_amd_nostore.so timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-check >> gpurun_out/nostore_bench.jsonl 2>&1 || exit 1
done
