#!/bin/bash
# config 3 (chain_mfma_wide_kernel<2>): timing-only ablation builds against the product build.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r03d_mw_ablate.txt
: > $out
for v in prod mw1 mw2 mw3 prod; do
  if [ $v = prod ]; then lib=$PWD/nip_amd/_lib/libnip_amd.so; else lib=$PWD/nip_amd/_lib/diag/libnip_amd_$v.so; fi
  echo -n "$v " >> $out
  NIPAMD_LIB=$lib timeout -k 10 200 python bench.py --workload config3 --steps 5 --warmup 1 --no-cpu-baseline --no-check \
    | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['roofline']['kernel_ms'], d['roofline']['kernel'])" >> $out || exit 1
done
