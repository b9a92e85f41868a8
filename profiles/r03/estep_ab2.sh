#!/bin/bash
# e_step A/B (diagnostics build): chain_estep16_kernel at 16 sequences per block
# (two waves per SIMD, KC = 8) vs 24 (three waves per SIMD, KC = 4), config 4 shard.
set -o pipefail
export PYTHONPATH=$PWD NIPAMD_LIB=$PWD/nip_amd/_lib/diag/libnip_amd_diag.so
out=gpurun_out/${1:-r03r}_estep_ab2.txt
: > $out
for v in 16 24 16 24; do
  r=$(NIPAMD_ESTEP16_SEQS=$v timeout -k 10 120 python bench.py --workload estep --no-secondary --steps 5 2>/dev/null | tail -1) || exit 1
  echo "seqs=$v $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel"])')" >> $out
done
