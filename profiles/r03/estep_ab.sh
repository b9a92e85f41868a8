#!/bin/bash
# e_step A/B on one box (diagnostics build): the round-2 DPP kernel (dpp8) vs
# chain_estep16_kernel at several phase split points, config 4 shard.
set -o pipefail
export PYTHONPATH=$PWD NIPAMD_LIB=$PWD/nip_amd/_lib/diag/libnip_amd_diag.so
out=gpurun_out/${1:-r03q}_estep_ab.txt
: > $out
for v in dpp8 e16:50 e16:45 e16:40 e16:55 dpp8 e16:50; do
  k=${v%%:*}; h=${v#*:}
  if [ "$k" = dpp8 ]; then export NIPAMD_ESTEP_KERNEL=dpp8; unset NIPAMD_ESTEP_H; else unset NIPAMD_ESTEP_KERNEL; export NIPAMD_ESTEP_H=$h; fi
  r=$(timeout -k 10 120 python bench.py --workload estep --no-secondary --steps 5 2>/dev/null | tail -1) || exit 1
  echo "$v $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel"])')" >> $out
done
