#!/bin/bash
# At the final HEAD: the e_step's per-wave phase stamps (stamps build) for the
# em iterations (proper mode, sparse forward rescaling) and the estep shard,
# then three back-to-back default bench lines on one box (run-to-run spread).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04f5; mkdir -p $O
for w in em estep; do
  timeout -k 10 300 env NIPAMD_LIB=$PWD/nip_amd/_lib/ab/stamps.so NIPAMD_PHASE_TIMES=1 python bench.py --workload $w \
    --steps 1 --warmup 1 --no-secondary --no-cpu-baseline --no-check > $O/stamps_$w.txt 2>&1 || exit 1
done
for i in 1 2 3; do
  timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench_$i.jsonl 2> $O/bench_$i.err || exit 1
done
echo done
