#!/bin/bash
# config 4 em iteration (proper-mode e_step): 16 vs 24 sequences per block
# (diagnostics build, NIPAMD_ESTEP16_SEQS), interleaved twice.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04r; mkdir -p $O
D=$PWD/nip_amd/_lib/diag/libnip_amd_diag.so
for rep in 1 2; do
  for n in 16 24; do
    r=$(env NIPAMD_LIB=$D NIPAMD_ESTEP16_SEQS=$n timeout -k 10 300 python bench.py --workload em --no-secondary --no-cpu-baseline 2>$O/err.txt | tail -1) || { cat $O/err.txt; exit 1; }
    echo "seqs=$n $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.3f ms  kernel %.3f ms  %s" % (d["ms_per_step"], d["roofline"]["kernel_ms"], d["roofline"]["kernel"]))')" >> $O/em_seqs_ab.txt
  done
done
cat $O/em_seqs_ab.txt
