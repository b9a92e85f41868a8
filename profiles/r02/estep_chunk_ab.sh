#!/bin/bash
# e_step launch size: sequences per e_step launch (NIPAMD_ESTEP_SEQS build
# flag: 16384 default, 65536, 131072 = the whole config-4 shard at once).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in es64k es128k; do
  NIPAMD_LIB=$PWD/nip_amd/_lib/diag/libnip_amd_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_estep.py tests/test_gpu_em_dist.py -x -q --timeout 200 --timeout-method thread > gpurun_out/esq_parity_$v.log 2>&1 || exit 1
done
for rep in 1 2; do
  for v in base es64k es128k; do
    L=$PWD/nip_amd/_lib/diag/libnip_amd_$v.so; [ $v = base ] && L=$PWD/nip_amd/_lib/libnip_amd.so
    echo "$v" >> gpurun_out/esq_bench.txt
    NIPAMD_LIB=$L timeout -k 10 200 python bench.py --workload estep --steps 5 --warmup 1 --no-cpu-baseline >> gpurun_out/esq_bench.txt 2>&1 || exit 1
  done
done
