#!/bin/bash
# DPP e_step (chain_kernel<true>) occupancy variants: steps per prefetch chunk
# KC and waves per SIMD W (builds nip_amd/_lib/diag/libnip_amd_es<KC>_<W>.so);
# parity of each on the e_step suite, then interleaved bench lines.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in es4_3 es4_2; do
  NIPAMD_LIB=$PWD/nip_amd/_lib/diag/libnip_amd_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_estep.py -x -q --timeout 200 --timeout-method thread > gpurun_out/occ_parity_$v.log 2>&1 || exit 1
done
for rep in 1 2; do
  for v in base es4_3 es4_2; do
    L=$PWD/nip_amd/_lib/diag/libnip_amd_$v.so; [ $v = base ] && L=$PWD/nip_amd/_lib/libnip_amd.so
    echo "$v" >> gpurun_out/occ_bench.txt
    NIPAMD_LIB=$L timeout -k 10 200 python bench.py --workload estep --steps 5 --warmup 1 --no-cpu-baseline >> gpurun_out/occ_bench.txt 2>&1 || exit 1
  done
done
