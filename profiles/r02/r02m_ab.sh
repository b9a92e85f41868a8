#!/bin/bash
# Round-2 pass m: the general engine with its plan staged in LDS (default)
# against the HBM-resident plan (NIPAMD_JT_STAGE=0), and the DPP e_step with
# its off-critical-path row sums on ds_swizzle (NIPAMD_ESTEP_SWZ=1 build in
# nip_amd/_lib/diag) against the default; parity first, then interleaved lines.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="--timeout 150 --timeout-method thread"
timeout -k 10 400 python -u -m pytest tests/test_gpu_jtree.py -x -q $T > gpurun_out/m_jt_tests.log 2>&1 || exit 1
NIPAMD_LIB=$PWD/nip_amd/_lib/diag/libnip_amd_swz.so timeout -k 10 400 python -u -m pytest tests/test_gpu_estep.py -x -q $T > gpurun_out/m_swz_parity.log 2>&1 || exit 1
for rep in 1 2; do
  for st in 1 0; do
    echo "stage=$st" >> gpurun_out/m_jt_bench.txt
    NIPAMD_JT_STAGE=$st timeout -k 10 200 python bench.py --workload jtree --steps 5 --warmup 1 --no-cpu-baseline >> gpurun_out/m_jt_bench.txt 2>&1 || exit 1
  done
  for v in base swz; do
    L=$PWD/nip_amd/_lib/diag/libnip_amd_$v.so; [ $v = base ] && L=$PWD/nip_amd/_lib/libnip_amd.so
    echo "$v" >> gpurun_out/m_estep_bench.txt
    NIPAMD_LIB=$L timeout -k 10 200 python bench.py --workload estep --steps 5 --warmup 1 --no-cpu-baseline >> gpurun_out/m_estep_bench.txt 2>&1 || exit 1
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/m_prof_jt -o run --output-format csv -- \
  python3 bench.py --workload jtree --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/m_prof_jt.log 2>&1 || exit 1
