#!/bin/bash
# General engine lanes per unit: the factorial-HMM plan at L = 64 (the
# default for cliques > 64 entries) against L = 16 (four sequences per wave);
# the general-engine parity suite at L = 16 first, then interleaved bench lines.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
NIPAMD_JT_L=16 timeout -k 10 400 python -u -m pytest tests/test_gpu_jtree.py -x -q --timeout 150 --timeout-method thread > gpurun_out/n_jt16_tests.log 2>&1 || exit 1
for rep in 1 2; do
  for l in 64 16; do
    echo "L=$l" >> gpurun_out/n_jt_bench.txt
    NIPAMD_JT_L=$l timeout -k 10 200 python bench.py --workload jtree --steps 5 --warmup 1 --no-cpu-baseline >> gpurun_out/n_jt_bench.txt 2>&1 || exit 1
  done
done
