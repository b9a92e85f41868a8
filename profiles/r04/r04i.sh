#!/bin/bash
# config 5: filter-wave cycle stamps of the HEAD and prefetch builds, then an
# interleaved A/B of the two, with the GPU wide-chain tests on the variant.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04i
for lib in nip_amd/_lib/ab/based.so nip_amd/_lib/ab/r64pfd.so; do
  echo "== $lib" >> gpurun_out/r04i/stamps.txt
  timeout -k 10 120 env NIPAMD_LIB=$PWD/$lib NIPAMD_PHASE_TIMES=1 python bench.py --workload config5 --no-secondary \
    --no-cpu-baseline --steps 1 --warmup 1 --no-check >> gpurun_out/r04i/stamps.txt 2>&1 || exit 1
done
timeout -k 10 300 env NIPAMD_LIB=$PWD/nip_amd/_lib/ab/r64pf.so python -u -m pytest -q -x --timeout 120 --timeout-method thread \
  -m gpu tests/test_gpu_wide.py tests/test_gpu_fold.py tests/test_gpu_filter.py > gpurun_out/r04i/tests.log 2>&1 || exit 1
bash profiles/r04/ab_tests.sh r04i/ab config5 "" nip_amd/_lib/ab/base.so nip_amd/_lib/ab/r64pf.so
