#!/bin/bash
# chain_estep16_kernel with phase B's count cells read one step ahead
# (NIPAMD_E16_PIPE=1, the product) against the pinned read (ab/pipe0.so):
# the e_step GPU tests, then interleaved A/B on the estep and em workloads.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04zp
bash profiles/r04/ab_tests.sh r04zp/estep estep "tests/test_gpu_estep.py tests/test_gpu_em_dist.py tests/test_gpu_joint.py tests/test_gpu_train.py tests/test_gpu_compat.py" nip_amd/_lib/ab/pipe0.so || exit 1
grep -q "tests rc=0" gpurun_out/r04zp/estep_tests.log || exit 1
bash profiles/r04/ab_tests.sh r04zp/em em "" nip_amd/_lib/ab/pipe0.so || exit 1
echo done
