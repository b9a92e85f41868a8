#!/bin/bash
# Proper-mode e_step: the forward rows rescale every 4th step (the product)
# against every step (ab/fwdsp0.so): the e_step GPU tests (incl. the peaked
# proper model), then interleaved A/B on the em workload, two calls.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04zq
bash profiles/r04/ab_tests.sh r04zq/em em "tests/test_gpu_estep.py tests/test_gpu_em_dist.py tests/test_gpu_joint.py tests/test_gpu_train.py tests/test_gpu_compat.py" nip_amd/_lib/ab/fwdsp0.so || exit 1
grep -q "tests rc=0" gpurun_out/r04zq/em_tests.log || exit 1
bash profiles/r04/ab_tests.sh r04zq/emb em "" nip_amd/_lib/ab/fwdsp0.so || exit 1
echo done
