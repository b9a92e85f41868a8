#!/bin/bash
# e_step backward rows rescaling by the row's largest exponent (the product)
# against the row sum's (ab/bmx0.so): the e_step GPU tests, then interleaved
# A/B on em and estep.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04zr
bash profiles/r04/ab_tests.sh r04zr/em em "tests/test_gpu_estep.py tests/test_gpu_em_dist.py tests/test_gpu_joint.py tests/test_gpu_train.py tests/test_gpu_compat.py tests/test_gpu_parity.py" nip_amd/_lib/ab/bmx0.so || exit 1
grep -q "tests rc=0" gpurun_out/r04zr/em_tests.log || exit 1
bash profiles/r04/ab_tests.sh r04zr/estep estep "" nip_amd/_lib/ab/bmx0.so || exit 1
bash profiles/r04/ab_tests.sh r04zr/emb em "" nip_amd/_lib/ab/bmx0.so || exit 1
echo done
