#!/bin/bash
# every e_step / EM GPU test file, then the ck stamps
set -o pipefail
tag=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_estep.py tests/test_gpu_estep_ck.py tests/test_gpu_em_dist.py tests/test_gpu_train.py tests/test_gpu_errors.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash $R/profiles/r06/ck_stamps.sh $tag
