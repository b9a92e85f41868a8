#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06e
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 600 python -u -m pytest -x -v --timeout 180 --timeout-method thread -m gpu tests/test_gpu_estep_ck.py > $O/ck_tests.log 2>&1
rc=$?
tail -40 $O/ck_tests.log
exit $rc
