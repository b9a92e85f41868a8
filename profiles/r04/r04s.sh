#!/bin/bash
# The operator chain at 17..64 states (op_wide_*): opchain tests, then the
# general-engine and joint suites the routing change reaches, and a bench
# of a wide operator-chain request.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04s; mkdir -p $O
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_opchain.py \
  > $O/tests_op.log 2>&1; rc=$?; echo "tests rc=$rc" >> $O/tests_op.log; [ $rc -le 1 ] || exit 1
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_jtree.py \
  tests/test_gpu_joint.py tests/test_gpu_opchain_estep.py > $O/tests_more.log 2>&1; rc=$?; echo "tests rc=$rc" >> $O/tests_more.log
echo done
