#!/bin/bash
# Last check at HEAD: the operator-chain e_step tests and smoke().
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04f9
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_opchain_estep.py tests/test_gpu_opchain.py \
  > gpurun_out/r04f9/tests.log 2>&1 || { tail -20 gpurun_out/r04f9/tests.log; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04f9/smoke.txt 2>&1 || exit 1
echo done
