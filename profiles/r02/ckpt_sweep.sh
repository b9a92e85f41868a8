#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest tests/test_gpu_ckpt.py -q --timeout 300 --timeout-method thread > gpurun_out/ckpt_sweep.log 2>&1
