#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
NIPAMD_FB_KERNEL=scratch timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_all_scratch.log 2>&1
echo "rc=$?" >> gpurun_out/gpu_all_scratch.log
