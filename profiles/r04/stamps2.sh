#!/bin/bash
# Per-wave cycle stamps of chain_fb_ckpt_kernel for several stamps builds on
# one box.  Usage: stamps2.sh TAG LIB.so...
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for lib in "$@"; do
  echo "== $lib" >> gpurun_out/${tag}_stamps.txt
  timeout -k 10 120 env NIPAMD_LIB=$PWD/$lib NIPAMD_PHASE_TIMES=1 python bench.py --no-secondary --no-cpu-baseline \
    --steps 1 --warmup 1 --no-check >> gpurun_out/${tag}_stamps.txt 2>&1 || exit 1
done
