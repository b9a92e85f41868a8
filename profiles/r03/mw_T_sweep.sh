#!/bin/bash
# config 3 kernel time against T (B = 65536): the per-block fixed cost (prologue) vs per-step cost.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r03d_mw_T.txt
: > $out
for T in 8 32 64 128 256; do
  echo -n "T=$T " >> $out
  timeout -k 10 200 python bench.py --workload config3 --T $T --steps 5 --warmup 1 --no-cpu-baseline \
    | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['roofline']['kernel_ms'], d['roofline']['kernel'])" >> $out || exit 1
done
