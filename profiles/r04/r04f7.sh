#!/bin/bash
# The default bench line after the warmup change (extra secondary warmup
# agreed across ranks before it runs), and one torchrun-launched N=1 line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04f7
timeout -k 10 400 python bench.py > gpurun_out/r04f7/bench_default.jsonl 2> gpurun_out/r04f7/bench_default.err || exit 1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 1 --steps 10 --warmup 2 > gpurun_out/r04f7/bench_torchrun.jsonl 2> gpurun_out/r04f7/bench_torchrun.err || exit 1
echo done
