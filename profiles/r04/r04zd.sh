#!/bin/bash
# Wave priorities on top of the store policy (ab/prioA.so: config 3's partners
# and config 2's partners at s_setprio 1), interleaved A/B, three rounds.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04zd
for wl in config3 fb; do
  bash profiles/r04/ab_tests.sh r04zd/$wl $wl "" nip_amd/_lib/ab/prioA.so || exit 1
  bash profiles/r04/ab_tests.sh r04zd/${wl}b $wl "" nip_amd/_lib/ab/prioA.so || exit 1
done
echo done
