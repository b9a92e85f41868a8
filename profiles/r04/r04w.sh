#!/bin/bash
# Final-candidate pass at HEAD: the whole GPU suite, smoke(), the default
# bench line; then A/B of configs 2, 3 and 5 against the build before the
# 64-bit lane-swap copies (ab/pre.so); the microbenchmark.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash profiles/r04/full_pass.sh r04w || exit 1
O=gpurun_out/r04w; mkdir -p $O
grep -q "tests rc=0" gpurun_out/r04w_gpu_all.txt || exit 1
bash profiles/r04/ab_tests.sh r04w/c2 fb "" nip_amd/_lib/ab/pre.so || exit 1
bash profiles/r04/ab_tests.sh r04w/c3 config3 "" nip_amd/_lib/ab/pre.so || exit 1
bash profiles/r04/ab_tests.sh r04w/c5 config5 "" nip_amd/_lib/ab/pre.so || exit 1
timeout -k 10 60 ./profiles/r04/mb_r64 > $O/mb_r64.txt 2>&1
echo done
