#!/bin/bash
# Round-4 final pass at HEAD (e_step count cells read one step ahead, the
# secondary lines' settled warmup): the whole GPU suite, smoke(), the default
# bench line, kernel traces of configs 2, 3 and 5, and the e_step workloads'
# PMC passes (profiles/collect.sh).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash profiles/r04/full_pass.sh r04f3 || exit 1
grep -q "tests rc=0" gpurun_out/r04f3_gpu_all.txt || exit 1
bash profiles/r04/r04x.sh r04h2 || exit 1
bash profiles/collect.sh r04f3 em estep > gpurun_out/r04f3_collect.txt 2>&1 || exit 1
echo done
