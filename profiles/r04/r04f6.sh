#!/bin/bash
# Round-4 final pass at HEAD (backward rows rescaling by the largest exponent; the proper-mode
# e_step): the whole GPU suite, smoke(), the default bench line, kernel traces
# of configs 2, 3 and 5, and the e_step workloads' PMC passes.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash profiles/r04/full_pass.sh r04f6 || exit 1
grep -q "tests rc=0" gpurun_out/r04f6_gpu_all.txt || exit 1
bash profiles/r04/r04x.sh r04h6 || exit 1
bash profiles/collect.sh r04f6 em estep > gpurun_out/r04f6_collect.txt 2>&1 || exit 1
echo done
