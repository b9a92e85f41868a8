#!/bin/bash
# Round-4 final profiles at HEAD (kernel traces + separate PMC passes,
# profiles/collect.sh) of the kernels the store policy changed, then the
# config-2 wave-priority A/B against ab/ckprio0.so once more.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash profiles/collect.sh r04f fb config3 config5 estep_config3 > gpurun_out/r04f_collect.txt 2>&1 || exit 1
mkdir -p gpurun_out/r04f
bash profiles/r04/ab_tests.sh r04f/fb fb "" nip_amd/_lib/ab/ckprio0.so || exit 1
bash profiles/r04/ab_tests.sh r04f/fbb fb "" nip_amd/_lib/ab/ckprio0.so || exit 1
echo done
