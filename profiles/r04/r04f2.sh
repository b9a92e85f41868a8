#!/bin/bash
# Round-4 final pass at HEAD: the whole GPU suite, smoke(), the default bench
# line, then kernel traces of configs 2, 3 and 5 with the bench's own steps.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash profiles/r04/full_pass.sh r04f2 || exit 1
grep -q "tests rc=0" gpurun_out/r04f2_gpu_all.txt || exit 1
bash profiles/r04/r04x.sh r04g || exit 1
echo done
