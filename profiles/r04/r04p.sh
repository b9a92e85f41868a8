#!/bin/bash
# Profile collection part B: config 4 (em iteration and its e_step alone) and
# the config-3 e_step, at HEAD.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash profiles/collect.sh r04p em estep estep_config3
echo done
