#!/bin/bash
# Kernel-trace summaries at the final HEAD of the secondary workloads outside
# the default line (joint-interface chain, general engine, operator chains,
# e_step variants, generate_data), with each bench line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash profiles/r04/prof_wl.sh r04f8 "joint jtree opchain opchain_wide estep_opchain estep_demo1 generate" || exit 1
echo done
