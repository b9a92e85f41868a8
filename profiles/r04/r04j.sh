#!/bin/bash
# Worktree build: wide/filter/estep GPU tests, config-5 stamps, A/B of
# config 5 and the config-3 e_step against HEAD's build (ab/base.so).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04j; mkdir -p $O
timeout -k 10 600 python -u -m pytest -q -x --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_wide.py tests/test_gpu_filter.py tests/test_gpu_estep_wide.py tests/test_gpu_estep.py \
  > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc" >> $O/tests.log; [ $rc -eq 0 ] || exit 1
# the operator chain's e_step (new) and everything its route change reaches:
# every failure reported (no -x); assertion failures (rc 1) do not stop the run
timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_opchain_estep.py tests/test_gpu_opchain.py tests/test_gpu_jtree.py tests/test_gpu_joint.py \
  > $O/tests_op.log 2>&1; rc=$?; echo "tests rc=$rc" >> $O/tests_op.log; [ $rc -le 1 ] || exit 1
timeout -k 10 120 env NIPAMD_LIB=$PWD/nip_amd/_lib/diag/libnip_amd_diag.so NIPAMD_PHASE_TIMES=1 python bench.py --workload config5 \
  --no-secondary --no-cpu-baseline --steps 1 --warmup 1 --no-check > $O/stamps.txt 2>&1 || exit 1
bash profiles/r04/ab_tests.sh r04j/c5 config5 "" nip_amd/_lib/ab/base.so || exit 1
bash profiles/r04/ab_tests.sh r04j/e3 estep_config3 "" nip_amd/_lib/ab/base.so || exit 1
bash profiles/r04/ab_tests.sh r04j/e4 estep "" nip_amd/_lib/ab/base.so || exit 1
cd /tmp && timeout -k 10 200 python3 $GRAFT_REPO_ROOT/bench.py --workload estep_opchain --no-secondary --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/estep_opchain.jsonl 2>&1
