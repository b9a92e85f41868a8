set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r05q
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 600 env NIPAMD_LIB=$R/nip_amd/_lib/ab/cksplit.so python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ckpt.py tests/test_gpu_parity.py > gpurun_out/r05q/tests_split.log 2>&1 || { tail -30 gpurun_out/r05q/tests_split.log; exit 1; }
tail -1 gpurun_out/r05q/tests_split.log
bash $R/profiles/r05/ab.sh r05q fb 5 nip_amd/_lib/ab/ckprio3.so nip_amd/_lib/ab/cksplit.so nip_amd/_lib/ab/cksplitprio.so || exit 1
