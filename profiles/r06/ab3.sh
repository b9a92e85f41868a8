#!/bin/bash
# fb ckw tests + wide tests on the product, config3 A/B against VL0, config5 A/B.
set -o pipefail
tag=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fb_ckw.py tests/test_gpu_wide.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash $R/profiles/r05/ab.sh $tag config3 3 nip_amd/_lib/ab/vl0.so || exit 1
bash $R/profiles/r05/ab.sh $tag config5 3 nip_amd/_lib/ab/w4old.so || exit 1
