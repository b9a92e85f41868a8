#!/bin/bash
# general engine pass: its tests, then an A/B of the jtree line (staged pools
# vs the round-3 form, NIPAMD_JT_STAGE=0 on the diagnostics build), then c5.
set -o pipefail
tag=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_jtree.py tests/test_gpu_joint.py tests/test_gpu_opchain.py > $O/jt_tests.log 2>&1 || { tail -40 $O/jt_tests.log; exit 1; }
tail -1 $O/jt_tests.log
for rep in 1 2; do
  for v in product stage0; do
    if [ $v = product ]; then env=(); else env=(NIPAMD_LIB=$R/nip_amd/_lib/diag/libnip_amd_diag.so NIPAMD_JT_STAGE=0); fi
    r=$(env "${env[@]}" timeout -k 10 300 python bench.py --workload jtree --no-secondary --no-cpu-baseline --min-warm 0.3 --detail "" 2>$O/err.txt | tail -1) || { tail -5 $O/err.txt; exit 1; }
    echo "$v $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.4f ms  %.4g seq-ts/s  %s" % (d["ms_per_step"], d["value"], d["roofline"]["kernel"]))')" | tee -a $O/ab_jtree.txt
  done
done
bash $R/profiles/r06/c5.sh $tag
