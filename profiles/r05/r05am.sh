set -o pipefail
# <= 16 joint states on the wide operator chain (leaf factors, LDS operators): NIPAMD_OP_WIDE=1
# in a diagnostics build, against the narrow kernels (op_fb_kernel / op_xi_sort_kernel)
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05am
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $R
NIPAMD_LIB=$R/nip_amd/_lib/ab/opdiag.so NIPAMD_OP_WIDE=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_opchain.py tests/test_gpu_opchain_estep.py > $O/tests_wide.log 2>&1; echo "wide tests rc=$?" >> $O/tests_wide.log
tail -3 $O/tests_wide.log
out=$O/ab.txt; : > $out
for rep in 1 2; do
  for wl in opchain estep_opchain; do
    for e in 0 1; do
      if [ $e = 1 ]; then ev="NIPAMD_OP_WIDE=1"; else ev="NIPAMD_OP_NARROW=1"; fi
      r=$(env NIPAMD_LIB=$R/nip_amd/_lib/ab/opdiag.so $ev timeout -k 10 200 python bench.py --workload $wl --steps 5 --warmup 2 --no-secondary --no-cpu-baseline --detail "" 2>$O/err.txt | tail -1) || { cat $O/err.txt; exit 1; }
      echo "$wl wide=$e $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.4f ms %s" % (d["ms_per_step"], d["roofline"]["kernel"]))')" >> $out
    done
  done
done
cat $out
