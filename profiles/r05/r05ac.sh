set -o pipefail
# general engine: lanes per unit (NIPAMD_JT_L, diagnostics build) on the jtree workload
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05ac
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $R
out=$O/jt_L.txt; : > $out
for rep in 1 2; do
  for L in 64 32 16; do
    r=$(NIPAMD_LIB=$R/nip_amd/_lib/ab/diag.so NIPAMD_JT_L=$L timeout -k 10 200 python bench.py --workload jtree --steps 3 --warmup 1 --no-secondary --no-cpu-baseline --detail "" 2>$O/err.txt | tail -1) || { cat $O/err.txt; exit 1; }
    echo "L=$L $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.4f ms" % d["ms_per_step"])')" >> $out
  done
done
cat $out
