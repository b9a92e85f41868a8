set -o pipefail
# general engine: register cap (waves per SIMD) x lanes per unit, diagnostics builds
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05ae
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $R
out=$O/jt_wpe.txt; : > $out
for rep in 1 2; do
  for W in 1 6 8; do
    for L in 64 32; do
      r=$(NIPAMD_LIB=$R/nip_amd/_lib/ab/jtw$W.so NIPAMD_JT_L=$L timeout -k 10 200 python bench.py --workload jtree --steps 3 --warmup 1 --no-secondary --no-cpu-baseline --detail "" 2>$O/err.txt | tail -1) || { cat $O/err.txt; exit 1; }
      echo "W=$W L=$L $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.4f ms" % d["ms_per_step"])')" >> $out
    done
  done
done
cat $out
