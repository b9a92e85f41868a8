set -o pipefail
# config 2: does the headline's short warmup (3 steps) cost it clock ramp-up? interleaved
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05av
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $R
out=$O/warm.txt; : > $out
for rep in 1 2 3 4; do
  for mw in 0 0.5; do
    r=$(timeout -k 10 200 python bench.py --workload fb --no-secondary --no-cpu-baseline --min-warm $mw --detail "" 2>$O/err.txt | tail -1) || { cat $O/err.txt; exit 1; }
    echo "min_warm=$mw $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.4f ms kernel %.4f warmup %s" % (d["ms_per_step"], d["roofline"]["kernel_ms"], d["warmup"]))')" >> $out
  done
done
cat $out
