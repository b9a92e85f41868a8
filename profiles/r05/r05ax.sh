set -o pipefail
# config 2: the warm-up length (3 steps + up to 64 untimed = ~16 ms, against 300 and 2000 steps)
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05ax
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $R
out=$O/warm_len.txt; : > $out
for rep in 1 2 3; do
  for w in 3 300 2000; do
    r=$(timeout -k 10 200 python bench.py --workload fb --no-secondary --no-cpu-baseline --warmup $w --detail "" 2>$O/err.txt | tail -1) || { cat $O/err.txt; exit 1; }
    echo "W=$w $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.4f ms kernel %.4f warmup %s" % (d["ms_per_step"], d["roofline"]["kernel_ms"], d["warmup"]))')" >> $out
  done
done
cat $out
