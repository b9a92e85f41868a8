set -o pipefail
# op_wide_xi_kernel phase cycles (keys / bitonic sort / staged MFMA sums) and, per wave, the
# batch loop's parts (stamps 1: the loads' latency lands in "accum"; 2: loads waited for on their own)
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05al
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $R
for v in xistamp xistamp2; do
  NIPAMD_LIB=$R/nip_amd/_lib/ab/$v.so timeout -k 10 200 python bench.py --workload estep_opchain_wide --steps 1 --warmup 1 --no-secondary --no-cpu-baseline --detail "" > $O/$v.txt 2>&1 || { tail -5 $O/$v.txt; exit 1; }
  grep "\[xi\]" $O/$v.txt | tail -20
done
