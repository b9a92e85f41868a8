# config 5's filter step alone (NIPAMD_R64_SOLO timing builds under nip_amd/_lib/var/<variant>/)
# against the diagnostics build: bash profiles/r06/solo_config5.sh TAG (VARIANTS="base solo ...")
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r06as}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$R"
for v in ${VARIANTS:-base solo base solo}; do
  if [ $v = base ]; then L=$R/nip_amd/_lib/diag/libnip_amd_diag.so; else L=$R/nip_amd/_lib/var/$v/libnip_amd_diag.so; fi
  NIPAMD_LIB=$L NIPAMD_PHASE_TIMES=1 timeout -k 10 300 python bench.py --workload config5 --steps 3 --warmup 2 --min-warm 0.3 --no-check \
    --no-secondary --no-cpu-baseline --detail "" > $O/$v.jsonl 2> $O/$v.err || { tail -20 $O/$v.err; exit 1; }
  echo "== $v"; grep "\[nipamd\]" $O/$v.err | tail -2
done
