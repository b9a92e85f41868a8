#!/bin/bash
# Kernel-trace every built variant (nip_amd/_lib/variants/*.so and the main
# library): mean duration of the fb kernel and mean gap between back-to-back
# launches, from rocprofv3 --kernel-trace over a short bench run.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for so in $R/nip_amd/_lib/libnip_amd.so $R/nip_amd/_lib/variants/*.so; do
  n=$(basename $so .so)
  rm -rf /tmp/vt_$n
  NIPAMD_LIB=$so timeout -k 10 120 rocprofv3 --kernel-trace -d /tmp/vt_$n -o run --output-format csv -- \
    python3 $R/bench.py --no-cpu-baseline --no-check --steps 12 --warmup 2 > /tmp/vt_$n.log 2>&1 || { echo "$n failed"; continue; }
  python3 - "$n" /tmp/vt_$n <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[2] + "/**/run_kernel_trace.csv", recursive=True)[0]
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(f))
            if "chain_fb_mfma" in r["Kernel_Name"])[2:]
d = [(e - s) / 1e3 for s, e in ks]
g = [(ks[i + 1][0] - ks[i][1]) / 1e3 for i in range(len(ks) - 1)]
print("%-24s kernel %.1f us (min %.1f)  gap %.1f us" % (sys.argv[1], sum(d) / len(d), min(d), sum(g) / max(len(g), 1)))
PY
done
