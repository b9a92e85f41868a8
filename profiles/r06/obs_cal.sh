#!/bin/bash
# FETCH_SIZE calibration of the e_step's observation reads (mb_obsread.hip)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06z
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 $R/profiles/r06/mb_obsread > $O/plain.txt 2>&1 || { cat $O/plain.txt; exit 1; }
cat $O/plain.txt
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc -o run --output-format csv -- $R/profiles/r06/mb_obsread > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
python3 - <<PY
import csv, glob
f = glob.glob("$O/pmc/**/run_counter_collection.csv", recursive=True) + glob.glob("$O/pmc/run_counter_collection.csv")
tot = {}
for r in csv.DictReader(open(f[0])):
    tot[r["Dispatch_Id"]] = tot.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
for k, v in sorted(tot.items()): print("dispatch", k, "FETCH_SIZE KiB", v, "MiB", v / 1024)
PY
