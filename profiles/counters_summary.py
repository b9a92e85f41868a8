#!/usr/bin/env python3
"""Mean per-launch counter values of the fb kernel from profiles/counters.sh output."""
import collections, csv, glob, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1]
key = sys.argv[2] if len(sys.argv) > 2 else "chain_"
agg = collections.defaultdict(list)
for f in glob.glob(os.path.join(ROOT, "gpurun_out", "cnt_" + tag, "p*", "run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if key in r["Kernel_Name"] and "tree64" not in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {k: sum(v) / len(v) for k, v in sorted(agg.items())}
print(json.dumps(out, indent=1))
