#!/usr/bin/env python3
"""Per-dispatch counter values (summed over a dispatch's rows, averaged over
dispatches) of one kernel from pmc_wl.sh output:  pmc_kernel.py TAG KEY"""
import collections, csv, glob, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag, key = sys.argv[1], sys.argv[2]
per = collections.defaultdict(lambda: collections.defaultdict(float))
for f in sorted(glob.glob(os.path.join(ROOT, "gpurun_out", tag, "pmc*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        if key in r["Kernel_Name"]:
            per[r["Counter_Name"]][(f, r["Dispatch_Id"])] += float(r["Counter_Value"])
for c, d in sorted(per.items()):
    v = list(d.values())
    print("%-28s %16.4g  (%d dispatches)" % (c, sum(v) / len(v), len(v)))
