#!/usr/bin/env python3
"""Summarise a profiles/collect.sh run into committed files under profiles/.

  python profiles/summarize.py <tag>     (reads gpurun_out/prof_<tag>/)

Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --stats of the bench),
profiles/<tag>_estep_kernel_stats.csv, profiles/<tag>_counters.json, and
profiles/pmc_traffic.json (HBM bytes per launch of the dominant kernel, read
by bench.py).  HBM bytes follow MI355X_MICROARCH.md's HBM section: FETCH_SIZE
and WRITE_SIZE are in KiB; FETCH_SIZE is doubled on gfx950 (it tallies 128-B
requests at 64 B), WRITE_SIZE is taken as is.
"""
import collections
import csv
import json
import os
import shutil
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
KERNEL = "chain_fb_mfma_kernel"


def per_kernel(path, counter):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            agg[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main(tag):
    src = os.path.join(ROOT, "gpurun_out", "prof_" + tag)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"),
                os.path.join(HERE, tag + "_kernel_stats.csv"))
    est = os.path.join(src, "trace_estep", "run_kernel_stats.csv")
    if os.path.exists(est):
        shutil.copy(est, os.path.join(HERE, tag + "_estep_kernel_stats.csv"))
    counters = {}
    for pas in ("pmc1", "pmc2", "pmc3"):
        f = os.path.join(src, pas, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        names = {r["Counter_Name"] for r in csv.DictReader(open(f))}
        for n in names:
            for k, v in per_kernel(f, n).items():
                if KERNEL in k:
                    counters[n] = v
    fetch = counters.get("FETCH_SIZE")
    write = counters.get("WRITE_SIZE")
    with open(os.path.join(HERE, tag + "_counters.json"), "w") as f:
        json.dump({"kernel": KERNEL, "per_launch_mean": counters}, f, indent=1)
    if fetch is not None and write is not None:
        rd = 2 * fetch * 1024
        wr = write * 1024
        d = {"workload": "config2: HMM-shaped DBN, 16 hidden x 16 observed states, B=4096 seq/GPU x T=1024",
             "kernel": KERNEL, "tag": tag,
             "fetch_size_kib": fetch, "write_size_kib": write,
             "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
             "hbm_bytes_per_launch": rd + wr,
             "correction": "FETCH_SIZE x2 (gfx950, MI355X_MICROARCH.md HBM section); KiB -> bytes"}
        with open(os.path.join(HERE, "pmc_traffic.json"), "w") as f:
            json.dump(d, f, indent=1)
        print(json.dumps(d))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "run")
