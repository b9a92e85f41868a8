#!/usr/bin/env python3
"""Summarise a profiles/collect.sh run into committed files under profiles/.

  python profiles/summarize.py <tag> [--fresh]   (reads gpurun_out/prof_<tag>/<workload>/;
                                                  --fresh: drop the entries of earlier tags)

For every workload collected, writes profiles/<tag>_<workload>_kernel_stats.csv
(rocprofv3 --stats) and profiles/<tag>_<workload>_counters.json, and records in
profiles/pmc_traffic.json the HBM bytes per launch of the workload's dominant
kernel (read by bench.py, keyed by the bench's config.workload string).  HBM
bytes follow MI355X_MICROARCH.md's HBM section: FETCH_SIZE and WRITE_SIZE are
in KiB; FETCH_SIZE is doubled on gfx950 (it tallies 128-B requests at 64 B),
WRITE_SIZE is taken as is.
"""
import collections
import csv
import json
import os
import shutil
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def per_kernel(path, counter):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            agg[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def bench_line(log):
    for line in open(log):
        if line.startswith("{"):
            return json.loads(line)
    return None


def dominant(stats_csv):
    # the runtime's own copy kernels (the PCIe-inclusive leg's H2D / D2H) never count
    rows = [r for r in csv.DictReader(open(stats_csv)) if not r["Name"].startswith("__amd_rocclr")]
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    return rows[0]["Name"]


def main(tag, fresh=False):
    src = os.path.join(ROOT, "gpurun_out", "prof_" + tag)
    tp = os.path.join(HERE, "pmc_traffic.json")
    try:
        table = json.load(open(tp))
        if "entries" not in table or fresh:
            table = {"entries": {}}
    except Exception:
        table = {"entries": {}}
    for w in sorted(os.listdir(src)):
        d = os.path.join(src, w)
        stats = os.path.join(d, "trace", "run_kernel_stats.csv")
        if not os.path.isdir(d) or not os.path.exists(stats):
            continue
        shutil.copy(stats, os.path.join(HERE, "%s_%s_kernel_stats.csv" % (tag, w)))
        kname = dominant(stats)
        rec = bench_line(os.path.join(d, "trace.log"))
        counters = {}
        for pas in ("pmc1", "pmc2", "pmc3", "pmc4"):
            f = os.path.join(d, pas, "run_counter_collection.csv")
            if not os.path.exists(f):
                continue
            for n in {r["Counter_Name"] for r in csv.DictReader(open(f))}:
                for k, v in per_kernel(f, n).items():
                    if k == kname:
                        counters[n] = v
        with open(os.path.join(HERE, "%s_%s_counters.json" % (tag, w)), "w") as f:
            json.dump({"kernel": kname, "per_launch_mean": counters}, f, indent=1)
        fetch, write = counters.get("FETCH_SIZE"), counters.get("WRITE_SIZE")
        if rec and fetch is not None and write is not None:
            rd, wr = 2 * fetch * 1024, write * 1024
            calls = [int(r["Calls"]) for r in csv.DictReader(open(stats)) if r["Name"] == kname][0]
            # e.g. 8 e_step chunks per em step; the PCIe-inclusive leg's two extra
            # calls (fb / config3 / config5 headlines) round away
            per_step = max(1, int(calls / float(rec["steps"] + rec["warmup"])))
            e = {"kernel": kname, "tag": tag, "fetch_size_kib": fetch, "write_size_kib": write,
                 "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
                 "hbm_bytes_per_launch": rd + wr, "launches_per_step": per_step,
                 "hbm_bytes_per_step": (rd + wr) * per_step,
                 "counters_per_launch": {k: v for k, v in counters.items()
                                         if k not in ("FETCH_SIZE", "WRITE_SIZE")},
                 "correction": "FETCH_SIZE x2 (gfx950, MI355X_MICROARCH.md HBM section); KiB -> bytes"}
            # every kernel of the step (e.g. the wide e_step's messages and
            # statistics kernels), the runtime's copies excepted
            allk = 0.0
            f2 = os.path.join(d, "pmc2", "run_counter_collection.csv")
            f3 = os.path.join(d, "pmc3", "run_counter_collection.csv")
            if os.path.exists(f2) and os.path.exists(f3):
                fr = [r for r in csv.DictReader(open(f2)) if r["Counter_Name"] == "FETCH_SIZE"]
                wrr = [r for r in csv.DictReader(open(f3)) if r["Counter_Name"] == "WRITE_SIZE"]
                n_disp = len({r["Dispatch_Id"] for r in fr if not r["Kernel_Name"].startswith("__amd")})
                tot = sum(2 * float(r["Counter_Value"]) * 1024 for r in fr if not r["Kernel_Name"].startswith("__amd"))
                tot += sum(float(r["Counter_Value"]) * 1024 for r in wrr if not r["Kernel_Name"].startswith("__amd"))
                steps = float(rec["steps"] + rec["warmup"])
                allk = tot / steps
                e["all_kernels_hbm_bytes_per_step"] = allk
                e["all_kernels_dispatches_per_step"] = n_disp / steps
            avg_ns = [float(r["AverageNs"]) for r in csv.DictReader(open(stats)) if r["Name"] == kname][0]
            e["kernel_avg_ns"] = avg_ns
            g = counters.get("GRBM_GUI_ACTIVE")
            if g:
                # GRBM_GUI_ACTIVE sums the 8 XCDs' busy cycles (MI355X_MICROARCH.md, DVFS note)
                e["effective_clock_ghz"] = g / 8.0 / avg_ns
            table["entries"][rec["config"]["workload"]] = e
            print(w, json.dumps(e))
    with open(tp, "w") as f:
        json.dump(table, f, indent=1)


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    main(args[0] if args else "run", fresh="--fresh" in sys.argv)
