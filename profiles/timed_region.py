#!/usr/bin/env python3
"""Timed-region check of a kernel trace against the bench line of the same run.

    python profiles/timed_region.py TAG DIR WORKLOAD...

DIR/<workload>/ holds one `rocprofv3 --kernel-trace --stats -d ... -o run
--output-format csv -- python3 bench.py --workload W --no-secondary
--no-cpu-baseline [--min-warm S] > trace.log` run (profiles/r05/traces.sh).
For each workload: the bench line (last JSON line of trace.log: steps, warmup,
ms_per_step, roofline.kernel_ms), the trace's kernels in dispatch order, and
the launches of the timed region -- the steps after the warmup steps (the
line's `warmup` count) -- split into the dominant kernel (the line's
roofline.kernel, first name) and every kernel of the step.  Writes
profiles/<TAG>_timed_region.txt; the check is that the dominant kernel's time
per step and every kernel's time per step are <= the line's ms_per_step.
"""
import csv
import glob
import json
import os
import sys


# bench labels (nipamd_last_kernel) whose kernel symbol differs
ALIAS = {"chain_row64_kernel": "chain_wide4_kernel", "chain_fb_ckw_kernel": "chain_estep_ckw_kernel"}


def trace_rows(d):
    f = sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True))
    if not f:
        raise SystemExit("no kernel trace under " + d)
    rows = []
    with open(f[0]) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def bench_line(d):
    with open(os.path.join(d, "trace.log")) as fh:
        lines = [x for x in fh.read().splitlines() if x.startswith("{")]
    return json.loads(lines[-1])


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "").replace("nipamd::", "")
    return n.split("(")[0]


def main():
    tag, base, wls = sys.argv[1], sys.argv[2], sys.argv[3:]
    out = ["# %s: rocprofv3 --kernel-trace --stats of `python3 bench.py --workload W --no-secondary "
           "--no-cpu-baseline` (the secondary workloads with --min-warm 0.5, as the default line warms "
           "them); timed region = the launches of the `steps` steps after the line's `warmup` steps." % tag,
           "# dominant_ms: the dominant kernel's time per timed step; all_ms: every kernel's time per "
           "timed step; both must be <= the line's ms_per_step (events around the steps).",
           "workload  dominant_kernel  launches/step  dominant_ms  all_ms  bench_ms_per_step  bench_kernel_ms  ok"]
    bad = False
    for w in wls:
        d = os.path.join(base, w)
        line = bench_line(d)
        rows = trace_rows(d)
        dom = line["roofline"]["kernel"].split(" + ")[0].split("<")[0].split(" (")[0]
        dom = ALIAS.get(dom, dom)
        steps, warm = int(line["steps"]), int(line["warmup"])
        # the dominant kernel's launches: per step = (total - the 2 launches of
        # the fb line's PCIe-inclusive calls, when present) / (warmup + steps)
        dl = [i for i, r in enumerate(rows) if dom in short(r[2])]
        extra = 2 if "pcie_inclusive" in line else 0
        per = (len(dl) - extra) // (warm + steps)
        if per < 1 or per * (warm + steps) + extra != len(dl):
            out.append("%s  %s  cannot split %d launches into %d warmup + %d timed steps" % (
                w, dom, len(dl), warm, steps))
            bad = True
            continue
        # step s's window: from its first dominant launch to the next step's
        # (every timed window holds one step's kernel mix, rotated); the last
        # one ends at the next dominant launch (the PCIe-inclusive call) or the
        # trace's end.  torch's own kernels (the bench's output checks) excluded.
        lo = dl[warm * per]
        hi = dl[(warm + steps) * per] if (warm + steps) * per < len(dl) else len(rows)
        region = [i for i in range(lo, hi) if "at::" not in rows[i][2]]
        dom_ms = sum(rows[i][1] - rows[i][0] for i in dl[warm * per:(warm + steps) * per]) / steps / 1e6
        all_ms = sum(rows[i][1] - rows[i][0] for i in region) / steps / 1e6
        ok = dom_ms <= line["ms_per_step"] and all_ms <= line["ms_per_step"]
        bad |= not ok
        out.append("%s  %s  %d  %.4f  %.4f  %.4f  %.4f  %s" % (
            w, dom, per, dom_ms, all_ms, line["ms_per_step"], line["roofline"]["kernel_ms"], "yes" if ok else "NO"))
        ds = [(rows[i][1] - rows[i][0]) / 1e6 for i in dl]
        out.append("  dominant launches (ms; warmup | timed | after): " +
                   " ".join("%.4f" % x for x in ds[:warm * per]) + " | " +
                   " ".join("%.4f" % x for x in ds[warm * per:(warm + steps) * per]) + " | " +
                   " ".join("%.4f" % x for x in ds[(warm + steps) * per:]))
        names = {}
        for i in region:
            k = short(rows[i][2])
            names[k] = names.get(k, 0.0) + (rows[i][1] - rows[i][0]) / 1e6 / steps
        out.append("  per timed step (ms): " + ", ".join("%s %.4f" % (k, v) for k, v in sorted(names.items(),
                                                                                             key=lambda x: -x[1])))
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "%s_timed_region.txt" % tag)
    with open(path, "w") as fh:
        fh.write("\n".join(out) + "\n")
    print("\n".join(out))
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
