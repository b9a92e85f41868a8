#!/usr/bin/env python3
"""CPU baselines for bench.py's cpu_baseline leg -- MEASUREMENT INFRASTRUCTURE,
the checker's code, never the product (oracle/__init__.py).

Times the reference's own compiled code (oracle/_ref/libnipref.so: the
reference's nippotential / nipjointree / ... sources compiled unmodified, with
nip.c's time loops restated in oracle/ref/nipref_harness.c) on the bench's
synthetic workloads, one process per granted core: the reference keeps global
state (SURVEY 8(b) Threading), so it scales over processes, not threads, as a
user of util/nipinference.c:125-132 or util/niptrain.c:151 would run it.  The
C port (oracle/nip_oracle.c) is timed the same way as a secondary figure.

bench.py runs this as a child process BEFORE its own process touches the GPU
(this process makes no device call: nip_amd is used only for its host-side
join-tree compiler, to describe the model to the port), then reads one JSON
object per workload from stdout:

    python oracle/cpu_bench.py --procs 16 --budget 8 fb config3 em config5
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import platform
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from nip_amd import synth  # noqa: E402  (numpy only)
from oracle import bind  # noqa: E402

# workload -> (spec, observed, query, T of the sample, kind, sequences to draw,
# observation seeds as bench.py draws them on rank 0 (column i: 1 + 104729 i))
WORKLOADS = {
    "fb": (lambda: synth.hmm_spec(16, 16), ["M1"], "P1", 1024, "fb", 4096),
    "config3": (lambda: synth.demo1_spec(32), ["A1", "B1"], "C1", 256, "fb", 512),
    "em": (lambda: synth.hmm_spec(16, 16), ["M1"], "P1", 1024, "estep", 4096),
    "estep_config3": (lambda: synth.demo1_spec(32), ["A1", "B1"], "C1", 256, "estep", 512),
    # config 5: the 16.7M-entry clique makes a slice cost seconds: two slices
    # per sequence (the first two of each bench sequence)
    "config5": (lambda: synth.wide_spec(64, 16), ["O1"], "X1", 2, "fb", 64),
}


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def sample_obs(name, n):
    spec, ov, _, T, _, _ = WORKLOADS[name]
    nodes, _ = spec()
    card = {s: c for s, c, _ in nodes}
    full_T = {"fb": 1024, "config3": 256, "em": 1024, "config5": 128, "estep_config3": 256}[name]
    cols = [synth.observations(n, full_T, card[v], seed=1 + 104729 * i) for i, v in enumerate(ov)]
    return np.ascontiguousarray(np.concatenate(cols, axis=2)[:, :T])


_ORC = {}


def _worker(name, p, procs, budget, obs, barrier, out):
    """One process (forked after the parent built the model, so every process
    holds its own copy of the reference's global state): wait for every
    process, then run sequences p, p + procs, ... until the budget is spent
    (at least one)."""
    _, ov, q, T, kind, _ = WORKLOADS[name]
    orc, ps = _ORC["orc"], _ORC["ps"]
    barrier.wait()
    t0 = time.perf_counter()
    k, units = p, 0
    while k < obs.shape[0]:
        if kind == "estep":
            orc.estep(obs[k:k + 1], ov, np.ones(ps))
        else:
            orc.fb(obs[k], ov, [q])
        units += T
        k += procs
        if time.perf_counter() - t0 >= budget:
            break
    out.put((p, units, time.perf_counter() - t0))


def run(which, name, procs, budget, desc=None):
    spec, ov_names, q_name, T, kind, n = WORKLOADS[name]
    obs = sample_obs(name, n)
    nodes, pots = spec()
    if which == "reference":
        orc = bind.RefHarness(synth.spec_to_replay(nodes, pots), cards=[x[1] for x in nodes])
    else:
        orc = bind.PortOracle(desc)
    _ORC.update(orc=orc, ps=orc.param_size() if kind == "estep" else 0)
    names = [x[0] for x in nodes]
    wl = (spec, [names.index(v) for v in ov_names], names.index(q_name), T, kind, n)
    WORKLOADS[name + "#idx"] = wl
    ctx = mp.get_context("fork")
    barrier = ctx.Barrier(procs)
    out = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(name + "#idx", p, procs, budget, obs, barrier, out))
          for p in range(procs)]
    for x in ps:
        x.start()
    res = [out.get() for _ in ps]
    for x in ps:
        x.join()
    _ORC.clear()
    del orc
    units = sum(r[1] for r in res)
    wall = max(r[2] for r in res)
    seqs = units // T
    what = "e_step" if kind == "estep" else "fwd-bwd + ll"
    # oracle/_ref: the reference's nippotential.c, nipjointree.c, ... compiled
    # unmodified, nip.c's time loop restated in oracle/ref/nipref_harness.c
    code = "oracle/_ref (reference sources, gcc -O2)" if which == "reference" else "oracle/nip_oracle.c (gcc -O2)"
    return {"value": units / wall, "unit": "sequence-timesteps/s", "cores": procs,
            "kind": which if which == "reference" else "port",
            "sample": "%d seq x T=%d of the bench inputs%s, %s, %s, %d procs, %.1f s" % (
                seqs, T, "" if name != "config5" else " (first slices)", what, code, procs, wall)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=16)
    ap.add_argument("--budget", type=float, default=8.0)
    ap.add_argument("--no-port", action="store_true")
    ap.add_argument("workloads", nargs="*", default=["fb", "config3", "em", "config5"])
    a = ap.parse_args()
    have_ref = bind.ref_available()
    for name in a.workloads:
        rec = {"workload": name, "cpu_model": cpu_model(), "host_cpus": os.cpu_count()}
        try:
            if have_ref:
                rec["reference"] = run("reference", name, a.procs, a.budget)
            if not a.no_port:
                # the port needs the compiled join-tree description: nip_amd's host
                # compiler (no device work; loaded here, not in bench.py's process)
                import nip_amd
                nodes, pots = WORKLOADS[name][0]()
                rec["port"] = run("port", name, a.procs, a.budget / 2,
                                  desc=nip_amd.Model.from_spec(nodes, pots).desc())
        except Exception as e:  # a baseline must never take the bench down
            rec["error"] = "%s: %s" % (type(e).__name__, str(e)[:300])
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
