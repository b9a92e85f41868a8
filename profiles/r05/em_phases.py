#!/usr/bin/env python3
"""Where an em_learn iteration's time goes outside the e_step kernels (config
4's shard, 131072 x 1024): each phase of nip_amd/em.py's iteration timed on
the host with a device synchronise after it, the bench's synthetic inputs.

    python profiles/r05/em_phases.py [iterations]
"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import nip_amd  # noqa: E402
from nip_amd import synth  # noqa: E402
from nip_amd import em as nem  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    m = nip_amd.Model.from_spec(*synth.hmm_spec(16, 16))
    ov = [m.variable("M1")]
    obs = torch.from_numpy(synth.observations(131072, 1024, 16, seed=1)).cuda()
    params = synth.uniform01(2024, m.param_size()) + 0.05
    be = nem.GpuEStep()
    rows = []
    for it in range(n):
        torch.cuda.synchronize()
        t = [time.perf_counter()]
        m.m_step(params)
        torch.cuda.synchronize(); t.append(time.perf_counter())
        counts = torch.ones((m.param_size(),), dtype=torch.float64, device="cuda")
        partial, ll, status = be.partial(m, obs, ov)
        t.append(time.perf_counter())                     # launches queued
        torch.cuda.synchronize(); t.append(time.perf_counter())
        partial, lsum, nbad = nem.exchange(partial, ll, status, None)
        torch.cuda.synchronize(); t.append(time.perf_counter())
        be.finalize(m, partial, counts)
        torch.cuda.synchronize(); t.append(time.perf_counter())
        params = counts.cpu().numpy()
        t.append(time.perf_counter())
        rows.append(np.diff(t) * 1e3)
    names = ["m_step", "e_step launch (host)", "e_step (device wait)", "exchange", "finalize", "counts D2H"]
    r = np.array(rows[2:])
    print("em iteration phases (ms; median of %d iterations after 2 warmup):" % len(r))
    for i, nm in enumerate(names):
        print("  %-22s %8.3f" % (nm, float(np.median(r[:, i]))))
    print("  %-22s %8.3f" % ("total", float(np.median(r.sum(axis=1)))))
    # the product iteration as the bench times it, events on the stream
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    ev0.record()
    for _ in range(5):
        params, _, _ = nem.iteration(m, params, obs, ov)
    ev1.record()
    torch.cuda.synchronize()
    print("  nem.iteration (events, mean of 5): %.3f ms" % (ev0.elapsed_time(ev1) / 5))


if __name__ == "__main__":
    main()
