#!/usr/bin/env python3
"""Golden e_step of config 5's structure (the wide clique, 64
states, O1 at 16) on gappy series, from the reference's own code (oracle/_ref).

Run in the build container (about 2 minutes: the reference propagates the
16.7M-entry in-clique per slice):  python tests/golden/make_golden_wide_prefix.py

Output tests/golden/wide64_prefix.npz:
  obs      int32 [B, T, 1]: series 0..T with leading missing runs of length
           L = 0..T, one with a missing step in the middle
  ll, bad  the reference's e_step per-series ll and BAD_LUCK flags
  idx, cnt the e_step counts of the accepted series (bad == 0): every count outside the big family X1 | X0 Y1 Z1 and a
           fixed random sample of 8192 of its 16.8M entries (big_off,
           big_len locate it); cnt_sum = the sum of all counts
Pins nipamd_estep_prefix_first_bad above 2^20 entries (simulated since
round 4) and the GPU chain e_step at 64 states (tests/test_gpu_estep_wide.py).
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from nip_amd import synth  # noqa: E402  (synthetic spec generator only)
from oracle import bind  # noqa: E402


def main():
    assert bind.ref_available(), "build oracle/_ref first"
    nodes, pots = synth.wide_spec(64, 16)
    orc = bind.RefHarness(synth.spec_to_replay(nodes, pots), cards=[n[1] for n in nodes])
    T = 4
    rng = np.random.default_rng(2024)
    obs = rng.integers(0, 16, size=(T + 2, T, 1)).astype(np.int32)
    for L in range(T + 1):
        obs[L, :L] = -1
    obs[T + 1, 2] = -1
    ps = orc.param_size()
    _, ll, bad = orc.estep(obs, [4], np.ones(ps))
    cnt, _, bad_ok = orc.estep(obs[bad == 0], [4], np.ones(ps))     # counts of the accepted series
    assert not bad_ok.any()
    # em_learn layout: one block per variable in declaration order (X0, Y1, Z1
    # priors, X1 | X0 Y1 Z1, O1 | X1), card x prod(parent cards) each
    big_off, big_len = 3 * 64, 64 ** 4
    assert ps == big_off + big_len + 16 * 64
    idx = np.sort(rng.choice(big_len, size=8192, replace=False)) + big_off
    idx = np.concatenate([np.arange(big_off), idx, np.arange(big_off + big_len, ps)])
    out = dict(obs=obs, ll=ll, bad=bad, idx=idx, cnt=cnt[idx], cnt_sum=np.array(cnt.sum()),
               big_off=np.array(big_off), big_len=np.array(big_len))
    np.savez_compressed(os.path.join(HERE, "wide64_prefix.npz"), **out)
    print("bad", bad, "ll", ll)


if __name__ == "__main__":
    main()
