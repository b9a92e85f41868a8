"""The e_step's BAD_LUCK verdict on leading missing runs (prefix.cpp) against
the reference.

The reference's e_step (src/nip.c:1827-1854) rejects a series when m1 <= 0,
m2 <= 0 or its running log-likelihood is > 0.  Over a leading run of missing
observations that running sum is pure rounding (0 in exact arithmetic), so it
can land on +1e-16 and the series is rejected.  nip_amd reproduces the
verdict with a host-side restatement of the reference's propagation over such
a run (nipamd_estep_prefix_first_bad: one step index per model version); the
flag kernel applies it per series.  Checked here on the CPU, against
  * the reference's own flags in the committed goldens
    (tests/golden/gen_*.npz, estep_bad, made by make_golden_general.py), and
  * the reference itself (oracle/_ref, or the bit-exact port when the
    reference is not built) on sweeps of the leading-run length L = 0..T,
    on chain and general models, before and after an m_step with random
    parameters (the state of each EM iteration).
Bit-exact: the predicted flag of every series equals the reference's.
"""
import glob
import json
import os

import numpy as np
import pytest

import nip_amd
from nip_amd import synth
from oracle import bind

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
GEN = sorted(glob.glob(os.path.join(GOLD, "gen_*.npz")))


def leading_run(obs):
    miss = (obs < 0).all(axis=2)
    return np.array([int(np.argmin(np.append(m, False))) for m in miss])


def predicted(model, obs):
    k = model.estep_prefix_first_bad(obs.shape[1])
    assert k >= -1
    return (k >= 0) & (leading_run(obs) > k)


@pytest.mark.parametrize("path", GEN, ids=[os.path.basename(p) for p in GEN])
def test_prefix_verdict_matches_golden_flags(path):
    z = np.load(path)
    nodes, pots = json.loads(str(z["spec"]))
    m = nip_amd.Model.from_spec([tuple(n) for n in nodes], [(c, p, d) for c, p, d in pots])
    assert np.array_equal(predicted(m, z["obs"]), z["estep_bad"] != 0)


def oracle_for(nodes, pots, m):
    if bind.ref_available():
        return bind.RefHarness(synth.spec_to_replay(nodes, pots), cards=[n[1] for n in nodes])
    return bind.PortOracle(m.desc())


def gen_spec(name):
    z = np.load(os.path.join(GOLD, name))
    nodes, pots = json.loads(str(z["spec"]))
    return [tuple(n) for n in nodes], [(c, p, d) for c, p, d in pots], [int(v) for v in z["obs_vars"]]


def chain_case(spec, osyms):
    def make():
        nodes, pots = spec()
        names = [n[0] for n in nodes]
        return nodes, pots, [names.index(s) for s in osyms]
    return make


CASES = {
    "hmm6x5": chain_case(lambda: synth.hmm_spec(6, 5, seed=99), ["M1"]),
    "hmm16": chain_case(lambda: synth.hmm_spec(16, 16), ["M1"]),
    "hmm3x4": chain_case(lambda: synth.hmm_spec(3, 4, seed=5), ["M1"]),
    "demo1_4": chain_case(lambda: synth.demo1_spec(4), ["A1", "B1"]),
    "wide_6": chain_case(lambda: synth.wide_spec(6, 4), ["O1"]),
    "coupled": lambda: gen_spec("gen_coupled.npz"),
    "fhmm": lambda: gen_spec("gen_fhmm.npz"),
    "nonleaf": lambda: gen_spec("gen_nonleaf.npz"),
    "rand30": lambda: gen_spec("gen_rand30.npz"),
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_prefix_verdict_matches_reference_sweep(name):
    nodes, pots, ov = CASES[name]()
    m = nip_amd.Model.from_spec(nodes, pots)
    orc = oracle_for(nodes, pots, m)
    cards = [n[1] for n in nodes]
    T = 40
    rng = np.random.default_rng(len(name))
    # one series per leading-run length L = 0..T, observed after the run
    obs = np.stack([rng.integers(0, cards[v], size=(T + 1, T)) for v in ov], axis=2).astype(np.int32)
    for L in range(T + 1):
        obs[L, :L] = -1
    ps = orc.param_size()
    assert ps == m.param_size()
    for it in range(4):
        if it:
            params = rng.random(ps) + 0.05
            orc.m_step(params)
            m.m_step(params)
        _, _, bad = orc.estep(obs, ov, np.ones(ps))
        pred = predicted(m, obs)
        assert np.array_equal(pred, bad != 0), (it, np.nonzero(pred)[0], np.nonzero(bad)[0])


def test_prefix_verdict_independent_of_T():
    """The verdict for a run does not depend on how long the series is: the
    first rejected step is the same for every T beyond it, and none for T at
    or below it."""
    m = nip_amd.Model.from_spec(*synth.hmm_spec(6, 5, seed=99))
    ks = {T: m.estep_prefix_first_bad(T) for T in (1, 2, 3, 5, 8, 40, 200, 5000)}
    first = [k for k in ks.values() if k >= 0]
    if first:
        k0 = min(first)
        for T, k in ks.items():
            assert k == (k0 if T > k0 else -1)


def test_prefix_work_is_bounded_on_a_long_period_chain():
    """A chain whose forward message cycles with a period above the repeat
    check's window never repeats within it: the simulation stops at its work
    bound instead of propagating T steps, and answers -2 (not
    simulated) or a verdict it reached before the bound."""
    import time
    N, M = 40, 3
    nodes = [("P0", N, "P1"), ("P1", N, None), ("M1", M, None)]
    trans = np.zeros((N, N))
    trans[np.arange(N), (np.arange(N) + 1) % N] = 1.0        # P1 = P0 + 1 (mod 40)
    prior = synth.cpt(7, N, 1)
    pots = [("M1", ["P1"], synth.cpt(3, M, N)), ("P1", ["P0"], trans.ravel()), ("P0", [], prior)]
    m = nip_amd.Model.from_spec(nodes, pots)
    t0 = time.time()
    k = m.estep_prefix_first_bad(20_000_000)
    assert time.time() - t0 < 60
    assert k >= -2
    # a short T within the bound is simulated to the end, as before
    k_short = m.estep_prefix_first_bad(200)
    assert k_short >= -1
    if k >= 0:
        assert k_short == (k if k < 200 else -1)


def test_prefix_verdict_on_a_wide_clique_model():
    """Config 5's structure (in-clique card^4 entries) is simulated too (it was
    skipped above 2^20 entries before round 4): at 64 states the reference's
    e_step rejects a series whose leading missing run reaches the step this
    returns.  The 16.7M-entry join tree takes about a second on the host."""
    import time
    m = nip_amd.Model.from_spec(*synth.wide_spec(64, 16))
    t0 = time.time()
    k = m.estep_prefix_first_bad(128)
    assert time.time() - t0 < 30
    assert k >= -1                          # simulated, not skipped (-2)


def test_prefix_verdict_matches_wide64_golden():
    """Config 5's structure at 64 states (16.8M join-tree entries, skipped by
    the simulation before round 4): the predicted BAD_LUCK flags equal the
    reference's own e_step flags on gappy series (tests/golden/
    wide64_prefix.npz, made by make_golden_wide_prefix.py from oracle/_ref)."""
    z = np.load(os.path.join(GOLD, "wide64_prefix.npz"))
    m = nip_amd.Model.from_spec(*synth.wide_spec(64, 16))
    assert np.array_equal(predicted(m, z["obs"]), z["bad"] != 0)
    assert (z["bad"] != 0).any()            # the reference does reject some of them
