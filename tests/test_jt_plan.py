"""The general engine's compiled schedule (jtree_plan.cpp), replayed on the
CPU (tests/jt_emul.py) against the reference's outputs and the oracle.

This pins the host planner -- message order, factor placement, projections,
Hugin distribute, interface messages, e_step families -- without a GPU; the
-m gpu tests (test_gpu_jtree.py) run the same schedule in the kernels."""
import glob
import json
import os

import numpy as np
import pytest

import nip_amd
from nip_amd import synth
from jt_emul import Replay
from oracle.bind import PortOracle

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
GEN = sorted(glob.glob(os.path.join(GOLD, "gen_*.npz")))
DBL_MAX = np.finfo(np.float64).max


def gen_model(z):
    nodes, pots = json.loads(str(z["spec"]))
    return nip_amd.Model.from_spec([tuple(n) for n in nodes], [(c, p, d) for c, p, d in pots])


def ll_close(a, b):
    return (a == -DBL_MAX and b == -DBL_MAX) or abs(a - b) <= 1e-12 * max(1.0, abs(b))


@pytest.mark.parametrize("path", GEN, ids=[os.path.basename(p) for p in GEN])
def test_schedule_replay_matches_reference(path):
    z = np.load(path)
    m = gen_model(z)
    r = Replay(m, list(z["obs_vars"]), list(z["query"]))
    for b in range(z["obs"].shape[0]):
        p, l = r.fb(z["obs"][b])
        assert np.abs(p - z["post"][b]).max() <= 1e-12 and ll_close(l, z["ll"][b])
        fp, fl = r.fb(z["obs"][b], filt=True)
        assert np.abs(fp - z["fpost"][b]).max() <= 1e-12 and ll_close(fl, z["fll"][b])


@pytest.mark.parametrize("path", GEN, ids=[os.path.basename(p) for p in GEN])
def test_schedule_replay_estep(path):
    z = np.load(path)
    if z["estep_bad"].any():
        pytest.skip("the reference reports BAD_LUCK for this set")
    m = gen_model(z)
    r = Replay(m, list(z["obs_vars"]), [], estep=True)
    tot = np.ones(m.param_size())
    for b in range(z["obs"].shape[0]):
        slab, l, bad = r.fb(z["obs"][b], estep=True)
        assert not bad and ll_close(l, z["estep_ll"][b])
        tot += slab
    assert np.all(np.abs(tot - z["counts"]) <= 1e-11 * np.maximum(1.0, np.abs(z["counts"])))


@pytest.mark.parametrize("spec,osyms,qsyms", [
    (lambda: synth.hmm_spec(5, 4, seed=3), ["M1"], ["P0", "P1", "M1"]),
    (lambda: synth.demo1_spec(3), ["A1", "B1"], ["C0", "C1", "D1", "A1", "B1"]),
    (lambda: synth.wide_spec(3, 2), ["O1"], ["X0", "Y1", "Z1", "X1", "O1"]),
    (lambda: synth.factorial_spec(3, 2, 4), ["O1"], ["X0", "Y0", "X1", "Y1", "O1"]),
])
def test_schedule_replay_vs_oracle(spec, osyms, qsyms):
    nodes, pots = spec()
    m = nip_amd.Model.from_spec(nodes, pots)
    ov, q = [m.variable(s) for s in osyms], [m.variable(s) for s in qsyms]
    rng = np.random.default_rng(7)
    obs = np.stack([rng.integers(-1, m.card(v), size=9) for v in ov], 1).astype(np.int32)
    r = Replay(m, ov, q)
    orc = PortOracle(m.desc())
    p, l = r.fb(obs)
    rp, rl = orc.fb(obs, ov, q)
    assert np.abs(p - rp).max() <= 1e-12 and ll_close(l, rl)
