"""niplikelihood on the GPU (nip_amd/csrc/likelihood.hip) against the
reference's own code (oracle/_ref harness nh_likelihood: the loop of
util/niplikelihood.c:111-133 over the reference's join tree).

Per step: m1 (mass after the unmarked columns' evidence), m2 (after all),
ll = log(m2) - log(m1).  Floating point: 1e-12 relative on m1, m2 and 1e-11
absolute on ll; zero masses give the same non-finite ll.  The
nipamd_likelihood tool prints them with "%g" (6 significant digits).
"""
import os
import re
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
pytest.importorskip("torch")

import nip_amd
from nip_amd import build, synth
from oracle import bind

from test_generate import spec
from test_gpu_tools import write_data

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

CASES = {
    "model": (lambda: spec("model"), ["M1", "P1"]),
    "demo1": (lambda: spec("demo1"), ["A1", "B1", "C1"]),
    "hmm16": (lambda: synth.hmm_spec(16, 16), ["M1"]),
    "demo1_card4": (lambda: synth.demo1_spec(4), ["A1", "B1"]),
    "wide8": (lambda: synth.wide_spec(8, 5), ["O1", "X1"]),
}


def check(got, want):
    m1, m2, ll = got
    assert np.allclose(m1, want[..., 0], rtol=1e-12, atol=0)
    assert np.allclose(m2, want[..., 1], rtol=1e-12, atol=0)
    fin = np.isfinite(want[..., 2])
    assert np.array_equal(np.isfinite(ll), fin)
    assert np.abs(ll[fin] - want[..., 2][fin]).max(initial=0) <= 1e-11
    assert np.array_equal(np.isnan(ll), np.isnan(want[..., 2]))


@pytest.mark.parametrize("name", sorted(CASES))
def test_likelihood_matches_reference(name):
    build_spec, cols = CASES[name]
    nodes, pots = build_spec()
    m = nip_amd.Model.from_spec(nodes, pots)
    ov = [m.variable(c) for c in cols]
    rng = np.random.default_rng(len(name))
    B, T = 6, 11
    obs = np.stack([rng.integers(-1, m.card(v), size=(B, T)) for v in ov], axis=2).astype(np.int32)
    ref = bind.RefHarness(synth.spec_to_replay(nodes, pots))
    for mask in range(1 << len(ov)):
        marked = [(mask >> i) & 1 for i in range(len(ov))]
        got = nip_amd.likelihood(m, obs, ov, marked)
        check(got, ref.likelihood(obs, ov, marked))


def test_likelihood_tool(tmp_path):
    """nipamd_likelihood model.net data P1: p(P1 | M1) per record, ragged series."""
    net = os.path.join(GOLD, "model.net")
    m = nip_amd.Model.from_net(net)
    pn, mn = m.state_names(m.variable("P1")), m.state_names(m.variable("M1"))
    rng = np.random.default_rng(3)
    series = [[[rng.choice(mn + ["null"]), rng.choice(pn)] for _ in range(T)] for T in (5, 9, 5, 1)]
    data = str(tmp_path / "data.txt")
    write_data(data, ["M1", "P1"], series)
    r = subprocess.run([os.path.join(build.LIB_DIR, "nipamd_likelihood"), net, data, "P1"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    blocks = r.stdout.split("\n", 1)[1].split("\n\n")
    nodes, pots = spec("model")
    ref = bind.RefHarness(synth.spec_to_replay(nodes, pots))
    ov = [m.variable("M1"), m.variable("P1")]
    for s, blk in zip(series, blocks):
        obs = np.array([[mn.index(a) if a in mn else -1, pn.index(b)] for a, b in s], np.int32)[None]
        want = ref.likelihood(obs, ov, [0, 1])[0]
        rows = [[float(x) for x in ln.split()] for ln in blk.strip("\n").split("\n")]
        assert len(rows) == len(s)
        for got, w in zip(rows, want):
            for g, x in zip(got, w):
                assert (np.isinf(x) and np.isinf(g) and np.sign(g) == np.sign(x)) or \
                    abs(g - x) <= 1e-5 * abs(x) + 1e-300
