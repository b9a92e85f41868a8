"""Marginals of every variable of an interface-chain slice on the GPU.

forward_backward_inference / forward_inference return the marginal of each
queried variable from its family clique (src/nip.c:1535-1552, 1273-1290).
The chain kernels compute the interface variable's; the previous-slice copy,
the hidden parents and the leaf children are derived from it on the GPU
(nip_amd/csrc/derive.hip).  Checked against the CPU oracle (bit-identical to
the reference, tests/test_oracle.py) and the reference's own fixture that
queries C1, D1 and A1 of demo1.  Tolerances as test_gpu_parity: 1e-12
absolute on marginals, 1e-12 relative on ll.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

import nip_amd
from nip_amd import synth
from oracle.bind import PortOracle

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
DBL_MAX = np.finfo(np.float64).max


def run(fn, model, obs, ov, q):
    o = torch.from_numpy(np.ascontiguousarray(obs, np.int32)).cuda()
    post, ll, st = fn(model, o, ov, q)
    torch.cuda.synchronize()
    return post.cpu().numpy(), ll.cpu().numpy(), st.cpu().numpy()


def check(m, obs, ov, q, filt, ptol=1e-12, ltol=1e-12):
    fn = nip_amd.forward_inference if filt else nip_amd.forward_backward_inference
    post, ll, st = run(fn, m, obs, ov, q)
    orc = PortOracle(m.desc())
    for b in range(obs.shape[0]):
        rp, rl = orc.fb(obs[b], ov, q, filter_only=filt)
        err = np.abs(post[b] - rp).max()
        assert err <= ptol, "sequence %d: marginal error %g (filter=%s)" % (b, err, filt)
        if rl == -DBL_MAX:
            assert ll[b] == -DBL_MAX and st[b]
        else:
            assert abs(ll[b] - rl) <= ltol * max(1.0, abs(rl)), (b, ll[b], rl)


@pytest.mark.parametrize("filt", [False, True])
def test_hmm_every_variable(filt):
    """P0 (previous slice), P1 and the observed child M1 (missing and
    out-of-range states included); the derived slots before and after P1."""
    nodes, pots = synth.hmm_spec(16, 16, seed=21)
    m = nip_amd.Model.from_spec(nodes, pots)
    rng = np.random.default_rng(5)
    obs = rng.integers(-1, 17, size=(12, 41, 1)).astype(np.int32)
    obs[3, :, 0] = -1
    obs[4] = np.clip(obs[4], 0, 15)
    ov = [m.variable("M1")]
    check(m, obs, ov, [m.variable("P0"), m.variable("P1"), m.variable("M1")], filt)
    check(m, obs, ov, [m.variable("M1"), m.variable("P0")], filt)          # no P1 slot


@pytest.mark.parametrize("filt", [False, True])
def test_model_net_interface_evidence(filt):
    """model.net (zero CPT entries) with P1 observed: M1 is an unobserved
    child, P0 derived; zero-mass sequences give all-zero marginals."""
    m = nip_amd.Model.from_net(os.path.join(GOLD, "model.net"))
    rng = np.random.default_rng(8)
    obs = rng.integers(-1, 3, size=(15, 24, 1)).astype(np.int32)
    check(m, obs, [m.variable("P1")], [m.variable("M1"), m.variable("P0"), m.variable("P1")], filt)


@pytest.mark.parametrize("filt", [False, True])
@pytest.mark.parametrize("card", [4, 32])
def test_demo1_every_variable(filt, card):
    """demo1: the hidden parent D1 (summed into the transition), the previous
    slice C0, the observed A1 and the never-observed B1."""
    m = nip_amd.Model.from_spec(*synth.demo1_spec(card))
    obs = synth.observations(7, 29, card, seed=card)
    obs[:, ::5, 0] = -1
    q = [m.variable(v) for v in ("A1", "B1", "C0", "C1", "D1")]
    check(m, obs, [m.variable("A1")], q, filt, ltol=1e-11)


@pytest.mark.parametrize("filt", [False, True])
def test_wide_clique_two_hidden_parents(filt):
    """Config 5's structure at 8 states: hidden parents Y1 and Z1."""
    m = nip_amd.Model.from_spec(*synth.wide_spec(8, 5))
    obs = synth.observations(6, 23, 5, seed=3)
    q = [m.variable(v) for v in ("X0", "Y1", "Z1", "X1", "O1")]
    check(m, obs, [m.variable("O1")], q, filt)


def test_reference_fixture_demo1():
    """The reference's own forward_backward_inference of demo1 over C1, D1, A1."""
    from test_gpu_estep import product_model
    z = np.load(os.path.join(GOLD, "fb_demo1.npz"))
    m = product_model(str(z["model"]))
    ov, q = [int(v) for v in z["obs_vars"]], [int(v) for v in z["query"]]
    assert m.gpu_supported(ov, q)
    post, ll, st = run(nip_amd.forward_backward_inference, m, z["obs"], ov, q)
    assert np.abs(post - z["post"]).max() <= 1e-12
    for b in range(len(z["ll"])):
        assert abs(ll[b] - z["ll"][b]) <= 1e-12 * max(1.0, abs(z["ll"][b]))
