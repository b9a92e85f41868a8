"""GPU parity: the gfx950 path (through the C-ABI) against the CPU oracle.

The oracle (oracle/nip_oracle.c) is bit-identical to the reference's own code
(tests/test_oracle.py); here the GPU results must agree with it within the
fp64 tolerance stated in DESIGN.md:
    posteriors  |gpu - ref| <= 1e-12 (absolute)
    ll          |gpu - ref| <= 1e-12 * max(1, |ref|), or both -DBL_MAX
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

import nip_amd
from nip_amd import synth
from oracle.bind import PortOracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
POST_TOL = 1e-12
LL_RTOL = 1e-12
DBL_MAX = np.finfo(np.float64).max


def gpu_fb(model, obs, obs_vars, query):
    o = torch.from_numpy(np.ascontiguousarray(obs, np.int32)).cuda()
    post, ll, st = nip_amd.forward_backward_inference(model, o, obs_vars, query)
    torch.cuda.synchronize()
    return post.cpu().numpy(), ll.cpu().numpy(), st.cpu().numpy()


def check(model, obs, obs_vars, query):
    post, ll, st = gpu_fb(model, obs, obs_vars, query)
    orc = PortOracle(model.desc())
    for b in range(obs.shape[0]):
        rp, rl = orc.fb(obs[b], obs_vars, query)
        err = np.abs(post[b] - rp).max()
        assert err <= POST_TOL, "sequence %d: posterior error %g" % (b, err)
        if rl == -DBL_MAX:
            assert ll[b] == -DBL_MAX and (st[b] & nip_amd.STATUS_ZERO_MASS)
        else:
            assert abs(ll[b] - rl) <= LL_RTOL * max(1.0, abs(rl)), (b, ll[b], rl)
            assert not (st[b] & nip_amd.STATUS_ZERO_MASS)


@pytest.mark.parametrize("N,M,B,T", [
    (16, 16, 9, 64), (16, 16, 8, 1), (16, 16, 8, 2), (16, 16, 3, 3),
    (4, 5, 13, 33), (7, 3, 17, 17), (2, 2, 1, 5), (16, 8, 24, 128),
])
def test_hmm_synthetic(N, M, B, T):
    nodes, pots = synth.hmm_spec(N, M, seed=100 + N * 7 + M)
    m = nip_amd.Model.from_spec(nodes, pots)
    obs = synth.observations(B, T, M, seed=T * 31 + B)
    check(m, obs, [m.variable("M1")], [m.variable("P1")])


def test_missing_and_invalid_observations():
    nodes, pots = synth.hmm_spec(16, 16, seed=5)
    m = nip_amd.Model.from_spec(nodes, pots)
    rng = np.random.default_rng(3)
    obs = rng.integers(-1, 17, size=(11, 40, 1)).astype(np.int32)   # -1 missing, 16 invalid
    obs[0, :, 0] = -1                                                 # all missing
    check(m, obs, [m.variable("M1")], [m.variable("P1")])


def test_model_net_zero_mass():
    """examples model has zero CPT entries: random data hits m2 == 0."""
    m = nip_amd.Model.from_net(os.path.join(ROOT, "tests", "golden", "model.net"))
    rng = np.random.default_rng(7)
    obs = rng.integers(-1, 5, size=(21, 24, 1)).astype(np.int32)
    check(m, obs, [m.variable("M1")], [m.variable("P1")])


def test_long_sequences_register_prefetch():
    """T = 2000: the observation codes leave no LDS room for the phase-B
    LDS-DMA buffers, so the matrix-core kernel prefetches into registers."""
    nodes, pots = synth.hmm_spec(16, 16, seed=11)
    m = nip_amd.Model.from_spec(nodes, pots)
    obs = synth.observations(18, 2000, 16, seed=9)
    check(m, obs, [m.variable("M1")], [m.variable("P1")])


def near_identity(n, eps):
    d = np.full((n, n), eps)
    np.fill_diagonal(d, 1.0)
    return (d / d.sum(axis=1, keepdims=True)).ravel()


def test_peaked_model_rescaling():
    """Near-identity transition (1e-50 off the diagonal) and emission (1e-60):
    random data makes every step's evidence mass about 1e-50, so the filters'
    sparse rescaling (every 4th step in phase A) runs at 1e-200 between
    rescales.  Results must still match the reference's per-step normalisation."""
    N = 16
    nodes = [("P0", N, "P1"), ("P1", N, None), ("M1", N, None)]
    pots = [("M1", ["P1"], near_identity(N, 1e-60)),
            ("P1", ["P0"], near_identity(N, 1e-50)),
            ("P0", [], np.full(N, 1.0 / N))]
    m = nip_amd.Model.from_spec(nodes, pots)
    obs = synth.observations(19, 77, N, seed=4)
    check(m, obs, [m.variable("M1")], [m.variable("P1")])


def test_large_batch_properties():
    """Config-2 scale: posteriors normalised, ll finite and <= 0, spot parity."""
    nodes, pots = synth.hmm_spec(16, 16)
    m = nip_amd.Model.from_spec(nodes, pots)
    B, T = 4096, 1024
    obs = synth.observations(B, T, 16, seed=1)
    post, ll, st = gpu_fb(m, obs, [m.variable("M1")], [m.variable("P1")])
    assert np.abs(post.sum(-1) - 1).max() < 1e-12
    assert np.all(np.isfinite(ll)) and np.all(ll < 0) and not st.any()
    orc = PortOracle(m.desc())
    for b in (0, 1, 2047, 4095):
        rp, rl = orc.fb(obs[b], [m.variable("M1")], [m.variable("P1")])
        assert np.abs(post[b] - rp).max() <= POST_TOL
        assert abs(ll[b] - rl) <= LL_RTOL * abs(rl)


def test_config2_all_sequences_vs_textbook():
    """Config 2 in full (4096 x 1024, the bench's batch and seed): every
    sequence's posteriors (abs 1e-12) and ll (rel 1e-12) against the textbook
    smoother in torch fp64 on the same GPU (tests/textbook_util.py
    smoother_torch, pinned to the reference by test_oracle_textbook.py)."""
    import torch
    from textbook_util import chain_tables, smoother_torch
    nodes, pots = synth.hmm_spec(16, 16)
    m = nip_amd.Model.from_spec(nodes, pots)
    B, T = 4096, 1024
    obs = synth.observations(B, T, 16, seed=1)
    post, ll, st = gpu_fb(m, obs, [m.variable("M1")], [m.variable("P1")])
    assert not st.any()
    A, pi, Es = chain_tables(m, m.variable("P0"), m.variable("P1"), [m.variable("M1")])
    tA, tpi, tE = (torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in (A, pi, Es[0]))
    tobs = torch.from_numpy(obs[:, :, 0].astype(np.int64)).cuda()
    wp, wl = smoother_torch(tA, tpi, [tE], [tobs])
    assert np.abs(post - wp.cpu().numpy()).max() <= POST_TOL
    wl = wl.cpu().numpy()
    assert np.all(np.abs(ll - wl) <= LL_RTOL * np.abs(wl)), np.abs(ll - wl).max()
