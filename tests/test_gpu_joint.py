"""Joint-interface chains (compile.cpp build_joint_chain_plan): slices with
several interface variables -- factorial and coupled HMMs -- run as interface
chains over the joint interface state on the matrix-core chain kernels, with
the interface variables' marginals derived from the joint posterior.

Checked against the general join-tree engine (NIPAMD_ENGINE_JTREE, itself
pinned to the reference's own code by test_gpu_jtree.py) on the same inputs,
and against the oracle on a few sequences.  Tolerances as every fb kernel
(DESIGN.md 6): posteriors abs 1e-12, ll rel 1e-12 or both -DBL_MAX."""
import numpy as np
import pytest
import torch

import nip_amd
from nip_amd import synth
from oracle.bind import PortOracle

pytestmark = pytest.mark.gpu

DBL_MAX = np.finfo(np.float64).max
POST_TOL = 1e-12
LL_RTOL = 1e-12


def close_ll(a, b):
    a, b = np.asarray(a), np.asarray(b)
    both_min = (a == -DBL_MAX) & (b == -DBL_MAX)
    return bool(np.all(both_min | (np.abs(a - b) <= LL_RTOL * np.maximum(1.0, np.abs(b)))))


def run(model, obs, ov, q, filt=False):
    o = torch.from_numpy(np.ascontiguousarray(obs, np.int32)).cuda()
    fn = nip_amd.forward_inference if filt else nip_amd.forward_backward_inference
    post, ll, st = fn(model, o, ov, q)
    torch.cuda.synchronize()
    return post.cpu().numpy(), ll.cpu().numpy(), st.cpu().numpy()


def both_engines(model, obs, ov, q, filt=False):
    model.set_engine(nip_amd.ENGINE_CHAIN)
    assert model.gpu_supported(ov, q), "expected a joint-interface chain plan"
    a = run(model, obs, ov, q, filt)
    model.set_engine(nip_amd.ENGINE_JTREE)
    b = run(model, obs, ov, q, filt)
    model.set_engine(nip_amd.ENGINE_AUTO)
    return a, b


def make_obs(rng, B, T, cards, missing=0.2, invalid=0.0):
    cols = []
    for M in cards:
        o = rng.integers(0, M, size=(B, T, 1)).astype(np.int32)
        o[rng.random(o.shape) < missing] = -1
        o[rng.random(o.shape) < invalid] = M          # out of range: zero evidence
        cols.append(o)
    return np.concatenate(cols, axis=2)


CASES = [
    # name, spec, observed, queried
    ("factorial4x4", synth.factorial_spec(4, 4, 16), ["O1"], ["X1"]),
    ("factorial4x3", synth.factorial_spec(4, 3, 5), ["O1"], ["X1", "Y1", "Y0", "X0"]),
    ("coupled", synth.coupled_spec(), ["A1", "B1"], ["Y1", "X1", "A1", "X0"]),
    ("coupled_one_obs", synth.coupled_spec(), ["B1"], ["X1", "A1"]),
    ("factorial_obs_iface", synth.factorial_spec(4, 3, 5), ["O1", "X1"], ["X1", "Y1"]),
    ("factorial8x8", synth.factorial_spec(8, 8, 6), ["O1"], ["Y1"]),
]


@pytest.mark.parametrize("name,spec,osyms,qsyms", CASES, ids=[c[0] for c in CASES])
@pytest.mark.parametrize("T", [1, 2, 37, 300])
def test_joint_chain_equals_general_engine(name, spec, osyms, qsyms, T):
    m = nip_amd.Model.from_spec(*spec)
    ov, q = [m.variable(v) for v in osyms], [m.variable(v) for v in qsyms]
    rng = np.random.default_rng(T * 31 + len(name))
    obs = make_obs(rng, 19, T, [m.card(v) for v in ov])
    for filt in (False, True):
        (pa, la, sa), (pb, lb, sb) = both_engines(m, obs, ov, q, filt)
        assert np.abs(pa - pb).max() <= POST_TOL, (filt, np.abs(pa - pb).max())
        assert close_ll(la, lb)
        assert np.array_equal(sa != 0, sb != 0)


@pytest.mark.parametrize("name,spec,osyms,qsyms", CASES[:3], ids=[c[0] for c in CASES[:3]])
def test_joint_chain_vs_oracle(name, spec, osyms, qsyms):
    m = nip_amd.Model.from_spec(*spec)
    ov, q = [m.variable(v) for v in osyms], [m.variable(v) for v in qsyms]
    rng = np.random.default_rng(7)
    obs = make_obs(rng, 6, 45, [m.card(v) for v in ov])
    obs[0] = -1                                       # a fully missing sequence
    post, ll, st = run(m, obs, ov, q)
    assert not st.any()
    # no evidence anywhere: ll = 0 up to rounding (the matrix-core kernel's m1
    # is alpha . (A s), m2 the sum of alpha's successor -- equal in exact arithmetic)
    assert abs(ll[0]) <= 1e-12
    orc = PortOracle(m.desc())
    for b in range(obs.shape[0]):
        rp, rl = orc.fb(obs[b], ov, q)
        assert np.abs(post[b] - rp).max() <= POST_TOL
        assert close_ll([ll[b]], [rl])


@pytest.mark.parametrize("name,spec,osyms,qsyms", [
    ("factorial4x4", synth.factorial_spec(4, 4, 16), ["O1"], ["X1", "Y1"]),
    ("factorial4x3", synth.factorial_spec(4, 3, 5), ["O1"], ["Y1"]),
    ("coupled_one_obs", synth.coupled_spec(), ["B1"], ["Y1", "X1"]),      # 12 joint states: 4 padding
], ids=["factorial4x4", "factorial4x3", "coupled_one_obs"])
def test_joint_marginals_fused_into_chain_kernel(name, spec, osyms, qsyms):
    """Queries that are all current interface variables: the checkpoint
    kernel writes their marginals itself (chain_ckpt.hip norm_store, no joint
    posterior in HBM).  Bit-identical to the unfused path -- joint posterior,
    then project_kernel -- taken when the request also names a previous-slice
    variable; and against the general engine and the oracle."""
    m = nip_amd.Model.from_spec(*spec)
    ov, q = [m.variable(v) for v in osyms], [m.variable(v) for v in qsyms]
    rng = np.random.default_rng(len(name))
    obs = make_obs(rng, 37, 41, [m.card(v) for v in ov], missing=0.15)
    obs[3, :5] = -1
    post, ll, st = run(m, obs, ov, q)
    assert nip_amd.last_kernel() == "chain_fb_ckpt_kernel<proj>", nip_amd.last_kernel()
    x0 = m.variable(qsyms[0][:-1] + "0")
    post2, ll2, st2 = run(m, obs, ov, q + [x0])
    assert nip_amd.last_kernel() != "chain_fb_ckpt_kernel<proj>"
    w = post.shape[2]
    joint16 = name.startswith("factorial4x4")
    if joint16:        # 16 joint states: the unfused path runs the same kernel, storing the joint
        assert np.array_equal(post, post2[:, :, :w])
        assert np.array_equal(ll, ll2) and np.array_equal(st, st2)
    else:              # fewer: the unfused path is chain_fb_mfma_kernel (16-wide rows only on ckpt)
        assert np.abs(post - post2[:, :, :w]).max() <= POST_TOL
        assert close_ll(ll, ll2) and np.array_equal(st, st2)
    (pa, la, sa), (pb, lb, sb) = both_engines(m, obs, ov, q)
    assert np.array_equal(pa, post)
    assert np.abs(pa - pb).max() <= POST_TOL
    assert close_ll(la, lb)
    orc = PortOracle(m.desc())
    for b in (0, 3, 36):
        rp, rl = orc.fb(obs[b], ov, q)
        assert np.abs(post[b] - rp).max() <= POST_TOL
        assert close_ll([ll[b]], [rl])


def test_joint_chain_zero_mass_and_ragged_batch():
    """Out-of-range codes (an all-zero likelihood) kill a sequence exactly as
    on the general engine; B not a multiple of the kernels' 16-sequence
    blocks and above one launch wave."""
    m = nip_amd.Model.from_spec(*synth.factorial_spec(4, 4, 16))
    ov, q = [m.variable("O1")], [m.variable("X1"), m.variable("Y1")]
    rng = np.random.default_rng(3)
    obs = make_obs(rng, 1000 + 13, 64, [16], missing=0.1, invalid=0.002)
    (pa, la, sa), (pb, lb, sb) = both_engines(m, obs, ov, q)
    assert (sa != 0).any() and (sa == 0).any()
    assert np.array_equal(sa != 0, sb != 0)
    assert close_ll(la, lb)
    assert np.abs(pa - pb).max() <= POST_TOL


def test_joint_chain_scale_properties():
    """The bench slice at a launch-filling batch: normalisation, filter ll ==
    smoothing ll, last filtered step == last smoothed step, spot oracle parity."""
    m = nip_amd.Model.from_spec(*synth.factorial_spec(4, 4, 16))
    ov, q = [m.variable("O1")], [m.variable("X1")]
    B, T = 4096, 256
    obs = synth.observations(B, T, 16, seed=5)
    post, ll, st = run(m, obs, ov, q)
    fpost, fll, _ = run(m, obs, ov, q, filt=True)
    assert not st.any()
    assert np.abs(post.sum(-1) - 1).max() < 1e-12
    assert close_ll(fll, ll)
    assert np.abs(post[:, -1] - fpost[:, -1]).max() < 1e-12
    orc = PortOracle(m.desc())
    for b in (0, 2049, 4095):
        rp, rl = orc.fb(obs[b], ov, q)
        assert np.abs(post[b] - rp).max() <= POST_TOL
        assert close_ll([ll[b]], [rl])


def estep(model, obs, ov):
    o = torch.from_numpy(np.ascontiguousarray(obs, np.int32)).cuda()
    counts, ll, st = nip_amd.e_step(model, o, ov)
    torch.cuda.synchronize()
    return counts.cpu().numpy(), ll.cpu().numpy(), st.cpu().numpy()


ESTEP_CASES = [
    ("factorial4x4", synth.factorial_spec(4, 4, 16), "O1"),
    ("factorial4x3", synth.factorial_spec(4, 3, 5), "O1"),
    ("factorial2x8", synth.factorial_spec(2, 8, 7), "O1"),
]


@pytest.mark.parametrize("name,spec,osym", ESTEP_CASES, ids=[c[0] for c in ESTEP_CASES])
@pytest.mark.parametrize("T", [1, 2, 41])
def test_joint_estep_equals_general_engine(name, spec, osym, T):
    """e_step of a joint-interface chain (the HMM e_step kernel over the joint
    state, counts projected onto every family) against the general engine's
    family sweep on the same inputs, with missing observations: counts rel
    1e-11, ll rel 1e-12."""
    m = nip_amd.Model.from_spec(*spec)
    ov = [m.variable(osym)]
    m.set_engine(nip_amd.ENGINE_CHAIN)
    assert m.estep_supported()
    rng = np.random.default_rng(T + 11)
    obs = make_obs(rng, 23, T, [m.card(ov[0])], missing=0.25)
    ca, la, sa = estep(m, obs, ov)
    m.set_engine(nip_amd.ENGINE_JTREE)
    cb, lb, sb = estep(m, obs, ov)
    m.set_engine(nip_amd.ENGINE_AUTO)
    assert np.array_equal(sa != 0, sb != 0)
    assert close_ll(la, lb)
    assert np.allclose(ca, cb, rtol=1e-11, atol=0), np.abs(ca - cb).max()


def test_joint_estep_vs_oracle():
    """The joint e_step against the oracle's e_step (src/nip.c:1925-1967):
    the round-2 failure (B = 23, T = 41, 25% missing: one sequence off by
    0.058 in Y1 | Y0) and its minimal forms -- a missing step right before
    the last observation, where the step mass is 1.0 up to rounding and the
    kernel's row sums must agree to the bit in every lane."""
    m = nip_amd.Model.from_spec(*synth.factorial_spec(4, 4, 16))
    ov = [m.variable("O1")]
    orc = PortOracle(m.desc())
    rng = np.random.default_rng(52)
    cases = []
    for B, T in ((23, 41), (70, 41), (24, 40)):
        obs = rng.integers(0, 16, size=(B, T, 1)).astype(np.int32)
        obs[rng.random(obs.shape) < 0.25] = -1
        obs[:, 0] = np.maximum(obs[:, 0], 0)
        cases.append(obs)
    cases.append(np.array([[[0], [-1], [13]]], np.int32))
    for obs in cases:
        c, ll, st = estep(m, obs, ov)
        rc, rl, rb = orc.estep(obs, ov, np.ones(m.param_size()))
        assert not rb.any() and not st.any()
        assert close_ll(ll, rl)
        assert np.allclose(c, rc, rtol=1e-11, atol=0), (obs.shape, np.abs(c - rc).max())
    # leading missing runs of every length: the reference's BAD_LUCK verdict
    # (prefix.cpp) flag for flag, parity on the sequences it accepts
    T = 30
    obs = rng.integers(0, 16, size=(T + 1, T, 1)).astype(np.int32)
    for L in range(T + 1):
        obs[L, :L] = -1
    c, ll, st = estep(m, obs, ov)
    rc, rl, rb = orc.estep(obs, ov, np.ones(m.param_size()))
    assert np.array_equal((st & nip_amd.STATUS_BAD_LUCK) != 0, rb != 0)
    ok = rb == 0
    assert close_ll(ll[ok], rl[ok])
    c, _, _ = estep(m, obs[ok], ov)
    rc, _, _ = orc.estep(obs[ok], ov, np.ones(m.param_size()))
    assert np.allclose(c, rc, rtol=1e-11, atol=0), np.abs(c - rc).max()
