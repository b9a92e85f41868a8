"""GPU parity of the general join-tree engine (jtree.hip, jtree_plan.cpp).

Slices outside the interface-chain plan -- several interface variables
(factorial HMM, coupled chains, random DBNs), evidence on a hidden parent or
on a non-leaf variable, slices without any interface -- against the
reference's own outputs (tests/golden/gen_*.npz, make_golden_general.py) and
the CPU oracle; and the interface-chain models run through the general
engine (NIPAMD_ENGINE_JTREE) against the same references, so both GPU
engines are checked on one footing.  Tolerances:
    posteriors  |gpu - ref| <= 1e-12 (absolute)
    ll          |gpu - ref| <= 1e-12 * max(1, |ref|), or both -DBL_MAX
    counts      |gpu - ref| <= 1e-11 * max(1, |ref|)
"""
import glob
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

import nip_amd
from nip_amd import synth
from nip_amd.em import em_learn, NIP_NO_ERROR, NIP_ERROR_BAD_LUCK
from oracle.bind import PortOracle
from em_util import check_em_curve

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
GEN = sorted(glob.glob(os.path.join(GOLD, "gen_*.npz")))
POST_TOL = 1e-12
LL_RTOL = 1e-12
CNT_RTOL = 1e-11
DBL_MAX = np.finfo(np.float64).max


def gen_model(z):
    nodes, pots = json.loads(str(z["spec"]))
    return nip_amd.Model.from_spec([tuple(n) for n in nodes], [(c, p, d) for c, p, d in pots])


def close_ll(a, b):
    a, b = np.asarray(a), np.asarray(b)
    both_min = (a == -DBL_MAX) & (b == -DBL_MAX)
    ok = np.abs(a - b) <= LL_RTOL * np.maximum(1.0, np.abs(b))
    return bool(np.all(both_min | ok))


def run(model, obs, ov, q, filt=False):
    o = torch.from_numpy(np.ascontiguousarray(obs, np.int32)).cuda()
    fn = nip_amd.forward_inference if filt else nip_amd.forward_backward_inference
    post, ll, st = fn(model, o, ov, q)
    torch.cuda.synchronize()
    return post.cpu().numpy(), ll.cpu().numpy(), st.cpu().numpy()


@pytest.mark.parametrize("path", GEN, ids=[os.path.basename(p) for p in GEN])
def test_general_slice_matches_reference(path):
    z = np.load(path)
    m = gen_model(z)
    ov, q = list(z["obs_vars"]), list(z["query"])
    post, ll, st = run(m, z["obs"], ov, q)
    assert np.abs(post - z["post"]).max() <= POST_TOL
    assert close_ll(ll, z["ll"])
    assert np.array_equal((st & nip_amd.STATUS_ZERO_MASS) != 0, z["ll"] == -DBL_MAX)
    fpost, fll, _ = run(m, z["obs"], ov, q, filt=True)
    assert np.abs(fpost - z["fpost"]).max() <= POST_TOL
    assert close_ll(fll, z["fll"])


@pytest.mark.parametrize("path", GEN, ids=[os.path.basename(p) for p in GEN])
def test_general_slice_matches_reference_on_general_engine(path):
    """The same fixtures with the general engine forced: slices with several
    interface variables otherwise run as joint-interface chains
    (test_gpu_joint.py), so this keeps the general engine's own coverage."""
    z = np.load(path)
    m = gen_model(z)
    m.set_engine(nip_amd.ENGINE_JTREE)
    ov, q = list(z["obs_vars"]), list(z["query"])
    post, ll, st = run(m, z["obs"], ov, q)
    assert np.abs(post - z["post"]).max() <= POST_TOL
    assert close_ll(ll, z["ll"])
    fpost, fll, _ = run(m, z["obs"], ov, q, filt=True)
    assert np.abs(fpost - z["fpost"]).max() <= POST_TOL
    assert close_ll(fll, z["fll"])


@pytest.mark.parametrize("path", GEN, ids=[os.path.basename(p) for p in GEN])
def test_general_estep_matches_reference(path):
    z = np.load(path)
    m = gen_model(z)
    ov = list(z["obs_vars"])
    o = torch.from_numpy(np.ascontiguousarray(z["obs"], np.int32)).cuda()
    cnt, ll, st = nip_amd.e_step(m, o, ov)
    cnt, ll, st = cnt.cpu().numpy(), ll.cpu().numpy(), st.cpu().numpy()
    bad = z["estep_bad"] != 0
    # flag for flag, including the verdict on leading missing runs (prefix.cpp)
    assert np.array_equal(st != 0, bad)
    assert close_ll(ll[~bad], z["estep_ll"][~bad])
    if not bad.any():
        assert close_ll(ll, z["estep_ll"])
        assert np.all(np.abs(cnt - z["counts"]) <= CNT_RTOL * np.maximum(1.0, np.abs(z["counts"])))


@pytest.mark.parametrize("path", GEN, ids=[os.path.basename(p) for p in GEN])
def test_general_em_learn_curve(path):
    z = np.load(path)
    m = gen_model(z)
    obs = torch.from_numpy(np.ascontiguousarray(z["obs"])).cuda()
    curve = []
    rc = em_learn(m, obs, list(z["obs_vars"]), 1e-6, curve, init=z["em_init"], max_iterations=8)
    check_em_curve(z, rc, curve, 1e-10)


CHAIN_CASES = [
    ("hmm16", lambda: synth.hmm_spec(16, 16), ["M1"], ["P0", "P1", "M1"], 9, 40),
    ("hmm4x5", lambda: synth.hmm_spec(4, 5, seed=77), ["M1"], ["P1"], 13, 33),
    ("demo1_4", lambda: synth.demo1_spec(4), ["A1", "B1"], ["C1", "D1", "C0"], 7, 21),
    ("demo1_16", lambda: synth.demo1_spec(16), ["A1", "B1"], ["C1"], 5, 12),
    ("wide_6", lambda: synth.wide_spec(6, 4), ["O1"], ["X1", "Y1"], 4, 9),
]


@pytest.mark.parametrize("name,spec,osyms,qsyms,B,T", CHAIN_CASES, ids=[c[0] for c in CHAIN_CASES])
def test_chain_models_through_general_engine(name, spec, osyms, qsyms, B, T):
    nodes, pots = spec()
    m = nip_amd.Model.from_spec(nodes, pots)
    ov, q = [m.variable(s) for s in osyms], [m.variable(s) for s in qsyms]
    rng = np.random.default_rng(len(name) * 7 + B)
    obs = np.stack([rng.integers(0, m.card(v), size=(B, T)) for v in ov], 2).astype(np.int32)
    obs[rng.random(obs.shape) < 0.1] = -1
    m.set_engine(nip_amd.ENGINE_JTREE)
    post, ll, st = run(m, obs, ov, q)
    fpost, fll, _ = run(m, obs, ov, q, filt=True)
    orc = PortOracle(m.desc())
    for b in range(B):
        rp, rl = orc.fb(obs[b], ov, q)
        assert np.abs(post[b] - rp).max() <= POST_TOL
        assert close_ll([ll[b]], [rl])
        fp, fl = orc.fb(obs[b], ov, q, filter_only=True)
        assert np.abs(fpost[b] - fp).max() <= POST_TOL
        assert close_ll([fll[b]], [fl])
    # and the chain kernels agree with it
    m.set_engine(nip_amd.ENGINE_AUTO)
    post2, ll2, _ = run(m, obs, ov, q)
    assert np.abs(post2 - post).max() <= POST_TOL and close_ll(ll2, ll)


def test_estep_general_engine_equals_chain_kernel():
    nodes, pots = synth.hmm_spec(16, 16, seed=3)
    m = nip_amd.Model.from_spec(nodes, pots)
    obs = torch.from_numpy(synth.observations(64, 50, 16, seed=9)).cuda()
    ov = [m.variable("M1")]
    c1, l1, s1 = nip_amd.e_step(m, obs, ov)
    m.set_engine(nip_amd.ENGINE_JTREE)
    c2, l2, s2 = nip_amd.e_step(m, obs, ov)
    c1, c2 = c1.cpu().numpy(), c2.cpu().numpy()
    assert np.all(np.abs(c1 - c2) <= CNT_RTOL * np.maximum(1.0, np.abs(c1)))
    assert close_ll(l1.cpu().numpy(), l2.cpu().numpy())
    assert not s1.any().item() and not s2.any().item()


@pytest.mark.parametrize("T", [48, 50, 3])
def test_general_estep_partial_shard_invariant(T):
    """The general engine's posterior sweep runs one unit per (sequence, time
    chunk) with a slab row each; the chunk count depends on T only, so four
    64-sequence shards combine into the 256-sequence batch bit for bit --
    T = 50 leaves a short last chunk (ceil(50 / 4) = 13 units per sequence)."""
    m = nip_amd.Model.from_spec(*synth.hmm_spec(16, 16, seed=4))
    m.set_engine(nip_amd.ENGINE_JTREE)
    obs = torch.from_numpy(synth.observations(256, T, 16, seed=T)).cuda().contiguous()
    ov = [m.variable("M1")]
    whole, _, _ = nip_amd.estep_partial(m, obs, ov)
    whole = whole.clone()
    again, _, _ = nip_amd.estep_partial(m, obs, ov)
    assert torch.equal(whole, again)
    parts = [nip_amd.estep_partial(m, obs[k * 64:(k + 1) * 64].contiguous(), ov)[0].clone() for k in range(4)]
    x = torch.stack(parts)
    comb = (x[0] + x[1]) + (x[2] + x[3])
    assert torch.equal(comb[:-3], whole[:-3])
    assert comb[-3:].tolist() == [0.0, 4.0, 0.0]
    # and the counts match the chain kernel's (a different summation order)
    m.set_engine(nip_amd.ENGINE_AUTO)
    c1, _, _ = nip_amd.e_step(m, obs, ov)
    m.set_engine(nip_amd.ENGINE_JTREE)
    c2, _, _ = nip_amd.e_step(m, obs, ov)
    c1, c2 = c1.cpu().numpy(), c2.cpu().numpy()
    assert np.all(np.abs(c1 - c2) <= CNT_RTOL * np.maximum(1.0, np.abs(c1)))


def test_zero_probability_data_general_engine():
    """model.net has zero CPT entries: impossible data -> ll = -DBL_MAX."""
    m = nip_amd.Model.from_net(os.path.join(GOLD, "model.net"))
    m.set_engine(nip_amd.ENGINE_JTREE)
    z = np.load(os.path.join(GOLD, "fb_model_T24.npz"))
    post, ll, st = run(m, z["obs"], list(z["obs_vars"]), list(z["query"]))
    assert np.abs(post - z["post"]).max() <= POST_TOL
    assert close_ll(ll, z["ll"])


@pytest.mark.parametrize("case", ["config2_T65536", "demo1_32_T8192"])
def test_long_sequences_no_T_cap(case):
    """No sequence-length cap: the chain kernels stage codes in LDS, so long
    sequences fall through to the next kernel and finally to the general
    engine (streamed codes); parity with the oracle on a few sequences."""
    if case == "config2_T65536":
        nodes, pots = synth.hmm_spec(16, 16)
        osyms, q, B, T = ["M1"], "P1", 2, 65536
    else:
        nodes, pots = synth.demo1_spec(32)
        osyms, q, B, T = ["A1", "B1"], "C1", 1, 8192
    m = nip_amd.Model.from_spec(nodes, pots)
    ov, qv = [m.variable(s) for s in osyms], [m.variable(q)]
    obs = np.concatenate([synth.observations(B, T, m.card(v), seed=5 + i) for i, v in enumerate(ov)], 2)
    post, ll, st = run(m, obs, ov, qv)
    assert not st.any()
    orc = PortOracle(m.desc())
    for b in range(B):
        rp, rl = orc.fb(obs[b], ov, qv)
        assert np.abs(post[b] - rp).max() <= POST_TOL
        assert close_ll([ll[b]], [rl])


def test_general_batch_scale_properties():
    """A factorial HMM (16-state joint interface) at a batch that spans many
    launch waves and a posterior chunking over time: normalisation, filter
    ll == smoothing ll, last filtered step == last smoothed step, spot parity."""
    nodes, pots = synth.factorial_spec(4, 4, 6)
    m = nip_amd.Model.from_spec(nodes, pots)
    ov, q = [m.variable("O1")], [m.variable("X1"), m.variable("Y1")]
    B, T = 3000, 200
    obs = synth.observations(B, T, 6, seed=2)
    post, ll, st = run(m, obs, ov, q)
    fpost, fll, _ = run(m, obs, ov, q, filt=True)
    assert not st.any()
    assert np.abs(post[:, :, :4].sum(-1) - 1).max() < 1e-12
    assert np.abs(post[:, :, 4:].sum(-1) - 1).max() < 1e-12
    assert close_ll(fll, ll)
    assert np.abs(post[:, -1] - fpost[:, -1]).max() < 1e-12
    orc = PortOracle(m.desc())
    for b in (0, 1234, 2999):
        rp, rl = orc.fb(obs[b], ov, q)
        assert np.abs(post[b] - rp).max() <= POST_TOL
        assert close_ll([ll[b]], [rl])
