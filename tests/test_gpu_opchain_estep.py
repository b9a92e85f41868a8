"""The operator chain's e_step (opchain.cpp op_estep_*, opchain.hip
op_fb_kernel e_step mode + op_xi_kernel): slices outside the chain plan with
a joint interface of <= 16 states train without the general join-tree engine.

The partial holds the per-evidence-combination xi sums; the finalize projects
them onto every family (nip.c:1925-1967, the previous interface's prior
families at t = 0 only) through the enumeration's CSR map.  Checked against
the general engine (NIPAMD_ENGINE_JTREE, itself pinned to the reference's
golden counts by test_gpu_jtree.py), against the oracle's e_step, and for the
partial's exchange properties (shard invariance, route refusal).
Tolerances: counts 1e-11 relative, ll 1e-12 relative or both
-DBL_MAX, BAD_LUCK flags equal."""
import glob
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

import nip_amd
from nip_amd import synth
from nip_amd.em import em_learn, tree_sum
from oracle.bind import PortOracle

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
DBL_MAX = np.finfo(np.float64).max
CNT_RTOL = 1e-11
LL_RTOL = 1e-12


def close_ll(a, b):
    a, b = np.asarray(a), np.asarray(b)
    both = (a == -DBL_MAX) & (b == -DBL_MAX)
    return bool(np.all(both | (np.abs(a - b) <= LL_RTOL * np.maximum(1.0, np.abs(b)))))


def close_cnt(a, b):
    return bool(np.all(np.abs(a - b) <= CNT_RTOL * np.maximum(1.0, np.abs(b))))


def estep(m, obs, ov, engine=nip_amd.ENGINE_AUTO):
    m.set_engine(engine)
    o = torch.from_numpy(np.ascontiguousarray(obs, np.int32)).cuda()
    c, ll, st = nip_amd.e_step(m, o, ov)
    torch.cuda.synchronize()
    k = nip_amd.last_kernel()
    m.set_engine(nip_amd.ENGINE_AUTO)
    return c.cpu().numpy(), ll.cpu().numpy(), st.cpu().numpy(), k


def demo1_hidden(T, B, seed, missing=True):
    """demo1.net with D1 (C1's hidden parent) observed: the chain plan rejects
    it, the operator chain takes it."""
    m = nip_amd.Model.from_net(os.path.join(GOLD, "demo1.net"))
    ov = [m.variable(s) for s in ("A1", "B1", "D1")]
    rng = np.random.default_rng(seed)
    lo = -1 if missing else 0
    obs = np.stack([rng.integers(lo, m.card(v), size=(B, T)) for v in ov], axis=2).astype(np.int32)
    return m, ov, obs


@pytest.mark.parametrize("T", [1, 2, 3, 40, 257])
def test_op_estep_equals_general_engine(T):
    m, ov, obs = demo1_hidden(T, 37, seed=T)
    a = estep(m, obs, ov)
    assert a[3].startswith("op_fb_kernel"), a[3]
    b = estep(m, obs, ov, nip_amd.ENGINE_JTREE)
    assert close_cnt(a[0], b[0]), np.abs(a[0] - b[0]).max()
    assert close_ll(a[1], b[1])
    assert np.array_equal(a[2], b[2])           # the status words, bit for bit


def test_op_estep_vs_oracle():
    m, ov, obs = demo1_hidden(30, 12, seed=4)
    c, ll, st, _ = estep(m, obs, ov)
    rc, rl, rb = PortOracle(m.desc()).estep(obs, ov, np.ones(m.param_size()))
    assert np.array_equal(st != 0, rb != 0)
    assert close_ll(ll, rl)
    assert close_cnt(c, rc), np.abs(c - rc).max()


def test_op_estep_demo1_at_6_states():
    """The opchain bench's model (demo1 @ 6 states, A1 B1 D1 observed:
    343 evidence combinations): op e_step vs the general engine."""
    nodes, pots = synth.demo1_spec(6)
    m = nip_amd.Model.from_spec(nodes, pots)
    ov = [m.variable(s) for s in ("A1", "B1", "D1")]
    rng = np.random.default_rng(6)
    obs = np.stack([rng.integers(-1, 6, size=(70, 64)) for _ in ov], axis=2).astype(np.int32)
    a = estep(m, obs, ov)
    assert a[3].startswith("op_fb_kernel"), a[3]
    b = estep(m, obs, ov, nip_amd.ENGINE_JTREE)
    assert close_cnt(a[0], b[0]), np.abs(a[0] - b[0]).max()
    assert close_ll(a[1], b[1])


def test_op_estep_zero_mass_sequences():
    """Out-of-range observations: zero-likelihood sequences are flagged and
    add nothing, as on the general engine."""
    m, ov, obs = demo1_hidden(20, 33, seed=9)
    obs[3, 5, 0] = m.card(ov[0])
    obs[17, 0, 2] = m.card(ov[2]) + 3
    a = estep(m, obs, ov)
    b = estep(m, obs, ov, nip_amd.ENGINE_JTREE)
    assert np.array_equal(a[2], b[2]) and (a[2] != 0).sum() == 2
    assert set(a[2][a[2] != 0].tolist()) == {3}   # ZERO_MASS | BAD_LUCK, as the general engine's e_step
    assert close_cnt(a[0], b[0])
    assert close_ll(a[1], b[1])


def test_op_partial_shard_invariant_and_refused_with_others():
    """16-sequence groups and power-of-two launch chunks: four 64-sequence
    shards combine into the 256-sequence partial bit for bit; the route tag is
    (-1, -1, -1) per partial, and a sum with another route's partial is
    refused by the finalize."""
    m, ov, obs = demo1_hidden(24, 256, seed=2)
    o = torch.from_numpy(obs).cuda().contiguous()
    whole, _, _ = nip_amd.estep_partial(m, o, ov)
    whole = whole.clone()
    again, _, _ = nip_amd.estep_partial(m, o, ov)
    assert torch.equal(whole, again)
    parts = [nip_amd.estep_partial(m, o[k * 64:(k + 1) * 64].contiguous(), ov)[0].clone() for k in range(4)]
    comb = tree_sum(torch.stack(parts))
    body = m.partial_size() - 3
    assert whole[body:body + 3].tolist() == [-1.0, -1.0, -1.0]
    assert comb[body:body + 3].tolist() == [-4.0, -4.0, -4.0]
    hdr = 1 + 2 * (3 + 8)                     # opchain.cpp kOpHdr: count, 11 request fields and their squares
    assert torch.equal(comb[body + 3 + hdr:], whole[body + 3 + hdr:])    # the xi sums and P0
    c1 = nip_amd.estep_finalize(m, whole, None).cpu().numpy()
    c4 = nip_amd.estep_finalize(m, comb, None).cpu().numpy()
    assert np.array_equal(c1, c4)
    # a general-engine partial of the same request: different layout, refused
    m.set_engine(nip_amd.ENGINE_JTREE)
    g, _, _ = nip_amd.estep_partial(m, o, ov)
    g = g.clone()
    m.set_engine(nip_amd.ENGINE_AUTO)
    mixed = whole.clone()
    mixed[:g.numel()] += g
    with pytest.raises(nip_amd.NipError):
        nip_amd.estep_finalize(m, mixed, None)


def test_plain_partial_api_never_overruns_the_model_level_size():
    """nipamd_estep_partial takes no capacity and promises only
    nipamd_estep_partial_size doubles, so it runs an operator-chain request on
    the general engine (route tag (0, 1, 0)) and writes nothing past that size;
    nipamd_estep_partial_ex with the request's size takes the operator chain,
    and one below the model-level size is refused."""
    import ctypes as C
    m, ov, obs = demo1_hidden(24, 64, seed=12)
    o = torch.from_numpy(obs).cuda().contiguous()
    L = nip_amd.lib()
    base = L.nipamd_estep_partial_size(m._h)
    req = m.partial_size(ov, 24)
    assert req > base
    buf = torch.full((req + 64,), 7.0, dtype=torch.float64, device="cuda")
    ll = torch.empty(64, dtype=torch.float64, device="cuda")
    st = torch.empty(64, dtype=torch.int32, device="cuda")
    ivars = (C.c_int * len(ov))(*ov)
    rc = L.nipamd_estep_partial(m._h, C.c_void_p(o.data_ptr()), len(ov), ivars, 64, 24, C.c_void_p(buf.data_ptr()),
                                C.c_void_p(ll.data_ptr()), C.c_void_p(st.data_ptr()), None)
    torch.cuda.synchronize()
    assert rc == 0
    assert nip_amd.last_kernel().startswith("jt_"), nip_amd.last_kernel()
    assert buf[base - 3:base].tolist() == [0.0, 1.0, 0.0]
    assert bool((buf[base:] == 7.0).all())                     # nothing written past the promised size
    g = nip_amd.estep_finalize(m, buf[:base], None).cpu().numpy()
    a = estep(m, obs, ov)
    assert a[3].startswith("op_fb_kernel")
    assert close_cnt(g, a[0]), np.abs(g - a[0]).max()
    rc = L.nipamd_estep_partial_ex(m._h, C.c_void_p(o.data_ptr()), len(ov), ivars, 64, 24,
                                   C.c_void_p(buf.data_ptr()), base - 1, C.c_void_p(ll.data_ptr()),
                                   C.c_void_p(st.data_ptr()), None)
    assert rc == nip_amd.NIP_ERROR_INVALID_ARGUMENT


def test_op_em_learn_matches_general_engine():
    """em_learn on the operator chain: the learning curve and the learned
    parameters follow the general engine's within the count tolerance."""
    m1, ov, obs = demo1_hidden(48, 64, seed=11)
    # no series starts with an unobserved step: the reference's verdict on
    # leading missing runs (prefix.cpp) is a comparison of masses that sit at
    # equal values, which the two engines' last-bit different parameters can
    # tip either way after a few iterations
    obs[:, 0, 0] = np.maximum(obs[:, 0, 0], 0)
    m2 = nip_amd.Model.from_net(os.path.join(GOLD, "demo1.net"))
    m2.set_engine(nip_amd.ENGINE_JTREE)
    o = torch.from_numpy(obs).cuda()
    c1, c2 = [], []
    # (a threshold of 0 would let a last-bit ll decrease end either run early)
    assert em_learn(m1, o, ov, 1e-9, c1, seed=5, max_iterations=4) == em_learn(m2, o, ov, 1e-9, c2, seed=5,
                                                                              max_iterations=4)
    l1, l2 = np.asarray(c1), np.asarray(c2)
    assert len(l1) == len(l2) > 1 and np.all(np.abs(l1 - l2) <= 1e-10 * np.maximum(1.0, np.abs(l2)))
    assert np.all(np.diff(l1) >= -1e-9 * np.abs(l1[1:]))
    for c in range(nip_amd.lib().nipamd_model_num_cliques(m1._h)):
        assert np.abs(m1.original(c) - m2.original(c)).max() <= 1e-10


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "gen_*.npz"))),
                         ids=lambda p: os.path.basename(p))
def test_op_estep_reference_goldens(path):
    """Random DBNs (make_golden_general.py): where the operator chain takes
    the request, its e_step against the reference's own counts."""
    z = np.load(path)
    nodes, pots = json.loads(str(z["spec"]))
    m = nip_amd.Model.from_spec([tuple(n) for n in nodes], [(c, p, d) for c, p, d in pots])
    ov = list(z["obs_vars"])
    c, ll, st, k = estep(m, z["obs"], ov)
    if not k.startswith("op_fb_kernel"):
        pytest.skip("not on the operator chain: " + k)
    bad = z["estep_bad"] != 0
    assert np.array_equal(st != 0, bad)
    assert close_ll(ll[~bad], z["estep_ll"][~bad])
    if not bad.any():
        assert close_cnt(c, z["counts"]), np.abs(c - z["counts"]).max()
