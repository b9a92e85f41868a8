"""The evidence-indexed interface chain (opchain.cpp / opchain.hip): slices the
interface-chain plan rejects -- evidence on a hidden parent (demo1 with D1
observed), evidence on non-leaf variables, random DBNs -- run as a chain over
the joint interface with one K x K operator per evidence combination.

Checked against the general join-tree engine (NIPAMD_ENGINE_JTREE, pinned to
the reference's own outputs by test_gpu_jtree.py), against the reference's
golden posteriors where the golden queries the interface, and the oracle.
Tolerances as every fb path: posteriors abs 1e-12, ll rel 1e-12
or both -DBL_MAX."""
import glob
import json
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
POST_TOL = 1e-12
LL_RTOL = 1e-12


def close_ll(a, b):
    a, b = np.asarray(a), np.asarray(b)
    both = (a == -DBL_MAX) & (b == -DBL_MAX)
    return bool(np.all(both | (np.abs(a - b) <= LL_RTOL * np.maximum(1.0, np.abs(b)))))


def run(m, obs, ov, q, filt=False, engine=nip_amd.ENGINE_AUTO):
    m.set_engine(engine)
    o = torch.from_numpy(np.ascontiguousarray(obs, np.int32)).cuda()
    fn = nip_amd.forward_inference if filt else nip_amd.forward_backward_inference
    post, ll, st = fn(m, o, ov, q)
    torch.cuda.synchronize()
    k = nip_amd.last_kernel()
    m.set_engine(nip_amd.ENGINE_AUTO)
    return post.cpu().numpy(), ll.cpu().numpy(), st.cpu().numpy(), k


def gen_model(z):
    nodes, pots = json.loads(str(z["spec"]))
    return nip_amd.Model.from_spec([tuple(n) for n in nodes], [(c, p, d) for c, p, d in pots])


def both(m, obs, ov, q, filt=False):
    a = run(m, obs, ov, q, filt)
    assert a[3] == "op_fb_kernel", a[3]
    b = run(m, obs, ov, q, filt, nip_amd.ENGINE_JTREE)
    assert np.abs(a[0] - b[0]).max() <= POST_TOL, np.abs(a[0] - b[0]).max()
    assert close_ll(a[1], b[1])
    assert np.array_equal(a[2] != 0, b[2] != 0)
    return a


@pytest.mark.parametrize("T", [1, 2, 3, 40, 257])
def test_demo1_with_hidden_parent_evidence(T):
    """demo1.net with D1 (C1's hidden parent) observed: not an interface chain
    for the chain plan (evidence on a summed-out parent); here a chain whose
    transition follows D1's state."""
    m = nip_amd.Model.from_net(os.path.join(GOLD, "demo1.net"))
    ov = [m.variable(s) for s in ("A1", "B1", "D1")]
    q = [m.variable("C1")]
    rng = np.random.default_rng(T)
    obs = np.stack([rng.integers(-1, m.card(v), size=(21, T)) for v in ov], axis=2).astype(np.int32)
    for filt in (False, True):
        post, ll, st, _ = both(m, obs, ov, q, filt)
        assert not st.any()
        assert np.abs(post.sum(-1) - 1).max() < 1e-12
    orc = PortOracle(m.desc())
    post, ll, _, _ = run(m, obs, ov, q)
    for b in (0, 7, 20):
        rp, rl = orc.fb(obs[b], ov, q)
        assert np.abs(post[b] - rp).max() <= POST_TOL
        assert close_ll([ll[b]], [rl])


def test_zero_mass_and_ragged_batch():
    """Out-of-range states (an all-zero likelihood) kill a sequence as on the
    general engine; B not a multiple of the 8-sequence blocks."""
    m = nip_amd.Model.from_net(os.path.join(GOLD, "demo1.net"))
    ov = [m.variable(s) for s in ("A1", "D1")]
    q = [m.variable("C1")]
    rng = np.random.default_rng(5)
    obs = np.stack([rng.integers(-1, m.card(v), size=(1003, 33)) for v in ov], axis=2).astype(np.int32)
    obs[5, 7, 1] = 2                                       # D1 has 2 states
    obs[900, 0, 0] = 3
    post, ll, st, _ = both(m, obs, ov, q)
    assert st[5] and st[900] and ll[5] == -DBL_MAX
    assert (st == 0).sum() == 1001


def test_filter_first_on_a_fresh_model():
    """forward_inference before any smoothing call (filter mode's
    masked lanes wrote to a sink sized for the first request only), with a
    ragged B and K < 16; then smoothing and filtering with larger B and T than
    any earlier call, each against the general engine."""
    m = nip_amd.Model.from_net(os.path.join(GOLD, "demo1.net"))
    ov = [m.variable(s) for s in ("A1", "B1", "D1")]
    q = [m.variable("C1")]
    rng = np.random.default_rng(11)
    for B, T, filt in ((13, 17, True), (5, 9, False), (301, 90, True), (517, 130, False), (900, 200, True)):
        obs = np.stack([rng.integers(-1, m.card(v), size=(B, T)) for v in ov], axis=2).astype(np.int32)
        post, ll, st, _ = both(m, obs, ov, q, filt)
        assert not st.any()
        assert np.abs(post.sum(-1) - 1).max() < 1e-12


def interface_queries(m, query):
    out = m.desc()["outgoing"]
    return [v for v in query if v in out]


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "gen_*.npz"))),
                         ids=lambda p: os.path.basename(p))
def test_general_goldens_on_the_operator_chain(path):
    """Every golden slice whose interface fits (K <= 16): the interface
    variables' marginals against the reference's own (the golden) and the
    general engine."""
    z = np.load(path)
    m = gen_model(z)
    ov = [int(v) for v in z["obs_vars"]]
    qall = [int(v) for v in z["query"]]
    q = interface_queries(m, qall)
    if not q:
        pytest.skip("no interface variable among the golden's queries")
    m.set_engine(nip_amd.ENGINE_AUTO)
    if not m.gpu_supported(ov, q):
        pytest.skip("not a GPU request")
    post, ll, st, k = run(m, z["obs"], ov, q)
    if k != "op_fb_kernel":
        pytest.skip("served by %s" % k)
    both(m, z["obs"], ov, q)
    # the golden's columns of these variables
    offs, o = {}, 0
    for v in qall:
        offs[v] = o
        o += m.card(v)
    cols = np.concatenate([np.arange(offs[v], offs[v] + m.card(v)) for v in q])
    assert np.abs(post - z["post"][:, :, cols]).max() <= POST_TOL
    assert close_ll(ll, z["ll"])


WIDE_CASES = [
    # (name, spec, observed, query, B, T): joint interfaces of 17..64 states
    # the chain plan rejects (evidence on a hidden parent): op_wide_* kernels
    ("demo1_20_D1", lambda: synth.demo1_spec(20), ["A1", "B1", "D1"], ["C1"], 9, 23),
    ("wide_34_Y1", lambda: synth.wide_spec(34, 4), ["Y1", "O1"], ["X1"], 5, 17),
    ("demo1_17_D1_T1", lambda: synth.demo1_spec(17), ["A1", "D1"], ["C1"], 6, 1),
]


@pytest.mark.parametrize("name,spec,osyms,qsyms,B,T", WIDE_CASES, ids=[c[0] for c in WIDE_CASES])
def test_wide_operator_chain(name, spec, osyms, qsyms, B, T):
    """17-64 joint interface states on the operator chain (op_wide_msgs_kernel
    + op_wide_post_kernel): smoothing and filtering against the general engine
    (posteriors 1e-12, ll 1e-12, zero-mass flags) and the oracle."""
    m = nip_amd.Model.from_spec(*spec())
    ov, q = [m.variable(s) for s in osyms], [m.variable(s) for s in qsyms]
    rng = np.random.default_rng(B * 31 + T)
    obs = np.stack([rng.integers(-1, m.card(v), size=(B, T)) for v in ov], axis=2).astype(np.int32)
    if B > 3:
        obs[3, 0, 0] = m.card(ov[0])                  # out of range: a zero-mass sequence
    for filt in (False, True):
        a = run(m, obs, ov, q, filt)
        assert a[3].startswith("op_wide_msgs_kernel"), a[3]
        b = run(m, obs, ov, q, filt, nip_amd.ENGINE_JTREE)
        assert np.abs(a[0] - b[0]).max() <= POST_TOL, np.abs(a[0] - b[0]).max()
        assert close_ll(a[1], b[1])
        assert np.array_equal(a[2] != 0, b[2] != 0)
    orc = PortOracle(m.desc())
    post, ll, _, _ = run(m, obs, ov, q)
    for bb in (0, B - 1):
        rp, rl = orc.fb(obs[bb], ov, q)
        assert np.abs(post[bb] - rp).max() <= POST_TOL
        assert close_ll([ll[bb]], [rl])
