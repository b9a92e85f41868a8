"""GPU parity of the batched e_step / em_learn (src/nip.c:1708-2243).

Expected counts, per-sequence log-likelihoods and BAD_LUCK flags from the
gfx950 path (through the C-ABI) against the reference's own outputs
(tests/golden/fb_*.npz, produced by oracle/_ref) and the CPU oracle.
Tolerances: counts |gpu - ref| <= 1e-11 * max(1, |ref|) (sums
of B*T normalised terms, summed in a different order); ll as in
test_gpu_parity; learning curves 1e-10 relative over <= 12 EM iterations.
The batch reduction must be bit-reproducible and shard-invariant.
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
from nip_amd.em import tree_sum, em_learn, NIP_NO_ERROR, NIP_ERROR_BAD_LUCK
from oracle.bind import PortOracle
from em_util import check_em_curve

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CONTRACT = json.load(open(os.path.join(GOLD, "index_contract.json")))
CNT_RTOL = 1e-11
LL_RTOL = 1e-12
CURVE_RTOL = 1e-10
DBL_MAX = np.finfo(np.float64).max


def product_model(name):
    c = CONTRACT[name]
    nodes = [tuple(n) for n in c["nodes"]]
    pots = [(ch, ps, d) for ch, ps, d in c["potentials"]]
    return nip_amd.Model.from_spec(nodes, pots)


def chain_fixtures():
    out = []
    for p in sorted(glob.glob(os.path.join(GOLD, "fb_*.npz"))):
        z = np.load(p)
        m = product_model(str(z["model"]))
        if m.estep_supported() and m.gpu_supported(list(z["obs_vars"]), []):
            out.append(p)
    return out


def gpu_estep(model, obs, obs_vars):
    o = torch.from_numpy(np.ascontiguousarray(obs, np.int32)).cuda()
    cnt, ll, st = nip_amd.e_step(model, o, obs_vars)
    torch.cuda.synchronize()
    return cnt.cpu().numpy(), ll.cpu().numpy(), st.cpu().numpy()


def close(a, b, rtol):
    return np.all(np.abs(a - b) <= rtol * np.maximum(1.0, np.abs(b)))


@pytest.mark.parametrize("path", chain_fixtures(), ids=lambda p: os.path.basename(p))
def test_estep_matches_reference_fixture(path):
    z = np.load(path)
    m = product_model(str(z["model"]))
    cnt, ll, st = gpu_estep(m, z["obs"], list(z["obs_vars"]))
    bad = z["estep_bad"]
    assert np.array_equal((st & nip_amd.STATUS_BAD_LUCK) != 0, bad != 0)
    ok = bad == 0
    assert close(ll[ok], z["estep_ll"][ok], LL_RTOL)
    if ok.all():
        err = np.abs(cnt - z["counts"]).max()
        assert close(cnt, z["counts"], CNT_RTOL), err


@pytest.mark.parametrize("N,M,B,T", [
    (16, 16, 9, 64), (16, 16, 8, 1), (16, 16, 8, 2), (16, 16, 3, 3),
    (4, 5, 13, 33), (7, 3, 17, 17), (2, 2, 1, 5), (16, 8, 70, 40),
])
def test_estep_synthetic_vs_oracle(N, M, B, T):
    nodes, pots = synth.hmm_spec(N, M, seed=200 + N * 7 + M)
    m = nip_amd.Model.from_spec(nodes, pots)
    obs = synth.observations(B, T, M, seed=T * 17 + B)
    ov = [m.variable("M1")]
    cnt, ll, st = gpu_estep(m, obs, ov)
    orc = PortOracle(m.desc())
    rc, rl, rb = orc.estep(obs, ov, np.ones(m.param_size()))
    assert not rb.any() and not st.any()
    assert close(ll, rl, LL_RTOL)
    assert close(cnt, rc, CNT_RTOL), np.abs(cnt - rc).max()


def test_estep_missing_observations_vs_oracle():
    """Missing values, with the reference's BAD_LUCK verdict on leading
    missing runs (nip.c:1838: the running ll of a run that observed nothing is
    0 up to the rounding of two propagations and can land on +1e-16): the
    engine reproduces it flag for flag (prefix.cpp, tests/test_estep_prefix.py);
    ll and counts are compared on the sequences the reference accepts."""
    nodes, pots = synth.hmm_spec(16, 16, seed=9)
    m = nip_amd.Model.from_spec(nodes, pots)
    rng = np.random.default_rng(4)
    obs = rng.integers(0, 16, size=(12, 37, 1)).astype(np.int32)
    obs[rng.random(obs.shape) < 0.3] = -1
    obs[0] = -1                                   # a fully missing sequence
    for L in range(1, 6):
        obs[L, :L] = -1                           # leading runs of length 1..5
    ov = [m.variable("M1")]
    _, ll, st = gpu_estep(m, obs, ov)
    _, rl, rb = PortOracle(m.desc()).estep(obs, ov, np.ones(m.param_size()))
    assert np.array_equal((st & nip_amd.STATUS_BAD_LUCK) != 0, rb != 0)
    assert np.array_equal(st != 0, rb != 0)
    ok = rb == 0
    assert close(ll[ok], rl[ok], LL_RTOL)
    cnt, _, _ = gpu_estep(m, obs[ok], ov)
    rc, _, _ = PortOracle(m.desc()).estep(obs[ok], ov, np.ones(m.param_size()))
    assert close(cnt, rc, CNT_RTOL), np.abs(cnt - rc).max()


@pytest.mark.parametrize("B,T,proper", [(23, 41, False), (70, 41, False), (24, 40, True), (70, 41, True),
                                          (2, 3, True)])
def test_estep_missing_multiblock_vs_oracle(B, T, proper):
    """The default e_step kernel (chain_kernel<true>, 8 sequences per block)
    with 25% missing values over several blocks and odd / even T.  proper=True:
    rows of A and E sum to 1, so the step masses of missing observations sit
    at 1.0, where a scale exponent taken from a lane-inconsistent sum differs
    by one between lanes (round 3: FMA contraction into the row sum's first
    add; the joint e_step's 0.058 error).  Leading missing runs included:
    the BAD_LUCK flags must equal the reference's."""
    m = nip_amd.Model.from_spec(*synth.hmm_spec(16, 16, seed=9, proper=proper))
    rng = np.random.default_rng(B * 100 + T)
    obs = rng.integers(0, 16, size=(B, T, 1)).astype(np.int32)
    obs[rng.random(obs.shape) < 0.25] = -1
    obs[:B // 3, :3] = -1
    if B == 2:
        obs[:, :, 0] = [[0, -1, 13], [5, -1, 2]]
    ov = [m.variable("M1")]
    cnt, ll, st = gpu_estep(m, obs, ov)
    orc = PortOracle(m.desc())
    rc, rl, rb = orc.estep(obs, ov, np.ones(m.param_size()))
    assert np.array_equal(st != 0, rb != 0)
    ok = rb == 0
    assert close(ll[ok], rl[ok], LL_RTOL)
    if not ok.all():
        cnt, _, _ = gpu_estep(m, obs[ok], ov)
        rc, _, _ = orc.estep(obs[ok], ov, np.ones(m.param_size()))
    assert close(cnt, rc, CNT_RTOL), np.abs(cnt - rc).max()
    # the same sequences through fb: posteriors and ll
    q = [m.variable("P1")]
    post, fll, _ = nip_amd.forward_backward_inference(m, torch.from_numpy(obs).cuda(), ov, q)
    post = post.cpu().numpy()
    for b in range(0, B, max(1, B // 6)):
        rp, r_ll = orc.fb(obs[b], ov, q)
        assert np.abs(post[b] - rp).max() <= 1e-12
        assert abs(fll[b].item() - r_ll) <= LL_RTOL * max(1.0, abs(r_ll))


def _near_identity(n, eps):
    d = np.full((n, n), eps)
    np.fill_diagonal(d, 1.0)
    return (d / d.sum(axis=1, keepdims=True)).ravel()


@pytest.mark.parametrize("T", [40, 203])
def test_estep_peaked_proper_model_sparse_rescaling(T):
    """A proper model (rows sum to 1: the kernel's proper mode) with a
    near-identity transition (1e-50 off the diagonal) and emission (1e-60):
    random data puts each step's evidence mass near 1e-50, so both filters'
    rescaling every 4th step runs at ~1e-200 between rescales.  Counts, ll
    and flags against the oracle (per-step normalisation, nip.c:1461-1474)."""
    N = 16
    nodes = [("P0", N, "P1"), ("P1", N, None), ("M1", N, None)]
    pots = [("M1", ["P1"], _near_identity(N, 1e-60)),
            ("P1", ["P0"], _near_identity(N, 1e-50)),
            ("P0", [], np.full(N, 1.0 / N))]
    m = nip_amd.Model.from_spec(nodes, pots)
    obs = synth.observations(37, T, N, seed=T)
    ov = [m.variable("M1")]
    cnt, ll, st = gpu_estep(m, obs, ov)
    assert nip_amd.last_kernel().startswith("chain_estep16_kernel")
    rc, rl, rb = PortOracle(m.desc()).estep(obs, ov, np.ones(m.param_size()))
    assert np.array_equal(st != 0, rb != 0) and not rb.any()
    assert close(ll, rl, LL_RTOL)
    assert close(cnt, rc, CNT_RTOL), np.abs(cnt - rc).max()


def test_estep_bad_luck_flags():
    """Invalid codes / impossible data: the reference's e_step BAD_LUCK."""
    nodes, pots = synth.hmm_spec(16, 16, seed=5)
    m = nip_amd.Model.from_spec(nodes, pots)
    rng = np.random.default_rng(3)
    obs = rng.integers(0, 16, size=(10, 20, 1)).astype(np.int32)
    obs[2, 7, 0] = 16                              # out of range -> zero likelihood
    obs[5, 0, 0] = 16
    ov = [m.variable("M1")]
    _, ll, st = gpu_estep(m, obs, ov)
    _, rl, rb = PortOracle(m.desc()).estep(obs, ov, np.ones(m.param_size()))
    assert np.array_equal((st & nip_amd.STATUS_BAD_LUCK) != 0, rb != 0)
    ok = rb == 0
    assert close(ll[ok], rl[ok], LL_RTOL)


def test_partial_is_shard_invariant_and_reproducible():
    """Binary-tree reduction: halves combined == whole batch, bit for bit."""
    nodes, pots = synth.hmm_spec(16, 16)
    m = nip_amd.Model.from_spec(nodes, pots)
    obs = torch.from_numpy(synth.observations(256, 48, 16, seed=8)).cuda().contiguous()
    ov = [m.variable("M1")]
    whole, _, _ = nip_amd.estep_partial(m, obs, ov)
    whole = whole.clone()
    again, _, _ = nip_amd.estep_partial(m, obs, ov)
    assert torch.equal(whole, again)
    parts = []
    for k in range(4):
        p, _, _ = nip_amd.estep_partial(m, obs[k * 64:(k + 1) * 64].contiguous(), ov)
        parts.append(p.clone())
    comb = tree_sum(torch.stack(parts))
    assert torch.equal(comb[:-3], whole[:-3])             # the body, bit for bit
    assert comb[-3:].tolist() == [4.0, 0.0, 0.0] and whole[-3:].tolist() == [1.0, 0.0, 0.0]   # route tag counts


def test_partials_of_different_routes_are_refused():
    """The e_step route depends on T (the 16-state kernel's LDS must hold the
    sequence; beyond it the wide chain e_step runs) and on the engine setting
    (the general engine): partials of the layouts have the same size, and
    combining them must fail in the finalize, not sum mismatched layouts
    (ADVICE r02).  Peaked tables (1e-50 / 1e-60 off the diagonal) fail the
    host's rescaling bound and keep the model off chain_estep_ck_kernel, whose
    LDS does not depend on T."""
    N = 4
    nodes = [("P0", N, "P1"), ("P1", N, None), ("M1", N, None)]
    pots = [("M1", ["P1"], _near_identity(N, 1e-60)), ("P1", ["P0"], _near_identity(N, 1e-50)),
            ("P0", [], np.full(N, 1.0 / N))]
    m = nip_amd.Model.from_spec(nodes, pots)
    ov = [m.variable("M1")]
    short = torch.from_numpy(synth.observations(2, 16, 4, seed=1)).cuda()
    long_ = torch.from_numpy(synth.observations(2, 16000, 4, seed=2)).cuda()   # > 96 KB of LDS
    a, _, _ = nip_amd.estep_partial(m, short, ov)
    a = a.clone()
    b, _, _ = nip_amd.estep_partial(m, long_, ov)
    b = b.clone()
    m.set_engine(nip_amd.ENGINE_JTREE)
    c, _, _ = nip_amd.estep_partial(m, short, ov)
    c = c.clone()
    m.set_engine(nip_amd.ENGINE_AUTO)
    assert a[-3:].tolist() == [1.0, 0.0, 0.0] and b[-3:].tolist() == [0.0, 0.0, 1.0]
    assert c[-3:].tolist() == [0.0, 1.0, 0.0]
    for p in (a, b, c):
        nip_amd.estep_finalize(m, p, None)               # each alone is fine
    for x, y in ((a, b), (a, c), (b, c)):
        with pytest.raises(nip_amd.NipError):
            nip_amd.estep_finalize(m, tree_sum(torch.stack([x, y])), None)


def test_chunked_batch_matches_tree():
    """B above one launch chunk (16384): chunk trees combine exactly."""
    nodes, pots = synth.hmm_spec(4, 4, seed=3)
    m = nip_amd.Model.from_spec(nodes, pots)
    B, T = 32768, 3
    obs = torch.from_numpy(synth.observations(B, T, 4, seed=12)).cuda().contiguous()
    ov = [m.variable("M1")]
    whole, _, _ = nip_amd.estep_partial(m, obs, ov)
    whole = whole.clone()
    a, _, _ = nip_amd.estep_partial(m, obs[:16384].contiguous(), ov)
    a = a.clone()
    b, _, _ = nip_amd.estep_partial(m, obs[16384:].contiguous(), ov)
    assert torch.equal(tree_sum(torch.stack([a, b.clone()]))[:-3], whole[:-3])


@pytest.mark.parametrize("path", chain_fixtures(), ids=lambda p: os.path.basename(p))
def test_em_learn_matches_reference_curve(path):
    z = np.load(path)
    m = product_model(str(z["model"]))
    obs = torch.from_numpy(np.ascontiguousarray(z["obs"])).cuda()
    curve = []
    rc = em_learn(m, obs, list(z["obs_vars"]), 1e-6, curve, init=z["em_init"], max_iterations=12)
    check_em_curve(z, rc, curve, CURVE_RTOL)



def test_estep_config2_scale_properties():
    """Config-2 size (4096 x 1024, N=M=16): count masses and spot parity."""
    nodes, pots = synth.hmm_spec(16, 16)
    m = nip_amd.Model.from_spec(nodes, pots)
    B, T, N, M = 4096, 1024, 16, 16
    obs_np = synth.observations(B, T, M)
    obs = torch.from_numpy(obs_np).cuda()
    ov = [m.variable("M1")]
    cnt, ll, st = nip_amd.e_step(m, obs, ov)
    cnt = cnt.cpu().numpy()
    assert not st.any().item()
    d = m.desc()
    sizes = []
    for v in d["vars"]:
        s = v["card"]
        for p in v["parents"]:
            s *= d["vars"][p]["card"]
        sizes.append(s)
    offs = np.concatenate([[0], np.cumsum(sizes)])
    mass = {d["vars"][i]["symbol"]: cnt[offs[i]:offs[i + 1]].sum() for i in range(3)}
    assert abs(mass["P0"] - (N + B)) <= 1e-9 * (N + B)
    assert abs(mass["P1"] - (N * N + B * T)) <= 1e-9 * B * T
    assert abs(mass["M1"] - (N * M + B * T)) <= 1e-9 * B * T
    sub = 64
    c64, l64, _ = nip_amd.e_step(m, obs[:sub].contiguous(), ov)
    rc, rl, _ = PortOracle(d).estep(obs_np[:sub], ov, np.ones(m.param_size()))
    assert close(c64.cpu().numpy(), rc, CNT_RTOL)
    assert close(l64.cpu().numpy(), rl, LL_RTOL)


def test_estep_host_buffers_match_device():
    """nipamd_estep_host (the C em_learn seam) == nipamd_estep on device."""
    import ctypes as C
    nodes, pots = synth.hmm_spec(16, 16, seed=21)
    m = nip_amd.Model.from_spec(nodes, pots)
    obs = synth.observations(33, 50, 16, seed=4)
    ov = [m.variable("M1")]
    cnt, ll, st = gpu_estep(m, obs, ov)
    hc = np.ones(m.param_size())
    hl = np.zeros(33)
    hs = np.zeros(33, np.uint32)
    o = np.ascontiguousarray(obs, np.int32)
    rc = nip_amd.lib().nipamd_estep_host(m._h, o.ctypes.data_as(C.c_void_p), 1,
                                         (C.c_int * 1)(*ov), 33, 50, hc.ctypes.data_as(C.c_void_p),
                                         hl.ctypes.data_as(C.c_void_p), hs.ctypes.data_as(C.c_void_p))
    assert rc == 0
    assert np.array_equal(hc, cnt) and np.array_equal(hl, ll) and not hs.any()


# The matrix-core e_step (chain_fb_mfma_kernel<estep>) is a measured
# alternative, selected by NIPAMD_ESTEP_KERNEL=mfma in the diagnostics build
# only (csrc/diag.h): its parity checks run in a worker process on that library.
def test_estep_mfma_kernel_in_diagnostics_build():
    import subprocess
    import sys
    from nip_amd import build as nb
    here = os.path.dirname(os.path.abspath(__file__))
    r = subprocess.run([sys.executable, os.path.join(here, "_estep_mfma_worker.py")],
                       env=dict(os.environ, NIPAMD_LIB=nb.DIAG_LIB), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "all passed" in r.stdout


GENERAL_CASES = [
    # name, spec, observed children: chain plans beyond the HMM (hidden
    # parents folded into the transition, several leaf children)
    ("demo1_4_AB", lambda: synth.demo1_spec(4), ["A1", "B1"]),
    ("demo1_6_B", lambda: synth.demo1_spec(6, seed=3), ["B1"]),
    ("demo1_16_AB", lambda: synth.demo1_spec(16, seed=5), ["A1", "B1"]),
    ("demo1_5_none", lambda: synth.demo1_spec(5, seed=7), []),
    ("wide_8", lambda: synth.wide_spec(8, 5), ["O1"]),
]


@pytest.mark.parametrize("name,spec,osyms", GENERAL_CASES, ids=[c[0] for c in GENERAL_CASES])
@pytest.mark.parametrize("B,T", [(37, 41), (16, 1), (3, 2)])
def test_general_chain_estep_vs_oracle_and_general_engine(name, spec, osyms, B, T):
    """The chain e_step for plans with hidden parents and several children
    (chain_estep16_kernel with one evidence table per child, ensure_chain_map):
    counts rel 1e-11 and ll rel 1e-12 against the oracle and the general
    join-tree engine, BAD_LUCK flags equal, missing and leading-missing data."""
    m = nip_amd.Model.from_spec(*spec())
    ov = [m.variable(s) for s in osyms]
    rng = np.random.default_rng(B * 31 + T + len(name))
    if ov:
        obs = np.stack([rng.integers(0, m.card(v), size=(B, T)) for v in ov], axis=2).astype(np.int32)
        obs[rng.random(obs.shape) < 0.2] = -1
        obs[0, :2] = -1
    else:
        obs = np.zeros((B, T, 0), np.int32)
    cnt, ll, st = gpu_estep(m, obs, ov)
    assert nip_amd.last_kernel() == "chain_estep16_kernel", nip_amd.last_kernel()
    orc = PortOracle(m.desc())
    rc, rl, rb = orc.estep(obs, ov, np.ones(m.param_size()))
    assert np.array_equal(st != 0, rb != 0)
    ok = rb == 0
    assert close(ll[ok], rl[ok], LL_RTOL)
    if not ok.all():
        cnt, _, _ = gpu_estep(m, obs[ok], ov)
        rc, _, _ = orc.estep(obs[ok], ov, np.ones(m.param_size()))
    assert close(cnt, rc, CNT_RTOL), np.abs(cnt - rc).max()
    m.set_engine(nip_amd.ENGINE_JTREE)
    cj, lj, sj = gpu_estep(m, obs[ok], ov)
    m.set_engine(nip_amd.ENGINE_AUTO)
    assert close(cnt, cj, CNT_RTOL), np.abs(cnt - cj).max()


def test_general_chain_em_learn_matches_general_engine():
    """em_learn on demo1's structure through the chain e_step against the same
    run on the general engine (curves rel 1e-10)."""
    nodes, pots = synth.demo1_spec(6, seed=11)
    obs_np = np.concatenate([synth.observations(64, 50, 6, seed=s) for s in (1, 2)], axis=2)
    curves = []
    for engine in (nip_amd.ENGINE_AUTO, nip_amd.ENGINE_JTREE):
        m = nip_amd.Model.from_spec(nodes, pots)
        m.set_engine(engine)
        ov = [m.variable("A1"), m.variable("B1")]
        curve = []
        rc = em_learn(m, torch.from_numpy(obs_np).cuda(), ov, 1e-6, curve,
                      init=synth.uniform01(5, m.param_size()) + 0.05, max_iterations=6)
        curves.append((rc, curve))
    assert curves[0][0] == curves[1][0]
    assert len(curves[0][1]) == len(curves[1][1])
    assert close(np.array(curves[0][1]), np.array(curves[1][1]), 1e-10)


# ---------------------------------------------------------------------------
# BAD_LUCK outside leading missing runs: the reference
# rejects a series as soon as its running ll is > 0 (nip.c:1827-1829).  An
# observed step adds log P(o_t | past) <= 0, so the test can only fire by
# rounding while every step so far had probability 1 exactly -- deterministic
# rows.  These models put the e_step there, in both kernel modes (proper: the
# rows sum to 1, the ll from the final mass; general: per-step masses), and
# compare every series' flag and ll with the reference's own code
# (oracle/_ref).  Findings:
#   * 0/1 and dyadic tables: the arithmetic is exact on both sides (ll 0, or
#     log of the first observation's probability), so nothing is flagged by
#     rounding and the flags agree;
#   * a one-state child observed at every step carries no evidence: the
#     reference's propagation is bit for bit the missing step's, so its
#     rounding verdict is the leading-missing-run verdict (prefix.cpp), which
#     the flag kernel applies to such columns too;
#   * non-dyadic deterministic rows (probability 1 from inexact sums) put the
#     running ll at +-1e-16 on the reference's side -- its verdict there is a
#     rounding accident the kernels do not reproduce; the case below records
#     the reference's outcome on it and checks the ll agree within 1e-15.
def _det_spec(E, A, pi, proper):
    """HMM-shaped slice M1 | P1, P1 | P0, P0 with the given tables (rows: parent
    state); proper=True declares M1 first, so the reference's CPT
    normalisation runs over the child (huginnet.y:635-636)."""
    N, M = E.shape
    nodes = [("P0", N, "P1"), ("P1", N, None), ("M1", M, None)]
    if proper:
        nodes = nodes[::-1]
    pots = [("M1", ["P1"], np.asarray(E, np.float64).ravel()), ("P1", ["P0"], np.asarray(A, np.float64).ravel()),
            ("P0", [], np.asarray(pi, np.float64))]
    return nodes, pots


def _det_cases():
    T = 40
    cyc = np.roll(np.eye(3), 1, axis=1)              # P1 = P0 + 1 mod 3
    good = np.array([[(t + 1) % 3 for t in range(T)]] * 8, np.int32)
    good[1, 5:12] = -1                                # a gap
    good[2, :9] = -1                                  # a leading missing run
    good[3, 17] = (good[3, 17] + 1) % 3               # an impossible step: zero mass
    out = [("identity_onehot_proper", np.eye(3), cyc, [1.0, 0.0, 0.0], True, good)]
    # 3 states, 2 symbols, states 0 and 1 emit symbol 0 (non-proper order: the
    # emission normalised over P1, rows 0.5 / 0.5 / 1)
    E2 = np.array([[1.0, 0.0], [1.0, 0.0], [0.0, 1.0]])
    A2 = np.array([[0.5, 0.5, 0.0], [0.5, 0.5, 0.0], [0.0, 0.0, 1.0]])
    obs2 = np.zeros((8, T), np.int32)
    obs2[1, 3:9] = -1
    obs2[2, :5] = -1
    obs2[3, 11] = 1                                   # impossible: zero mass
    out.append(("dyadic_nonproper", E2, A2, [0.25, 0.75, 0.0], False, obs2))
    out.append(("dyadic_proper", E2, A2, [0.25, 0.75, 0.0], True, obs2))
    # a one-state child: every observation is uninformative
    E3 = np.ones((3, 1))
    A3 = np.array([[0.1, 0.2, 0.7], [0.3, 0.3, 0.4], [0.5, 0.25, 0.25]])
    obs3 = np.zeros((8, T), np.int32)
    obs3[1, 4:10] = -1
    obs3[2, :3] = -1
    out.append(("one_state_child_proper", E3, A3, [0.2, 0.3, 0.5], True, obs3))
    out.append(("one_state_child_nonproper", E3, A3, [0.2, 0.3, 0.5], False, obs3))
    # non-dyadic transition and prior behind a deterministic emission: every
    # observed step has probability 1 from inexact sums (the reference's ll
    # ends at -1.1e-16 here, nothing flagged; a rounding accident either way)
    A4 = np.array([[0.3, 0.7, 0.0], [0.6, 0.4, 0.0], [0.0, 0.0, 1.0]])
    obs4 = np.zeros((8, T), np.int32)
    obs4[1, 6:14] = -1
    out.append(("deterministic_emission_nondyadic", E2, A4, [0.1, 0.9, 0.0], True, obs4))
    return out


@pytest.mark.parametrize("name,E,A,pi,proper,obs", _det_cases(), ids=[c[0] for c in _det_cases()])
def test_bad_luck_on_deterministic_rows_vs_reference(name, E, A, pi, proper, obs):
    from oracle import bind
    if not bind.ref_available():
        pytest.skip("oracle/_ref not built")
    nodes, pots = _det_spec(E, A, pi, proper)
    m = nip_amd.Model.from_spec(nodes, pots)
    ov = [m.variable("M1")]
    obs = obs[..., None]
    cnt, ll, st = gpu_estep(m, obs, ov)
    # chain_estep16_kernel, or chain_estep_ck_kernel where the tables pass its rescaling bound
    assert nip_amd.last_kernel().startswith(("chain_estep16_kernel", "chain_estep_ck_kernel")), nip_amd.last_kernel()
    ref = bind.RefHarness(synth.spec_to_replay(nodes, pots), cards=[n[1] for n in nodes])
    rc, rl, rb = ref.estep(obs, [nodes.index(next(n for n in nodes if n[0] == "M1"))], np.ones(m.param_size()))
    assert np.array_equal(st != 0, rb != 0), (st.tolist(), rb.tolist())
    ok = rb == 0
    assert np.all(np.abs(ll[ok] - rl[ok]) <= 1e-15 + 1e-12 * np.abs(rl[ok])), np.abs(ll[ok] - rl[ok]).max()
    if ok.any():
        c2, _, _ = gpu_estep(m, obs[ok], ov)
        rc2, _, _ = ref.estep(obs[ok], [nodes.index(next(n for n in nodes if n[0] == "M1"))],
                              np.ones(m.param_size()))
        assert close(c2, rc2, CNT_RTOL), np.abs(c2 - rc2).max()
