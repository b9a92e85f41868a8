"""GPU parity of the interface-chain plan beyond the plain HMM: hidden
independent parents folded into the transition, several observed children,
and up to 64 interface states (SURVEY 8(d) configs 3 and 5 shapes).

Reference: the reference's own outputs (tests/golden/fb_demo1*.npz) and the
CPU oracle.  Tolerances as test_gpu_parity: posteriors 1e-12 absolute, ll
1e-12 relative (configs with 32/64 states: 1e-11, longer fp64 sums).
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


def gpu_fb(model, obs, ov, q):
    o = torch.from_numpy(np.ascontiguousarray(obs, np.int32)).cuda()
    post, ll, st = nip_amd.forward_backward_inference(model, o, ov, q)
    torch.cuda.synchronize()
    return post.cpu().numpy(), ll.cpu().numpy(), st.cpu().numpy()


def check_vs_oracle(m, obs, ov, q, ptol=1e-12, ltol=1e-12):
    post, ll, st = gpu_fb(m, obs, ov, q)
    orc = PortOracle(m.desc())
    for b in range(obs.shape[0]):
        rp, rl = orc.fb(obs[b], ov, q)
        err = np.abs(post[b] - rp).max()
        assert err <= ptol, "sequence %d: posterior error %g" % (b, err)
        if rl == -DBL_MAX:
            assert ll[b] == -DBL_MAX and st[b]
        else:
            assert abs(ll[b] - rl) <= ltol * max(1.0, abs(rl)), (b, ll[b], rl)


@pytest.mark.parametrize("fixture", ["fb_demo1.npz", "fb_demo1_card4.npz"])
def test_demo1_vs_reference_fixture(fixture):
    """Both observed children (A1, B1), the reference's own posteriors of C1."""
    z = np.load(os.path.join(GOLD, fixture))
    name = str(z["model"])
    if name == "demo1":
        m = nip_amd.Model.from_net(os.path.join(GOLD, "demo1.net"))
    else:
        m = nip_amd.Model.from_spec(*synth.demo1_spec(4))
    c1 = m.variable("C1")
    q = [int(x) for x in z["query"]]
    assert q[0] == c1
    post, ll, st = gpu_fb(m, z["obs"], list(z["obs_vars"]), [c1])
    N = m.card(c1)
    assert np.abs(post - z["post"][:, :, :N]).max() <= 1e-12
    assert np.all(np.abs(ll - z["ll"]) <= 1e-12 * np.maximum(1, np.abs(z["ll"])))


@pytest.mark.parametrize("observed", [["A1", "B1"], ["B1", "A1"], ["B1"], ["A1"], []])
def test_demo1_observed_subsets(observed):
    m = nip_amd.Model.from_net(os.path.join(GOLD, "demo1.net"))
    ov = [m.variable(s) for s in observed]
    rng = np.random.default_rng(len(observed) * 7 + 1)
    cards = [m.card(v) for v in ov]
    obs = np.stack([rng.integers(-1, c, size=(9, 29)) for c in cards], axis=2) if ov else \
        np.zeros((9, 29, 0), np.int32)
    check_vs_oracle(m, obs.astype(np.int32), ov, [m.variable("C1")])


def test_demo1_card32_config3_shape():
    m = nip_amd.Model.from_spec(*synth.demo1_spec(32))
    ov = [m.variable("A1"), m.variable("B1")]
    obs = synth.observations(5, 24, 32, seed=3, n_obs=2)
    obs[0, 3, 1] = -1
    check_vs_oracle(m, obs, ov, [m.variable("C1")], 1e-12, 1e-11)


@pytest.mark.parametrize("card,ocard,B,T", [(8, 5, 6, 19), (16, 16, 3, 12)])
def test_wide_clique_config5_shape(card, ocard, B, T):
    m = nip_amd.Model.from_spec(*synth.wide_spec(card, ocard))
    ov = [m.variable("O1")]
    obs = synth.observations(B, T, ocard, seed=card)
    check_vs_oracle(m, obs, ov, [m.variable("X1")], 1e-12, 1e-11)


def test_wide_clique_32_states_vs_oracle():
    """Config 5 shape at 32 states: 32^4-entry in-clique through the oracle."""
    m = nip_amd.Model.from_spec(*synth.wide_spec(32, 16))
    ov = [m.variable("O1")]
    obs = synth.observations(2, 4, 16, seed=5)
    check_vs_oracle(m, obs, ov, [m.variable("X1")], 1e-12, 1e-11)


def test_wide_clique_64_states_properties():
    """Config 5 at full width (64 states, 64^4-entry in-clique): B=256, T=128."""
    m = nip_amd.Model.from_spec(*synth.wide_spec(64, 16))
    ov = [m.variable("O1")]
    obs = torch.from_numpy(synth.observations(256, 128, 16, seed=6)).cuda()
    post, ll, st = nip_amd.forward_backward_inference(m, obs, ov, [m.variable("X1")])
    torch.cuda.synchronize()
    assert not st.any().item()
    s = post.sum(dim=2)
    assert torch.allclose(s, torch.ones_like(s), atol=1e-12, rtol=0)
    assert bool((ll <= 0).all()) and bool(torch.isfinite(ll).all())
    # time reversal of a single step sequence: posterior of T=1 = prior-propagated evidence
    one = obs[:4, :1].contiguous()
    p1, l1, _ = nip_amd.forward_backward_inference(m, one, ov, [m.variable("X1")])
    torch.cuda.synchronize()
    assert torch.allclose(p1.sum(dim=2), torch.ones(4, 1, dtype=torch.float64, device="cuda"), atol=1e-12)


def test_config3_scale_properties():
    """demo1 @ 32 states, 2048 sequences x T=256: normalised posteriors, ll <= 0."""
    m = nip_amd.Model.from_spec(*synth.demo1_spec(32))
    ov = [m.variable("A1"), m.variable("B1")]
    obs = torch.from_numpy(synth.observations(2048, 256, 32, seed=9, n_obs=2)).cuda()
    post, ll, st = nip_amd.forward_backward_inference(m, obs, ov, [m.variable("C1")])
    torch.cuda.synchronize()
    assert not st.any().item()
    s = post.sum(dim=2)
    assert torch.allclose(s, torch.ones_like(s), atol=1e-12, rtol=0)
    assert bool((ll <= 0).all()) and bool(torch.isfinite(ll).all())
    orc = PortOracle(m.desc())
    o = obs.cpu().numpy()
    for b in (0, 2047):
        rp, rl = orc.fb(o[b], ov, [m.variable("C1")])
        assert np.abs(post[b].cpu().numpy() - rp).max() <= 1e-12
        assert abs(ll[b].item() - rl) <= 1e-11 * abs(rl)


def test_config3_full_size_properties_and_parity():
    """Config 3 at its bench size: demo1 @ 32 states, 65,536 sequences x
    T=256 (chain_mfma_wide_kernel<2>: every launch-grid and LDS path at full B).  Normalised posteriors, finite
    ll <= 0, filter ll == smoothing ll and the last filtered step == the last
    smoothed step; 1,024 sequences spread over the batch (first and last
    block included) against the textbook smoother over the model's own
    tables, two against the oracle."""
    from textbook_util import chain_tables, smoother
    m = nip_amd.Model.from_spec(*synth.demo1_spec(32))
    ov = [m.variable("A1"), m.variable("B1")]
    q = [m.variable("C1")]
    B, T = 65536, 256
    obs_np = synth.observations(B, T, 32, seed=9, n_obs=2)
    obs_np[B - 1, :4, :] = -1                           # a leading missing run, last sequence
    obs_np[1000, 100:140, 0] = -1
    obs = torch.from_numpy(obs_np).cuda()
    post, ll, st = nip_amd.forward_backward_inference(m, obs, ov, q)
    fpost, fll, fst = nip_amd.forward_inference(m, obs, ov, q)
    torch.cuda.synchronize()
    assert not st.any().item() and not fst.any().item()
    s = post.sum(dim=2)
    assert torch.allclose(s, torch.ones_like(s), atol=1e-12, rtol=0)
    assert bool((ll <= 0).all()) and bool(torch.isfinite(ll).all())
    assert bool(((fll - ll).abs() <= 1e-11 * ll.abs()).all())
    assert float((post[:, -1] - fpost[:, -1]).abs().max()) <= 1e-12
    idx = np.unique(np.concatenate([np.arange(0, B, 64), [1, 255, 256, 1000, B - 256, B - 2, B - 1]]))
    A, pi, Es = chain_tables(m, m.variable("C0"), q[0], ov)
    tp, tf, tl = smoother(A, pi, Es, [obs_np[idx, :, 0], obs_np[idx, :, 1]])
    sel = torch.from_numpy(idx).cuda()
    assert np.abs(post[sel].cpu().numpy() - tp).max() <= 1e-12
    assert np.abs(fpost[sel].cpu().numpy() - tf).max() <= 1e-12
    assert np.all(np.abs(ll[sel].cpu().numpy() - tl) <= 1e-11 * np.abs(tl))
    orc = PortOracle(m.desc())
    for b in (0, B - 1):
        rp, rl = orc.fb(obs_np[b], ov, q)
        assert np.abs(post[b].cpu().numpy() - rp).max() <= 1e-12
        assert abs(ll[b].item() - rl) <= 1e-11 * abs(rl)


@pytest.mark.parametrize("T", [4096, 8192])
def test_config3_long_sequences_analytic_normalisation(T):
    """chain_mfma_wide_kernel<2>'s phase B normalises every
    posterior with one mass c* taken at the partner's first phase-B step
    (NIPAMD_MW_ANALYTIC); the rounding drift grows with |t - t*|.  At T = 4096
    and 8192 (16x / 32x config 3's length) every row still sums to 1 within
    1e-12 and every posterior and ll matches the textbook smoother (1e-12 /
    1e-11), missing runs included."""
    from textbook_util import chain_tables, smoother
    m = nip_amd.Model.from_spec(*synth.demo1_spec(32))
    ov = [m.variable("A1"), m.variable("B1")]
    q = [m.variable("C1")]
    B = 48
    obs_np = synth.observations(B, T, 32, seed=T + 1, n_obs=2)
    obs_np[3, 500:900, :] = -1
    obs_np[7, :, 1] = -1
    obs = torch.from_numpy(obs_np).cuda()
    post, ll, st = nip_amd.forward_backward_inference(m, obs, ov, q)
    torch.cuda.synchronize()
    assert not st.any().item()
    s = post.sum(dim=2)
    assert float((s - 1.0).abs().max()) <= 1e-12
    A, pi, Es = chain_tables(m, m.variable("C0"), q[0], ov)
    tp, tf, tl = smoother(A, pi, Es, [obs_np[:, :, 0], obs_np[:, :, 1]])
    assert np.abs(post.cpu().numpy() - tp).max() <= 1e-12
    assert np.all(np.abs(ll.cpu().numpy() - tl) <= 1e-11 * np.abs(tl))


# 33..64 states: chain_row64_kernel (one filter wave per direction; chain_wide4_kernel, four per direction, one
# barrier per step, sparse rescaling, partner waves for scratch/posterior/ll)
@pytest.mark.parametrize("card,B,T", [(48, 3, 21), (40, 2, 2), (64, 2, 9), (33, 3, 1)])
def test_wide4_demo1_vs_oracle(card, B, T):
    m = nip_amd.Model.from_spec(*synth.demo1_spec(card, seed=card))
    ov = [m.variable("A1"), m.variable("B1")]
    obs = synth.observations(B, T, card, seed=card + T, n_obs=2)
    obs[0, ::4, 0] = -1                               # missing values on one child
    check_vs_oracle(m, obs, ov, [m.variable("C1")], 1e-12, 1e-11)


def test_wide4_filter_vs_oracle():
    m = nip_amd.Model.from_spec(*synth.demo1_spec(50, seed=3))
    ov = [m.variable("A1"), m.variable("B1")]
    q = [m.variable("C1")]
    obs = synth.observations(3, 17, 50, seed=11, n_obs=2)
    o = torch.from_numpy(obs).cuda()
    post, ll, st = nip_amd.forward_inference(m, o, ov, q)
    torch.cuda.synchronize()
    post, ll = post.cpu().numpy(), ll.cpu().numpy()
    orc = PortOracle(m.desc())
    for b in range(obs.shape[0]):
        rp, rl = orc.fb(obs[b], ov, q, filter_only=True)
        assert np.abs(post[b] - rp).max() <= 1e-12
        assert abs(ll[b] - rl) <= 1e-11 * max(1.0, abs(rl))


def test_wide4_matches_one_wave_kernel_config5():
    """Config 5 at full size: the four-wave kernel against the one-wave kernel
    (NIPAMD_WIDE_KERNEL=wave1 in a child process: the switch is read once)."""
    import subprocess, sys, os
    code = (
        "import numpy as np, torch, nip_amd\n"
        "from nip_amd import synth\n"
        "m = nip_amd.Model.from_spec(*synth.wide_spec(64, 16))\n"
        "obs = torch.from_numpy(synth.observations(64, 128, 16, seed=6)).cuda()\n"
        "p, l, s = nip_amd.forward_backward_inference(m, obs, [m.variable('O1')], [m.variable('X1')])\n"
        "torch.cuda.synchronize()\n"
        "np.savez(sys.argv[1], p=p.cpu().numpy(), l=l.cpu().numpy())\n")
    outs = []
    from nip_amd import build as nb
    for env in ({}, {"NIPAMD_WIDE_KERNEL": "wave1", "NIPAMD_LIB": nb.DIAG_LIB}):   # a diagnostics-build switch
        path = os.path.join(os.environ.get("TMPDIR", "/tmp"), "wide4_%d.npz" % len(outs))
        r = subprocess.run([sys.executable, "-c", "import sys\n" + code, path],
                           env=dict(os.environ, **env), timeout=300)
        assert r.returncode == 0
        outs.append(np.load(path))
    assert np.abs(outs[0]["p"] - outs[1]["p"]).max() <= 1e-12
    assert np.all(np.abs(outs[0]["l"] - outs[1]["l"]) <= 1e-11 * np.maximum(1.0, np.abs(outs[1]["l"])))


def _four_child_spec(card=36, m=5, seed=7):
    """A 36-state chain observed through up to four leaf children (the
    row-form 33..64-state kernel is instantiated per observed-column count)."""
    nodes = [("X0", card, "X1"), ("X1", card, None)] + [("O%d" % i, m, None) for i in range(1, 5)]
    pots = [("X1", ["X0"], synth.cpt(seed, card, card)), ("X0", [], synth.cpt(seed + 1, card, 1))]
    pots += [("O%d" % i, ["X1"], synth.cpt(seed + 1 + i, m, card)) for i in range(1, 5)]
    return nodes, pots


@pytest.mark.parametrize("cols", [["O1"], ["O2", "O4"], ["O1", "O2", "O3"], ["O4", "O3", "O2", "O1"]])
def test_row64_observed_columns_vs_oracle(cols):
    m = nip_amd.Model.from_spec(*_four_child_spec())
    ov = [m.variable(c) for c in cols]
    obs = synth.observations(3, 19, 5, seed=len(cols) + 3, n_obs=len(cols))
    obs[1, ::3, 0] = -1                               # missing values on one child
    obs[2, 5, -1] = 7                                 # out of range: zero mass from step 5
    check_vs_oracle(m, obs, ov, [m.variable("X1")], 1e-12, 1e-11)
    assert nip_amd.last_kernel() == "chain_row64_kernel"
