"""GPU parity of batched forward_inference (filtering, src/nip.c:1103-1315).

The filtered marginals P(X_t | y_0..y_t) and the log-likelihood from the GPU
(nipamd_filter, through the C-ABI) against the reference's own filtered
outputs (tests/golden/fb_*.npz: fpost, fll) and the CPU oracle's filter.
Tolerances as test_gpu_parity: posteriors 1e-12 absolute, ll 1e-12 relative.
"""
import glob
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


def check_vs_oracle(m, obs, ov, q, ptol=1e-12, ltol=1e-12):
    post, ll, st = run(nip_amd.forward_inference, m, obs, ov, q)
    orc = PortOracle(m.desc())
    for b in range(obs.shape[0]):
        rp, rl = orc.fb(obs[b], ov, q, filter_only=True)
        err = np.abs(post[b] - rp).max()
        assert err <= ptol, "sequence %d: filtered posterior error %g" % (b, err)
        if rl == -DBL_MAX:
            assert ll[b] == -DBL_MAX and st[b]
        else:
            assert abs(ll[b] - rl) <= ltol * max(1.0, abs(rl)), (b, ll[b], rl)


def fixtures():
    out = []
    for p in sorted(glob.glob(os.path.join(GOLD, "fb_*.npz"))):
        z = np.load(p)
        if "fpost" in z.files:
            out.append(os.path.basename(p))
    return out


@pytest.mark.parametrize("fixture", fixtures())
def test_filter_vs_reference_fixture(fixture):
    """The reference's own forward_inference outputs (fpost, fll)."""
    from test_gpu_estep import product_model
    z = np.load(os.path.join(GOLD, fixture))
    m = product_model(str(z["model"]))
    ov, q = [int(v) for v in z["obs_vars"]], [int(v) for v in z["query"]]
    if not m.gpu_supported(ov, q):
        pytest.skip("outside the GPU plan")
    post, ll, st = run(nip_amd.forward_inference, m, z["obs"], ov, q)
    ref, rll = z["fpost"], z["fll"]
    assert np.abs(post - ref[:, :, :post.shape[2]]).max() <= 1e-12
    for b in range(len(rll)):
        if rll[b] == -DBL_MAX:
            assert ll[b] == -DBL_MAX and st[b]
        else:
            assert abs(ll[b] - rll[b]) <= 1e-12 * max(1.0, abs(rll[b])), (b, ll[b], rll[b])


@pytest.mark.parametrize("N,M,B,T", [(16, 16, 9, 64), (16, 16, 8, 1), (16, 16, 3, 2),
                                     (4, 5, 13, 33), (7, 3, 17, 17), (32, 8, 5, 40)])
def test_filter_hmm(N, M, B, T):
    nodes, pots = synth.hmm_spec(N, M, seed=300 + N + M)
    m = nip_amd.Model.from_spec(nodes, pots)
    obs = synth.observations(B, T, M, seed=T + 7 * B)
    check_vs_oracle(m, obs, [m.variable("M1")], [m.variable("P1")])


def test_filter_missing_invalid_and_zero_mass():
    nodes, pots = synth.hmm_spec(16, 16, seed=9)
    m = nip_amd.Model.from_spec(nodes, pots)
    rng = np.random.default_rng(11)
    obs = rng.integers(-1, 17, size=(10, 37, 1)).astype(np.int32)
    obs[1, :, 0] = -1
    check_vs_oracle(m, obs, [m.variable("M1")], [m.variable("P1")])
    mz = nip_amd.Model.from_net(os.path.join(GOLD, "model.net"))
    obs = rng.integers(-1, 5, size=(21, 24, 1)).astype(np.int32)
    check_vs_oracle(mz, obs, [mz.variable("M1")], [mz.variable("P1")])


def test_filter_demo1_two_children():
    m = nip_amd.Model.from_spec(*synth.demo1_spec(32))
    ov = [m.variable("A1"), m.variable("B1")]
    obs = np.concatenate([synth.observations(6, 48, 32, seed=4), synth.observations(6, 48, 32, seed=5)], axis=2)
    check_vs_oracle(m, obs, ov, [m.variable("C1")], ltol=1e-11)


def test_filter_wide_64_properties():
    """64 states (the DPP wide kernel): normalised, the last step equals the
    smoothed posterior, ll identical to forward_backward_inference's."""
    m = nip_amd.Model.from_spec(*synth.wide_spec(64, 16))
    ov, q = [m.variable("O1")], [m.variable("X1")]
    obs = synth.observations(12, 40, 16, seed=2)
    fp, fl, fs = run(nip_amd.forward_inference, m, obs, ov, q)
    sp, sl, ss = run(nip_amd.forward_backward_inference, m, obs, ov, q)
    assert np.abs(fp.sum(axis=2) - 1).max() <= 1e-12
    assert np.abs(fp[:, -1] - sp[:, -1]).max() <= 1e-12
    assert np.array_equal(fl, sl) and not fs.any() and not ss.any()


def test_filter_ll_equals_smoothing_ll():
    nodes, pots = synth.hmm_spec(16, 16)
    m = nip_amd.Model.from_spec(nodes, pots)
    obs = synth.observations(64, 256, 16, seed=8)
    ov, q = [m.variable("M1")], [m.variable("P1")]
    fp, fl, _ = run(nip_amd.forward_inference, m, obs, ov, q)
    sp, sl, _ = run(nip_amd.forward_backward_inference, m, obs, ov, q)
    assert np.all(np.abs(fl - sl) <= 1e-12 * np.abs(sl))
    assert np.abs(fp[:, -1] - sp[:, -1]).max() <= 1e-12
