"""The interface chain's transition folded on the GPU (fold.hip, SURVEY 8(d)
config 5's LDS-tiled marginalise): the in-clique's hidden parents summed out
under their priors -- what the reference's nip_general_marginalise does to
the in-clique every time slice (src/nippotential.c:267-311).

Checked against a numpy contraction of the model's own tables (tolerance
1e-14 relative: sums of up to 4096 positive terms in another order), for the
transition and for each hidden parent's kept-dimension table; at config 5's
64^4 entries the engine defers the fold to the GPU, and forward-backward
through it is checked against the CPU oracle at T = 2 (the oracle
propagates the whole 16.7M-entry clique; no fold involved).
"""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

import nip_amd
from nip_amd import synth
from oracle.bind import PortOracle

FOLD_RTOL = 1e-14


def clique_vars(m, c):
    vars_ = (C.c_int * 64)()
    links = (C.c_int * 64)()
    nv, nl = C.c_int(0), C.c_int(0)
    assert nip_amd.lib().nipamd_model_clique(m._h, c, vars_, C.byref(nv), links, C.byref(nl)) == 0
    return list(vars_[:nv.value])


def numpy_fold(m, prev, cur, hidden, keep=-1):
    """A[x][y] (or G_keep[g][x][y]) from the in-clique's original table."""
    cin = next(c for c in range(nip_amd.lib().nipamd_model_num_cliques(m._h))
               if prev in clique_vars(m, c))
    cv = clique_vars(m, cin)
    arr = m.original(cin).reshape([m.card(v) for v in reversed(cv)])   # axes: last var first
    letters = "abcdefgh"
    ax = {v: letters[len(cv) - 1 - i] for i, v in enumerate(cv)}
    ops, subs = [arr], ["".join(ax[v] for v in reversed(cv))]
    for h in hidden:
        ops.append(m.prior(h))
        subs.append(ax[h])
    outs = (ax[hidden[keep]] if keep >= 0 else "") + ax[prev] + ax[cur]
    return np.einsum(",".join(subs) + "->" + outs, *ops)


@pytest.mark.parametrize("card", [4, 8, 16, 32])
def test_fold_matches_numpy(card):
    m = nip_amd.Model.from_spec(*synth.wide_spec(card, 5))
    X0, X1, Y1, Z1 = (m.variable(s) for s in ("X0", "X1", "Y1", "Z1"))
    A, ms, nbytes = m.fold()
    ref = numpy_fold(m, X0, X1, [Y1, Z1])
    assert np.all(A[card:, :] == 0) and np.all(A[:, card:] == 0)
    assert np.allclose(A[:card, :card], ref, rtol=FOLD_RTOL, atol=0)
    assert nbytes == card ** 4 * 8 and ms > 0
    for j in range(2):
        G, _, _ = m.fold(j, card)
        gref = numpy_fold(m, X0, X1, [Y1, Z1], keep=j)
        assert np.allclose(G[:, :card, :card], gref, rtol=FOLD_RTOL, atol=0)
        # the kept tables sum to the transition
        assert np.allclose(G.sum(axis=0), A, rtol=1e-13, atol=0)


def test_fold_config5_size_and_bandwidth():
    """64^4 entries (134 MB): the engine's deferred fold, against numpy."""
    m = nip_amd.Model.from_spec(*synth.wide_spec(64, 16))
    X0, X1, Y1, Z1 = (m.variable(s) for s in ("X0", "X1", "Y1", "Z1"))
    A, ms, nbytes = m.fold()
    A2, _, _ = m.fold()
    assert np.array_equal(A, A2)                       # deterministic
    ref = numpy_fold(m, X0, X1, [Y1, Z1])
    assert np.allclose(A, ref, rtol=FOLD_RTOL, atol=0)
    assert nbytes == 64 ** 4 * 8
    print("fold: %.3f ms, %.0f GB/s" % (ms, nbytes / ms / 1e6))


def test_deferred_fold_fb_matches_oracle_64_states():
    """Config 5 at full width through the deferred GPU fold, against the CPU
    oracle's propagation of the whole in-clique (T = 2, one sequence)."""
    m = nip_amd.Model.from_spec(*synth.wide_spec(64, 16))
    ov, q = [m.variable("O1")], [m.variable("X1")]
    obs = synth.observations(1, 2, 16, seed=9)
    post, ll, st = nip_amd.forward_backward_inference(m, torch.from_numpy(obs).cuda(), ov, q)
    torch.cuda.synchronize()
    post, ll = post.cpu().numpy(), ll.cpu().numpy()
    assert not st.any().item()
    rp, rl = PortOracle(m.desc()).fb(obs[0], ov, q)
    assert np.abs(post[0] - rp).max() <= 1e-12
    assert abs(ll[0] - rl) <= 1e-11 * max(1.0, abs(rl))


def test_config5_full_size_vs_textbook():
    """Config 5 at its bench size (256 x 128, 64 states) through the deferred
    fold and chain_wide4_kernel, every sequence against the textbook smoother
    over the model's own tables (tests/textbook_util.py)."""
    from textbook_util import chain_tables, smoother
    m = nip_amd.Model.from_spec(*synth.wide_spec(64, 16))
    X0, X1, O1 = m.variable("X0"), m.variable("X1"), m.variable("O1")
    obs = synth.observations(256, 128, 16, seed=6)
    obs[7, :5, 0] = -1                                  # a leading missing run
    obs[9, 40:50, 0] = -1
    o = torch.from_numpy(obs).cuda()
    post, ll, st = nip_amd.forward_backward_inference(m, o, [O1], [X1])
    fpost, fll, _ = nip_amd.forward_inference(m, o, [O1], [X1])
    torch.cuda.synchronize()
    assert not st.any().item()
    A, pi, Es = chain_tables(m, X0, X1, [O1])
    tp, tf, tl = smoother(A, pi, Es, [obs[:, :, 0]])
    assert np.abs(post.cpu().numpy() - tp).max() <= 1e-12
    assert np.abs(fpost.cpu().numpy() - tf).max() <= 1e-12
    assert np.all(np.abs(ll.cpu().numpy() - tl) <= 1e-11 * np.abs(tl))
    assert np.all(np.abs(fll.cpu().numpy() - tl) <= 1e-11 * np.abs(tl))
