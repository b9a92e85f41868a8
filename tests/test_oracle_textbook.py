"""Pin of the oracle's time-slice loops against an independent textbook.

oracle/_ref compiles the reference's propagation primitives unmodified, but
nip.c's time loops (forward_backward_inference, forward_inference, e_step,
nip.c:1103-2007) are restated in oracle/ref/nipref_harness.c.  These tests
check that restatement -- and through test_oracle.py's bit-exactness the C
port oracle/nip_oracle.c -- against a textbook scaled forward-backward
smoother written here in numpy straight from the CPT data (no join tree, no
reference code), i.e. the interface-chain algebra SURVEY.md 8(a)/DESIGN.md 2
derive:

  A[x][y] = sum_h P(cur=y | prev=x, h) prod prior(h)      (hidden parents folded)
  e_t[y]  = prod_k E_k[y][m_k,t]  (row sum for a missing value)
  alpha_t = e_t o A^T alpha_{t-1},  alpha_{-1} = prior(prev)
  beta_t  = A (e_{t+1} o beta_{t+1}), beta_{T-1} = 1
  ll      = sum_t log sum(A^T alpha^_{t-1} o e_t) - log sum(A^T alpha^_{t-1} o s)

on the HMM of config 2 (fb, filter, e_step counts) and on demo1's structure
(two observed children and a hidden parent: fb and filter).  Tolerances:
posteriors 1e-12 absolute, ll 1e-12 relative, counts 1e-11 relative.

The e_step's BAD_LUCK rule (nip.c:1827-1854: m1 <= 0, m2 <= 0 or a running ll
> 0) is checked on missing data: the reference flags only sequences whose
running ll sits at 0 up to rounding, i.e. within a leading run of missing
observations -- the divergence DESIGN.md 6 records (nip_amd accepts them).
"""
import numpy as np
import pytest

from nip_amd import synth
from oracle import bind

pytestmark = pytest.mark.skipif(not bind.ref_available(), reason="oracle/_ref not built")


def harness(nodes, pots):
    return bind.RefHarness(synth.spec_to_replay(nodes, pots), cards=[n[1] for n in nodes])


def pot(pots, child):
    return next(np.asarray(d, np.float64) for ch, ps, d in pots if ch == child)


def evidence(E_list, cols, t, N):
    """e_t[y] over the observed children (missing = -1: the row sum)."""
    e = np.ones(N)
    for E, m in zip(E_list, cols):
        e = e * (E.sum(axis=1) if m[t] < 0 else E[:, m[t]])
    return e


def textbook(A, pi, E_list, cols, s_all):
    """Scaled two-filter smoother; returns smoothed, filtered, ll, and the
    per-step pieces the e_step counts need."""
    T = len(cols[0])
    N = A.shape[0]
    ah = np.zeros((T, N))
    ll = 0.0
    prev = pi.copy()
    for t in range(T):
        u = A.T @ prev
        al = u * evidence(E_list, cols, t, N)
        ll += np.log(al.sum()) - np.log((u * s_all).sum())
        prev = al / al.sum()
        ah[t] = prev
    be = np.zeros((T, N))
    b = np.ones(N)
    be[T - 1] = b
    for t in range(T - 2, -1, -1):
        b = A @ (evidence(E_list, cols, t + 1, N) * b)
        b = b / b.sum()
        be[t] = b
    post = ah * be
    post /= post.sum(axis=1, keepdims=True)
    return post, ah, ll, be


def quirk(t, axis):
    """The reference's CPT normalisation (huginnet.y:635-636): along the
    family's lowest-ID variable, which is the parent when the parent was
    declared first (nip_normalise_cpd over dimension 0 of the ID-sorted
    potential; compile.cpp reproduces it)."""
    return t / t.sum(axis=axis, keepdims=True)


def hmm_tables(N, M, seed):
    nodes, pots = synth.hmm_spec(N, M, seed=seed)
    A = quirk(pot(pots, "P1").reshape(N, N), 0)   # [prev x][cur y], normalised over x (P0 < P1)
    E = quirk(pot(pots, "M1").reshape(N, M), 0)   # [y][m], normalised over y (P1 < M1)
    pi = pot(pots, "P0")
    return nodes, pots, A, E, pi


@pytest.mark.parametrize("N,M,B,T,miss", [(5, 4, 6, 17, 0.0), (16, 16, 4, 40, 0.0), (7, 3, 5, 23, 0.3)])
def test_hmm_fb_filter_vs_textbook(N, M, B, T, miss):
    nodes, pots, A, E, pi = hmm_tables(N, M, seed=N * 31 + M)
    ref = harness(nodes, pots)
    obs = synth.observations(B, T, M, seed=N + T)
    rng = np.random.default_rng(N)
    obs[rng.random(obs.shape) < miss] = -1
    for b in range(B):
        cols = [obs[b, :, 0]]
        post, ah, ll, _ = textbook(A, pi, [E], cols, E.sum(axis=1))
        rp, rl = ref.fb(obs[b], [2], [1])
        fp, fl = ref.fb(obs[b], [2], [1], filter_only=True)
        assert np.abs(rp - post).max() <= 1e-12
        assert np.abs(fp - ah).max() <= 1e-12
        assert abs(rl - ll) <= 1e-12 * max(1.0, abs(ll)) and abs(fl - ll) <= 1e-12 * max(1.0, abs(ll))


def test_demo1_structure_fb_filter_vs_textbook():
    """demo1.net's slice: C0 -> C1 with hidden parent D1, children A1, B1."""
    card = 4
    nodes, pots = synth.demo1_spec(card, seed=77)
    # ids: A1 0, B1 1, C0 2, C1 3, D1 4; C1's family is normalised over C0
    P = quirk(pot(pots, "C1").reshape(card, card, card), 1)   # [D1][C0][C1] (first parent outermost)
    pD = pot(pots, "D1")
    A = np.einsum("dxy,d->xy", P, pD)
    EA = quirk(pot(pots, "A1").reshape(card, card), 1)        # [C1][A1], over A1 (A1 < C1)
    EB = quirk(pot(pots, "B1").reshape(card, card), 1)
    pi = pot(pots, "C0")
    ref = harness(nodes, pots)
    names = [n[0] for n in nodes]
    ia, ib, ic = names.index("A1"), names.index("B1"), names.index("C1")
    obs = synth.observations(5, 19, card, seed=3, n_obs=2)
    obs[1, 4:9, 0] = -1
    for b in range(obs.shape[0]):
        cols = [obs[b, :, 0], obs[b, :, 1]]
        s_all = EA.sum(axis=1) * EB.sum(axis=1)
        post, ah, ll, _ = textbook(A, pi, [EA, EB], cols, s_all)
        rp, rl = ref.fb(obs[b], [ia, ib], [ic])
        fp, fl = ref.fb(obs[b], [ia, ib], [ic], filter_only=True)
        assert np.abs(rp - post).max() <= 1e-12
        assert np.abs(fp - ah).max() <= 1e-12
        assert abs(rl - ll) <= 1e-12 * max(1.0, abs(ll))


def textbook_estep(A, pi, E, obs):
    """Expected counts in the em_learn layout [P0 | P1|P0 (y + N x) | M1|P1 (m + M y)]."""
    N, M = E.shape
    c0, c1, c2 = np.zeros(N), np.zeros((N, N)), np.zeros((N, M))
    s = E.sum(axis=1)
    for o in obs:
        m = o[:, 0]
        post, ah, _, be = textbook(A, pi, [E], [m], s)
        T = len(m)
        prevs = np.vstack([pi, ah[:-1]])
        for t in range(T):
            e = s if m[t] < 0 else E[:, m[t]]
            xi = prevs[t][:, None] * A * (e * be[t])[None, :]
            c1 += xi / xi.sum()
            if m[t] < 0:
                c2 += post[t][:, None] * E / s[:, None]
            else:
                c2[:, m[t]] += post[t]
        g = pi * (A @ (evidence([E], [m], 0, N) * be[0]))
        c0 += g / g.sum()
    return np.concatenate([c0, c1.ravel(), c2.ravel()])


@pytest.mark.parametrize("N,M,miss", [(5, 4, 0.0), (6, 3, 0.25)])
def test_hmm_estep_vs_textbook(N, M, miss):
    nodes, pots, A, E, pi = hmm_tables(N, M, seed=N * 7 + M)
    ref = harness(nodes, pots)
    obs = synth.observations(8, 21, M, seed=N)
    rng = np.random.default_rng(M)
    obs[rng.random(obs.shape) < miss] = -1
    obs[:, 0] = np.where(obs[:, 0] < 0, 0, obs[:, 0])     # no leading missing run (see below)
    cnt, ll, bad = ref.estep(obs, [2], np.zeros(ref.param_size()))
    assert not bad.any()
    want = textbook_estep(A, pi, E, obs)
    assert np.all(np.abs(cnt - want) <= 1e-11 * np.maximum(1.0, np.abs(want)))
    for b in range(obs.shape[0]):
        _, _, l, _ = textbook(A, pi, [E], [obs[b, :, 0]], E.sum(axis=1))
        assert abs(ll[b] - l) <= 1e-12 * max(1.0, abs(l))


def test_bad_luck_only_on_leading_missing_runs():
    """The reference's e_step BAD_LUCK on missing data (nip.c:1838): its
    running ll is exactly 0 in exact arithmetic until the first observed
    value, and m1, m2 come from two propagations, so rounding can push it to
    +1e-16 there.  Flags therefore fall only on sequences that start with a
    missing value; elsewhere the running ll is clearly negative."""
    N, M = 6, 5
    nodes, pots, A, E, pi = hmm_tables(N, M, seed=99)
    ref = harness(nodes, pots)
    obs = synth.observations(64, 12, M, seed=5)
    rng = np.random.default_rng(7)
    obs[rng.random(obs.shape) < 0.35] = -1
    obs[:8] = -1                                      # fully missing sequences
    _, ll, bad = ref.estep(obs, [2], np.zeros(ref.param_size()))
    lead = obs[:, 0, 0] < 0
    assert not (bad.astype(bool) & ~lead).any()
    assert np.all(np.abs(ll[:8]) <= 1e-13)             # fully missing: ll = 0 up to rounding
    ok = bad == 0
    for b in np.nonzero(ok)[0]:
        _, _, l, _ = textbook(A, pi, [E], [obs[b, :, 0]], E.sum(axis=1))
        assert abs(ll[b] - l) <= 1e-12 * max(1.0, abs(l))


@pytest.mark.parametrize("N,M,miss", [(5, 4, 0.0), (16, 16, 0.2)])
def test_torch_textbook_estep_vs_reference(N, M, miss):
    """tests/textbook_util.py's torch e_step (the full-shard check of
    test_gpu_em_dist.py, run there on the GPU) against the reference's own
    e_step, here on the CPU: counts 1e-11, ll 1e-12."""
    torch = pytest.importorskip("torch")
    from textbook_util import hmm_estep_torch, smoother_torch
    nodes, pots, A, E, pi = hmm_tables(N, M, seed=N * 5 + M)
    ref = harness(nodes, pots)
    obs = synth.observations(9, 23, M, seed=N + 1)
    rng = np.random.default_rng(M + 1)
    obs[rng.random(obs.shape) < miss] = -1
    obs[:, 0] = np.where(obs[:, 0] < 0, 0, obs[:, 0])     # no leading missing run
    cnt, ll, bad = ref.estep(obs, [2], np.zeros(ref.param_size()))
    assert not bad.any()
    tA, tE, tpi = (torch.from_numpy(x) for x in (A, E, pi))
    tobs = torch.from_numpy(obs[:, :, 0].astype(np.int64))
    got, gll = hmm_estep_torch(tA, tpi, tE, tobs)
    got = got.numpy()
    assert np.all(np.abs(got - cnt) <= 1e-11 * np.maximum(1.0, np.abs(cnt))), np.abs(got - cnt).max()
    assert np.all(np.abs(gll.numpy() - ll) <= 1e-12 * np.maximum(1.0, np.abs(ll)))
    post, sll = smoother_torch(tA, tpi, [tE], [tobs])
    for b in range(obs.shape[0]):
        rp, rl = ref.fb(obs[b], [2], [1])
        assert np.abs(post[b].numpy() - rp).max() <= 1e-12
        assert abs(sll[b].item() - rl) <= 1e-12 * max(1.0, abs(rl))
