"""A textbook scaled forward-backward smoother over an interface chain,
vectorised over sequences (numpy, fp64), built from a compiled model's own
tables -- no join tree, no kernel code.  The check of the GPU chain kernels at
full config sizes, where the oracle's join-tree propagation is too slow
(config 5's 16.7M-entry in-clique costs seconds per slice).

  A[x][y] = sum_H in-clique(x, y, H) prod prior(h)    (hidden parents folded)
  e_t[y]  = prod_k E_k[y][m_k,t]   (the row sum s_k[y] for a missing value)
  alpha_t = e_t o A^T alpha_{t-1} (normalised), alpha_{-1} = prior(prev)
  beta_t  = A (e_{t+1} o beta_{t+1}) (normalised), beta_{T-1} = 1
  ll      = sum_t log sum(A^T alpha_{t-1} o e_t) - log sum(A^T alpha_{t-1} o s)
"""
import ctypes as C

import numpy as np

import nip_amd


def clique_vars(m, c):
    vars_ = (C.c_int * 64)()
    links = (C.c_int * 64)()
    nv, nl = C.c_int(0), C.c_int(0)
    assert nip_amd.lib().nipamd_model_clique(m._h, c, vars_, C.byref(nv), links, C.byref(nl)) == 0
    return list(vars_[:nv.value])


def table(m, want, out):
    """The original table of the clique holding every variable of `want`,
    summed under the priors of its other variables (none for the chain's
    cliques but the hidden parents), as an array over `out`."""
    nc = nip_amd.lib().nipamd_model_num_cliques(m._h)
    cin = next(c for c in range(nc) if set(want) <= set(clique_vars(m, c)))
    cv = clique_vars(m, cin)
    arr = m.original(cin).reshape([m.card(v) for v in reversed(cv)])   # axes: last variable first
    letters = "abcdefghij"
    ax = {v: letters[len(cv) - 1 - i] for i, v in enumerate(cv)}
    ops, subs = [arr], ["".join(ax[v] for v in reversed(cv))]
    for v in cv:
        if v not in out:
            ops.append(m.prior(v))
            subs.append(ax[v])
    return np.einsum(",".join(subs) + "->" + "".join(ax[v] for v in out), *ops)


def chain_tables(m, prev, cur, children):
    A = table(m, [prev, cur], [prev, cur])
    Es = [table(m, [cur, o], [cur, o]) for o in children]
    return A, m.prior(prev), Es


def smoother(A, pi, Es, cols):
    """cols: one [B, T] int array per child (-1 missing).  Returns smoothed
    [B, T, N], filtered [B, T, N] and ll [B]."""
    B, T = cols[0].shape
    N = A.shape[0]
    s_all = np.ones(N)
    for E in Es:
        s_all = s_all * E.sum(axis=1)

    def ev(t):
        e = np.ones((B, N))
        for E, c in zip(Es, cols):
            x = c[:, t]
            ee = E[:, np.maximum(x, 0)].T.copy()
            ee[x < 0] = E.sum(axis=1)
            e *= ee
        return e

    ah = np.zeros((B, T, N))
    ll = np.zeros(B)
    prev = np.tile(pi, (B, 1))
    for t in range(T):
        u = prev @ A
        al = u * ev(t)
        c = al.sum(axis=1)
        ll += np.log(c) - np.log((u * s_all).sum(axis=1))
        prev = al / c[:, None]
        ah[:, t] = prev
    post = np.empty_like(ah)
    post[:, T - 1] = ah[:, T - 1]
    b = np.ones((B, N))
    for t in range(T - 2, -1, -1):
        b = (ev(t + 1) * b) @ A.T
        b = b / b.sum(axis=1, keepdims=True)
        p = ah[:, t] * b
        post[:, t] = p / p.sum(axis=1, keepdims=True)
    return post, ah, ll
