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


# ---------------------------------------------------------------------------
# The same textbook recursions in torch fp64 on the GPU, for the full-size
# checks (config 2: 4096 x 1024; config 4: 131072 x 1024), where numpy would
# take minutes.  Independent of the engine: plain matmuls and elementwise ops
# over the model's compiled tables (chain_tables).

def _ev_torch(Es, s_list, cols, t):
    """e_t [B, N] over the children (cols: [B, T] long tensors, -1 missing)."""
    e = None
    for E, s, c in zip(Es, s_list, cols):
        x = c[:, t]
        ee = E[:, x.clamp(min=0)].T
        ee = torch_where(x < 0, s, ee)
        e = ee if e is None else e * ee
    return e


def torch_where(mask, s, ee):
    import torch
    return torch.where(mask[:, None], s[None, :].expand_as(ee), ee)


def smoother_torch(A, pi, Es, cols):
    """Smoothed [B, T, N] and ll [B] (torch, on the device of A)."""
    import torch
    B, T = cols[0].shape
    N = A.shape[0]
    s_list = [E.sum(dim=1) for E in Es]
    s_all = torch.ones(N, dtype=A.dtype, device=A.device)
    for s in s_list:
        s_all = s_all * s
    ah = torch.empty((B, T, N), dtype=A.dtype, device=A.device)
    ll = torch.zeros(B, dtype=A.dtype, device=A.device)
    prev = pi[None, :].expand(B, N)
    for t in range(T):
        u = prev @ A
        al = u * _ev_torch(Es, s_list, cols, t)
        c = al.sum(dim=1)
        ll += torch.log(c) - torch.log((u * s_all).sum(dim=1))
        prev = al / c[:, None]
        ah[:, t] = prev
    post = torch.empty_like(ah)
    post[:, T - 1] = ah[:, T - 1]
    b = torch.ones((B, N), dtype=A.dtype, device=A.device)
    for t in range(T - 2, -1, -1):
        b = (_ev_torch(Es, s_list, cols, t + 1) * b) @ A.T
        b = b / b.sum(dim=1, keepdim=True)
        p = ah[:, t] * b
        post[:, t] = p / p.sum(dim=1, keepdim=True)
    return post, ll


def hmm_estep_torch(A, pi, E, obs):
    """The e_step of an HMM slice (prev, cur, one child) in the em_learn
    layout [P0 | P1|P0 (y + N x) | M1|P1 (m + M y)] (nip.c:1925-1967: each
    family marginal normalised per step, P0 at t = 0 only, a missing
    observation split as E(y, m) / s(y)), and the per-sequence ll.
    obs: [B, T] long tensor (-1 missing).  Sums over sequences and steps in
    torch's order (a check at 1e-11 relative, not a bit-exact one)."""
    import torch
    B, T = obs.shape
    N, M = E.shape
    s = E.sum(dim=1)
    dev, dt = A.device, A.dtype
    # forward: alpha^_t normalised; backward: beta^_t normalised
    ah = torch.empty((B, T, N), dtype=dt, device=dev)
    ll = torch.zeros(B, dtype=dt, device=dev)
    prev = pi[None, :].expand(B, N)
    for t in range(T):
        u = prev @ A
        al = u * _ev_torch([E], [s], [obs], t)
        c = al.sum(dim=1)
        ll += torch.log(c) - torch.log((u * s).sum(dim=1))
        prev = al / c[:, None]
        ah[:, t] = prev
    c0 = torch.zeros(N, dtype=dt, device=dev)
    c1 = torch.zeros((N, N), dtype=dt, device=dev)
    c2 = torch.zeros((N, M), dtype=dt, device=dev)
    b = torch.ones((B, N), dtype=dt, device=dev)
    ar = torch.arange(M, device=dev)
    for t in range(T - 1, -1, -1):
        if t < T - 1:
            b = (_ev_torch([E], [s], [obs], t + 1) * b) @ A.T
            b = b / b.sum(dim=1, keepdim=True)
        e = _ev_torch([E], [s], [obs], t)
        w = e * b
        pv = ah[:, t - 1] if t > 0 else pi[None, :].expand(B, N)
        n = ((pv @ A) * w).sum(dim=1)
        c1 += A * ((pv / n[:, None]).T @ w)
        g = ah[:, t] * b
        g = g / g.sum(dim=1, keepdim=True)
        m = obs[:, t]
        miss = m < 0
        oh = (m[:, None] == ar[None, :]).to(dt)
        c2 += g.T @ oh
        if bool(miss.any()):
            c2 += g[miss].sum(dim=0)[:, None] * E / s[:, None]
        if t == 0:
            g0 = pi[None, :] * (w @ A.T)
            c0 += (g0 / g0.sum(dim=1, keepdim=True)).sum(dim=0)
    return torch.cat([c0, c1.reshape(-1), c2.reshape(-1)]), ll


def chain_sums_torch(A, pi, Es, cols):
    """The wide chain e_step's three sums (estep_wide.hip / estep_mw.hip, DESIGN.md
    4) over B sequences of an interface chain with children Es (cols: one [B, T]
    long tensor per child, -1 missing; every child observed):
      K [N, N]   = sum_t alpha_{t-1}(x) e_t(y) beta_t(y) / Z   (alpha_{-1} = prior)
      H_k [M_k + 2, N] = sum_t [row of child k's code at t] gamma_t(y)
                   (rows: the states, then missing, then out of range)
      P0 [N]     = gamma_{-1} = prior o beta_{-1} / Z,
    and the per-sequence ll -- each step normalised on its own, as the
    reference's family marginals are (nip.c:1925-1967); sums in torch's order."""
    import torch
    B, T = cols[0].shape
    N = A.shape[0]
    dev, dt = A.device, A.dtype
    s_list = [E.sum(dim=1) for E in Es]
    s_all = torch.ones(N, dtype=dt, device=dev)
    for s in s_list:
        s_all = s_all * s
    ah = torch.empty((B, T, N), dtype=dt, device=dev)
    ll = torch.zeros(B, dtype=dt, device=dev)
    prev = pi[None, :].expand(B, N)
    for t in range(T):
        u = prev @ A
        al = u * _ev_torch(Es, s_list, cols, t)
        c = al.sum(dim=1)
        ll += torch.log(c) - torch.log((u * s_all).sum(dim=1))
        prev = al / c[:, None]
        ah[:, t] = prev
    K = torch.zeros((N, N), dtype=dt, device=dev)
    Hs = [torch.zeros((E.shape[1] + 2, N), dtype=dt, device=dev) for E in Es]
    P0 = torch.zeros(N, dtype=dt, device=dev)
    b = torch.ones((B, N), dtype=dt, device=dev)
    for t in range(T - 1, -1, -1):
        if t < T - 1:
            b = (_ev_torch(Es, s_list, cols, t + 1) * b) @ A.T
            b = b / b.sum(dim=1, keepdim=True)
        w = _ev_torch(Es, s_list, cols, t) * b
        pv = ah[:, t - 1] if t > 0 else pi[None, :].expand(B, N)
        n = ((pv @ A) * w).sum(dim=1)
        K += (pv / n[:, None]).T @ w
        g = ah[:, t] * b
        g = g / g.sum(dim=1, keepdim=True)
        for H, E, c in zip(Hs, Es, cols):
            M = E.shape[1]
            r = c[:, t]
            r = torch.where(r < 0, torch.full_like(r, M), torch.where(r >= M, torch.full_like(r, M + 1), r))
            H.index_add_(0, r, g)
        if t == 0:
            g0 = pi[None, :] * (w @ A.T)
            P0 += (g0 / g0.sum(dim=1, keepdim=True)).sum(dim=0)
    return K, Hs, P0, ll
