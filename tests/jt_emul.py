"""TEST INFRASTRUCTURE: a sequential CPU replay of the general join-tree
engine's compiled schedule (nip_amd/csrc/jtree.h, jtree_plan.cpp).

The host planner's output -- visits, factors, projections, distribute passes,
outputs -- is dumped through the test hook nipamd_jt_plan_dump (no device
work) and executed here exactly as jtree.hip's kernels execute it, one
sequence at a time.  CPU tests compare the replay with the oracle, so the
schedule the GPU runs is checked without a GPU; the GPU tests then compare
the kernels with the same oracle.  Never imported by the product.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

import nip_amd

HDR = ["ncl", "K", "ws", "fwd", "bwd", "post", "down", "ndown", "out", "nout", "fac", "maps", "pres",
       "fwd_root_proj", "bwd_root_proj", "fwd_root_psi", "fwd_root_size", "bwd_root_psi",
       "bwd_root_size", "pi_off", "w_off", "ws_alpha", "ws_beta", "ws_out", "ws_slab", "slab", "L",
       "lds", "stride"]
DBL_MAX = np.finfo(np.float64).max


def dump(model, obs_vars, query, estep=False):
    L = nip_amd.lib()
    L.nipamd_jt_plan_dump.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_int,
                                      C.c_void_p, C.c_int, C.c_void_p, C.c_long, C.c_void_p, C.c_long,
                                      C.c_void_p]
    hdr = np.zeros(len(HDR), np.int32)
    sizes = np.zeros(2, np.int64)
    ov = np.ascontiguousarray(obs_vars, np.int32)
    q = np.ascontiguousarray(query, np.int32)
    args = [model._h, len(ov), ov.ctypes.data, len(q), q.ctypes.data, int(estep), hdr.ctypes.data, len(HDR)]
    rc = L.nipamd_jt_plan_dump(*args, None, 0, None, 0, sizes.ctypes.data)
    if rc:
        raise nip_amd.NipError(rc, L.nipamd_last_error().decode())
    ip = np.zeros(max(1, sizes[0]), np.int32)
    dp = np.zeros(max(1, sizes[1]), np.float64)
    rc = L.nipamd_jt_plan_dump(*args, ip.ctypes.data, len(ip), dp.ctypes.data, len(dp), sizes.ctypes.data)
    assert rc == 0
    return dict(zip(HDR, (int(x) for x in hdr))), ip, dp


class Replay:
    def __init__(self, model, obs_vars, query, estep=False):
        self.h, self.ip, self.dp = dump(model, obs_vars, query, estep)
        h = self.h
        self.dp = self.dp.copy()
        self.maps = self.ip[h["maps"]:]
        self.pres = self.ip[h["pres"]:]
        self.ws = np.zeros(h["ws"])
        # m1 weights: evidence-free backward sweep with beta = 1, unnormalised
        ws = self.ws
        ws[h["ws_beta"]:h["ws_beta"] + h["K"]] = 1.0
        self.collect(h["bwd"], None)
        self.dp[h["w_off"]:h["w_off"] + h["K"]] = self.marg(h["bwd_root_psi"], h["bwd_root_size"],
                                                            h["bwd_root_proj"], h["K"])

    def visits(self, off):
        v = self.ip[off:off + 8 * self.h["ncl"]].reshape(self.h["ncl"], 8)
        return [dict(zip(["size", "base", "psi", "fac0", "nfac", "up_proj", "up_D", "up_msg"], map(int, r)))
                for r in v]

    def slot(self, off, n):
        """A workspace slot; the kernels index one unit's workspace the
        same way, so a slot past its end would hit the next unit's."""
        assert 0 <= off and off + n <= len(self.ws), ("workspace overrun", off, n, len(self.ws))
        return slice(off, off + n)

    def marg(self, psi, size, proj, D):
        src = self.ws[self.slot(psi, size)]
        R = size // D
        pre = self.pres[proj:proj + size].reshape(D, R)
        return np.array([sum(src[pre[j, r]] for r in range(R)) for j in range(D)])

    def collect(self, off, orow):
        h, ws = self.h, self.ws
        F = self.ip[h["fac"]:]
        for v in self.visits(off):
            x = self.dp[v["base"]:v["base"] + v["size"]].copy()
            for k in range(v["nfac"]):
                kind, proj, arg = (int(a) for a in F[3 * (v["fac0"] + k):3 * (v["fac0"] + k) + 3])
                mp = self.maps[proj:proj + v["size"]]
                if kind == 0:
                    c = -1 if orow is None else int(orow[arg])
                    if c >= 0:
                        x = np.where(mp == c, x, 0.0)
                else:
                    x = x * ws[arg + mp]
            ws[self.slot(v["psi"], v["size"])] = x
            if v["up_proj"] >= 0:
                ws[self.slot(v["up_msg"], v["up_D"])] = self.marg(v["psi"], v["size"], v["up_proj"], v["up_D"])

    def fb(self, obs, filt=False, estep=False):
        """(post [T, stride], ll) of one sequence, obs [T, n_obs]; with
        estep (a plan built with estep=True): (counts slab, ll, bad)."""
        h, ws = self.h, self.ws
        T, K = obs.shape[0], h["K"]
        a = h["ws_alpha"]
        ws[a:a + K] = self.dp[h["pi_off"]:h["pi_off"] + K]
        msgA = np.zeros((T, K))
        ll = 0.0
        bad = False
        for t in range(T):
            m1 = float(np.dot(ws[a:a + K], self.dp[h["w_off"]:h["w_off"] + K]))
            self.collect(h["fwd"], obs[t])
            out = self.marg(h["fwd_root_psi"], h["fwd_root_size"], h["fwd_root_proj"], K)
            self.slot(h["ws_out"], K)
            m2 = float(out.sum())
            ws[a:a + K] = out / m2 if m2 != 0 else out
            msgA[t] = ws[a:a + K]
            if (obs[t] >= 0).any() and m1 > 0 and m2 > 0:
                ll += np.log(m2) - np.log(m1)
            if m2 == 0:
                ll = -DBL_MAX
            if m1 <= 0 or m2 <= 0 or ll > 0:
                bad = True
        msgB = np.ones((T, K))
        if not filt:
            b = h["ws_beta"]
            ws[b:b + K] = 1.0
            for t in range(T - 1, 0, -1):
                self.collect(h["bwd"], obs[t])
                out = self.marg(h["bwd_root_psi"], h["bwd_root_size"], h["bwd_root_proj"], K)
                s = out.sum()
                ws[b:b + K] = out / s if s != 0 else out
                msgB[t - 1] = ws[b:b + K]
        post = np.zeros((T, h["stride"]))
        slab = np.zeros(h["slab"])
        D = self.ip[h["down"]:h["down"] + 9 * h["ndown"]].reshape(-1, 9)
        O = self.ip[h["out"]:h["out"] + 6 * h["nout"]].reshape(-1, 6)
        for t in range(T):
            ws[a:a + K] = self.dp[h["pi_off"]:h["pi_off"] + K] if t == 0 else msgA[t - 1]
            ws[h["ws_beta"]:h["ws_beta"] + K] = 1.0 if (filt or t == T - 1) else msgB[t]
            self.collect(h["post"], obs[t])
            for p_psi, p_size, pS, S_D, mu, tmp, c_psi, c_size, cS in D:
                self.slot(tmp, S_D)
                self.slot(mu, S_D)
                new = self.marg(p_psi, p_size, pS, S_D)
                mp = self.maps[cS:cS + c_size]
                old = ws[mu + mp]
                x = ws[c_psi:c_psi + c_size] * new[mp]
                ws[c_psi:c_psi + c_size] = np.where(old != 0, x / np.where(old != 0, old, 1.0), 0.0)
            for psi, size, proj, Dn, dst, t0_only in O:
                if estep and t0_only and t > 0:
                    continue
                m = self.marg(psi, size, proj, Dn)
                self.slot(h["ws_out"], Dn)
                if estep:
                    self.slot(h["ws_slab"] + dst, Dn)
                s = m.sum()
                m = m / s if s != 0 else m
                if estep:
                    slab[dst:dst + Dn] += m
                else:
                    post[t, dst:dst + Dn] = m
        if estep:
            return slab, ll, bad
        return post, ll
