"""ctypes bindings for the oracle libraries -- TEST INFRASTRUCTURE ONLY."""
from __future__ import annotations

import ctypes as C
import json
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# NIPAMD_ORACLE_SO: another build of the port (the sanitizer test loads an ASan/UBSan one)
PORT_SO = os.environ.get("NIPAMD_ORACLE_SO", os.path.join(HERE, "libnip_oracle.so"))
REF_SO = os.path.join(HERE, "_ref", "libnipref.so")
REF_SRC = os.environ.get("NIP_REFERENCE_SRC", "/root/reference/src")

_i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")


def build(ref: bool | None = None) -> None:
    """Compile the port (always) and the reference build (when its sources exist)."""
    targets = ["port"]
    if ref or (ref is None and os.path.isdir(REF_SRC)):
        targets.append("ref")
    subprocess.check_call(["make", "-s", "-C", HERE, "REF=" + REF_SRC] + targets)


def ref_available() -> bool:
    return os.path.exists(REF_SO)


class NoDesc(C.Structure):
    _fields_ = [
        ("nvars", C.c_int), ("card", C.c_void_p), ("ifs", C.c_void_p),
        ("par_off", C.c_void_p), ("par", C.c_void_p),
        ("prior_off", C.c_void_p), ("priors", C.c_void_p),
        ("family", C.c_void_p), ("fmap_off", C.c_void_p), ("fmap", C.c_void_p),
        ("ncliques", C.c_int), ("cv_off", C.c_void_p), ("cv", C.c_void_p),
        ("lk_off", C.c_void_p), ("lk", C.c_void_p),
        ("orig_off", C.c_void_p), ("orig", C.c_void_p),
        ("nsepsets", C.c_int), ("sa", C.c_void_p), ("sb", C.c_void_p),
        ("sv_off", C.c_void_p), ("sv", C.c_void_p),
        ("in_clique", C.c_int), ("out_clique", C.c_int),
        ("nout", C.c_int), ("outgoing", C.c_void_p), ("prev_outgoing", C.c_void_p),
        ("nindep", C.c_int), ("independent", C.c_void_p),
    ]


def _csr(lists, dtype):
    off = np.zeros(len(lists) + 1, np.int32)
    for i, l in enumerate(lists):
        off[i + 1] = off[i] + len(l)
    flat = np.array([x for l in lists for x in l] or [0], dtype=dtype)
    return off, flat


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p)


def make_desc(d: dict):
    """Flatten a JSON join-tree description into a NoDesc (+ keep-alive list)."""
    keep = []

    def arr(x, dt=np.int32):
        a = np.ascontiguousarray(np.array(x if len(x) else [0], dtype=dt))
        keep.append(a)
        return a

    vs = d["vars"]
    nd = NoDesc()
    nd.nvars = len(vs)
    nd.card = _ptr(arr([v["card"] for v in vs]))
    nd.ifs = _ptr(arr([v["if"] for v in vs]))
    o, f = _csr([v["parents"] for v in vs], np.int32); keep += [o, f]
    nd.par_off, nd.par = _ptr(o), _ptr(f)
    prior_off, priors, acc = [], [], 0
    for v in vs:
        if v["prior"] is None:
            prior_off.append(-1)
        else:
            prior_off.append(acc); priors += v["prior"]; acc += len(v["prior"])
    nd.prior_off = _ptr(arr(prior_off)); nd.priors = _ptr(arr(priors, np.float64))
    nd.family = _ptr(arr([v["family"] for v in vs]))
    o, f = _csr([v["family_mapping"] for v in vs], np.int32); keep += [o, f]
    nd.fmap_off, nd.fmap = _ptr(o), _ptr(f)
    cs = d["cliques"]
    nd.ncliques = len(cs)
    o, f = _csr([c["vars"] for c in cs], np.int32); keep += [o, f]
    nd.cv_off, nd.cv = _ptr(o), _ptr(f)
    o, f = _csr([c["links"] for c in cs], np.int32); keep += [o, f]
    nd.lk_off, nd.lk = _ptr(o), _ptr(f)
    o, f = _csr([c["original"] for c in cs], np.float64); keep += [o, f]
    nd.orig_off, nd.orig = _ptr(o), _ptr(f)
    ss = d["sepsets"]
    nd.nsepsets = len(ss)
    nd.sa = _ptr(arr([s["a"] for s in ss])); nd.sb = _ptr(arr([s["b"] for s in ss]))
    o, f = _csr([s["vars"] for s in ss], np.int32); keep += [o, f]
    nd.sv_off, nd.sv = _ptr(o), _ptr(f)
    nd.in_clique, nd.out_clique = d["in_clique"], d["out_clique"]
    nd.nout = len(d["outgoing"])
    nd.outgoing = _ptr(arr(d["outgoing"])); nd.prev_outgoing = _ptr(arr(d["previous_outgoing"]))
    nd.nindep = len(d["independent"]); nd.independent = _ptr(arr(d["independent"]))
    return nd, keep


def _post_stride(desc, vint):
    return int(sum(desc["vars"][v]["card"] for v in vint))


def _obs2d(obs, T, nobs):
    return np.ascontiguousarray(np.asarray(obs, np.int32).reshape(T, nobs))


class PortOracle:
    """The standalone C restatement (bit-identical to the reference by design)."""

    _lib = None

    @classmethod
    def lib(cls):
        if cls._lib is None:
            if not os.path.exists(PORT_SO):
                build(ref=False)
            L = C.CDLL(PORT_SO)
            L.no_create.restype = C.c_void_p
            L.no_create.argtypes = [C.POINTER(NoDesc)]
            L.no_free.argtypes = [C.c_void_p]
            L.no_param_size.argtypes = [C.c_void_p]
            for name in ("no_fb", "no_filter"):
                getattr(L, name).argtypes = [C.c_void_p, C.c_int, C.c_int, _i32p, _i32p,
                                             C.c_int, _i32p, _f64p, C.POINTER(C.c_double)]
            L.no_fb_batch.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, _i32p, _i32p,
                                      C.c_int, _i32p, _f64p, _f64p, C.c_int]
            L.no_estep.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, _i32p, _i32p,
                                   _f64p, _f64p, _f64p, _i32p]
            L.no_m_step.argtypes = [C.c_void_p, _f64p]
            L.no_em.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, _i32p, _i32p,
                                _f64p, C.c_double, C.c_int, _f64p]
            L.no_original.argtypes = [C.c_void_p, C.c_int, _f64p, C.c_int]
            L.no_prior.argtypes = [C.c_void_p, C.c_int, _f64p]
            L.no_query.argtypes = [C.c_void_p, C.c_int, C.c_int, _i32p, _f64p, C.c_int, _f64p]
            cls._lib = L
        return cls._lib

    def __init__(self, desc: dict):
        self.desc = desc
        nd, keep = make_desc(desc)
        self.h = self.lib().no_create(C.byref(nd))
        del keep

    def __del__(self):
        try:
            self.lib().no_free(self.h)
        except Exception:
            pass

    def fb(self, obs, obs_vars, vint, filter_only=False):
        obs_vars = np.asarray(obs_vars, np.int32)
        a = np.asarray(obs)
        T = a.shape[0] if a.ndim == 2 else int(a.size // max(len(obs_vars), 1))
        o = _obs2d(obs, T, len(obs_vars))
        vint = np.asarray(vint, np.int32)
        post = np.zeros((T, _post_stride(self.desc, vint)))
        ll = C.c_double(0)
        fn = self.lib().no_filter if filter_only else self.lib().no_fb
        fn(self.h, T, len(obs_vars), obs_vars, o, len(vint), vint, post, C.byref(ll))
        return post, ll.value

    def fb_batch(self, obs, obs_vars, vint, nthreads=1):
        obs = np.ascontiguousarray(np.asarray(obs, np.int32))
        B, T = obs.shape[0], obs.shape[1]
        obs_vars = np.asarray(obs_vars, np.int32)
        vint = np.asarray(vint, np.int32)
        post = np.zeros((B, T, _post_stride(self.desc, vint)))
        ll = np.zeros(B)
        self.lib().no_fb_batch(self.h, B, T, len(obs_vars), obs_vars, obs.reshape(-1),
                               len(vint), vint, post, ll, nthreads)
        return post, ll

    def param_size(self):
        return self.lib().no_param_size(self.h)

    def estep(self, obs, obs_vars, counts_in):
        obs = np.ascontiguousarray(np.asarray(obs, np.int32))
        ns, T = obs.shape[0], obs.shape[1]
        obs_vars = np.asarray(obs_vars, np.int32)
        cin = np.ascontiguousarray(counts_in, np.float64)
        cout = np.zeros_like(cin)
        ll = np.zeros(ns)
        bad = np.zeros(ns, np.int32)
        self.lib().no_estep(self.h, ns, T, len(obs_vars), obs_vars, obs.reshape(-1),
                            cin, cout, ll, bad)
        return cout, ll, bad

    def m_step(self, params):
        self.lib().no_m_step(self.h, np.ascontiguousarray(params, np.float64))

    def em(self, obs, obs_vars, init, threshold, max_iter):
        obs = np.ascontiguousarray(np.asarray(obs, np.int32))
        ns, T = obs.shape[0], obs.shape[1]
        obs_vars = np.asarray(obs_vars, np.int32)
        curve = np.zeros(max_iter)
        it = self.lib().no_em(self.h, ns, T, len(obs_vars), obs_vars, obs.reshape(-1),
                              np.ascontiguousarray(init, np.float64), threshold, max_iter, curve)
        return it, curve[:max(it, 0)] if it >= 0 else curve

    def original(self, c):
        n = len(self.desc["cliques"][c]["original"])
        out = np.zeros(n)
        self.lib().no_original(self.h, c, out, n)
        return out

    def prior(self, v):
        out = np.zeros(self.desc["vars"][v]["card"])
        n = self.lib().no_prior(self.h, v, out)
        return out if n else None

    def query(self, root, evidence, q):
        """evidence: {var: vector}; marginal of q after propagation from root."""
        ev_vars = np.array(list(evidence.keys()), np.int32)
        ev = np.concatenate([np.asarray(evidence[v], np.float64) for v in evidence]) \
            if evidence else np.zeros(1)
        out = np.zeros(self.desc["vars"][q]["card"])
        self.lib().no_query(self.h, root, len(ev_vars), ev_vars, np.ascontiguousarray(ev), q, out)
        return out


class RefHarness:
    """The reference's own compiled code (oracle/_ref/libnipref.so)."""

    _lib = None

    @classmethod
    def lib(cls):
        if cls._lib is None:
            if not os.path.exists(REF_SO):
                build(ref=True)
            L = C.CDLL(REF_SO)
            L.nh_build.argtypes = [C.c_char_p]
            L.nh_desc.argtypes = [C.c_int, C.c_char_p, C.c_int]
            for name in ("nh_fb", "nh_filter"):
                getattr(L, name).argtypes = [C.c_int, C.c_int, C.c_int, _i32p, _i32p,
                                             C.c_int, _i32p, _f64p, C.POINTER(C.c_double)]
            L.nh_estep.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, _i32p, _i32p,
                                   _f64p, _f64p, _f64p, _i32p]
            L.nh_param_size.argtypes = [C.c_int]
            L.nh_m_step.argtypes = [C.c_int, _f64p]
            L.nh_em.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, _i32p, _i32p,
                                _f64p, C.c_double, C.c_int, _f64p]
            L.nh_clique_original.argtypes = [C.c_int, C.c_int, _f64p, C.c_int]
            L.nh_prior.argtypes = [C.c_int, C.c_int, _f64p]
            L.nh_graph_cliques.argtypes = [C.c_int, _i32p, C.c_int, _i32p, C.c_int, _i32p,
                                           _i32p, C.c_int]
            cls._lib = L
        return cls._lib

    def __init__(self, replay: str, cards=None):
        """cards: the variables' cardinalities in declaration order, when known;
        then the JSON description (which prints every clique table -- 16.7M
        entries for the wide-clique model) is only produced if .desc is read."""
        self.h = self.lib().nh_build(replay.encode())
        if self.h < 0:
            raise RuntimeError("reference harness failed to build the model")
        self._desc = None if cards is not None else self._load_desc()
        self._cards = list(cards) if cards is not None else [v["card"] for v in self._desc["vars"]]

    def _load_desc(self):
        cap = 1 << 26
        while True:
            buf = C.create_string_buffer(cap)
            n = self.lib().nh_desc(self.h, buf, cap)
            if n < cap:
                return json.loads(buf.value.decode())
            cap *= 4

    @property
    def desc(self):
        if self._desc is None:
            self._desc = self._load_desc()
        return self._desc

    def fb(self, obs, obs_vars, vint, filter_only=False):
        obs_vars = np.asarray(obs_vars, np.int32)
        a = np.asarray(obs)
        T = a.shape[0] if a.ndim == 2 else int(a.size // max(len(obs_vars), 1))
        o = _obs2d(obs, T, len(obs_vars))
        vint = np.asarray(vint, np.int32)
        post = np.zeros((T, int(sum(self._cards[v] for v in vint))))
        ll = C.c_double(0)
        fn = self.lib().nh_filter if filter_only else self.lib().nh_fb
        fn(self.h, T, len(obs_vars), obs_vars, o, len(vint), vint, post, C.byref(ll))
        return post, ll.value

    def param_size(self):
        return self.lib().nh_param_size(self.h)

    def estep(self, obs, obs_vars, counts_in):
        obs = np.ascontiguousarray(np.asarray(obs, np.int32))
        ns, T = obs.shape[0], obs.shape[1]
        obs_vars = np.asarray(obs_vars, np.int32)
        cin = np.ascontiguousarray(counts_in, np.float64)
        cout = np.zeros_like(cin)
        ll = np.zeros(ns)
        bad = np.zeros(ns, np.int32)
        self.lib().nh_estep(self.h, ns, T, len(obs_vars), obs_vars, obs.reshape(-1),
                            cin, cout, ll, bad)
        return cout, ll, bad

    def m_step(self, params):
        self.lib().nh_m_step(self.h, np.ascontiguousarray(params, np.float64))

    def em(self, obs, obs_vars, init, threshold, max_iter):
        obs = np.ascontiguousarray(np.asarray(obs, np.int32))
        ns, T = obs.shape[0], obs.shape[1]
        obs_vars = np.asarray(obs_vars, np.int32)
        curve = np.zeros(max_iter)
        it = self.lib().nh_em(self.h, ns, T, len(obs_vars), obs_vars, obs.reshape(-1),
                              np.ascontiguousarray(init, np.float64), threshold, max_iter, curve)
        return it, curve[:max(it, 0)] if it >= 0 else curve

    def original(self, c):
        n = len(self.desc["cliques"][c]["original"])
        out = np.zeros(n)
        self.lib().nh_clique_original(self.h, c, out, n)
        return out

    def prior(self, v):
        out = np.zeros(self.desc["vars"][v]["card"])
        n = self.lib().nh_prior(self.h, v, out)
        return out if n else None

    def likelihood(self, obs, obs_vars, marked):
        """util/niplikelihood.c over the reference's code: [ns][T][3] of
        (m1, m2, log(m2) - log(m1)) per step."""
        obs = np.ascontiguousarray(np.asarray(obs, np.int32))
        ns, T, nobs = obs.shape
        out = np.zeros((ns, T, 3))
        L = self.lib()
        L.nh_likelihood.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, _i32p, _i32p, _i32p, _f64p]
        L.nh_likelihood(self.h, ns, T, nobs, np.asarray(obs_vars, np.int32),
                        np.asarray([1 if x else 0 for x in marked], np.int32), obs.reshape(-1), out.reshape(-1))
        return out

    def generate(self, seed, n_series, T):
        """generate_data (nip.c:2325-2478) n_series times from srand(seed):
        (order [nv], data [n_series][T][nv] in sampling-order columns)."""
        nv = len(self._cards)
        order = np.zeros(nv, np.int32)
        data = np.zeros((n_series, T, nv), np.int32)
        L = self.lib()
        L.nh_generate.argtypes = [C.c_int, C.c_long, C.c_int, C.c_int, _i32p, _i32p]
        L.nh_generate(self.h, seed, n_series, T, order, data.reshape(-1))
        return order, data


def ref_graph_cliques(card, edges, set_parents=True):
    """Cliques of a DAG through the reference's own triangulation."""
    L = RefHarness.lib()
    n = len(card)
    off = np.zeros(n + 1, np.int32)
    out = np.zeros(n * n, np.int32)
    flat = np.array([x for e in edges for x in e] or [0], np.int32)
    nc = L.nh_graph_cliques(n, np.asarray(card, np.int32), len(edges), flat, int(set_parents),
                            off, out, n * n)
    return [list(out[off[i]:off[i + 1]]) for i in range(nc)]
