"""nip_amd -- MI355X-native forward-backward join-tree engine for NIP's DBNs.

Python mirror of the reference's top-level interface for this path
(src/nip.h): ``parse_model`` / ``model_variable`` / ``forward_backward_inference``
/ ``em_learn``-pieces, batched over sequences and backed by the gfx950 C-ABI
library ``_lib/libnip_amd.so`` (include/nip_amd.h).  The library is loaded
through ctypes with plain pointers; torch is only used by callers for device
memory and streams.  There is no CPU fallback: if the library or a GPU is
missing, calls raise ``NipError``.
"""
from __future__ import annotations

import ctypes as C
import json
import os

import numpy as np

from . import build as _build

__all__ = ["NipError", "Model", "parse_model", "lib", "forward_backward_inference",
           "forward_backward_inference_host", "forward_inference", "forward_inference_host",
           "e_step", "estep_partial", "estep_finalize", "em_learn", "read_timeseries",
           "write_uncertainseries", "write_model", "em_learn_series", "LIB_PATH"]

LIB_PATH = os.environ.get("NIPAMD_LIB", _build.LIB)

NIP_NO_ERROR = 0
NIP_ERROR_NULLPOINTER = 1
NIP_ERROR_DIVBYZERO = 2
NIP_ERROR_INVALID_ARGUMENT = 3
NIP_ERROR_OUTOFMEMORY = 4
NIP_ERROR_IO = 5
NIP_ERROR_GENERAL = 6
NIP_ERROR_FILENOTFOUND = 7
NIP_ERROR_BAD_LUCK = 8
NIPAMD_ERROR_UNSUPPORTED = 100
NIPAMD_ERROR_DEVICE = 101
STATUS_ZERO_MASS = 1
STATUS_BAD_LUCK = 2
ENGINE_AUTO = 0          # interface-chain kernels where they apply, else the general engine
ENGINE_CHAIN = 1         # interface-chain kernels only
ENGINE_JTREE = 2         # the general join-tree engine for every request

# every entry point declared in include/nip_amd.h
EXPORTS = [
    "nipamd_model_from_spec", "nipamd_model_from_net", "nipamd_model_free",
    "nipamd_model_num_vars", "nipamd_model_var_index", "nipamd_model_var_card",
    "nipamd_model_desc_json", "nipamd_model_param_size", "nipamd_model_gpu_supported",
    "nipamd_fb", "nipamd_fb_host", "nipamd_estep", "nipamd_m_step",
    "nipamd_model_original", "nipamd_model_prior", "nipamd_last_error", "nipamd_last_kernel",
    "nipamd_graph_cliques", "nipamd_estep_partial_size", "nipamd_estep_partial_size_req", "nipamd_estep_partial",
    "nipamd_estep_partial_ex",
    "nipamd_estep_finalize", "nipamd_estep_prefix_first_bad", "nipamd_tree_sum", "nipamd_estep_tail", "nipamd_estep_host", "nipamd_filter", "nipamd_filter_host",
    "nipamd_model_state_name", "nipamd_read_timeseries", "nipamd_series_count",
    "nipamd_series_num_observed", "nipamd_series_observed", "nipamd_series_length",
    "nipamd_series_data", "nipamd_series_free", "nipamd_write_uncertainseries",
    "nipamd_em_learn", "nipamd_write_model", "nipamd_model_var_symbol",
    "nipamd_model_var_label", "nipamd_model_var_info",
    "nipamd_generate_order", "nipamd_generate", "nipamd_generate_host", "nipamd_rand_windows",
    "nipamd_generate_host_draws", "nipamd_likelihood", "nipamd_likelihood_host",
    "nipamd_model_set_engine", "nipamd_jt_plan_dump", "nipamd_hugin_passes",
    "nipamd_model_num_cliques", "nipamd_model_num_sepsets", "nipamd_model_clique",
    "nipamd_model_sepset", "nipamd_model_interface_cliques", "nipamd_model_set_tables", "nipamd_model_fold",
]


class NipError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("nip_amd error %d: %s" % (code, msg))
        self.code = code


_lib = None


def lib():
    """Load the gfx950 C-ABI library (raises if it was never built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NipError(NIPAMD_ERROR_DEVICE,
                           "native library missing: %s (run __graft_entry__.build())" % LIB_PATH)
        L = C.CDLL(LIB_PATH)
        vp, ip, dp = C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_double)
        L.nipamd_model_from_spec.argtypes = [C.c_int, C.POINTER(C.c_char_p), ip, ip, C.c_int,
                                             ip, ip, ip, ip, dp, C.POINTER(vp)]
        L.nipamd_model_from_net.argtypes = [C.c_char_p, C.POINTER(vp)]
        L.nipamd_model_free.argtypes = [vp]
        L.nipamd_model_free.restype = None
        L.nipamd_model_num_vars.argtypes = [vp]
        L.nipamd_model_var_index.argtypes = [vp, C.c_char_p]
        L.nipamd_model_var_card.argtypes = [vp, C.c_int]
        L.nipamd_model_desc_json.argtypes = [vp, C.c_char_p, C.c_int]
        L.nipamd_model_param_size.argtypes = [vp]
        L.nipamd_model_gpu_supported.argtypes = [vp, C.c_int, ip, C.c_int, ip]
        L.nipamd_fb.argtypes = [vp, vp, C.c_int, ip, C.c_int, C.c_int, C.c_int, ip,
                                vp, vp, vp, vp]
        L.nipamd_fb_host.argtypes = [vp, vp, C.c_int, ip, C.c_int, C.c_int, C.c_int, ip,
                                     vp, vp, vp]
        L.nipamd_filter.argtypes = L.nipamd_fb.argtypes
        L.nipamd_filter_host.argtypes = L.nipamd_fb_host.argtypes
        L.nipamd_estep.argtypes = [vp, vp, C.c_int, ip, C.c_int, C.c_int, vp, vp, vp, vp]
        L.nipamd_estep_partial_size.argtypes = [vp]
        if hasattr(L, "nipamd_estep_partial_size_req"):      # (absent from A/B builds of older revisions)
            L.nipamd_estep_partial_size_req.argtypes = [vp, C.c_int, ip, C.c_int]
        L.nipamd_estep_partial.argtypes = [vp, vp, C.c_int, ip, C.c_int, C.c_int, vp, vp, vp, vp]
        if hasattr(L, "nipamd_estep_partial_ex"):            # (absent from A/B builds of older revisions)
            L.nipamd_estep_partial_ex.argtypes = [vp, vp, C.c_int, ip, C.c_int, C.c_int, vp, C.c_long, vp, vp, vp]
        L.nipamd_estep_finalize.argtypes = [vp, vp, vp, vp]
        L.nipamd_estep_prefix_first_bad.argtypes = [vp, C.c_int]
        L.nipamd_tree_sum.argtypes = [vp, C.c_long, C.c_int, vp, vp, vp]
        if hasattr(L, "nipamd_estep_tail"):                  # (absent from A/B builds of older revisions)
            L.nipamd_estep_tail.argtypes = [vp, vp, C.c_long, vp, vp, vp]
        L.nipamd_estep_host.argtypes = [vp, vp, C.c_int, ip, C.c_int, C.c_int, vp, vp, vp]
        L.nipamd_m_step.argtypes = [vp, dp]
        L.nipamd_model_original.argtypes = [vp, C.c_int, dp, C.c_int]
        L.nipamd_model_prior.argtypes = [vp, C.c_int, dp]
        L.nipamd_last_error.restype = C.c_char_p
        L.nipamd_last_kernel.restype = C.c_char_p
        L.nipamd_graph_cliques.argtypes = [C.c_int, ip, C.c_int, ip, C.c_int, ip, ip, C.c_int]
        L.nipamd_model_state_name.argtypes = [vp, C.c_int, C.c_int, C.c_char_p, C.c_int]
        L.nipamd_read_timeseries.argtypes = [vp, C.c_char_p, C.POINTER(vp)]
        L.nipamd_series_count.argtypes = [vp]
        L.nipamd_series_num_observed.argtypes = [vp]
        L.nipamd_series_observed.argtypes = [vp, ip]
        L.nipamd_series_length.argtypes = [vp, C.c_int]
        L.nipamd_series_data.argtypes = [vp, C.c_int]
        L.nipamd_series_data.restype = C.POINTER(C.c_int32)
        L.nipamd_series_free.argtypes = [vp]
        L.nipamd_series_free.restype = None
        L.nipamd_write_uncertainseries.argtypes = [vp, C.c_char_p, C.c_int, C.c_int, ip, dp, C.c_int,
                                                   C.c_int]
        L.nipamd_em_learn.argtypes = [vp, C.c_int, ip, vp, C.c_int, ip, C.c_double, dp, C.c_int, dp,
                                      C.c_int, ip]
        L.nipamd_write_model.argtypes = [vp, C.c_char_p]
        L.nipamd_model_var_symbol.argtypes = [vp, C.c_int, C.c_char_p, C.c_int]
        _lib = L
    return _lib


def _check(rc):
    if rc != 0:
        raise NipError(rc, lib().nipamd_last_error().decode())


def last_kernel() -> str:
    """The dominant kernel of the library's last hot-path launch (a label for
    measurements, nipamd_last_kernel)."""
    return lib().nipamd_last_kernel().decode()


def _ints(xs):
    a = (C.c_int * max(len(xs), 1))()
    for i, x in enumerate(xs):
        a[i] = int(x)
    return a


class Model:
    """A compiled DBN time slice (the reference's nip_model, src/nip.h:71-104)."""

    def __init__(self, handle):
        self._h = C.c_void_p(handle)
        self._desc = None

    def __del__(self):
        try:
            if self._h:
                lib().nipamd_model_free(self._h)
        except Exception:
            pass

    # -- construction ---------------------------------------------------
    @classmethod
    def from_net(cls, path: str) -> "Model":
        h = C.c_void_p()
        _check(lib().nipamd_model_from_net(path.encode(), C.byref(h)))
        return cls(h.value)

    @classmethod
    def from_spec(cls, nodes, potentials) -> "Model":
        """nodes: [(symbol, card, next_symbol_or_None)] in declaration order;
        potentials: [(child, [parents in file order], data_or_None)]."""
        syms = [n[0] for n in nodes]
        idx = {s: i for i, s in enumerate(syms)}
        card = [int(n[1]) for n in nodes]
        nxt = [idx[n[2]] if n[2] else -1 for n in nodes]
        child, npar, par, nd, data = [], [], [], [], []
        for ch, ps, d in potentials:
            child.append(idx[ch]); npar.append(len(ps)); par += [idx[p] for p in ps]
            d = [] if d is None else list(np.asarray(d, np.float64).ravel())
            nd.append(len(d)); data += d
        csyms = (C.c_char_p * len(syms))(*[s.encode() for s in syms])
        dbuf = (C.c_double * max(len(data), 1))(*data)
        h = C.c_void_p()
        _check(lib().nipamd_model_from_spec(len(syms), csyms, _ints(card), _ints(nxt), len(child),
                                            _ints(child), _ints(npar), _ints(par), _ints(nd),
                                            dbuf, C.byref(h)))
        return cls(h.value)

    # -- introspection (the index contract) -----------------------------
    def desc(self) -> dict:
        if self._desc is None:
            n = lib().nipamd_model_desc_json(self._h, None, 0)
            buf = C.create_string_buffer(n + 1)
            lib().nipamd_model_desc_json(self._h, buf, n + 1)
            self._desc = json.loads(buf.value.decode())
        return self._desc

    @property
    def num_vars(self):
        return lib().nipamd_model_num_vars(self._h)

    def variable(self, symbol: str) -> int:
        """model_variable() (src/nip.c:1584): index of a symbol, or -1."""
        return lib().nipamd_model_var_index(self._h, symbol.encode())

    def state_names(self, v: int):
        """The variable's state names (nip_variable_state_name)."""
        out = []
        for st in range(self.card(v)):
            n = lib().nipamd_model_state_name(self._h, v, st, None, 0)
            buf = C.create_string_buffer(n + 1)
            lib().nipamd_model_state_name(self._h, v, st, buf, n + 1)
            out.append(buf.value.decode())
        return out

    def card(self, v: int) -> int:
        return lib().nipamd_model_var_card(self._h, int(v))

    def param_size(self) -> int:
        return lib().nipamd_model_param_size(self._h)

    def gpu_supported(self, obs_vars, query) -> bool:
        return bool(lib().nipamd_model_gpu_supported(self._h, len(obs_vars), _ints(obs_vars),
                                                     len(query), _ints(query)))

    def partial_size(self, obs_vars=None, T: int = 0) -> int:
        """Doubles in an e_step partial: the count body plus the 3-slot route
        tag (nipamd_estep_partial_size), and for a request (obs_vars, T) that
        runs the operator chain's e_step its section as well
        (nipamd_estep_partial_size_req); -1 without an e_step plan."""
        if obs_vars is None:
            return lib().nipamd_estep_partial_size(self._h)
        return lib().nipamd_estep_partial_size_req(self._h, len(obs_vars), _ints(obs_vars), int(T))

    def estep_prefix_first_bad(self, T: int) -> int:
        """nipamd_estep_prefix_first_bad: the first step k < T at which the
        reference's e_step rejects a series that observed nothing at steps
        0..k (-1: none; -2: model too large to simulate).  Host only."""
        return lib().nipamd_estep_prefix_first_bad(self._h, int(T))

    def estep_supported(self) -> bool:
        """Whether the batched e_step has a GPU plan for this model under the
        selected engine (the chain kernel's HMM slice, or the general engine)."""
        return lib().nipamd_estep_partial_size(self._h) >= 0

    def set_engine(self, engine: int) -> int:
        """nipamd_model_set_engine: ENGINE_AUTO / ENGINE_CHAIN / ENGINE_JTREE;
        returns the previous setting."""
        L = lib()
        L.nipamd_model_set_engine.argtypes = [C.c_void_p, C.c_int]
        prev = L.nipamd_model_set_engine(self._h, int(engine))
        if prev < 0:
            raise NipError(NIP_ERROR_INVALID_ARGUMENT, "bad engine %r" % engine)
        return prev

    def fold(self, keep: int = -1, cards: int = 0):
        """nipamd_model_fold: the interface chain's transition summed over the
        in-clique's hidden parents on the GPU ([64][64], row = previous state),
        or hidden parent `keep`'s table ([card][64][64], `cards` = its card).
        Returns (table, kernel_ms, bytes streamed)."""
        n = (cards if keep >= 0 else 1) * 64 * 64
        out = np.zeros(n)
        ms, by = C.c_double(0.0), C.c_double(0.0)
        L = lib()
        L.nipamd_model_fold.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_long, C.c_void_p, C.c_void_p]
        _check(L.nipamd_model_fold(self._h, int(keep), out.ctypes.data_as(C.c_void_p), n,
                                   C.byref(ms), C.byref(by)))
        return (out.reshape(64, 64) if keep < 0 else out.reshape(cards, 64, 64)), ms.value, by.value

    def original(self, c: int) -> np.ndarray:
        n = lib().nipamd_model_original(self._h, c, None, 0)
        out = np.zeros(n)
        lib().nipamd_model_original(self._h, c, out.ctypes.data_as(C.POINTER(C.c_double)), n)
        return out

    def prior(self, v: int):
        out = np.zeros(self.card(v))
        n = lib().nipamd_model_prior(self._h, v, out.ctypes.data_as(C.POINTER(C.c_double)))
        return out if n > 0 else None

    def m_step(self, params) -> None:
        """m_step() (src/nip.c:2010): params in the em_learn layout."""
        p = np.ascontiguousarray(params, np.float64)
        assert p.size == self.param_size()
        _check(lib().nipamd_m_step(self._h, p.ctypes.data_as(C.POINTER(C.c_double))))
        self._desc = None


def graph_cliques(card, edges, set_parents=True):
    """Clique array of a DAG through the join-tree compiler (index contract)."""
    n = len(card)
    flat = [x for e in edges for x in e]
    off = (C.c_int * (n + 1))()
    cap = n * n
    out = (C.c_int * cap)()
    nc = lib().nipamd_graph_cliques(n, _ints(card), len(edges), _ints(flat), int(set_parents),
                                    off, out, cap)
    if nc < 0:
        raise NipError(-nc, lib().nipamd_last_error().decode())
    return [[out[j] for j in range(off[i], off[i + 1])] for i in range(nc)]


def parse_model(path: str) -> Model:
    """parse_model() (src/nip.c:122): read a Hugin .net file."""
    return Model.from_net(path)


def _stream_ptr(stream):
    if stream is None:
        import torch
        return C.c_void_p(torch.cuda.current_stream().cuda_stream)
    if isinstance(stream, int):
        return C.c_void_p(stream)
    return C.c_void_p(stream.cuda_stream)


def _out_buf(t, shape, dtype, dev, name):
    """A caller-supplied output buffer must be exactly what the kernels write
    through its raw pointer: shape, dtype, device and dense layout; None
    allocates one."""
    import torch
    if t is None:
        return torch.empty(shape, dtype=dtype, device=dev)
    if (tuple(t.shape) != tuple(shape) or t.dtype != dtype or t.device != dev
            or not t.is_contiguous()):
        raise NipError(NIP_ERROR_INVALID_ARGUMENT,
                       "%s must be a contiguous %s tensor of shape %s on %s (got %s %s on %s)"
                       % (name, dtype, tuple(shape), dev, t.dtype, tuple(t.shape), t.device))
    return t


def _run_device(fn, model, obs, obs_vars, query, post, ll, status, stream):
    import torch
    if obs.dim() == 2:
        obs = obs.unsqueeze(-1)
    assert obs.dtype == torch.int32 and obs.is_cuda and obs.is_contiguous()
    B, T, nobs = obs.shape
    assert nobs == len(obs_vars)
    width = sum(model.card(v) for v in query)
    dev = obs.device
    post = _out_buf(post, (B, T, width), torch.float64, dev, "post")
    ll = _out_buf(ll, (B,), torch.float64, dev, "ll")
    status = _out_buf(status, (B,), torch.int32, dev, "status")
    _check(fn(model._h, C.c_void_p(obs.data_ptr()), nobs, _ints(obs_vars), B, T,
              len(query), _ints(query), C.c_void_p(post.data_ptr()),
              C.c_void_p(ll.data_ptr()), C.c_void_p(status.data_ptr()), _stream_ptr(stream)))
    return post, ll, status


def _run_host(fn, model, obs, obs_vars, query):
    obs = np.ascontiguousarray(np.asarray(obs, np.int32))
    if obs.ndim == 2:
        obs = obs[:, :, None]
    B, T, nobs = obs.shape
    width = sum(model.card(v) for v in query)
    post = np.zeros((B, T, width))
    ll = np.zeros(B)
    status = np.zeros(B, np.uint32)
    _check(fn(model._h, obs.ctypes.data_as(C.c_void_p), nobs, _ints(obs_vars),
              B, T, len(query), _ints(query), post.ctypes.data_as(C.c_void_p),
              ll.ctypes.data_as(C.c_void_p), status.ctypes.data_as(C.c_void_p)))
    return post, ll, status


def forward_backward_inference(model: Model, obs, obs_vars, query, post=None, ll=None,
                               status=None, stream=None):
    """Batched forward_backward_inference() (src/nip.c:1320) on the GPU.

    obs: torch int32 CUDA tensor [B, T, n_obs] (state index, <0 missing).
    Returns (post [B, T, sum card(query)] float64, ll [B] float64, status [B] int32),
    all CUDA tensors, computed asynchronously on ``stream`` (default: torch's
    current stream).  ll is the SUM over t, as the reference returns it.
    """
    return _run_device(lib().nipamd_fb, model, obs, obs_vars, query, post, ll, status, stream)


def forward_inference(model: Model, obs, obs_vars, query, post=None, ll=None, status=None,
                      stream=None):
    """Batched forward_inference() (src/nip.c:1103-1315) on the GPU: filtered
    marginals P(X_t | y_0..y_t) of the query variables, and the same ll (sum
    over t).  Buffers and conventions as forward_backward_inference."""
    return _run_device(lib().nipamd_filter, model, obs, obs_vars, query, post, ll, status, stream)


def forward_backward_inference_host(model: Model, obs, obs_vars, query):
    """Same, from host numpy buffers (PCIe-inclusive, synchronous)."""
    return _run_host(lib().nipamd_fb_host, model, obs, obs_vars, query)


def forward_inference_host(model: Model, obs, obs_vars, query):
    """forward_inference from host numpy buffers (PCIe-inclusive, synchronous)."""
    return _run_host(lib().nipamd_filter_host, model, obs, obs_vars, query)


def generate_order(model: Model):
    """The sampling order of generate_data (src/nip.c:2343-2375): the model
    variable of each data column."""
    L = lib()
    n = L.nipamd_generate_order(model._h, None)
    order = (C.c_int * max(n, 1))()
    L.nipamd_generate_order(model._h, order)
    return list(order)[:n]


def generate_data(model: Model, seed: int, B: int, T: int, out=None, stream=None):
    """generate_data (src/nip.c:2325-2478) B times from srand(seed), on the
    GPU: (order, int32 tensor [B][T][nv]); column i holds variable order[i]
    (the reference's ts->observed)."""
    import torch
    order = generate_order(model)
    if out is None:
        out = torch.empty((B, T, len(order)), dtype=torch.int32, device="cuda")
    assert out.dtype == torch.int32 and out.is_cuda and out.is_contiguous()
    assert tuple(out.shape) == (B, T, len(order))
    L = lib()
    L.nipamd_generate.argtypes = [C.c_void_p, C.c_long, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
    _check(L.nipamd_generate(model._h, seed, B, T, C.c_void_p(out.data_ptr()), _stream_ptr(stream)))
    return order, out


def likelihood(model: Model, obs, obs_vars, marked):
    """util/niplikelihood.c batched on the GPU: (m1, m2, ll) [B][T] -- the
    mass after the unmarked columns' evidence, after all, and log(m2/m1)
    per step, each step on its own (niplikelihood.c:111-133)."""
    obs = np.ascontiguousarray(np.asarray(obs, np.int32))
    if obs.ndim == 2:
        obs = obs[:, :, None]
    B, T, nobs = obs.shape
    if not (len(obs_vars) == nobs == len(marked)):
        raise NipError(NIP_ERROR_INVALID_ARGUMENT, "obs_vars (%d) and marked (%d) must name every "
                       "one of the %d columns" % (len(obs_vars), len(marked), nobs))
    out = [np.zeros((B, T)) for _ in range(3)]
    L = lib()
    L.nipamd_likelihood_host.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p,
                                         C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
    _check(L.nipamd_likelihood_host(model._h, obs.ctypes.data_as(C.c_void_p), nobs, _ints(obs_vars),
                                    _ints([1 if m else 0 for m in marked]), B, T,
                                    *[o.ctypes.data_as(C.c_void_p) for o in out]))
    return tuple(out)


def rand_windows(seed: int, B: int, draws_per_series: int):
    """glibc rand() state window [B][31] of each series (nipamd_rand_windows)."""
    out = np.zeros((B, 31), np.uint32)
    L = lib()
    L.nipamd_rand_windows.argtypes = [C.c_long, C.c_int, C.c_long, C.c_void_p]
    _check(L.nipamd_rand_windows(seed, B, draws_per_series, out.ctypes.data_as(C.c_void_p)))
    return out


def read_timeseries(model: Model, path):
    """read_timeseries() (src/nip.c:512-667) of the reference's data-file format.

    Returns (series, obs_vars): a list of int32 arrays [T_i, n_obs] (state
    index, -1 missing) and the model variable of each column (file order).
    """
    h = C.c_void_p()
    _check(lib().nipamd_read_timeseries(model._h, os.fsencode(path), C.byref(h)))
    try:
        L = lib()
        n, k = L.nipamd_series_count(h), L.nipamd_series_num_observed(h)
        ov = (C.c_int * max(k, 1))()
        _check(L.nipamd_series_observed(h, ov))
        out = []
        for i in range(n):
            T = L.nipamd_series_length(h, i)
            if k == 0:
                out.append(np.zeros((T, 0), np.int32))
                continue
            p = L.nipamd_series_data(h, i)
            out.append(np.ctypeslib.as_array(p, shape=(T * k,)).reshape(T, k).copy())
        return out, [ov[i] for i in range(k)]
    finally:
        lib().nipamd_series_free(h)


def write_model(model: Model, path):
    """write_model() (src/nip.c:298-484): the model as a Hugin .net file."""
    _check(lib().nipamd_write_model(model._h, os.fsencode(path)))


def em_learn_series(model: Model, series, obs_vars, threshold, init=None, max_iterations=0):
    """em_learn() for series of any lengths on one GPU (nipamd_em_learn).

    series: list of int32 arrays [T_i, n_obs].  init: initial parameters in the
    em_learn layout, or None for rand()/RAND_MAX draws like the reference (C
    rand(); seed it with libc's srand).  Returns (rc, learning_curve)."""
    series = [np.ascontiguousarray(np.asarray(s, np.int32).reshape(len(s), -1)) for s in series]
    k = len(obs_vars)
    flat = np.ascontiguousarray(np.concatenate(series, axis=0)) if k else np.zeros(1, np.int32)
    lengths = np.array([len(s) for s in series], np.int32)
    cap = 100000
    curve = np.zeros(cap)
    n = C.c_int(0)
    ini = None if init is None else np.ascontiguousarray(init, np.float64)
    rc = lib().nipamd_em_learn(model._h, len(series), lengths.ctypes.data_as(C.POINTER(C.c_int)),
                               flat.ctypes.data_as(C.c_void_p), k, _ints(obs_vars), threshold,
                               None if ini is None else ini.ctypes.data_as(C.POINTER(C.c_double)),
                               max_iterations, curve.ctypes.data_as(C.POINTER(C.c_double)), cap,
                               C.byref(n))
    if rc not in (0, 8):
        _check(rc)
    return rc, list(curve[:n.value])


def write_uncertainseries(model: Model, path, var: int, posts):
    """write_uncertainseries() (src/nip.c:815-893): `posts` is a list of
    arrays [T_i, card(var)] (or wider rows with the variable first)."""
    posts = [np.ascontiguousarray(p, np.float64) for p in posts]
    stride = posts[0].shape[1]
    flat = np.ascontiguousarray(np.concatenate(posts, axis=0))
    lengths = np.array([p.shape[0] for p in posts], np.int32)
    _check(lib().nipamd_write_uncertainseries(
        model._h, os.fsencode(path), var, len(posts), lengths.ctypes.data_as(C.POINTER(C.c_int)),
        flat.ctypes.data_as(C.POINTER(C.c_double)), stride, 0))


def _obs3(obs, obs_vars):
    import torch
    if obs.dim() == 2:
        obs = obs.unsqueeze(-1)
    assert obs.dtype == torch.int32 and obs.is_cuda and obs.is_contiguous()
    assert obs.shape[2] == len(obs_vars)
    return obs


def estep_partial(model: Model, obs, obs_vars, partial=None, ll=None, status=None, stream=None):
    """First half of the batched e_step (src/nip.c:1708): the fixed-order tree
    sum of the per-sequence count slabs of obs [B, T, n_obs] (CUDA int32).
    Returns (partial [partial_size] float64, ll [B], status [B]) on the GPU."""
    import torch
    obs = _obs3(obs, obs_vars)
    B, T, nobs = obs.shape
    L = lib()
    S = (L.nipamd_estep_partial_size_req(model._h, nobs, _ints(obs_vars), T)
         if hasattr(L, "nipamd_estep_partial_size_req") else L.nipamd_estep_partial_size(model._h))
    if S < 0:
        raise NipError(NIPAMD_ERROR_UNSUPPORTED, "model has no GPU e_step plan")
    dev = obs.device
    partial = _out_buf(partial, (S,), torch.float64, dev, "partial")
    ll = _out_buf(ll, (B,), torch.float64, dev, "ll")
    status = _out_buf(status, (B,), torch.int32, dev, "status")
    if hasattr(L, "nipamd_estep_partial_ex"):
        # with the request's capacity: the operator chain may take the request
        _check(L.nipamd_estep_partial_ex(model._h, C.c_void_p(obs.data_ptr()), nobs, _ints(obs_vars), B, T,
                                         C.c_void_p(partial.data_ptr()), int(partial.numel()),
                                         C.c_void_p(ll.data_ptr()), C.c_void_p(status.data_ptr()),
                                         _stream_ptr(stream)))
    else:
        _check(L.nipamd_estep_partial(model._h, C.c_void_p(obs.data_ptr()), nobs, _ints(obs_vars),
                                      B, T, C.c_void_p(partial.data_ptr()), C.c_void_p(ll.data_ptr()),
                                      C.c_void_p(status.data_ptr()), _stream_ptr(stream)))
    return partial, ll, status


def tree_sum(rows, out=None, stream=None):
    """Fixed-order binary-tree sum of rows [n, S] (CUDA float64) over dim 0
    (nipamd_tree_sum): pairs (2i, 2i + 1) level by level, the shape of the
    e_step's count tree.  Returns out [S]."""
    import torch
    x = rows.reshape(rows.shape[0], -1) if rows.dim() > 1 else rows.reshape(-1, 1)
    x = x.to(torch.float64).contiguous()
    n, S = int(x.shape[0]), int(x.shape[1])
    out = _out_buf(out, (S,), torch.float64, x.device, "out")
    work = torch.empty((2 * ((n + 63) // 64) * S,), dtype=torch.float64, device=x.device) if n > 64 else None
    _check(lib().nipamd_tree_sum(C.c_void_p(x.data_ptr()), n, S,
                                 C.c_void_p(work.data_ptr() if work is not None else 0),
                                 C.c_void_p(out.data_ptr()), _stream_ptr(stream)))
    return out


def estep_tail(ll, status, out=None, stream=None):
    """out [2] = [nipamd_tree_sum of ll [B], number of nonzero status words]
    (nipamd_estep_tail): the scalars em_learn exchanges with its counts,
    written on the GPU next to them (em.py).  Returns out."""
    import torch
    B = int(ll.numel())
    out = _out_buf(out, (2,), torch.float64, ll.device, "out")
    if ll.dtype != torch.float64 or not ll.is_contiguous() or status.numel() != B or status.element_size() != 4 \
            or not status.is_contiguous():
        raise NipError(NIP_ERROR_INVALID_ARGUMENT, "ll must be contiguous float64 [B], status contiguous 32-bit [B]")
    work = torch.empty((2 * ((B + 63) // 64) + (B + 4095) // 4096 + 1,), dtype=torch.float64, device=ll.device)
    _check(lib().nipamd_estep_tail(C.c_void_p(ll.data_ptr()), C.c_void_p(status.data_ptr()), B,
                                   C.c_void_p(work.data_ptr()), C.c_void_p(out.data_ptr()), _stream_ptr(stream)))
    return out


def estep_finalize(model: Model, partial, counts, stream=None):
    """counts (CUDA float64 [param_size], em_learn layout) += families of partial.
    counts=None starts from the em_learn pseudo-counts (ones, nip.c:2172)."""
    import torch
    if counts is None:
        counts = torch.ones((model.param_size(),), dtype=torch.float64, device=partial.device)
    counts = _out_buf(counts, (model.param_size(),), torch.float64, partial.device, "counts")
    _check(lib().nipamd_estep_finalize(model._h, C.c_void_p(partial.data_ptr()),
                                       C.c_void_p(counts.data_ptr()), _stream_ptr(stream)))
    return counts


def e_step(model: Model, obs, obs_vars, counts=None, ll=None, status=None, stream=None):
    """Batched e_step() (src/nip.c:1708-2007) of B sequences on the GPU.

    counts: CUDA float64 [param_size] accumulated into (default: ones, the
    em_learn pseudo-counts of nip.c:2172).  Returns (counts, ll [B], status [B]);
    status bit NIPAMD_STATUS_BAD_LUCK marks the sequences for which the
    reference's e_step returns NIP_ERROR_BAD_LUCK.
    """
    import torch
    obs = _obs3(obs, obs_vars)
    B, T, nobs = obs.shape
    dev = obs.device
    if counts is None:
        counts = torch.ones((model.param_size(),), dtype=torch.float64, device=dev)
    counts = _out_buf(counts, (model.param_size(),), torch.float64, dev, "counts")
    ll = _out_buf(ll, (B,), torch.float64, dev, "ll")
    status = _out_buf(status, (B,), torch.int32, dev, "status")
    _check(lib().nipamd_estep(model._h, C.c_void_p(obs.data_ptr()), nobs, _ints(obs_vars), B, T,
                              C.c_void_p(counts.data_ptr()), C.c_void_p(ll.data_ptr()),
                              C.c_void_p(status.data_ptr()), _stream_ptr(stream)))
    return counts, ll, status


from .em import em_learn  # noqa: E402
