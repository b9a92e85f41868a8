"""Debug: replicate nipamd_em_learn's second iteration with nipamd_estep_host per length group."""
import os, sys, ctypes as C
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, ROOT)
import nip_amd
from nip_amd import synth, lib, _ints
nodes, pots = synth.hmm_spec(6, 5, seed=21)
m = nip_amd.Model.from_spec(nodes, pots)
ov = [m.variable("M1")]
rng = np.random.default_rng(3)
series = [rng.integers(-1, 5, size=(T, 1)).astype(np.int32) for T in (5, 1, 17, 5, 33, 2, 9, 17)]
init = rng.random(m.param_size())
for mi in (1, 2, 3):
    rc, curve = nip_amd.em_learn_series(m, series, ov, 1e-6, init=init, max_iterations=mi)
    print("max_it", mi, "rc", rc, "curve", curve, lib().nipamd_last_error().decode())
params = init.copy()
groups = {}
for s in series: groups.setdefault(len(s), []).append(s)
for it in range(2):
    m.m_step(params)
    counts = np.ones(m.param_size())
    for T in sorted(groups):
        g = np.ascontiguousarray(np.stack(groups[T]))
        B = len(g)
        ll = np.zeros(B); st = np.zeros(B, np.uint32)
        rc = lib().nipamd_estep_host(m._h, g.ctypes.data_as(C.c_void_p), 1, _ints(ov), B, T,
                                     counts.ctypes.data_as(C.POINTER(C.c_double)),
                                     ll.ctypes.data_as(C.POINTER(C.c_double)),
                                     st.ctypes.data_as(C.POINTER(C.c_uint32)))
        print("it", it, "T", T, "rc", rc, nip_amd.last_kernel(), "ll", ll, "st", st, "first_bad",
              lib().nipamd_estep_prefix_first_bad(m._h, T) if hasattr(lib(), "nipamd_estep_prefix_first_bad") else None)
    params = counts
