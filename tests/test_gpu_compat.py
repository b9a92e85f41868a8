"""libnip.so on the GPU: the reference's nip.h API over the engine
(SURVEY 8(b) drop-in).

1. The reference's OWN util/nipinference.c, util/nipmap.c and
   util/niptrain.c, compiled unmodified against include/compat and linked
   with libnip.so (oracle/_ref/compat, built by nip_amd.build in the container
   that has the reference tree), run end to end and are checked exactly like
   the nipamd_* counterparts (tests/test_gpu_tools.py: against the CPU oracle
   on the same files; "%f" output within 5e-7).
2. forward_inference / forward_backward_inference / the batched extension
   through ctypes, with marks: only MARKED observed variables' evidence is
   entered (insert_ts_step with NIP_MARK_ON, nip.c:982-1003).  Against the
   oracle, 1e-12 absolute on marginals and relative on ll (test_gpu_parity).
"""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
pytest.importorskip("torch")

import nip_amd
from nip_amd import build
from oracle import datafile as ref
from oracle.bind import PortOracle

import test_compat as tc
import test_gpu_tools as tt

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def ref_program(name):
    p = os.path.join(build.REF_BIN_DIR, name)
    if not os.access(p, os.X_OK):
        pytest.skip("reference util programs not built (no reference tree where the build ran)")
    return p


def test_reference_nipinference(tmp_path):
    """util/nipinference.c itself over libnip.so: model.net, ragged series with nulls."""
    rng = np.random.default_rng(4)
    series = [[[rng.choice(["0", "1", "2", "null"], p=[0.4, 0.3, 0.2, 0.1])] for _ in range(T)]
              for T in (24, 1, 7, 24, 13, 2)]
    tt.check(os.path.join(GOLD, "model.net"), ["M1"], series, "P1", tmp_path,
             tool=ref_program("nipinference"))


def test_reference_nipinference_demo1(tmp_path):
    m = nip_amd.Model.from_net(os.path.join(GOLD, "demo1.net"))
    a, b = m.state_names(m.variable("A1")), m.state_names(m.variable("B1"))
    rng = np.random.default_rng(1)
    series = [[[rng.choice(a + ["null"]), "x", rng.choice(b)] for _ in range(T)] for T in (5, 9, 5)]
    tt.check(os.path.join(GOLD, "demo1.net"), ["A1", "junk", "B1"], series, "C1", tmp_path,
             tool=ref_program("nipinference"))


def test_reference_nipmap(tmp_path):
    """util/nipmap.c itself: MAP of C0, C1 and the hidden parent D1 of demo1."""
    m = nip_amd.Model.from_net(os.path.join(GOLD, "demo1.net"))
    a, b = m.state_names(m.variable("A1")), m.state_names(m.variable("B1"))
    rng = np.random.default_rng(2)
    series = [[[rng.choice(a + ["null"]), rng.choice(b)] for _ in range(T)] for T in (6, 6, 11)]
    tt.check_map(os.path.join(GOLD, "demo1.net"), ["A1", "B1"], series, tmp_path,
                 tool=ref_program("nipmap"))


def test_reference_niptrain(tmp_path):
    """util/niptrain.c itself: em_learn from random starts drawn after its own
    random_seed(NULL) (printed).  Replaying the same rand() stream through
    nip_amd.em_learn_series (one parameter draw per run it reports) and
    write_model gives the same .net file, byte for byte, and the learning
    curve it prints is that replay's (rounded to the threshold, niptrain.c:198)."""
    from test_gpu_train import libc_rand_init
    net = os.path.join(GOLD, "model.net")
    rng = np.random.default_rng(6)
    series = [[[rng.choice(["0", "1", "2"], p=[0.5, 0.3, 0.2])] for _ in range(T)] for T in (30, 30, 17)]
    data, out = str(tmp_path / "data.txt"), str(tmp_path / "learned.net")
    tt.write_data(data, ["M1"], series)
    r = subprocess.run([ref_program("niptrain"), net, data, "0.0001", "-100", out],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    seed = int(re.search(r"Random seed = (-?\d+)", r.stdout).group(1))
    runs = r.stdout.count("  Run ")
    m = nip_amd.Model.from_net(net)
    ser, ov = nip_amd.read_timeseries(m, data)
    for init in libc_rand_init(seed, m.param_size(), runs):
        rc, curve = nip_amd.em_learn_series(m, ser, ov, 0.0001, init=init)
    assert rc == 0
    replay = str(tmp_path / "replay.net")
    nip_amd.write_model(m, replay)
    assert open(out).read() == open(replay).read()
    printed = [float(x) for x in re.findall(r"average loglikelihood = (\S+)", r.stdout)]
    assert len(printed) == len(curve)
    assert np.allclose(printed, np.rint(np.asarray(curve) / 0.0001) * 0.0001, rtol=1e-5, atol=1e-9)


@pytest.fixture(scope="module")
def lib():
    L = tc.load()
    for f in ("forward_inference", "forward_backward_inference"):
        getattr(L, f).restype = C.c_void_p
        getattr(L, f).argtypes = [C.POINTER(tc.Series), C.POINTER(tc.VarP), C.c_int, C.POINTER(C.c_double)]
    L.forward_backward_inference_batch.argtypes = [C.POINTER(C.POINTER(tc.Series)), C.c_int,
                                                   C.POINTER(tc.VarP), C.c_int, C.POINTER(C.c_void_p),
                                                   C.POINTER(C.c_double)]
    L.free_uncertainseries.argtypes = [C.c_void_p]
    return L


class UCS(C.Structure):
    _fields_ = [("num_of_vars", C.c_int), ("variables", tc.VarPP), ("length", C.c_int),
                ("data", C.POINTER(C.POINTER(C.POINTER(C.c_double))))]


def ucs_array(p, cards):
    u = C.cast(p, C.POINTER(UCS)).contents
    return np.array([[u.data[t][i][j] for i, c in enumerate(cards) for j in range(c)]
                     for t in range(u.length)]).reshape(u.length, sum(cards))


@pytest.mark.parametrize("marked", [("A1", "B1"), ("A1",), ()])
def test_marks_and_batch(lib, tmp_path, marked):
    """demo1 with A1 and B1 in the file: only the marked columns count."""
    net = os.path.join(GOLD, "demo1.net")
    m = nip_amd.Model.from_net(net)
    a, b = m.state_names(m.variable("A1")), m.state_names(m.variable("B1"))
    rng = np.random.default_rng(7)
    series = [[[rng.choice(a + ["null"]), rng.choice(b)] for _ in range(T)] for T in (8, 8, 3, 8)]
    data = str(tmp_path / "data.txt")
    tt.write_data(data, ["A1", "B1"], series)
    pm = lib.parse_model(net.encode())
    ts = C.POINTER(C.POINTER(tc.Series))()
    n = lib.read_timeseries(pm, data.encode(), C.byref(ts))
    assert n == 4
    for s in marked:
        lib.nip_mark_variable(lib.model_variable(pm, s.encode()))
    qs = ("C1", "D1", "A1")
    q = (tc.VarP * 3)(*[lib.model_variable(pm, s.encode()) for s in qs])
    oq = [m.variable(s) for s in qs]
    cards = [m.card(v) for v in oq]
    syms = [d["symbol"] for d in m.desc()["vars"]]
    rs, ov = ref.read_timeseries(data, syms, [m.state_names(i) for i in range(m.num_vars)])
    keep = [k for k, v in enumerate(ov) if syms[v] in marked]
    orc = PortOracle(m.desc())
    batch = (C.c_void_p * n)()
    bll = (C.c_double * n)()
    assert lib.forward_backward_inference_batch(ts, n, q, 3, batch, bll) == 0
    for i in range(n):
        obs = np.array(rs[i], np.int32).reshape(len(rs[i]), len(ov))[:, keep]
        for filt, fn in ((False, lib.forward_backward_inference), (True, lib.forward_inference)):
            ll = C.c_double()
            u = fn(ts[i], q, 3, C.byref(ll))
            assert u
            got = ucs_array(u, cards)
            want, wl = orc.fb(np.ascontiguousarray(obs), [ov[k] for k in keep], oq, filter_only=filt)
            assert np.abs(got - want).max() <= 1e-12
            assert abs(ll.value - wl) <= 1e-12 * max(1.0, abs(wl))
            if not filt:
                assert np.array_equal(ucs_array(batch[i], cards), got)
                assert bll[i] == ll.value
            lib.free_uncertainseries(u)
        lib.free_uncertainseries(batch[i])
    for i in range(n):
        lib.free_timeseries(ts[i])
    lib.free_model(pm)
