"""libnip.so, the reference's nip.h API over the engine (include/compat,
nip_amd/compat/compat.cpp), host side on the CPU.

The public structs are read through ctypes mirrors of the reference's layouts
(nip_variable_struct nipvariable.h:51-78, nip_model_struct nip.h:71-104,
time_series_struct nip.h:112-122, nip_double_list niplists.h:73-86) and
checked against the engine's compiled model (tests/test_compiler.py pins
that to the reference).  Data files go through read_timeseries /
write_timeseries and are compared with oracle/datafile.py, the restatement of
nip.c:512-789.  Inference and em_learn need the GPU: tests/test_gpu_compat.py.
"""
import ctypes as C
import os
import re

import numpy as np
import pytest

import nip_amd
from nip_amd import build
from oracle import datafile as ref

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
HEADERS = ["nip.h", "niplists.h", "nipvariable.h", "niperrorhandler.h"]


class Var(C.Structure):
    pass


Var._fields_ = [("id", C.c_ulong), ("symbol", C.c_char_p), ("name", C.c_char_p),
                ("cardinality", C.c_int), ("state_names", C.POINTER(C.c_char_p)),
                ("likelihood", C.POINTER(C.c_double)), ("prior", C.POINTER(C.c_double)),
                ("prior_entered", C.c_int), ("previous", C.POINTER(Var)), ("next", C.POINTER(Var)),
                ("num_of_parents", C.c_int), ("parents", C.POINTER(C.POINTER(Var))),
                ("family_clique", C.c_void_p), ("family_mapping", C.POINTER(C.c_int)),
                ("interface_status", C.c_int), ("mark", C.c_char), ("pos_x", C.c_int),
                ("pos_y", C.c_int)]
VarP = C.POINTER(Var)
VarPP = C.POINTER(VarP)


class Model(C.Structure):
    _fields_ = [("num_of_cliques", C.c_int), ("cliques", C.c_void_p), ("num_of_vars", C.c_int),
                ("variables", VarPP), ("num_of_nexts", C.c_int), ("next", VarPP),
                ("previous", VarPP), ("outgoing_interface_size", C.c_int),
                ("outgoing_interface", VarPP), ("previous_outgoing_interface", VarPP),
                ("incoming_interface_size", C.c_int), ("incoming_interface", VarPP),
                ("in_clique", C.c_void_p), ("out_clique", C.c_void_p), ("num_of_children", C.c_int),
                ("children", VarPP), ("independent", VarPP), ("node_size_x", C.c_int),
                ("node_size_y", C.c_int)]


class Series(C.Structure):
    _fields_ = [("model", C.POINTER(Model)), ("num_of_hidden", C.c_int), ("hidden", VarPP),
                ("num_of_observed", C.c_int), ("observed", VarPP), ("length", C.c_int),
                ("data", C.POINTER(C.POINTER(C.c_int)))]


class Link(C.Structure):
    pass


Link._fields_ = [("data", C.c_double), ("fwd", C.POINTER(Link)), ("bwd", C.POINTER(Link))]


class DList(C.Structure):
    _fields_ = [("length", C.c_int), ("first", C.POINTER(Link)), ("last", C.POINTER(Link))]


def load():
    nip_amd.lib()                        # libnip.so sits on top of libnip_amd.so
    L = C.CDLL(build.COMPAT_LIB)
    L.parse_model.restype = C.POINTER(Model)
    L.parse_model.argtypes = [C.c_char_p]
    L.free_model.argtypes = [C.POINTER(Model)]
    L.model_variable.restype = VarP
    L.model_variable.argtypes = [C.POINTER(Model), C.c_char_p]
    L.read_timeseries.argtypes = [C.POINTER(Model), C.c_char_p, C.POINTER(C.POINTER(C.POINTER(Series)))]
    L.write_timeseries.argtypes = [C.POINTER(C.POINTER(Series)), C.c_int, C.c_char_p]
    L.free_timeseries.argtypes = [C.POINTER(Series)]
    L.timeseries_length.argtypes = [C.POINTER(Series)]
    L.get_observation.restype = C.c_char_p
    L.get_observation.argtypes = [C.POINTER(Series), VarP, C.c_int]
    L.set_observation.argtypes = [C.POINTER(Series), VarP, C.c_int, C.c_char_p]
    L.nip_new_double_list.restype = C.POINTER(DList)
    L.nip_append_double.argtypes = [C.POINTER(DList), C.c_double]
    L.nip_prepend_double.argtypes = [C.POINTER(DList), C.c_double]
    L.nip_double_list_to_array.restype = C.POINTER(C.c_double)
    L.nip_double_list_to_array.argtypes = [C.POINTER(DList)]
    L.nip_empty_double_list.argtypes = [C.POINTER(DList)]
    L.random_seed.restype = C.c_long
    L.random_seed.argtypes = [C.POINTER(C.c_long)]
    L.lottery.argtypes = [C.POINTER(C.c_double), C.c_int]
    L.nip_report_error.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_int]
    L.nip_variable_state_index.argtypes = [VarP, C.c_char_p]
    L.nip_variable_marked.argtypes = [VarP]
    L.nip_mark_variable.argtypes = [VarP]
    return L


@pytest.fixture(scope="module")
def lib():
    return load()


def declared(header):
    text = open(os.path.join(build.ROOT, "include", "compat", header)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return re.findall(r"^[A-Za-z][\w \*]*?\**\b(\w+)\((?!\*)", text, flags=re.M)


def test_exports(lib):
    names = [n for h in HEADERS for n in declared(h)]
    assert len(names) > 30, names
    for n in names:
        assert hasattr(lib, n), n


@pytest.mark.parametrize("net", ["model.net", "demo1.net"])
def test_model_struct(lib, net):
    """parse_model fills the reference's records: ids, symbols, cards, states,
    parents (v->parents order), next/previous, interface flags, priors, and
    the special-purpose arrays of nip.c:216-247."""
    path = os.path.join(GOLD, net)
    m = nip_amd.Model.from_net(path)
    d = m.desc()
    pm = lib.parse_model(path.encode())
    assert pm
    M = pm.contents
    assert M.num_of_vars == m.num_vars == len(d["vars"])
    assert M.num_of_cliques == len(d["cliques"])
    idx = {C.addressof(M.variables[i].contents): i for i in range(M.num_of_vars)}
    for i, dv in enumerate(d["vars"]):
        v = M.variables[i].contents
        # consecutive IDs from the one process-wide counter the parser shares
        # with nip_new_variable (nipvariable.c:60): a later model continues it
        assert v.id == M.variables[0].contents.id + i >= 1
        assert v.symbol.decode() == dv["symbol"]
        assert v.cardinality == dv["card"]
        assert [v.state_names[s].decode() for s in range(v.cardinality)] == m.state_names(i)
        assert v.interface_status == dv["if"]
        assert [idx[C.addressof(v.parents[k].contents)] for k in range(v.num_of_parents)] == dv["parents"]
        nxt = idx[C.addressof(v.next.contents)] if v.next else -1
        prv = idx[C.addressof(v.previous.contents)] if v.previous else -1
        assert (nxt, prv) == (dv["next"], dv["previous"])
        if dv["prior"] is not None:
            assert [v.prior[s] for s in range(v.cardinality)] == dv["prior"]
        assert v.mark == bytes([1])                       # NIP_MARK_OFF
        assert lib.model_variable(pm, dv["symbol"].encode()).contents.id == v.id
    assert not lib.model_variable(pm, b"no such variable")
    out = [idx[C.addressof(M.outgoing_interface[k].contents)] for k in range(M.outgoing_interface_size)]
    old = [idx[C.addressof(M.previous_outgoing_interface[k].contents)]
           for k in range(M.outgoing_interface_size)]
    assert out == d["outgoing"] and old == d["previous_outgoing"]
    ch = [idx[C.addressof(M.children[k].contents)] for k in range(M.num_of_children)]
    ind = [idx[C.addressof(M.independent[k].contents)] for k in range(M.num_of_vars - M.num_of_children)]
    assert ch == d["children"] and ind == d["independent"]
    lib.free_model(pm)


def write_data(path, header, series, sep=" "):
    with open(path, "w") as f:
        f.write(sep.join(header) + "\n")
        for s in series:
            for row in s:
                f.write(sep.join(row) + "\n")
            f.write("\n")


def test_timeseries_round_trip(lib, tmp_path):
    """read_timeseries (columns not in the model ignored, nulls missing, the
    hidden variables in model order) and write_timeseries (',' separators,
    "null", a blank line after each series) against oracle/datafile.py."""
    path = os.path.join(GOLD, "demo1.net")
    m = nip_amd.Model.from_net(path)
    a, b = m.state_names(m.variable("A1")), m.state_names(m.variable("B1"))
    rng = np.random.default_rng(3)
    series = [[[rng.choice(a + ["null"]), "x", rng.choice(b + ["N/A"])] for _ in range(T)]
              for T in (4, 1, 7)]
    series[0][0][0] = a[0]
    data = str(tmp_path / "in.txt")
    write_data(data, ["A1", "junk", "B1"], series)
    pm = lib.parse_model(path.encode())
    ts = C.POINTER(C.POINTER(Series))()
    n = lib.read_timeseries(pm, data.encode(), C.byref(ts))
    syms = [dv["symbol"] for dv in m.desc()["vars"]]
    names = [m.state_names(i) for i in range(m.num_vars)]
    want, ov = ref.read_timeseries(data, syms, names)
    assert n == len(want) == 3
    for i in range(n):
        s = ts[i].contents
        assert s.length == len(want[i]) == lib.timeseries_length(ts[i])
        id0 = pm.contents.variables[0].contents.id
        assert [s.observed[k].contents.id - id0 for k in range(s.num_of_observed)] == ov
        assert [s.hidden[k].contents.id - id0 for k in range(s.num_of_hidden)] == \
               [v for v in range(m.num_vars) if v not in ov]
        got = [[s.data[t][k] for k in range(s.num_of_observed)] for t in range(s.length)]
        assert got == want[i]
    # get/set_observation (nip.c:918-948)
    a1 = lib.model_variable(pm, b"A1")
    assert lib.get_observation(ts[0], a1, 0) == a[0].encode()
    assert lib.get_observation(ts[0], a1, 99) is None
    assert lib.set_observation(ts[0], a1, 0, a[1].encode()) == 0
    assert ts[0].contents.data[0][0] == 1
    assert lib.set_observation(ts[0], a1, 0, b"no such state") == nip_amd.NIP_ERROR_INVALID_ARGUMENT
    out = str(tmp_path / "out.txt")
    assert lib.write_timeseries(ts, n, out.encode()) == 0
    want[0][0][0] = 1
    lines = [",".join(syms[v] for v in ov)]
    for s in want:
        for row in s:
            lines.append(",".join(names[ov[k]][x] if x >= 0 else "null" for k, x in enumerate(row)))
        lines.append("")
    assert open(out).read() == "\n".join(lines) + "\n"
    for i in range(n):
        lib.free_timeseries(ts[i])
    lib.free_model(pm)


def test_double_list(lib):
    """niplists.c: append / prepend / to_array / empty, walked as niptrain.c does."""
    lst = lib.nip_new_double_list()
    for x in (1.5, 2.5):
        assert lib.nip_append_double(lst, x) == 0
    assert lib.nip_prepend_double(lst, 0.5) == 0
    L = lst.contents
    assert L.length == 3
    vals, k = [], L.first
    while k:
        vals.append(k.contents.data)
        k = k.contents.fwd
    assert vals == [0.5, 1.5, 2.5]
    assert L.last.contents.bwd.contents.data == 1.5
    arr = lib.nip_double_list_to_array(lst)
    assert [arr[i] for i in range(3)] == vals
    lib.nip_empty_double_list(lst)
    assert lst.contents.length == 0 and not lst.contents.first


def test_lottery_and_seed(lib):
    """random_seed seeds rand(); lottery draws rand()/RAND_MAX against the
    running sum (nip.c:2482-2520)."""
    libc = C.CDLL(None)
    seed = C.c_long(12345)
    assert lib.random_seed(C.byref(seed)) == 12345
    dist = (C.c_double * 4)(0.1, 0.2, 0.3, 0.4)
    got = [lib.lottery(dist, 4) for _ in range(200)]
    libc.srand(12345)
    cum = np.cumsum([0.1, 0.2, 0.3, 0.4])
    want = []
    for _ in range(200):
        r = libc.rand() / 2147483647.0
        i = 0
        while cum[i] < r:
            i += 1
        want.append(i)
    assert got == want


def test_error_handler(lib, capfd):
    """niperrorhandler.c:32-69: errno-coded messages, last code and counter."""
    import errno
    capfd.readouterr()
    lib.nip_reset_error_handler()
    assert lib.nip_report_error(b"f.c", 7, errno.EINVAL, 1) == errno.EINVAL
    assert lib.nip_report_error(b"f.c", 8, nip_amd.NIP_ERROR_BAD_LUCK, 0) == nip_amd.NIP_ERROR_BAD_LUCK
    assert lib.nip_check_error_type() == nip_amd.NIP_ERROR_BAD_LUCK
    assert lib.nip_check_error_counter() == 2
    assert capfd.readouterr().err == "In f.c (7): Invalid argument given.\n"
    lib.nip_reset_error_handler()
    assert lib.nip_check_error_counter() == 0


def test_reference_programs_built():
    """The reference's util programs compile unmodified against the compat
    headers and link against libnip.so (built by nip_amd.build where the
    reference tree exists)."""
    if not os.path.isdir(build.REF_UTIL):
        pytest.skip("reference tree absent")
    for p in build.REF_PROGRAMS:
        assert os.access(os.path.join(build.REF_BIN_DIR, p), os.X_OK), p
