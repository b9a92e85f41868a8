"""libnip.so's single-slice propagation on the GPU (SURVEY 8(a) A2-A4, A10-A15,
8(b) hot symbols, 8(f) row 4): nip_collect_evidence / nip_distribute_evidence
/ make_consistent record the reference's message passes and run them through
nipamd_hugin_passes (nip_amd/csrc/hugin.hip), bit-identical to the
reference's own nipjointree.c / nippotential.c.

  - test/cliquetest.c, the reference's own unit test (hand-built join tree,
    evidence, collect + distribute from a middle clique), compiled unmodified
    against include/compat + libnip.so: output identical to the same program
    over the reference's sources, incl. the known answer P(A) = [0.49225,
    0.2973, 0.21045];
  - seeded single-slice scripts with propagation (make_consistent and
    collect/distribute pairs from random cliques, hard and soft evidence,
    retractions, masses, marginals, joints, full dumps of every clique and
    sepset) on 67 models, incl. one whose 160,000-entry clique takes the
    multi-launch path: every printed double identical (%a);
  - util/niplikelihood.c and util/nipjoint.c, unmodified, over libnip.so:
    their printed output equals the reference's numbers formatted the same
    way (niplikelihood.c:129 "%g %g %g"; nipjoint.c:134-143);
  - insert_hard_evidence / insert_soft_evidence / get_probability through
    ctypes.
"""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
pytest.importorskip("torch")

from nip_amd import build, synth
from oracle import bind, netfile

import slice_util as su

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def need(path):
    if not os.access(path, os.X_OK):
        pytest.skip(f"{path} not built (no reference tree where the build ran)")
    return path


def test_cliquetest_identical_to_reference():
    ours = subprocess.run([need(os.path.join(build.REF_BIN_DIR, "cliquetest"))],
                          capture_output=True, text=True, timeout=120)
    ref = subprocess.run([need(os.path.join(ROOT, "oracle", "_ref", "reftests", "cliquetest"))],
                         capture_output=True, text=True, timeout=120)
    assert ours.returncode == 0, ours.stderr
    assert ours.stdout == ref.stdout
    assert "result[0] = 0.49225\nresult[1] = 0.2973\nresult[2] = 0.21045\n" in ours.stdout


@pytest.fixture(scope="module")
def nets(tmp_path_factory):
    d = tmp_path_factory.mktemp("nets")
    out = {name: su.spec_to_net(nodes, pots, str(d / (name + ".net")))
           for name, (nodes, pots) in sorted(su.contract_models().items())}
    out["model"] = os.path.join(su.GOLD, "model.net")
    out["demo1"] = os.path.join(su.GOLD, "demo1.net")
    nodes, pots = synth.wide_spec(20, 6)          # {X0,Y1,Z1,X1}: 160,000 entries
    out["wide20"] = su.spec_to_net(nodes, pots, str(d / "wide20.net"))
    return out


def compare(net, script):
    ref = su.ref_slice(net, script)
    cut = script
    if ref is None:                 # the reference's gather corrupted its heap
        cut = script.split(" joint ")[0]
        ref = su.ref_slice(net, cut)
    got = su.compat_slice(net, cut)
    rl, gl = ref.splitlines(), got.splitlines()
    assert len(rl) == len(gl)
    for a, b in zip(rl, gl):
        if b == "joint null":       # undefined in the reference (tests/test_slice.py)
            continue
        assert a == b, su.first_diff(ref, got)
    return ref


@pytest.mark.skipif(not os.path.exists(su.REF_DRIVER), reason="oracle/_ref not built")
def test_propagation_scripts_bit_identical(nets):
    for name in sorted(nets):
        if name == "wide20":
            continue
        for seed in range(2):
            compare(nets[name], su.random_script(nets[name], 100 + seed))


@pytest.mark.skipif(not os.path.exists(su.REF_DRIVER), reason="oracle/_ref not built")
def test_propagation_large_clique_multilaunch(nets):
    """a 160,000-entry clique (> 65,536: one launch per half-pass)"""
    net = nets["wide20"]
    compare(net, "reset priors 0 consistent mass dump obs 4 3 consistent mass prob 0 prob 3 "
                 "soft 1 " + " ".join(["0.5"] * 19 + ["0"]) + " collect 1 distribute 1 mass dump")


def fmt_g(x):
    return "%g" % x


def test_reference_niplikelihood(tmp_path):
    """util/niplikelihood.c over libnip.so vs the reference's numbers"""
    prog = need(os.path.join(build.REF_BIN_DIR, "niplikelihood"))
    net = os.path.join(su.GOLD, "demo1.net")
    rng = np.random.default_rng(3)
    spec = netfile.read_net(net)
    syms = [n.symbol for n in spec.nodes]
    cols = ["A1", "B1", "D1"]
    cards = [len(spec.nodes[syms.index(c)].states) for c in cols]
    lens = (6, 1, 9)
    data = [rng.integers(-1, np.array(cards)[None, :], size=(T, 3)) for T in lens]
    with open(tmp_path / "data.txt", "w") as f:
        f.write(",".join(cols) + "\n")
        for s in data:
            for row in s:
                f.write(",".join("null" if x < 0 else spec.nodes[syms.index(c)].states[x]
                                 for x, c in zip(row, cols)) + "\n")
            f.write("\n")
    out = subprocess.run([prog, net, str(tmp_path / "data.txt"), "A1", "D1"], capture_output=True,
                         text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    ref = bind.RefHarness(spec.replay())
    want = ["niplikelihood:"]
    for s in data:
        r = ref.likelihood(s[None].astype(np.int32), [syms.index(c) for c in cols], [1, 0, 1])[0]
        want += [" ".join(fmt_g(x) for x in row) for row in r] + [""]
    assert out.stdout.splitlines() == want


def test_reference_nipjoint(tmp_path):
    """util/nipjoint.c over libnip.so vs the reference's join tree: masses
    before / after the first step's evidence and the joint distribution of
    the hidden variables (or of the given ones)"""
    prog = need(os.path.join(build.REF_BIN_DIR, "nipjoint"))
    net = os.path.join(su.GOLD, "model.net")
    with open(tmp_path / "d.txt", "w") as f:
        f.write("M1\n3\n1\n")
    spec = netfile.read_net(net)
    syms = [n.symbol for n in spec.nodes]
    # (without variable arguments nipjoint frees ts->hidden twice, nipjoint.c:118
    # then :145 and free_timeseries, nip.c:800 -- the reference program's own
    # double free, so that form is not run)
    for args, vs in ((["P1"], [1]), (["P0", "P1"], [0, 1]), (["P1", "P0"], [1, 0])):
        out = subprocess.run([prog, net, str(tmp_path / "d.txt"), *args], capture_output=True,
                             text=True, timeout=120)
        assert out.returncode == 0, out.stderr
        ref = su.ref_slice(net, "priors 0 consistent mass obs 2 3 consistent mass joint %d %s"
                           % (len(vs), " ".join(map(str, vs))))
        lines = ref.splitlines()
        m1, m2 = (float.fromhex(l.split()[1]) for l in lines[:2])
        head, vals = lines[2].split(":")
        dims = [int(x) for x in head.split()[1:]]
        p = [float.fromhex(x) for x in vals.split()]
        want = ["nipjoint:", "P(" + ", ".join(syms[v] for v in vs) + ") equals: "]
        for i, x in enumerate(p):
            idx, r = [], i
            for d in dims:
                idx.append(r % d)
                r //= d
            want.append("P(" + ", ".join(map(str, idx)) + ") = %f" % x)
        want += ["Marginal probability before evidence: m1 = %s" % fmt_g(m1),
                 "Marginal probability after evidence : m2 = %s" % fmt_g(m2),
                 "Log. likelihood: ln(m2/m1) = %s" % fmt_g(np.log(m2 / m1))]
        assert out.stdout.splitlines() == want


class Var(C.Structure):   # the leading fields of nip_variable_struct (nipvariable.h:51-56)
    _fields_ = [("id", C.c_ulong), ("symbol", C.c_char_p), ("name", C.c_char_p), ("cardinality", C.c_int)]


def test_insert_evidence_and_get_probability():
    lib = C.CDLL(build.COMPAT_LIB)
    lib.parse_model.restype = C.c_void_p
    lib.parse_model.argtypes = [C.c_char_p]
    lib.model_variable.restype = C.POINTER(Var)
    lib.model_variable.argtypes = [C.c_void_p, C.c_char_p]
    lib.get_probability.restype = C.POINTER(C.c_double)
    lib.get_probability.argtypes = [C.c_void_p, C.POINTER(Var)]
    lib.insert_hard_evidence.argtypes = [C.c_void_p, C.c_char_p, C.c_char_p]
    lib.insert_soft_evidence.argtypes = [C.c_void_p, C.c_char_p, C.POINTER(C.c_double)]
    for f in ("reset_model", "make_consistent", "free_model"):
        getattr(lib, f).argtypes = [C.c_void_p]
    lib.use_priors.argtypes = [C.c_void_p, C.c_int]
    lib.model_prob_mass.restype = C.c_double
    lib.model_prob_mass.argtypes = [C.c_void_p]
    net = os.path.join(su.GOLD, "demo1.net")
    m = lib.parse_model(net.encode())
    assert m
    lib.reset_model(m)
    lib.use_priors(m, 0)
    lib.make_consistent(m)
    assert lib.insert_hard_evidence(m, b"A1", b"1") == 0
    soft = (C.c_double * 2)(0.3, 0.7)
    assert lib.insert_soft_evidence(m, b"D1", soft) == 0
    assert lib.insert_hard_evidence(m, b"nosuch", b"1") == 3      # NIP_ERROR_INVALID_ARGUMENT
    got = []
    for sym in (b"A1", b"B1", b"C0", b"C1", b"D1"):
        v = lib.model_variable(m, sym)
        r = lib.get_probability(m, v)
        got.append([r[i] for i in range(v.contents.cardinality)])
    mass = lib.model_prob_mass(m)
    lib.free_model(m)
    ref = su.ref_slice(net, "reset priors 0 consistent obs 0 1 consistent soft 4 0.3 0.7 consistent "
                            "prob 0 prob 1 prob 2 prob 3 prob 4 mass")
    lines = ref.splitlines()
    for v, line in enumerate(lines[:5]):
        assert [float.fromhex(x) for x in line.split()[2:]] == got[v]
    assert float.fromhex(lines[5].split()[1]) == mass
