"""The C-ABI library loads and exports every entry point of include/*.h
(no compute calls: this runs without a GPU)."""
import ctypes
import glob
import os
import re

import nip_amd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    syms = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        text = open(h).read()
        syms |= set(re.findall(r"^\s*(?:const\s+)?\w+\**\s+\**(nipamd_\w+)\s*\(", text, re.M))
    return syms


def test_exports_every_declared_symbol():
    lib = ctypes.CDLL(nip_amd.LIB_PATH)
    syms = declared_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(lib, s), s
    assert syms == set(nip_amd.EXPORTS)


def test_gfx950_code_object():
    data = open(nip_amd.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_host_side_errors():
    try:
        nip_amd.Model.from_net("/nonexistent.net")
    except nip_amd.NipError as e:
        assert e.code == nip_amd.NIP_ERROR_FILENOTFOUND
    else:
        raise AssertionError("expected NipError")


def test_request_sized_estep_partials():
    """nipamd_estep_partial_size_req (host only): the model-level size for
    requests the chain routes take, plus the operator chain's section --
    header (23: count, 11 request fields, their squares) + (ncomb + 1) K^2 + K -- for one they decline (demo1 with its
    hidden parent D1 observed: K = 2 joint states of C, 3 x 3 x 3 evidence
    combinations); the general engine's requests keep the model size."""
    m = nip_amd.Model.from_net(os.path.join(ROOT, "tests", "golden", "demo1.net"))
    base = m.partial_size()
    ab = [m.variable("A1"), m.variable("B1")]
    assert m.partial_size(ab, 40) == base                      # the chain e_step's request
    abd = ab + [m.variable("D1")]
    K = m.card(m.variable("C1"))
    ncomb = 1
    for v in abd:
        ncomb *= m.card(v) + 1
    assert m.partial_size(abd, 40) == base + 23 + (ncomb + 1) * K * K + K
    m.set_engine(nip_amd.ENGINE_JTREE)
    assert m.partial_size(abd, 40) == m.partial_size()
