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
