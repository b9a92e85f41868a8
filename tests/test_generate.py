"""generate_data host side on the CPU (nip_amd/csrc/generate.cpp).

* The per-series rand() windows reproduce glibc's rand() stream: stepping
  r[n] = r[n-31] + r[n-3] from series b's window gives exactly the draws
  b*D .. b*D+D-1 that libc's own rand() returns after srand(seed) (the stream
  the reference's generate_data consumes series after series,
  util/nipsample.c:100-110, nip.c:2510).
* The sampling order is the reference's (nip.c:2343-2375), checked against
  the reference's own code (oracle/_ref harness, nh_generate).
The draws themselves need the GPU: tests/test_gpu_generate.py.
"""
import ctypes as C
import json
import os

import numpy as np
import pytest

import nip_amd
from nip_amd import synth

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CONTRACT = json.load(open(os.path.join(GOLD, "index_contract.json")))


def draws_from_window(w, n):
    st = [int(x) for x in w]
    out = []
    for _ in range(n):
        v = (st[-31] + st[-3]) & 0xFFFFFFFF
        st.append(v)
        out.append(v >> 1)
    return out


@pytest.mark.parametrize("seed", [1, 0, 12345, -7, 2**31 + 5, 987654321])
@pytest.mark.parametrize("D", [1, 7, 31, 32, 100, 1000])
def test_rand_windows_match_libc(seed, D):
    libc = C.CDLL(None)
    B = 5
    win = nip_amd.rand_windows(seed, B, D)
    libc.srand(C.c_uint(seed & 0xFFFFFFFF))
    want = [libc.rand() for _ in range(B * D)]
    got = []
    for b in range(B):
        got += draws_from_window(win[b], D)
    assert got == want


def test_rand_windows_far_offsets():
    """A long stream: series 3 of 1e5 draws each starts where libc is after 3e5 calls."""
    libc = C.CDLL(None)
    D = 100000
    win = nip_amd.rand_windows(42, 4, D)
    libc.srand(42)
    for _ in range(3 * D):
        libc.rand()
    assert draws_from_window(win[3], 50) == [libc.rand() for _ in range(50)]


def spec(name):
    if name == "demo1_card32":
        return synth.demo1_spec(32)
    if name == "wide8":
        return synth.wide_spec(8, 5)
    if name in ("model", "demo1"):
        e = CONTRACT[name]
        return [tuple(n) for n in e["nodes"]], [tuple(p) for p in e["potentials"]]
    return synth.hmm_spec(4, 3, seed=1)


@pytest.mark.parametrize("name", ["model", "demo1", "hmm", "wide8"])
def test_sampling_order_matches_reference(name):
    from oracle import bind
    nodes, pots = spec(name)
    m = nip_amd.Model.from_spec(nodes, pots)
    ref = bind.RefHarness(synth.spec_to_replay(nodes, pots))
    order, _ = ref.generate(1, 1, 1)
    assert nip_amd.generate_order(m) == list(order)
