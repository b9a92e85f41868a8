"""generate_data on the GPU (nip_amd/csrc/generate.hip) against the
reference's own generate_data (oracle/_ref harness nh_generate: src/nip.c
code compiled unmodified, the sampling loop of nip.c:2325-2478 restated)
from the same srand(seed) stream, B series after one another.

Integer draws: the bar is bit-exact equality.  (The GPU's conditional tables
are summed in a different order from the reference's join tree, so a draw
could only differ when rand()/RAND_MAX falls within a few ulps of a
cumulative boundary -- none does in these cases.)
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

import nip_amd
from nip_amd import synth
from oracle import bind

from test_generate import spec

CASES = {
    "model": lambda: spec("model"),
    "demo1": lambda: spec("demo1"),
    "hmm4x3": lambda: synth.hmm_spec(4, 3, seed=1),
    "hmm16": lambda: synth.hmm_spec(16, 16),
    "demo1_card4": lambda: synth.demo1_spec(4),
    "demo1_card32": lambda: synth.demo1_spec(32),
    "wide8": lambda: synth.wide_spec(8, 5),
}


def gen(nodes, pots, seed, B, T):
    m = nip_amd.Model.from_spec(nodes, pots)
    order, out = nip_amd.generate_data(m, seed, B, T)
    torch.cuda.synchronize()
    return order, out.cpu().numpy()


@pytest.mark.parametrize("name", sorted(CASES))
@pytest.mark.parametrize("seed", [12345, 7])
def test_generate_matches_reference(name, seed):
    nodes, pots = CASES[name]()
    order, got = gen(nodes, pots, seed, 9, 17)
    ref = bind.RefHarness(synth.spec_to_replay(nodes, pots))
    rorder, want = ref.generate(seed, 9, 17)
    assert order == list(rorder)
    assert np.array_equal(got, want), np.argwhere(got != want)[:5]


@pytest.mark.parametrize("net", ["model", "demo1"])
def test_reference_nipsample(tmp_path, net):
    """util/nipsample.c itself, compiled against include/compat and linked
    with libnip.so (generate_data on the GPU from its rand() stream): the file
    it writes is the reference's generate_data from the seed it prints, in
    write_timeseries' format (nip.c:670-789)."""
    import os
    import re
    import subprocess
    from test_gpu_compat import ref_program, GOLD
    path = os.path.join(GOLD, net + ".net")
    out = str(tmp_path / "sample.txt")
    n, T = 4, 13
    r = subprocess.run([ref_program("nipsample"), path, str(n), str(T), out],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    seed = int(re.search(r"Random seed = (-?\d+)", r.stdout).group(1))
    nodes, pots = spec(net)
    order, want = bind.RefHarness(synth.spec_to_replay(nodes, pots)).generate(seed & 0xFFFFFFFF, n, T)
    m = nip_amd.Model.from_net(path)                  # the state names of the file
    names = [m.state_names(v) for v in range(m.num_vars)]
    syms = [d["symbol"] for d in m.desc()["vars"]]
    lines = [",".join(syms[v] for v in order)]
    for s in range(n):
        for t in range(T):
            lines.append(",".join(names[v][want[s, t, i]] for i, v in enumerate(order)))
        lines.append("")
    assert open(out).read() == "\n".join(lines) + "\n"


def test_generate_many_series():
    """300 series: every series' rand() window is derived on the GPU
    (rand_window_kernel: x^(b T nv) by square-and-multiply on b's bits),
    including the last ones, far into the stream."""
    nodes, pots = synth.hmm_spec(4, 3, seed=1)
    _, got = gen(nodes, pots, 31337, 300, 7)
    want = bind.RefHarness(synth.spec_to_replay(nodes, pots)).generate(31337, 300, 7)[1]
    assert np.array_equal(got, want), np.argwhere(got != want)[:5]


def test_generate_edge_lengths():
    """T = 1 (first slice only), B = 1, and B*T = 0 (nothing drawn)."""
    nodes, pots = synth.demo1_spec(4)
    ref = bind.RefHarness(synth.spec_to_replay(nodes, pots))
    for B, T in ((5, 1), (1, 40)):
        _, got = gen(nodes, pots, 99, B, T)
        assert np.array_equal(got, ref.generate(99, B, T)[1])
    m = nip_amd.Model.from_spec(nodes, pots)
    order, out = nip_amd.generate_data(m, 1, 0, 5)
    assert out.shape == (0, 5, len(order))


def test_generate_large_batch_properties():
    """B = 20000 series: the first two equal the reference's; every later
    slice's previous-slice column repeats the interface draw before it (the
    forward message is a point mass, nip.c:2439-2446); the empirical emission
    frequencies match the model's table."""
    nodes, pots = synth.hmm_spec(16, 16)
    m = nip_amd.Model.from_spec(nodes, pots)
    B, T = 20000, 50
    order, out = nip_amd.generate_data(m, 4242, B, T)
    got = out.cpu().numpy()
    ref = bind.RefHarness(synth.spec_to_replay(nodes, pots))
    assert np.array_equal(got[:2], ref.generate(4242, 2, T)[1])
    ip, ic = order.index(m.variable("P0")), order.index(m.variable("P1"))
    assert np.array_equal(got[:, 1:, ip], got[:, :-1, ic])
    io = order.index(m.variable("M1"))
    x, o = got[:, :, ic].ravel(), got[:, :, io].ravel()
    counts = np.zeros((16, 16))
    np.add.at(counts, (x, o), 1)
    emp = counts / counts.sum(1, keepdims=True)
    # the emission clique {P1, M1} as the reference's parser leaves it (its CPT
    # quirk normalises along the lowest-ID variable, P1), conditioned on P1
    d = m.desc()
    c = [k for k, cl in enumerate(d["cliques"]) if cl["vars"] == sorted([m.variable("P1"), m.variable("M1")])][0]
    E = np.asarray(d["cliques"][c]["original"]).reshape(16, 16).T       # [P1][M1]
    E = E / E.sum(1, keepdims=True)
    n = counts.sum(1, keepdims=True)
    assert (np.abs(emp - E) <= 5 * np.sqrt(E * (1 - E) / n) + 1e-9).all()     # 5 sigma per cell
