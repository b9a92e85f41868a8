"""em_learn over series of any lengths on one GPU (nipamd_em_learn) and the
niptrain counterpart (nip_amd/_lib/nipamd_train), against the reference's
recorded EM curves (tests/golden/fb_*.npz) and the CPU oracle.

Tolerances as test_gpu_estep: learning curves rel 1e-10, counts rel 1e-11.
"""
import ctypes
import glob
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
pytest.importorskip("torch")

import nip_amd
from nip_amd import build, synth
from oracle.bind import PortOracle

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
TRAIN = os.path.join(build.LIB_DIR, "nipamd_train")
CURVE_RTOL = 1e-10


def hmm_fixtures():
    from test_gpu_estep import product_model
    out = []
    for p in sorted(glob.glob(os.path.join(GOLD, "fb_*.npz"))):
        z = np.load(p)
        m = product_model(str(z["model"]))
        if m.estep_supported() and int(z["em_iters"]) >= 0:
            out.append(os.path.basename(p))
    return out


@pytest.mark.parametrize("fixture", hmm_fixtures())
def test_em_learn_series_matches_reference_curve(fixture):
    from test_gpu_estep import product_model
    z = np.load(os.path.join(GOLD, fixture))
    m = product_model(str(z["model"]))
    rc, curve = nip_amd.em_learn_series(m, list(z["obs"]), list(z["obs_vars"]), 1e-6,
                                        init=z["em_init"], max_iterations=12)
    it = int(z["em_iters"])
    assert rc == 0 and len(curve) == it
    ref = z["em_curve"][:it]
    assert np.all(np.abs(np.array(curve) - ref) <= CURVE_RTOL * np.abs(ref))


def test_em_learn_ragged_series_vs_oracle():
    """Series of 7 different lengths: two iterations against the oracle's
    per-series e_step + m_step (counts summed in series order)."""
    nodes, pots = synth.hmm_spec(6, 5, seed=21)
    m = nip_amd.Model.from_spec(nodes, pots)
    ov = [m.variable("M1")]
    rng = np.random.default_rng(3)
    series = [rng.integers(-1, 5, size=(T, 1)).astype(np.int32) for T in (5, 1, 17, 5, 33, 2, 9, 17)]
    # every series observes its first step: a leading missing run meets the
    # reference's BAD_LUCK verdict (prefix.cpp), which after an m_step flips
    # with ulp-level differences of the learned tables (the
    # em_util.check_em_curve tests cover it) -- not what this test is about
    for s in series:
        s[0, 0] = abs(int(s[0, 0]))
    init = rng.random(m.param_size())
    rc, curve = nip_amd.em_learn_series(m, series, ov, 1e-6, init=init, max_iterations=2)
    assert rc == 0 and len(curve) == 2
    orc = PortOracle(m.desc())
    steps = sum(len(s) for s in series)
    params = init
    for k in range(2):
        orc.m_step(params)
        counts = np.ones(m.param_size())
        total = 0.0
        for s in series:
            counts, ll, bad = orc.estep(s[None], ov, counts)
            assert not bad.any()
            total += ll[0]
        assert abs(curve[k] - total / steps) <= CURVE_RTOL * abs(total / steps)
        params = counts


def libc_rand_init(seed, P, runs=1):
    libc = ctypes.CDLL("libc.so.6")
    libc.srand(ctypes.c_uint(seed))
    return [np.array([libc.rand() / 2147483647.0 for _ in range(P)]) for _ in range(runs)]


def test_train_tool_matches_em_learn(tmp_path):
    """nipamd_train (seeded) writes the same model as em_learn_series from the
    same rand() draws followed by write_model."""
    net = os.path.join(GOLD, "model.net")
    m = nip_amd.Model.from_net(net)
    rng = np.random.default_rng(8)
    names = m.state_names(m.variable("M1"))
    data = tmp_path / "data.txt"
    with open(data, "w") as f:
        f.write("M1\n")
        for T in (24, 24, 10, 24):
            for _ in range(T):
                f.write(rng.choice(names[:3]) + "\n")
            f.write("\n")
    out = tmp_path / "trained.net"
    env = dict(os.environ, NIPAMD_SEED="12345")
    r = subprocess.run([TRAIN, net, str(data), "0.0001", "-5", str(out)], capture_output=True,
                       text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    runs = r.stdout.count("  Run ")
    # replay: the same rand() stream, one draw of the parameters per run
    series, ov = nip_amd.read_timeseries(m, str(data))
    inits = libc_rand_init(12345, m.param_size(), runs)
    m2 = nip_amd.Model.from_net(net)
    for init in inits:
        rc, curve = nip_amd.em_learn_series(m2, series, ov, 0.0001, init=init)
    assert rc == 0 and curve[-1] >= -5
    ref_out = tmp_path / "replay.net"
    nip_amd.write_model(m2, str(ref_out))
    assert out.read_text() == ref_out.read_text()
    assert "  Iteration %d:" % (len(curve) - 1) in r.stdout
