"""The checkpoint + recompute forward-backward kernel (chain_ckpt.hip).

NIPAMD_FB_KERNEL selects the 16-state fb kernel once per process in the
diagnostics build (csrc/diag.h): this process runs the default (the
checkpoint kernel), a worker process (tests/_fb_worker.py) on the diagnostics
library with NIPAMD_FB_KERNEL=scratch the scratch-round-trip kernel
(chain_mfma.hip).  Both are checked against the oracle (1e-12, as
tests/test_gpu_parity.py) and against each other: the recomputed messages and
the sparse phase-B rescaling change only the powers of two the vectors carry
and the rounding of the last bits, so the two kernels agree to 4e-16
(posteriors, absolute) and 1e-14 (ll, relative).
"""
import os
import subprocess
import sys
import tempfile

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

import nip_amd
from oracle.bind import PortOracle

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import _fb_worker  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
DBL_MAX = np.finfo(np.float64).max


@pytest.fixture(scope="module")
def scratch_results():
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "scratch.npz")
        from nip_amd import build as nb
        env = dict(os.environ, NIPAMD_FB_KERNEL="scratch", NIPAMD_LIB=nb.DIAG_LIB)   # a diagnostics-build switch
        r = subprocess.run([sys.executable, os.path.join(HERE, "_fb_worker.py"), out], env=env,
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stdout + r.stderr
        with np.load(out) as z:
            return {k: z[k] for k in z.files}


@pytest.mark.parametrize("name", list(_fb_worker.CASES))
def test_ckpt_vs_scratch_and_oracle(name, scratch_results):
    m, obs, ov, q = _fb_worker.build_case(name)
    cp, cl, cs = _fb_worker.run(m, obs, ov, q)      # checkpoint kernel (this process)
    post, ll, st = scratch_results[name + "/post"], scratch_results[name + "/ll"], scratch_results[name + "/st"]
    orc = PortOracle(m.desc())
    idx = range(obs.shape[0]) if obs.shape[0] <= 32 else (0, 1, obs.shape[0] // 2, obs.shape[0] - 1)
    if obs.shape[1] > 300:                     # long sweeps: the scratch kernel is the reference, oracle spot check
        idx = (0, obs.shape[0] - 1)
    for b in idx:
        rp, rl = orc.fb(obs[b], ov, q)
        assert np.abs(cp[b] - rp).max() <= 1e-12
        if rl == -DBL_MAX:
            assert cl[b] == -DBL_MAX
        else:
            assert abs(cl[b] - rl) <= 1e-12 * max(1.0, abs(rl))
    assert np.abs(post - cp).max() <= 4e-16
    assert np.all(np.abs(ll - cl) <= 1e-14 * np.maximum(1.0, np.abs(cl)))
    assert np.array_equal(st, cs)
