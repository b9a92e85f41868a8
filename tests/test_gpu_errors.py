"""Error codes through the C ABI: a request the host refuses before queueing
anything is NIPAMD_ERROR_UNSUPPORTED (100) with the kernel's name, a failed
HIP call NIPAMD_ERROR_DEVICE (101) -- launchers return kLaunchRefused for the
first (nip_amd/csrc/chain_kernels.h), engine.cpp / opchain.cpp map it
(launch_fail).  The refusal is forced in a worker process on the diagnostics
library with NIPAMD_LDS_CAP=1024 (every dynamic-LDS kernel then refuses); the
product library ignores that switch (csrc/diag.h) and serves the same calls.
Error conventions: SURVEY 8(b), include/nip_amd.h."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

import nip_amd
from nip_amd import synth

HERE = os.path.dirname(os.path.abspath(__file__))


def test_host_refusal_is_unsupported_not_device_error():
    from nip_amd import build as nb
    env = dict(os.environ, NIPAMD_LIB=nb.DIAG_LIB, NIPAMD_LDS_CAP="1024")
    r = subprocess.run([sys.executable, os.path.join(HERE, "_refusal_worker.py")], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count(": ok ") == 3, r.stdout


def test_product_library_ignores_the_lds_cap(monkeypatch):
    monkeypatch.setenv("NIPAMD_LDS_CAP", "1024")
    m = nip_amd.Model.from_spec(*synth.hmm_spec(16, 16))
    obs = torch.from_numpy(synth.observations(32, 64, 16, seed=4)).cuda()
    post, ll, st = nip_amd.forward_backward_inference(m, obs, [m.variable("M1")], [m.variable("P1")])
    torch.cuda.synchronize()
    assert not st.any().item()
    assert float((post.sum(dim=2) - 1).abs().max()) <= 1e-12
