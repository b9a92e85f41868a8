"""Worker for tests/test_gpu_errors.py: with the diagnostics library
(NIPAMD_LIB=nip_amd/_lib/diag/libnip_amd_diag.so) and NIPAMD_LDS_CAP=1024 every
launcher's LDS check refuses on the host (chain_kernels.h ensure_dyn_lds).
Through the C ABI (nipamd_fb, nipamd_estep via ctypes) the engine must then
report NIPAMD_ERROR_UNSUPPORTED naming the kernel, never NIPAMD_ERROR_DEVICE
"kernel launch failed: no error" (VERDICT r05 weak 8).  Prints one line per
case; exit code 0 = every case refused with code 100."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import nip_amd  # noqa: E402
from nip_amd import synth  # noqa: E402


def main():
    assert os.environ.get("NIPAMD_LDS_CAP"), "run with NIPAMD_LDS_CAP set"
    m = nip_amd.Model.from_spec(*synth.hmm_spec(16, 16))
    ov, q = [m.variable("M1")], [m.variable("P1")]
    obs = torch.from_numpy(synth.observations(32, 64, 16, seed=4)).cuda()
    counts = torch.zeros(m.param_size(), dtype=torch.float64, device="cuda")
    bad = 0
    cases = [("fb", lambda: nip_amd.forward_backward_inference(m, obs, ov, q)),
             ("filter", lambda: nip_amd.forward_inference(m, obs, ov, q)),
             ("estep", lambda: nip_amd.e_step(m, obs, ov, counts))]
    for name, call in cases:
        try:
            call()
            torch.cuda.synchronize()
            print("%s: no error" % name)
            bad += 1
        except nip_amd.NipError as e:
            ok = e.code == nip_amd.NIPAMD_ERROR_UNSUPPORTED and "refused on the host" in str(e)
            print("%s: %s %s" % (name, "ok" if ok else "WRONG", e))
            bad += 0 if ok else 1
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
