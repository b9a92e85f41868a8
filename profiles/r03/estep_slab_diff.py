"""The joint e_step partials of the DPP kernel (chain_kernel<true>) and the
matrix-core kernel on the minimal failing sequence (T = 3: [0, -1, 13]),
region by region (Kf + Kb, Hf + Hb rows, P0).  NIPAMD_JOINT_ESTEP=1 build."""
import os

import numpy as np
import torch

import nip_amd
from nip_amd import synth

np.set_printoptions(precision=4, linewidth=200, suppress=True)
m = nip_amd.Model.from_spec(*synth.factorial_spec(4, 4, 16))
ov = [m.variable("O1")]
M = 16


def partial(seq, kern):
    if kern:
        os.environ["NIPAMD_ESTEP_KERNEL"] = kern
    else:
        os.environ.pop("NIPAMD_ESTEP_KERNEL", None)
    o = torch.tensor(np.array(seq, np.int32).reshape(1, -1, 1)).cuda()
    p, ll, st = nip_amd.estep_partial(m, o, ov)
    torch.cuda.synchronize()
    return p.cpu().numpy().copy()


for seq in ([0, -1, 13], [0, -1, 12], [0, 5, 13], [-1, 13], [13]):
    a = partial(seq, None)
    b = partial(seq, "mfma")
    K = (a[0:256] + a[256:512]).reshape(16, 16) - (b[0:256] + b[256:512]).reshape(16, 16)
    Ha = a[512:512 + (M + 2) * 16].reshape(M + 2, 16) + a[512 + (M + 2) * 16:512 + 2 * (M + 2) * 16].reshape(M + 2, 16)
    Hb = b[512:512 + (M + 2) * 16].reshape(M + 2, 16) + b[512 + (M + 2) * 16:512 + 2 * (M + 2) * 16].reshape(M + 2, 16)
    p0 = 512 + 2 * (M + 2) * 16
    print("seq", seq, "| K diff %.3e | H diff %.3e | P0 diff %.3e" %
          (np.abs(K).max(), np.abs(Ha - Hb).max(), np.abs(a[p0:p0 + 16] - b[p0:p0 + 16]).max()))
    if np.abs(K).max() > 1e-12 or np.abs(Ha - Hb).max() > 1e-12:
        print(" Kf sum %.6f Kb sum %.6f | mfma Kf %.6f Kb %.6f" %
              (a[0:256].sum(), a[256:512].sum(), b[0:256].sum(), b[256:512].sum()))
        print(" H rows (dpp) sums", Ha.sum(axis=1))
        print(" H rows (mfma) sums", Hb.sum(axis=1))
        print(" K diff\n", K)
        print(" dpp Kf\n", a[0:256].reshape(16, 16))
        print(" dpp Kb\n", a[256:512].reshape(16, 16))

np.set_printoptions(precision=17, linewidth=250)
for seq in ([-1, 13], [-1, 12], [13]):
    a = partial(seq, None)
    b = partial(seq, "mfma")
    p0 = 512 + 2 * (M + 2) * 16
    print("P0", seq, "dpp ", repr(a[p0:p0 + 16]))
    print("P0", seq, "mfma", repr(b[p0:p0 + 16]))
