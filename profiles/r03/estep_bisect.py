"""Bisect the joint e_step error to a time step: the failing factorial
sequence of estep_missing_diag.py (case 1, b = 9), alone, with each missing
value filled in turn and with the sequence truncated.  Run under the
NIPAMD_JOINT_ESTEP=1 build."""
import os

import numpy as np
import torch

import nip_amd
from nip_amd import synth
from oracle.bind import PortOracle

rng = np.random.default_rng(52)
obs = rng.integers(0, 16, size=(23, 41, 1)).astype(np.int32)
obs[rng.random(obs.shape) < 0.25] = -1
obs[:, 0] = np.maximum(obs[:, 0], 0)
seq = obs[9:10].copy()
m = nip_amd.Model.from_spec(*synth.factorial_spec(4, 4, 16))
ov = [m.variable("O1")]
orc = PortOracle(m.desc())


def err(o):
    c, _, _ = nip_amd.e_step(m, torch.from_numpy(np.ascontiguousarray(o)).cuda(), ov)
    torch.cuda.synchronize()
    rc, _, rb = orc.estep(o, ov, np.ones(m.param_size()))
    e = np.abs(c.cpu().numpy() - rc)
    return e.max(), int(e.argmax())


print("alone: %.3e at %d" % err(seq))
os.environ["NIPAMD_ESTEP_KERNEL"] = "mfma"
print("alone, mfma e_step kernel: %.3e at %d" % err(seq))
del os.environ["NIPAMD_ESTEP_KERNEL"]
q = [m.variable("X1"), m.variable("Y1")]
post, ll, _ = nip_amd.forward_backward_inference(m, torch.from_numpy(seq).cuda(), ov, q)
rp, rl = orc.fb(seq[0], ov, q)
print("fb: post max abs %.3e, ll %.17g vs %.17g" % (np.abs(post.cpu().numpy()[0] - rp).max(), ll.item(), rl))
for t in range(seq.shape[1]):
    if seq[0, t, 0] < 0:
        s2 = seq.copy()
        s2[0, t, 0] = 0
        print("fill t=%2d: %.3e at %d" % ((t,) + err(s2)))
for T in range(1, seq.shape[1] + 1):
    print("T'=%2d: %.3e at %d" % ((T,) + err(seq[:, :T].copy())))
for t0 in range(1, seq.shape[1] - 1):
    s2 = seq[:, t0:].copy()
    if s2[0, 0, 0] < 0:
        continue
    print("from t0=%2d: %.3e at %d" % ((t0,) + err(s2)))
