"""Which e_step is off on a factorial HMM at T = 41: the joint route (a
NIPAMD_JOINT_ESTEP=1 build), the general engine, or both -- each against the
oracle's e_step, per family of the em_learn layout."""
import numpy as np
import torch

import nip_amd
from nip_amd import synth
from oracle.bind import PortOracle

m = nip_amd.Model.from_spec(*synth.factorial_spec(4, 4, 16))
ov = [m.variable("O1")]
rng = np.random.default_rng(52)
for B, T, miss in ((23, 41, 0.25), (23, 41, 0.0), (16, 41, 0.0), (9, 41, 0.0), (5, 41, 0.25)):
    obs = rng.integers(0, 16, size=(B, T, 1)).astype(np.int32)
    obs[rng.random(obs.shape) < miss] = -1
    obs[:, 0] = np.maximum(obs[:, 0], 0)
    o = torch.from_numpy(obs).cuda()
    res = {}
    for eng, name in ((nip_amd.ENGINE_AUTO, "auto"), (nip_amd.ENGINE_JTREE, "jtree")):
        m.set_engine(eng)
        c, ll, st = nip_amd.e_step(m, o, ov)
        torch.cuda.synchronize()
        res[name] = c.cpu().numpy()
    m.set_engine(nip_amd.ENGINE_AUTO)
    rc, rl, rb = PortOracle(m.desc()).estep(obs, ov, np.ones(m.param_size()))
    print("B", B, "T", T, "missing", miss, "oracle bad", int(np.sum(rb)))
    for name, c in res.items():
        err = np.abs(c - rc)
        print("  %-6s max abs vs oracle %.3e  argmax %d" % (name, err.max(), int(err.argmax())))
