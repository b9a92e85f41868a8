"""Debug: test_em_learn_ragged_series_vs_oracle, both iterations."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, ROOT)
import nip_amd
from nip_amd import synth
from oracle.bind import PortOracle
nodes, pots = synth.hmm_spec(6, 5, seed=21)
m = nip_amd.Model.from_spec(nodes, pots)
ov = [m.variable("M1")]
rng = np.random.default_rng(3)
series = [rng.integers(-1, 5, size=(T, 1)).astype(np.int32) for T in (5, 1, 17, 5, 33, 2, 9, 17)]
init = rng.random(m.param_size())
rc, curve = nip_amd.em_learn_series(m, series, ov, 1e-6, init=init, max_iterations=2)
print("em_learn_series rc", rc, "curve", curve, nip_amd.last_kernel())
orc = PortOracle(m.desc())
steps = sum(len(s) for s in series)
params = init
m2 = nip_amd.Model.from_spec(nodes, pots)
for k in range(2):
    orc.m_step(params)
    m2.m_step(params)
    counts = np.ones(m.param_size())
    gcounts = np.ones(m.param_size())
    total = 0.0; gtotal = 0.0
    for s in series:
        counts, ll, bad = orc.estep(s[None], ov, counts)
        total += ll[0]
        o = torch.from_numpy(np.ascontiguousarray(s[None])).cuda()
        c, l, st = nip_amd.e_step(m2, o, ov, torch.from_numpy(gcounts).cuda())
        torch.cuda.synchronize()
        gcounts = c.cpu().numpy(); gtotal += float(l[0]); 
        print("  it", k, "T", len(s), nip_amd.last_kernel(), "ll", float(l[0]), ll[0], "st", int(st[0]), bad[0])
    print("it", k, "oracle", total / steps, "gpu", gtotal / steps, "counts err", np.abs(gcounts - counts).max())
    params = counts
