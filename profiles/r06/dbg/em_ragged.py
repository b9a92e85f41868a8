"""Debug: test_em_learn_ragged_series_vs_oracle's first iteration, group by group."""
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
m.m_step(init)
orc = PortOracle(m.desc())
orc.m_step(init)
for T in sorted(set(len(s) for s in series)):
    g = np.stack([s for s in series if len(s) == T])
    o = torch.from_numpy(np.ascontiguousarray(g)).cuda()
    cnt, ll, st = nip_amd.e_step(m, o, ov, torch.zeros(m.param_size(), dtype=torch.float64, device="cuda"))
    torch.cuda.synchronize()
    k = nip_amd.last_kernel()
    rc, rl, rb = orc.estep(g, ov, np.zeros(m.param_size()))
    print("T", T, "B", len(g), k, "ll", ll.cpu().numpy(), "ref", rl, "st", st.cpu().numpy(), "rb", rb,
          "cnt err", float(np.abs(cnt.cpu().numpy() - rc).max()))
    print("   obs", g[:, :, 0].tolist())
