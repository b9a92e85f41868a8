import sys, os
import numpy as np
import torch
sys.path.insert(0, os.getcwd())
import nip_amd
from nip_amd import synth
from oracle.bind import PortOracle
for seed, B, T in ((3, 64, 50), (3, 9, 64), (200 + 16 * 7 + 16, 9, 64)):
    nodes, pots = synth.hmm_spec(16, 16, seed=seed)
    m = nip_amd.Model.from_spec(nodes, pots)
    obs = synth.observations(B, T, 16, seed=9)
    ov = [m.variable("M1")]
    c1, l1, s1 = nip_amd.e_step(m, torch.from_numpy(obs).cuda(), ov)
    rc, rl, rb = PortOracle(m.desc()).estep(obs, ov, np.ones(m.param_size()))
    c1 = c1.cpu().numpy()
    print(seed, B, T, "chain vs oracle", np.abs(c1 - rc).max(), np.abs(l1.cpu().numpy() - rl).max())
