"""Debug helper: general-engine e_step vs the CPU schedule replay."""
import sys, os
import numpy as np
import torch
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import nip_amd
from nip_amd import synth
from jt_emul import Replay

for N, M, B, T in ((16, 16, 2, 5), (6, 5, 3, 7), (16, 16, 64, 50)):
    nodes, pots = synth.hmm_spec(N, M, seed=3)
    m = nip_amd.Model.from_spec(nodes, pots)
    obs = synth.observations(B, T, M, seed=9)
    ov = [m.variable("M1")]
    r = Replay(m, ov, [], estep=True)
    tot = np.ones(m.param_size())
    lls = []
    for b in range(B):
        s, l, bad = r.fb(obs[b], estep=True)
        tot += s
        lls.append(l)
    m.set_engine(nip_amd.ENGINE_JTREE)
    c, ll, st = nip_amd.e_step(m, torch.from_numpy(obs).cuda(), ov)
    c = c.cpu().numpy()
    d = np.abs(c - tot)
    print(N, M, B, T, "L", r.h["L"], "lds", r.h["lds"], "max diff", d.max(), "argmax", int(d.argmax()),
          "blocks P0/P1/M1", d[:N].max(), d[N:N + N * N].max(), d[N + N * N:].max(),
          "ll diff", np.abs(ll.cpu().numpy() - np.array(lls)).max(), "status", st.cpu().numpy().max())
