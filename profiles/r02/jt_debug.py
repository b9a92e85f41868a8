"""Debug helper: general engine on one fixture vs the CPU schedule replay."""
import json, sys, os
import numpy as np
import torch
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import nip_amd
from jt_emul import Replay

name = sys.argv[1] if len(sys.argv) > 1 else "rand30"
z = np.load("tests/golden/gen_%s.npz" % name)
nodes, pots = json.loads(str(z["spec"]))
m = nip_amd.Model.from_spec([tuple(n) for n in nodes], [(c, p, d) for c, p, d in pots])
ov, q = list(z["obs_vars"]), list(z["query"])
r = Replay(m, ov, q)
print("hdr", r.h)
obs = torch.from_numpy(np.ascontiguousarray(z["obs"][:1])).cuda()
for filt in (False, True):
    fn = nip_amd.forward_inference if filt else nip_amd.forward_backward_inference
    post, ll, st = fn(m, obs, ov, q)
    post = post.cpu().numpy()[0]
    ep, el = r.fb(z["obs"][0], filt)
    print("filter" if filt else "fb", "ll gpu", float(ll[0]), "emul", el)
    for t in range(post.shape[0]):
        d = np.abs(post[t] - ep[t]).max()
        print(t, z["obs"][0][t], "%.3g" % d, np.round(post[t], 4) if d > 1e-12 else "")
