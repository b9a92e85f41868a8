"""Worker for tests/test_gpu_ckpt.py: runs the fb cases through the C-ABI in
this process (kernel choice from NIPAMD_FB_KERNEL) and saves the outputs.

    python tests/_fb_worker.py OUT.npz
"""
import os
import sys

import numpy as np
import torch  # noqa: F401  (first: nip_amd's library then binds to torch's HIP runtime)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import nip_amd  # noqa: E402
from nip_amd import synth  # noqa: E402


def near_identity(n, eps):
    d = np.full((n, n), eps)
    np.fill_diagonal(d, 1.0)
    return (d / d.sum(axis=1, keepdims=True)).ravel()


# name -> (seed of the model, B, T, kind); all 16-state interface chains with
# 16-wide posterior rows (the checkpoint kernel's requests)
CASES = {
    "t1": (1, 8, 1, "plain"),
    "t2": (2, 8, 2, "plain"),
    "t3": (3, 3, 3, "plain"),
    "t9": (4, 5, 9, "plain"),
    "t17": (5, 7, 17, "plain"),
    "t64": (6, 9, 64, "plain"),
    "t77_ragged_b": (7, 21, 77, "plain"),
    "t128": (8, 24, 128, "plain"),
    "t130": (9, 16, 130, "plain"),
    "t1000": (10, 18, 1000, "plain"),
    "missing": (11, 11, 40, "missing"),
    "peaked": (12, 19, 77, "peaked"),
    "config2_slice": (13, 512, 1024, "plain"),
}
# every T around the chunk (8) and checkpoint (4) boundaries, odd batch sizes,
# and lengths across the LDS budget of the checkpoint kernel (it falls back to
# the scratch kernel beyond it)
for _T in list(range(4, 41)) + [63, 64, 65, 127, 129, 255, 257, 511, 513, 1023, 1025, 1500, 1601]:
    CASES["sweep_T%d" % _T] = (100 + _T, 17 if _T < 100 else 9, _T, "missing" if _T % 3 == 0 else "plain")


def build_case(name):
    seed, B, T, kind = CASES[name]
    if kind == "peaked":
        N = 16
        nodes = [("P0", N, "P1"), ("P1", N, None), ("M1", N, None)]
        pots = [("M1", ["P1"], near_identity(N, 1e-60)),
                ("P1", ["P0"], near_identity(N, 1e-50)),
                ("P0", [], np.full(N, 1.0 / N))]
    else:
        nodes, pots = synth.hmm_spec(16, 16, seed=seed)
    m = nip_amd.Model.from_spec(nodes, pots)
    obs = synth.observations(B, T, 16, seed=seed * 7 + T)
    if kind == "missing":
        rng = np.random.default_rng(seed)
        obs = rng.integers(-1, 17, size=(B, T, 1)).astype(np.int32)   # -1 missing, 16 invalid
        obs[0, :, 0] = -1
    return m, obs, [m.variable("M1")], [m.variable("P1")]


def run(m, obs, ov, q):
    o = torch.from_numpy(np.ascontiguousarray(obs, np.int32)).cuda()
    post, ll, st = nip_amd.forward_backward_inference(m, o, ov, q)
    torch.cuda.synchronize()
    return post.cpu().numpy(), ll.cpu().numpy(), st.cpu().numpy()


def main(out):
    res = {}
    for name in CASES:
        post, ll, st = run(*build_case(name))
        res[name + "/post"], res[name + "/ll"], res[name + "/st"] = post, ll, st
    np.savez(out, **res)


if __name__ == "__main__":
    main(sys.argv[1])
