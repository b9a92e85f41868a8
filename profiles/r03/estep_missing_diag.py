"""Round-3 diagnosis of the joint e_step error.

Per case: the batched e_step against the oracle's e_step of the whole batch,
and every sequence alone (B = 1) against the oracle of that sequence, so the
fault is pinned to the batch (block / slab / reduction) or to one sequence's
recursion.  Runs the plain HMM route (chain_kernel<true> + estep_finalize)
and the factorial slice (joint route when the library was built with
NIPAMD_JOINT_ESTEP=1, else the general engine).
"""
import sys

import numpy as np
import torch

import nip_amd
from nip_amd import synth
from oracle.bind import PortOracle


def run(m, ov, obs, label):
    o = torch.from_numpy(obs).cuda()
    c, ll, st = nip_amd.e_step(m, o, ov)
    torch.cuda.synchronize()
    c = c.cpu().numpy()
    orc = PortOracle(m.desc())
    rc, rl, rb = orc.estep(obs, ov, np.ones(m.param_size()))
    err = np.abs(c - rc)
    print("%s B %d T %d: oracle bad %d, batch max abs %.3e at %d" %
          (label, obs.shape[0], obs.shape[1], int(rb.sum()), err.max(), int(err.argmax())))
    worst = []
    for b in range(obs.shape[0]):
        cb, _, _ = nip_amd.e_step(m, torch.from_numpy(obs[b:b + 1].copy()).cuda(), ov)
        torch.cuda.synchronize()
        rcb, _, _ = orc.estep(obs[b:b + 1], ov, np.ones(m.param_size()))
        e = np.abs(cb.cpu().numpy() - rcb)
        worst.append((e.max(), b, int(e.argmax())))
    worst.sort(reverse=True)
    print("   per-sequence worst:", ["%.2e(b=%d,i=%d)" % w for w in worst[:4]])
    # sum of single-sequence e_steps (each starts from ones: subtract them)
    return err.max()


def main():
    rng = np.random.default_rng(52)
    hmm = nip_amd.Model.from_spec(*synth.hmm_spec(16, 16, seed=9))
    fac = nip_amd.Model.from_spec(*synth.factorial_spec(4, 4, 16))
    for B, T, miss in ((23, 41, 0.25), (70, 41, 0.25), (23, 41, 0.0), (5, 41, 0.25), (24, 40, 0.25)):
        obs = rng.integers(0, 16, size=(B, T, 1)).astype(np.int32)
        obs[rng.random(obs.shape) < miss] = -1
        obs[:, 0] = np.maximum(obs[:, 0], 0)
        run(hmm, [hmm.variable("M1")], obs, "hmm    miss %.2f" % miss)
        run(fac, [fac.variable("O1")], obs, "factor miss %.2f" % miss)
    sys.stdout.flush()


if __name__ == "__main__":
    main()
