"""Worker for tests/test_gpu_opchain_estep_wide.py::test_wide_op_estep_over_launch_chunks:
the wide operator chain's e_step (op_wide_msgs_kernel + op_wide_xi_kernel,
demo1 @ 20 with A1 B1 D1 observed) with its per-launch message budget lowered
(NIPAMD_OP_WIDE_BYTES, read by the diagnostics build,
NIPAMD_LIB=nip_amd/_lib/diag/libnip_amd_diag.so) so that one batch runs as
several launch chunks of 32 sequences.  Chunks are powers of two, so their
trees are subtrees of the batch tree: the batch's partial must equal the
rank-ordered combination of four power-of-two shards bit for bit, and the
counts must match the general engine's.  Exit code 0 = every check passed.
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import nip_amd  # noqa: E402
from nip_amd import synth  # noqa: E402
from nip_amd.em import tree_sum  # noqa: E402

T = 20
NP = 32


def main():
    per = 2 * T * NP * 8 + T * 4                  # opchain.cpp op_wide_estep: messages + scale exponents
    os.environ["NIPAMD_OP_WIDE_BYTES"] = str(40 * per)
    m = nip_amd.Model.from_spec(*synth.demo1_spec(20))
    ov = [m.variable(s) for s in ("A1", "B1", "D1")]
    rng = np.random.default_rng(5)
    obs_np = np.stack([rng.integers(-1, 20, size=(128, T)) for _ in ov], axis=2).astype(np.int32)
    obs = torch.from_numpy(obs_np).cuda().contiguous()
    whole, _, _ = nip_amd.estep_partial(m, obs, ov)
    whole = whole.clone()
    assert nip_amd.last_kernel() == "op_wide_msgs_kernel (e_step) + op_wide_xi_kernel", nip_amd.last_kernel()
    parts = [nip_amd.estep_partial(m, obs[k * 32:(k + 1) * 32].contiguous(), ov)[0].clone() for k in range(4)]
    comb = tree_sum(torch.stack(parts))
    body = m.partial_size() - 3
    hdr = 1 + 2 * (3 + 8)
    assert torch.equal(comb[body + 3 + hdr:], whole[body + 3 + hdr:]), "shard partials do not combine into the batch's"
    a = nip_amd.estep_finalize(m, whole, None).cpu().numpy()
    m.set_engine(nip_amd.ENGINE_JTREE)
    b, _, _ = nip_amd.e_step(m, obs, ov)
    b = b.cpu().numpy()
    assert np.all(np.abs(a - b) <= 1e-11 * np.maximum(1.0, np.abs(b))), np.abs(a - b).max()
    print("all passed")


if __name__ == "__main__":
    main()
