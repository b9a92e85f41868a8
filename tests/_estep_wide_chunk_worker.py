"""Worker for tests/test_gpu_estep_wide.py::test_wide_partial_shard_invariant_over_launch_chunks:
the wide chain e_step (msgs + stats kernels, 64 states) with its per-launch
byte budget lowered (NIPAMD_ESTEP_WIDE_BYTES, read by the diagnostics build,
NIPAMD_LIB=nip_amd/_lib/diag/libnip_amd_diag.so) so that one batch runs as
several launch chunks whose size the budget alone would make 48 sequences.
The chunk is rounded down to a power of two, so the chunk trees
are subtrees of the batch tree: partials of power-of-two shards must combine
into the whole batch's partial bit for bit, and the counts must still match
the oracle.  Exit code 0 = every check passed.
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
from oracle.bind import PortOracle  # noqa: E402

T = 24
NP = 64


def per_seq_bytes(T):
    # engine.cpp / estep_wide.hip estep_wide_scratch_bytes(N, 1, T)
    return (2 * T + 1) * NP * 8 + T * 4 + 256


def main():
    os.environ["NIPAMD_ESTEP_WIDE_BYTES"] = str(48 * per_seq_bytes(T))
    m = nip_amd.Model.from_spec(*synth.hmm_spec(64, 16, seed=11))
    ov = [m.variable("M1")]
    obs_np = synth.observations(256, T, 16, seed=21)
    obs = torch.from_numpy(obs_np).cuda().contiguous()
    whole, _, _ = nip_amd.estep_partial(m, obs, ov)
    whole = whole.clone()
    assert nip_amd.last_kernel() == "chain_msgs_kernel + chain_stats_kernel", nip_amd.last_kernel()
    parts = []
    for k in range(4):
        p, _, _ = nip_amd.estep_partial(m, obs[k * 64:(k + 1) * 64].contiguous(), ov)
        parts.append(p.clone())
    comb = tree_sum(torch.stack(parts))
    assert torch.equal(comb[:-3], whole[:-3]), "shard partials do not combine into the batch's"
    cnt = torch.ones(m.param_size(), dtype=torch.float64, device="cuda")
    nip_amd.e_step(m, obs, ov, cnt)
    torch.cuda.synchronize()
    rc, _, _ = PortOracle(m.desc()).estep(obs_np, ov, np.ones(m.param_size()))
    c = cnt.cpu().numpy()
    assert np.all(np.abs(c - rc) <= 1e-11 * np.maximum(1.0, np.abs(rc))), np.abs(c - rc).max()
    print("all passed")


if __name__ == "__main__":
    main()
