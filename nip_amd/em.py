"""em_learn() (src/nip.c:2076-2243) over the batched GPU e_step.

Mirrors the reference's driver loop exactly -- m_step first (entering the
initial parameters), pseudo-counts 1.0 (nip.c:2172), per-iteration average
log-likelihood appended to the learning curve (nip.c:2208-2222), the
BAD_LUCK exits (e_step failure nip.c:2182-2198; decreasing / positive /
-inf likelihood nip.c:2224-2234) and the stopping rule with
MIN_EM_ITERATIONS = 3 (nip.c:29, 2240-2241) -- with the sequence loop
replaced by one batched e_step per iteration.

Data-parallel (util/niptrain.c:151 trains one model on a sequence set): with
``group`` set, each process owns a shard of the sequences on its own GPU.
Every iteration it computes its e_step partial (nipamd_estep_partial), the
partials are all-gathered over RCCL and combined by the fixed pairwise tree
(`tree_sum`) in rank order, and every rank applies the same finalize and
m_step -- so all ranks keep bit-identical models, and with power-of-two
shards the counts are bit-identical to the single-GPU run.  The only
collectives are one all-gather of partial_size doubles and one of the
per-sequence log-likelihoods per iteration.
"""
from __future__ import annotations

import numpy as np

MIN_EM_ITERATIONS = 3          # src/nip.c:29
NIP_NO_ERROR = 0
NIP_ERROR_BAD_LUCK = 8


def tree_sum(rows):
    """Pairwise binary-tree sum over dim 0 (pairs (2i, 2i+1), odd tail padded
    with 0) -- the same tree the GPU's radix-64 levels implement
    (tree64_kernel), so it extends that tree across shards and ranks."""
    import torch
    x = rows
    while x.shape[0] > 1:
        if x.shape[0] & 1:
            x = torch.cat([x, torch.zeros_like(x[:1])])
        x = x[0::2] + x[1::2]
    return x[0]


def combine_partials(partial, group=None):
    """All-gather every rank's e_step partial and combine in rank order."""
    import torch
    import torch.distributed as dist
    if group is None or dist.get_world_size(group) == 1:
        return partial
    W = dist.get_world_size(group)
    out = [torch.empty_like(partial) for _ in range(W)]
    dist.all_gather(out, partial.contiguous(), group=group)
    return tree_sum(torch.stack(out))


def gather_sequence_ll(ll, status, group=None):
    """Per-sequence log-likelihoods / statuses of all ranks, in global order
    (host numpy).  Shards must have equal length."""
    import torch
    import torch.distributed as dist
    if group is None or dist.get_world_size(group) == 1:
        return ll.cpu().numpy(), status.cpu().numpy()
    W = dist.get_world_size(group)
    both = torch.stack([ll, status.to(torch.float64)]).contiguous()
    out = [torch.empty_like(both) for _ in range(W)]
    dist.all_gather(out, both, group=group)
    out = torch.stack(out).cpu().numpy()
    return out[:, 0].reshape(-1), out[:, 1].reshape(-1).astype(np.int64)


class GpuEStep:
    """The product e_step backend: nipamd_estep_partial / _finalize."""

    def partial(self, model, obs, obs_vars):
        from . import estep_partial
        return estep_partial(model, obs, obs_vars)

    def finalize(self, model, partial, counts):
        from . import estep_finalize
        return estep_finalize(model, partial, counts)


def em_learn(model, obs, obs_vars, threshold, learning_curve=None, init=None,
             max_iterations=None, seed=None, group=None, backend=None):
    """em_learn(ts, n_ts, threshold, learning_curve) (src/nip.c:2076).

    obs: this rank's sequences, CUDA int32 [B, T, n_obs] (all ranks the same
    B and T).  init: initial parameters in the em_learn layout (the
    reference draws them with rand()/RAND_MAX, nippotential.c:222-229; here
    numpy's generator seeded by ``seed`` when init is None, identical on every
    rank).  max_iterations: optional cap the reference does not have.
    Returns NIP_NO_ERROR or NIP_ERROR_BAD_LUCK; the model keeps the
    parameters of the last m_step, as in the reference.
    """
    import torch
    be = backend or GpuEStep()
    if learning_curve is not None:
        del learning_curve[:]
    P = model.param_size()
    if init is None:
        init = np.random.default_rng(seed).random(P)
    params = np.array(init, dtype=np.float64).reshape(P)
    dev = obs.device
    B, T = int(obs.shape[0]), int(obs.shape[1])
    world = 1
    if group is not None:
        import torch.distributed as dist
        world = dist.get_world_size(group)
    ts_steps = B * T * world                      # nip.c:2141-2143
    loglikelihood = -np.finfo(np.float64).max     # -DBL_MAX, nip.c:2082
    i = 0
    while True:
        model.m_step(params)                      # nip.c:2154
        old_loglikelihood = loglikelihood
        counts = torch.ones((P,), dtype=torch.float64, device=dev)   # nip.c:2172
        partial, ll, status = be.partial(model, obs, obs_vars)
        partial = combine_partials(partial, group)
        lls, sts = gather_sequence_ll(ll, status, group)
        if np.any(sts != 0):                      # e_step BAD_LUCK, nip.c:2182-2198
            return NIP_ERROR_BAD_LUCK
        loglikelihood = float(np.sum(lls))
        be.finalize(model, partial, counts)
        params = counts.cpu().numpy()
        if learning_curve is not None:
            learning_curve.append(loglikelihood / ts_steps)
        if (old_loglikelihood > loglikelihood + ts_steps * threshold or
                loglikelihood > 0 or loglikelihood == -np.inf):
            return NIP_ERROR_BAD_LUCK             # nip.c:2224-2234
        i += 1
        if max_iterations is not None and i >= max_iterations:
            return NIP_NO_ERROR
        if not ((loglikelihood - old_loglikelihood) > ts_steps * threshold or i < MIN_EM_ITERATIONS):
            return NIP_NO_ERROR
