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
Every iteration it computes its e_step partial (nipamd_estep_partial); the
partial, the tree sum of its sequences' log-likelihoods and its failure
count are packed into one buffer, all-gathered over RCCL and combined by the
fixed pairwise tree (`tree_sum`) in rank order (`exchange`), and every rank
applies the same finalize and m_step -- so all ranks keep bit-identical
models, and with power-of-two shards the counts and the ll are bit-identical
to the single-GPU run.  That all-gather (partial_size + 2 doubles per rank,
4.2 KB for the 16-state HMM) is the only collective of an iteration.
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
    x = partial.contiguous()
    dev = x.device
    if dist.get_backend(group) == "gloo" and x.is_cuda:
        x = x.cpu()          # gloo rehearsal of the RCCL path (tests)
    out = [torch.empty_like(x) for _ in range(W)]
    dist.all_gather(out, x, group=group)
    return tree_sum(torch.stack(out)).to(dev)


def exchange(partial, ll, status, group=None):
    """The one collective of an EM iteration.

    Each rank packs [its count partial | the tree sum of its per-sequence
    log-likelihoods | its number of failed sequences] into one buffer of
    partial_size + 2 doubles; one all-gather over RCCL (xGMI) and the same
    rank-ordered pairwise tree on every rank give the global partial and the
    global ll.  The ll tree has the shape of the count tree, so for
    power-of-two shards both are bit-identical to the 1-GPU run.
    Returns (partial, ll_total (python float), n_bad (int))."""
    import torch
    if ll.is_cuda:                                # one tree kernel per 64x level (nipamd_tree_sum)
        from . import tree_sum as gpu_tree_sum
        ll_part = gpu_tree_sum(ll.to(torch.float64))
    else:
        ll_part = tree_sum(ll.to(torch.float64).reshape(-1, 1))
    bad = (status != 0).sum().to(torch.float64).reshape(1).to(partial.device)
    packed = torch.cat([partial.reshape(-1), ll_part.reshape(1).to(partial.device), bad])
    comb = combine_partials(packed, group)
    P = partial.numel()
    tail = comb[P:].cpu()
    return comb[:P], float(tail[0]), int(round(float(tail[1])))


class GpuEStep:
    """The product e_step backend: nipamd_estep_partial / _finalize."""

    def partial(self, model, obs, obs_vars):
        from . import estep_partial
        return estep_partial(model, obs, obs_vars)

    def finalize(self, model, partial, counts):
        from . import estep_finalize
        return estep_finalize(model, partial, counts)

    def packed(self, model, obs, obs_vars):
        """The e_step partial written straight into the exchange buffer
        [partial | ll tree sum | failed series] (nipamd_estep_tail fills the
        two scalars on the GPU): no pack kernels, no host round trip before the
        collective.  Returns (packed, partial size)."""
        import torch
        from . import NIPAMD_ERROR_UNSUPPORTED, NipError, _ints, _obs3, estep_partial, estep_tail, lib
        o = _obs3(obs, obs_vars)
        S = lib().nipamd_estep_partial_size_req(model._h, int(o.shape[2]), _ints(obs_vars), int(o.shape[1]))
        if S < 0:                                 # no GPU e_step plan for this model / request
            raise NipError(NIPAMD_ERROR_UNSUPPORTED, "model has no GPU e_step plan")
        buf = torch.empty((S + 2,), dtype=torch.float64, device=obs.device)
        _, ll, status = estep_partial(model, o, obs_vars, partial=buf[:S])
        estep_tail(ll, status, out=buf[S:])
        return buf, S


def iteration(model, params, obs, obs_vars, group=None, backend=None, timing=None):
    """One em_learn iteration (src/nip.c:2154-2207): m_step(params), e_step
    of this rank's shard with pseudo-counts 1.0, the one exchange, finalize.
    Returns (new params (host), global ll, number of failed sequences).
    ``timing``: optional dict; 'exchange_ms' receives the collective's time
    (events on the stream: no synchronisation inside the iteration)."""
    import time
    import torch
    be = backend or GpuEStep()
    P = model.param_size()
    model.m_step(params)                          # nip.c:2154
    if isinstance(be, GpuEStep) and obs.is_cuda:
        # the product path: one buffer from the e_step to the finalize, and
        # one device-to-host synchronisation per iteration (the counts)
        packed, S = be.packed(model, obs, obs_vars)
        if timing is not None:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        comb = combine_partials(packed, group)
        if timing is not None:
            e1.record()
        counts = be.finalize(model, comb[:S], None)   # pseudo-counts 1.0 (nip.c:2172) + the families
        host = counts.cpu().numpy()
        tail = comb[S:].cpu()
        if timing is not None:
            timing["exchange_ms"] = e0.elapsed_time(e1)
        return host, float(tail[0]), int(round(float(tail[1])))
    counts = torch.ones((P,), dtype=torch.float64, device=obs.device)   # nip.c:2172
    partial, ll, status = be.partial(model, obs, obs_vars)
    if timing is not None and obs.is_cuda:
        torch.cuda.synchronize(obs.device)
        t0 = time.perf_counter()
    partial, loglikelihood, n_bad = exchange(partial, ll, status, group)
    if timing is not None and obs.is_cuda:
        timing["exchange_ms"] = (time.perf_counter() - t0) * 1e3
    be.finalize(model, partial, counts)
    return counts.cpu().numpy(), loglikelihood, n_bad


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
    if learning_curve is not None:
        del learning_curve[:]
    P = model.param_size()
    if init is None:
        init = np.random.default_rng(seed).random(P)
    params = np.array(init, dtype=np.float64).reshape(P)
    B, T = int(obs.shape[0]), int(obs.shape[1])
    world = 1
    if group is not None:
        import torch.distributed as dist
        world = dist.get_world_size(group)
    ts_steps = B * T * world                      # nip.c:2141-2143
    loglikelihood = -np.finfo(np.float64).max     # -DBL_MAX, nip.c:2082
    i = 0
    while True:
        old_loglikelihood = loglikelihood
        new, loglikelihood, n_bad = iteration(model, params, obs, obs_vars, group, backend)
        if n_bad:                                 # e_step BAD_LUCK, nip.c:2182-2198
            return NIP_ERROR_BAD_LUCK
        params = new
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
