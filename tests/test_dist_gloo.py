"""Data-parallel EM plumbing on CPU: world_size 2 over gloo.

The GPU e_step is replaced by an injected CPU backend (the oracle's e_step on
this rank's shard: test infrastructure only), so these tests exercise the
distributed driver in nip_amd/em.py exactly as the RCCL run does: shard-wise
partials, all-gather + rank-ordered tree combination, global ll gather,
identical m_step on every rank.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import nip_amd
from nip_amd import synth
from nip_amd.em import tree_sum, combine_partials, exchange, em_learn, NIP_NO_ERROR


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class OracleEStep:
    """partial = counts of this shard without pseudo-counts (em_learn layout)."""

    def partial(self, model, obs, obs_vars):
        from oracle.bind import PortOracle
        orc = PortOracle(model.desc())
        cnt, ll, bad = orc.estep(obs.numpy(), obs_vars, np.zeros(model.param_size()))
        return (torch.from_numpy(cnt), torch.from_numpy(ll), torch.from_numpy(bad.astype(np.int32)))

    def finalize(self, model, partial, counts):
        counts += partial
        return counts


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = dist.group.WORLD
        out = {}
        # 1. partial combination: shard trees + rank-ordered tree == global tree
        rng = np.random.default_rng(5)
        rows = torch.from_numpy(rng.random((64, 37)) * 10.0 ** rng.integers(-3, 4, size=(64, 1)))
        shard = rows[rank * 32:(rank + 1) * 32]
        comb = combine_partials(tree_sum(shard), g)
        out["combine_exact"] = bool(torch.equal(comb, tree_sum(rows)))
        # 2. the packed exchange: partial, ll tree sum and failure count in one all-gather
        ll = torch.from_numpy(rng.random(8) * 1e3)
        mine = ll[rank * 4:(rank + 1) * 4]
        st = torch.tensor([0, 0, rank, 0], dtype=torch.int32)
        p, llt, nbad = exchange(tree_sum(shard), mine, st, g)
        out["ex_partial"] = bool(torch.equal(p, tree_sum(rows)))
        out["ex_ll"] = llt == float(tree_sum(ll.reshape(-1, 1))[0])
        out["ex_bad"] = nbad
        # 3. em_learn over sharded sequences
        nodes, pots = synth.hmm_spec(4, 5, seed=77)
        m = nip_amd.Model.from_spec(nodes, pots)
        obs = synth.observations(8, 20, 5, seed=3)
        mine = torch.from_numpy(obs[rank * 4:(rank + 1) * 4].copy())
        init = synth.uniform01(2024, m.param_size()) + 0.05
        curve = []
        rc = em_learn(m, mine, [m.variable("M1")], 1e-6, curve, init=init, max_iterations=8,
                      group=g, backend=OracleEStep())
        out["rc"] = rc
        out["curve"] = curve
        out["orig"] = np.concatenate([m.original(c) for c in range(2)]).tolist()
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_two_rank_em_driver():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = {}
    import queue, time
    t0 = time.time()
    while len(res) < 2 and time.time() - t0 < 240:
        try:
            r, out = q.get(timeout=2)
            res[r] = out
        except queue.Empty:
            if any(p.exitcode not in (None, 0) for p in ps):
                break
    assert len(res) == 2, [p.exitcode for p in ps]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0]["combine_exact"] and res[1]["combine_exact"]
    for r in range(2):
        assert res[r]["ex_partial"] and res[r]["ex_ll"] and res[r]["ex_bad"] == 1
    # every rank ends with the same model
    assert res[0]["curve"] == res[1]["curve"] and res[0]["orig"] == res[1]["orig"]
    assert res[0]["rc"] == NIP_NO_ERROR
    # and it is the single-process em_learn of the whole set (oracle no_em)
    from oracle.bind import PortOracle
    nodes, pots = synth.hmm_spec(4, 5, seed=77)
    m = nip_amd.Model.from_spec(nodes, pots)
    obs = synth.observations(8, 20, 5, seed=3)
    init = synth.uniform01(2024, m.param_size()) + 0.05
    it, ref_curve = PortOracle(m.desc()).em(obs, [m.variable("M1")], init, 1e-6, 8)
    assert it == len(res[0]["curve"])
    np.testing.assert_allclose(res[0]["curve"], ref_curve, rtol=1e-13)
