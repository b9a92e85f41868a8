"""Data-parallel EM on the GPU: the product
e_step backend (GpuEStep: nipamd_estep_partial / _finalize through the C-ABI)
in a world_size-2 process group on the one GPU of the test box.

Both ranks run on cuda:0 (RCCL refuses two ranks on one device, so the group
is gloo; em.exchange moves the packed buffer through host memory for gloo and
over RCCL/xGMI in bench.py --workload em).  Asserted:
  * the 2-rank learning curve, final model and per-iteration ll are
    bit-identical to the 1-rank run over the same sequences (power-of-two
    shards: the rank trees are subtrees of the 1-GPU tree);
  * at the full per-GPU shard of config 4 (131072 x 1024), count masses and
    spot oracle parity (per-sequence ll and counts of a 32-sequence subset).
"""
import os
import queue
import socket
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

import nip_amd
from nip_amd import synth
from nip_amd import em as nem
from oracle.bind import PortOracle

B_TOTAL, T, ITERS = 1024, 96, 5


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(rank, world, group):
    nodes, pots = synth.hmm_spec(16, 16, seed=31)
    m = nip_amd.Model.from_spec(nodes, pots)
    obs = synth.observations(B_TOTAL, T, 16, seed=77)
    per = B_TOTAL // world
    mine = torch.from_numpy(np.ascontiguousarray(obs[rank * per:(rank + 1) * per])).cuda()
    params = synth.uniform01(2024, m.param_size()) + 0.05
    lls = []
    for _ in range(ITERS):
        params, ll, bad = nem.iteration(m, params, mine, [m.variable("M1")], group)
        assert bad == 0
        lls.append(ll)
    orig = np.concatenate([m.original(c) for c in range(len(m.desc()["cliques"]))])
    return {"lls": lls, "params": params.tolist(), "orig": orig.tolist()}


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, _run(rank, world, dist.group.WORLD)))
    except Exception as e:  # report, do not hang the parent
        q.put((rank, {"error": repr(e)}))
    finally:
        dist.destroy_process_group()


def test_two_rank_em_on_gpu_bit_identical_to_one_rank():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = {}
    t0 = time.time()
    while len(res) < 2 and time.time() - t0 < 100:
        try:
            r, out = q.get(timeout=2)
            res[r] = out
        except queue.Empty:
            if any(p.exitcode not in (None, 0) for p in ps):
                break
    for p in ps:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    assert len(res) == 2, [p.exitcode for p in ps]
    for r in range(2):
        assert "error" not in res[r], res[r]
    one = _run(0, 1, None)
    for r in range(2):
        assert res[r]["lls"] == one["lls"]          # bit-identical, not approximately
        assert res[r]["params"] == one["params"]
        assert res[r]["orig"] == one["orig"]


def test_config4_shard_scale_and_spot_parity():
    """One e_step over config 4's per-GPU shard (131072 x 1024)."""
    nodes, pots = synth.hmm_spec(16, 16)
    m = nip_amd.Model.from_spec(nodes, pots)
    B, Tn, N, M = 131072, 1024, 16, 16
    obs_np = synth.observations(B, Tn, M, seed=4)
    obs = torch.from_numpy(obs_np).cuda()
    del obs_np
    ov = [m.variable("M1")]
    partial, ll, st = nip_amd.estep_partial(m, obs, ov)
    counts = torch.ones((m.param_size(),), dtype=torch.float64, device="cuda")
    nip_amd.estep_finalize(m, partial, counts)
    cnt = counts.cpu().numpy()
    assert not st.any().item()
    assert bool(torch.isfinite(ll).all()) and float(ll.max()) < 0
    d = m.desc()
    sizes = []
    for v in d["vars"]:
        s = v["card"]
        for p in v["parents"]:
            s *= d["vars"][p]["card"]
        sizes.append(s)
    offs = np.concatenate([[0], np.cumsum(sizes)])
    mass = {d["vars"][i]["symbol"]: cnt[offs[i]:offs[i + 1]].sum() for i in range(3)}
    assert abs(mass["P0"] - (N + B)) <= 1e-9 * (N + B)
    assert abs(mass["P1"] - (N * N + B * Tn)) <= 1e-9 * B * Tn
    assert abs(mass["M1"] - (N * M + B * Tn)) <= 1e-9 * B * Tn
    # spot parity: 32 sequences spread over the shard, per-sequence ll from
    # the full-shard launch, counts of the subset against the oracle
    idx = np.linspace(0, B - 1, 32).astype(np.int64)
    sub = obs[torch.from_numpy(idx).cuda()].contiguous()
    sub_np = sub.cpu().numpy()
    rc, rl, rb = PortOracle(d).estep(sub_np, ov, np.ones(m.param_size()))
    assert not rb.any()
    llf = ll.cpu().numpy()[idx]
    assert np.all(np.abs(llf - rl) <= 1e-12 * np.abs(rl))
    c32, _, _ = nip_amd.e_step(m, sub, ov)
    c32 = c32.cpu().numpy()
    assert np.all(np.abs(c32 - rc) <= 1e-11 * np.maximum(1.0, np.abs(rc)))


@pytest.mark.parametrize("n,S", [(1, 1), (63, 1), (64, 1), (65, 3), (4097, 1), (131072, 1), (130001, 2)])
def test_gpu_tree_sum_bit_identical_to_pairwise_tree(n, S):
    """nipamd_tree_sum (the exchange's ll tree) is the pairwise tree of
    em.tree_sum, bit for bit, for any n (odd tails paired with 0)."""
    import torch
    rng = np.random.default_rng(n + S)
    x = torch.tensor(rng.standard_normal((n, S)) * 10.0 ** rng.integers(-8, 8, (n, S)), dtype=torch.float64)
    want = nem.tree_sum(x.clone())
    got = nip_amd.tree_sum(x.cuda()).cpu()
    assert torch.equal(got, want.reshape(-1))


@pytest.mark.parametrize("B", [0, 1, 64, 65, 4096, 4097, 131072, 130001])
def test_estep_tail_is_the_exchange_pack(B):
    """nipamd_estep_tail (em.iteration's pack): [the pairwise-tree sum of ll,
    the number of nonzero status words], bit for bit what exchange() packs."""
    import torch
    rng = np.random.default_rng(B)
    ll = torch.tensor(-rng.random(B) * 10.0 ** rng.integers(0, 4, B), dtype=torch.float64)
    st = torch.tensor(rng.integers(0, 4, B) * (rng.random(B) < 0.01), dtype=torch.int32)
    out = nip_amd.estep_tail(ll.cuda(), st.cuda()).cpu()
    want = nem.tree_sum(ll.reshape(-1, 1)).reshape(-1)[0] if B else torch.tensor(0.0, dtype=torch.float64)
    assert out[0].item() == want.item()
    assert out[1].item() == float(int((st != 0).sum()))


def test_config4_full_shard_counts_vs_textbook():
    """The whole config-4 shard (131072 x 1024) element by element: the
    e_step counts of the full launch (8 chunks of 16384 sequences, the
    fixed-order trees) against a textbook e_step in torch fp64 on the same
    GPU (tests/textbook_util.py hmm_estep_torch, pinned to the reference by
    test_oracle_textbook.py), counts rel 1e-11, every sequence's ll rel 1e-12."""
    from textbook_util import chain_tables, hmm_estep_torch
    nodes, pots = synth.hmm_spec(16, 16)
    m = nip_amd.Model.from_spec(nodes, pots)
    B, Tn = 131072, 1024
    obs = torch.from_numpy(synth.observations(B, Tn, 16, seed=4)).cuda()
    ov = [m.variable("M1")]
    counts, ll, st = nip_amd.e_step(m, obs, ov, torch.zeros((m.param_size(),), dtype=torch.float64, device="cuda"))
    assert not st.any().item()
    A, pi, Es = chain_tables(m, m.variable("P0"), m.variable("P1"), [m.variable("M1")])
    tA, tpi, tE = (torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in (A, pi, Es[0]))
    want = torch.zeros_like(counts)
    wll = torch.empty_like(ll)
    for b0 in range(0, B, 16384):
        c, l = hmm_estep_torch(tA, tpi, tE, obs[b0:b0 + 16384, :, 0].long())
        want += c
        wll[b0:b0 + 16384] = l
        del c
        torch.cuda.empty_cache()
    got, want = counts.cpu().numpy(), want.cpu().numpy()
    err = np.abs(got - want) / np.maximum(1.0, np.abs(want))
    assert err.max() <= 1e-11, err.max()
    lg, lw = ll.cpu().numpy(), wll.cpu().numpy()
    assert np.all(np.abs(lg - lw) <= 1e-12 * np.abs(lw)), np.abs(lg - lw).max()


def _rccl_worker(port, q):
    """One rank over the "nccl" backend (RCCL on ROCm): the exchange's
    all-gather of a packed config-4 partial on cuda:0."""
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=0, world_size=1)
        nodes, pots = synth.hmm_spec(16, 16, seed=31)
        m = nip_amd.Model.from_spec(nodes, pots)
        obs = torch.from_numpy(synth.observations(256, 64, 16, seed=5)).cuda()
        partial, ll, st = nip_amd.estep_partial(m, obs, [m.variable("M1")])
        packed, llt, bad = nem.exchange(partial, ll, st, None)
        x = torch.cat([packed, torch.tensor([llt, float(bad)], dtype=torch.float64, device="cuda")])
        out = [torch.empty_like(x)]
        dist.all_gather(out, x)                       # RCCL, one rank
        torch.cuda.synchronize()
        q.put({"same": bool(torch.equal(out[0], x)), "backend": dist.get_backend(), "n": x.numel()})
        dist.destroy_process_group()
    except Exception as e:  # report, do not hang the parent
        q.put({"error": repr(e)})


def test_rccl_all_gather_one_rank():
    """The exchange's collective through RCCL on the test box's one GPU (two
    ranks cannot share a device under RCCL; the 2-rank path above is gloo).
    Executes the nccl backend's init and all-gather with the packed buffer."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_free_port(), q))
    p.start()
    try:
        res = q.get(timeout=100)
    finally:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    assert "error" not in res, res
    assert res["backend"] == "nccl" and res["same"] and res["n"] > 2
