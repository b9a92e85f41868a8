"""The checkpoint + recompute e_step at 17..32 states (nip_amd/csrc/
estep_ckw.hip, chain_estep_ckw_kernel): config 3's default e_step (demo1 @ 32
states, one or two observed leaf children, hidden parents) when the host's
rescaling bound holds (engine.cpp ckw_sparse_ok).

Against the CPU oracle (nip.c:1708-2007 restated, pinned to the reference by
tests/test_oracle.py) on proper and non-proper models, every T mod 4, ragged
batches, missing and out-of-range observations, one and two columns, an
unobserved child; at long T against the textbook e_step in torch fp64; shard
invariance of its partials; the same slab as chain_estep_mw_kernel (route tag
(0, 0, 1)).  Tolerances as tests/test_gpu_estep_wide.py: counts rel 1e-11, ll
rel 1e-12, BAD_LUCK flags exact.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

import nip_amd
from nip_amd import synth
from nip_amd.em import tree_sum
from oracle.bind import PortOracle

CNT_RTOL = 1e-11
LL_RTOL = 1e-12
CKW = "chain_estep_ckw_kernel"


def gpu_estep(model, obs, obs_vars):
    o = torch.from_numpy(np.ascontiguousarray(obs, np.int32)).cuda()
    cnt, ll, st = nip_amd.e_step(model, o, obs_vars)
    torch.cuda.synchronize()
    return cnt.cpu().numpy(), ll.cpu().numpy(), st.cpu().numpy()


def close(a, b, rtol):
    return np.all(np.abs(a - b) <= rtol * np.maximum(1.0, np.abs(b)))


def demo1(card, seed, proper):
    """demo1 @ card; proper=True declares C1 before C0 and D1, so the
    reference's CPT normalisation of (C1 | D1 C0) runs over C1 (its lowest
    ID) and every table row sums to 1."""
    nodes, pots = synth.demo1_spec(card, seed=seed)
    if proper:
        nodes = [nodes[0], nodes[1], nodes[3], nodes[2], nodes[4]]
    return nip_amd.Model.from_spec(nodes, pots)


def check_vs_oracle(m, obs, ov):
    cnt, ll, st = gpu_estep(m, obs, ov)
    assert nip_amd.last_kernel() == CKW, nip_amd.last_kernel()
    rc, rl, rb = PortOracle(m.desc()).estep(obs, ov, np.ones(m.param_size()))
    assert np.array_equal(st != 0, rb != 0), (st.tolist(), rb.tolist())
    ok = rb == 0
    assert close(ll[ok], rl[ok], LL_RTOL), np.abs(ll[ok] - rl[ok]).max()
    if ok.all():
        assert close(cnt, rc, CNT_RTOL), np.abs(cnt - rc).max()
    else:
        c2, _, _ = gpu_estep(m, obs[ok], ov)
        rc2, _, _ = PortOracle(m.desc()).estep(obs[ok], ov, np.ones(m.param_size()))
        assert close(c2, rc2, CNT_RTOL), np.abs(c2 - rc2).max()


def gappy(B, T, cards, seed, frac=0.15):
    rng = np.random.default_rng(seed)
    obs = np.stack([rng.integers(0, c, size=(B, T)) for c in cards], axis=2).astype(np.int32)
    obs[rng.random(obs.shape) < frac] = -1
    obs[:, 0, 0] = np.abs(obs[:, 0, 0])           # every series observes its first step (prefix.cpp verdicts aside)
    return obs


@pytest.mark.parametrize("proper", [False, True])
@pytest.mark.parametrize("B,T", [(37, 41), (16, 1), (3, 2), (17, 3), (21, 4), (33, 5), (70, 33), (9, 203)])
def test_ckw_two_columns_vs_oracle(B, T, proper):
    m = demo1(32, 300 + T, proper)
    ov = [m.variable("A1"), m.variable("B1")]
    check_vs_oracle(m, gappy(B, T, (32, 32), B * 31 + T), ov)


@pytest.mark.parametrize("proper", [False, True])
@pytest.mark.parametrize("card,B,T", [(32, 29, 38), (20, 13, 27), (17, 40, 9)])
def test_ckw_one_column_and_an_unobserved_child_vs_oracle(card, B, T, proper):
    """One column (A1): B1 is an unobserved child, whose rows take every step's
    posterior on the missing row."""
    m = demo1(card, 40 + card, proper)
    ov = [m.variable("A1")]
    check_vs_oracle(m, gappy(B, T, (card,), card + T), ov)


@pytest.mark.parametrize("card,M", [(32, 20), (24, 7)])
def test_ckw_hmm_shapes_vs_oracle(card, M):
    m = nip_amd.Model.from_spec(*synth.hmm_spec(card, M, seed=card + M, proper=card == 32))
    check_vs_oracle(m, gappy(45, 30, (M,), M), [m.variable("M1")])


def test_ckw_missing_and_invalid_vs_oracle():
    """Missing runs (inner, trailing, whole columns), out-of-range codes in
    either column (zero mass: BAD_LUCK), with the reference's flags."""
    m = demo1(32, 77, False)
    ov = [m.variable("A1"), m.variable("B1")]
    B, T = 37, 61
    obs = gappy(B, T, (32, 32), 5)
    obs[1, 10:30] = -1
    obs[2, 50:] = -1
    obs[3, 1:, :] = -1
    obs[4, ::2, 1] = -1
    obs[6, 3, 0] = 32                            # out of range: an impossible step
    obs[8, 40, 1] = 99
    obs[36, 5:9] = -1
    check_vs_oracle(m, obs, ov)


def test_ckw_is_the_config3_default():
    m = nip_amd.Model.from_spec(*synth.demo1_spec(32))
    ov = [m.variable("A1"), m.variable("B1")]
    gpu_estep(m, gappy(64, 32, (32, 32), 1), ov)
    assert nip_amd.last_kernel() == CKW, nip_amd.last_kernel()


@pytest.mark.parametrize("T", [1024, 1027])
def test_ckw_long_sequences_vs_textbook(T):
    """Long T: the partial's sums and every ll against the textbook e_step in
    torch fp64 (tests/textbook_util.py chain_sums_torch, pinned to the
    reference by test_oracle_textbook.py); counts rel 1e-11, ll rel 1e-11."""
    from textbook_util import chain_tables, clique_vars, chain_sums_torch
    m = nip_amd.Model.from_spec(*synth.demo1_spec(32, seed=8))
    ov = [m.variable("A1"), m.variable("B1")]
    B = 48
    obs_np = np.concatenate([synth.observations(B, T, 32, seed=T + 7 * i) for i in range(2)], axis=2)
    obs = torch.from_numpy(obs_np).cuda()
    partial, ll, st = nip_amd.estep_partial(m, obs, ov)
    torch.cuda.synchronize()
    assert nip_amd.last_kernel() == CKW
    assert not bool(st.any())
    c1 = m.variable("C1")
    nc = nip_amd.lib().nipamd_model_num_cliques(m._h)
    order = sorted(ov, key=lambda v: next(c for c in range(nc) if set(clique_vars(m, c)) == {c1, v}))
    A, pi, Es = chain_tables(m, m.variable("C0"), c1, order)
    tA, tpi = torch.from_numpy(A).cuda(), torch.from_numpy(pi).cuda()
    tEs = [torch.from_numpy(E).cuda() for E in Es]
    k, h, p, lr = chain_sums_torch(tA, tpi, tEs, [obs[:, :, ov.index(v)].long() for v in order])
    ref = torch.cat([k.reshape(-1)] + [x.reshape(-1) for x in h] + [p]).cpu().numpy()
    got = partial[:ref.size].cpu().numpy()
    assert close(got, ref, CNT_RTOL), np.abs(got - ref).max()
    assert close(ll.cpu().numpy(), lr.cpu().numpy(), 1e-11), np.abs(ll.cpu().numpy() - lr.cpu().numpy()).max()


def test_ckw_partials_are_shard_invariant_and_reproducible():
    """One slab row per 16 sequences and fixed-order trees: the partial of 256
    sequences is the pairwise tree of four 64-sequence shards' partials, bit
    for bit, and a rerun repeats it bit for bit."""
    m = nip_amd.Model.from_spec(*synth.demo1_spec(32, seed=3))
    ov = [m.variable("A1"), m.variable("B1")]
    obs = torch.from_numpy(gappy(256, 24, (32, 32), 6)).cuda().contiguous()
    whole, _, _ = nip_amd.estep_partial(m, obs, ov)
    whole = whole.clone()
    assert nip_amd.last_kernel() == CKW
    again, _, _ = nip_amd.estep_partial(m, obs, ov)
    assert torch.equal(whole, again)
    parts = []
    for k in range(4):
        p, _, _ = nip_amd.estep_partial(m, obs[64 * k:64 * (k + 1)].contiguous(), ov)
        parts.append(p.clone())
    comb = tree_sum(torch.stack(parts))
    torch.cuda.synchronize()
    assert torch.equal(comb[:-3], whole[:-3])
    assert comb[-3:].tolist() == [0.0, 0.0, 4.0] and whole[-3:].tolist() == [0.0, 0.0, 1.0]


def test_ckw_peaked_model_takes_the_mw_kernel():
    """A1 emits only its own state (1e-40 elsewhere): the smallest evidence
    of every state falls below 1e-30, the rescaling bound fails and the
    e_step runs on chain_estep_mw_kernel (per-step rescaling), still matching
    the oracle."""
    nodes, pots = synth.demo1_spec(32, seed=21)
    name, par, _ = pots[0]
    d = np.full((32, 32), 1e-40)
    np.fill_diagonal(d, 1.0)
    pots = [(name, par, (d / d.sum(axis=1, keepdims=True)).ravel())] + list(pots[1:])
    m = nip_amd.Model.from_spec(nodes, pots)
    ov = [m.variable("A1"), m.variable("B1")]
    obs = gappy(20, 17, (32, 32), 3)
    cnt, ll, st = gpu_estep(m, obs, ov)
    assert nip_amd.last_kernel() == "chain_estep_mw_kernel", nip_amd.last_kernel()
    rc, rl, rb = PortOracle(m.desc()).estep(obs, ov, np.ones(m.param_size()))
    ok = rb == 0
    assert np.array_equal(st != 0, rb != 0)
    assert close(ll[ok], rl[ok], LL_RTOL)


def test_ckw_batch_over_two_launches_matches_tree():
    """B above one launch (65,536 sequences): the launch trees combine into
    the batch tree exactly (power-of-two chunks)."""
    m = nip_amd.Model.from_spec(*synth.demo1_spec(32, seed=4))
    ov = [m.variable("A1"), m.variable("B1")]
    B, T = 81920, 5
    obs = torch.from_numpy(gappy(B, T, (32, 32), 17)).cuda().contiguous()
    whole, _, _ = nip_amd.estep_partial(m, obs, ov)
    whole = whole.clone()
    assert nip_amd.last_kernel() == CKW
    a, _, _ = nip_amd.estep_partial(m, obs[:65536].contiguous(), ov)
    a = a.clone()
    b, _, _ = nip_amd.estep_partial(m, obs[65536:].contiguous(), ov)
    torch.cuda.synchronize()
    assert torch.equal(tree_sum(torch.stack([a, b.clone()]))[:-3], whole[:-3])
