"""The checkpoint + recompute e_step (nip_amd/csrc/estep_ck.hip,
chain_estep_ck_kernel): the default e_step of HMM-shaped slices (16 or fewer
hidden states, one observed child) whose tables pass the host's underflow
bound for rescaling every 4th step (engine.cpp estep16_sparse_ok).

Against the CPU oracle (nip.c:1708-2007 restated, pinned to the reference by
tests/test_oracle.py) on proper and non-proper models, every T mod 4, ragged
batches, missing and out-of-range observations; at long T against the
textbook e_step in torch fp64; shard invariance of its partials (one slab row
per 16 sequences, fixed-order trees).  Tolerances as tests/test_gpu_estep.py:
counts rel 1e-11, ll rel 1e-12, BAD_LUCK flags exact.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

import nip_amd
from nip_amd import synth
from oracle.bind import PortOracle

CNT_RTOL = 1e-11
LL_RTOL = 1e-12
CK = "chain_estep_ck_kernel"


def gpu_estep(model, obs, obs_vars):
    o = torch.from_numpy(np.ascontiguousarray(obs, np.int32)).cuda()
    cnt, ll, st = nip_amd.e_step(model, o, obs_vars)
    torch.cuda.synchronize()
    return cnt.cpu().numpy(), ll.cpu().numpy(), st.cpu().numpy()


def close(a, b, rtol):
    return np.all(np.abs(a - b) <= rtol * np.maximum(1.0, np.abs(b)))


def check_vs_oracle(m, obs, ov):
    cnt, ll, st = gpu_estep(m, obs, ov)
    assert nip_amd.last_kernel().startswith(CK), nip_amd.last_kernel()
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


@pytest.mark.parametrize("proper", [False, True])
@pytest.mark.parametrize("N,M,B,T", [
    (16, 16, 16, 64), (16, 16, 13, 1), (16, 16, 17, 2), (16, 16, 5, 3), (16, 16, 9, 4),
    (16, 16, 33, 5), (16, 16, 16, 7), (16, 16, 3, 8), (16, 16, 21, 9), (16, 16, 40, 203),
    (4, 5, 13, 33), (7, 3, 17, 18), (2, 2, 1, 6), (16, 8, 70, 40), (12, 30, 19, 27), (16, 16, 2, 1000),
])
def test_ck_estep_vs_oracle(N, M, B, T, proper):
    m = nip_amd.Model.from_spec(*synth.hmm_spec(N, M, seed=300 + N * 7 + M, proper=proper))
    obs = synth.observations(B, T, M, seed=T * 31 + B)
    check_vs_oracle(m, obs, [m.variable("M1")])


@pytest.mark.parametrize("proper", [False, True])
def test_ck_estep_missing_and_invalid_vs_oracle(proper):
    """Missing runs (leading, inner, trailing, whole sequences), out-of-range
    codes (zero mass: BAD_LUCK), with the reference's flags."""
    m = nip_amd.Model.from_spec(*synth.hmm_spec(16, 16, seed=77, proper=proper))
    B, T = 37, 61
    obs = synth.observations(B, T, 16, seed=5)
    obs[1, 10:30] = -1
    obs[2, 50:] = -1
    obs[3, :] = -1
    obs[4, ::2] = -1
    obs[6, 3] = 16                               # out of range: an impossible step
    obs[20, :7] = -1
    obs[36, 5:9] = -1
    check_vs_oracle(m, obs, [m.variable("M1")])


def test_ck_estep_is_the_config4_default():
    m = nip_amd.Model.from_spec(*synth.hmm_spec(16, 16))
    obs = synth.observations(64, 32, 16, seed=1)
    gpu_estep(m, obs, [m.variable("M1")])
    assert nip_amd.last_kernel().startswith(CK), nip_amd.last_kernel()


@pytest.mark.parametrize("T", [4096, 4097])
def test_ck_estep_long_sequences_vs_textbook(T):
    """Long T: the per-chunk exact mass keeps the analytic normalisation from
    drifting (counts 1e-11, ll 1e-12 against hmm_estep_torch, the textbook
    e_step pinned to the reference by test_oracle_textbook.py)."""
    from textbook_util import chain_tables, hmm_estep_torch
    m = nip_amd.Model.from_spec(*synth.hmm_spec(16, 16, seed=8))
    B = 64
    obs = torch.from_numpy(synth.observations(B, T, 16, seed=T)).cuda()
    ov = [m.variable("M1")]
    counts, ll, st = nip_amd.e_step(m, obs, ov, torch.zeros((m.param_size(),), dtype=torch.float64, device="cuda"))
    torch.cuda.synchronize()
    assert nip_amd.last_kernel().startswith(CK)
    assert not st.any().item()
    A, pi, Es = chain_tables(m, m.variable("P0"), m.variable("P1"), [m.variable("M1")])
    tA, tpi, tE = (torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in (A, pi, Es[0]))
    want, wll = hmm_estep_torch(tA, tpi, tE, obs[:, :, 0].long())
    got, want = counts.cpu().numpy(), want.cpu().numpy()
    assert np.all(np.abs(got - want) <= 1e-11 * np.maximum(1.0, np.abs(want))), np.abs(got - want).max()
    lg, lw = ll.cpu().numpy(), wll.cpu().numpy()
    assert np.all(np.abs(lg - lw) <= 1e-12 * np.abs(lw)), np.abs(lg - lw).max()


def test_ck_partials_are_shard_invariant():
    """One slab row per 16 sequences: the partial of 256 sequences is the
    pairwise tree of four 64-sequence shards' partials, bit for bit."""
    from nip_amd.em import tree_sum
    m = nip_amd.Model.from_spec(*synth.hmm_spec(16, 16, seed=12))
    obs = torch.from_numpy(synth.observations(256, 48, 16, seed=3)).cuda()
    ov = [m.variable("M1")]
    whole, _, _ = nip_amd.estep_partial(m, obs, ov)
    whole = whole.clone()
    assert nip_amd.last_kernel().startswith(CK)
    parts = []
    for k in range(4):
        p, _, _ = nip_amd.estep_partial(m, obs[64 * k:64 * (k + 1)].contiguous(), ov)
        parts.append(p.clone())
    comb = tree_sum(torch.stack(parts))
    torch.cuda.synchronize()
    assert torch.equal(comb[:-3], whole[:-3])             # the body, bit for bit
    assert comb[-3:].tolist() == [4.0, 0.0, 0.0] and whole[-3:].tolist() == [1.0, 0.0, 0.0]   # route tag counts


def test_ck_batch_over_two_launches_matches_tree():
    """B above one launch (131072 sequences): the launch trees combine into
    the batch tree exactly (power-of-two chunks)."""
    from nip_amd.em import tree_sum
    m = nip_amd.Model.from_spec(*synth.hmm_spec(4, 4, seed=3))
    B, T = 163840, 5
    obs = torch.from_numpy(synth.observations(B, T, 4, seed=12)).cuda().contiguous()
    ov = [m.variable("M1")]
    whole, _, _ = nip_amd.estep_partial(m, obs, ov)
    whole = whole.clone()
    assert nip_amd.last_kernel().startswith(CK)
    a, _, _ = nip_amd.estep_partial(m, obs[:131072].contiguous(), ov)
    a = a.clone()
    b, _, _ = nip_amd.estep_partial(m, obs[131072:].contiguous(), ov)
    assert torch.equal(tree_sum(torch.stack([a, b.clone()]))[:-3], whole[:-3])
