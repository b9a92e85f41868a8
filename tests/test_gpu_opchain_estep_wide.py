"""The operator chain's e_step at 17..64 joint interface states (opchain.cpp
op_wide_estep: estep_wide.hip op_wide_msgs_kernel in e_step mode +
op_wide_xi_kernel): slices outside the chain plan whose joint interface has
17-64 states train without the general join-tree engine.

Same partial layout and finalize as the <= 16-state operator chain
(test_gpu_opchain_estep.py); checked against the general engine
(NIPAMD_ENGINE_JTREE, pinned to the reference's golden counts by
test_gpu_jtree.py), against the oracle's e_step, and for shard invariance.
Tolerances: counts 1e-11 relative, ll 1e-12 relative or both
-DBL_MAX, status words equal."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

import nip_amd
from nip_amd import synth
from nip_amd.em import em_learn, tree_sum
from oracle.bind import PortOracle

from test_gpu_opchain_estep import close_cnt, close_ll, estep

WIDE = "op_wide_msgs_kernel (e_step) + op_wide_xi_kernel"


def demo1_20(T, B, seed, names=("D1",), missing=True):
    """demo1's structure at 20 states with C1's hidden parent D1 observed: the
    chain plan rejects it; the joint interface (C1) has 20 states."""
    m = nip_amd.Model.from_spec(*synth.demo1_spec(20))
    ov = [m.variable(s) for s in names]
    rng = np.random.default_rng(seed)
    lo = -1 if missing else 0
    obs = np.stack([rng.integers(lo, m.card(v), size=(B, T)) for v in ov], axis=2).astype(np.int32)
    return m, ov, obs


def factorial(a, b, T, B, seed):
    """A two-variable interface {X1, Y1} (a * b joint states) with evidence on
    the interface variable X1 and the shared child O1: the operator chain."""
    m = nip_amd.Model.from_spec(*synth.factorial_spec(a, b, 5))
    ov = [m.variable("X1"), m.variable("O1")]
    rng = np.random.default_rng(seed)
    obs = np.stack([rng.integers(-1, m.card(v), size=(B, T)) for v in ov], axis=2).astype(np.int32)
    return m, ov, obs


@pytest.mark.parametrize("T", [1, 2, 3, 40, 129])
def test_wide_op_estep_equals_general_engine(T):
    m, ov, obs = demo1_20(T, 37, seed=T)
    a = estep(m, obs, ov)
    assert a[3] == WIDE, a[3]
    b = estep(m, obs, ov, nip_amd.ENGINE_JTREE)
    assert close_cnt(a[0], b[0]), np.abs(a[0] - b[0]).max()
    assert close_ll(a[1], b[1])
    assert np.array_equal(a[2], b[2])


@pytest.mark.parametrize("ab", [(4, 6), (6, 7), (8, 8)], ids=["K24", "K42", "K64"])
def test_wide_op_estep_joint_interfaces(ab):
    """24, 42 and 64 joint states: both block layouts (32 and 64 lanes per
    message) and every cells-per-thread instance of op_wide_xi_kernel."""
    m, ov, obs = factorial(*ab, T=33, B=21, seed=ab[0])
    a = estep(m, obs, ov)
    assert a[3] == WIDE, a[3]
    b = estep(m, obs, ov, nip_amd.ENGINE_JTREE)
    assert close_cnt(a[0], b[0]), np.abs(a[0] - b[0]).max()
    assert close_ll(a[1], b[1])
    assert np.array_equal(a[2], b[2])


def test_wide_op_estep_many_combinations_and_tiles():
    """Two observed variables (441 combinations; A1 a leaf factor of the
    operators, not of the sums' keys) and 16 x 1100 steps per group: two
    sorted tiles per slab row (16,384 steps each), combinations recurring in
    the second (its sums read-add-written)."""
    m, ov, obs = demo1_20(1100, 20, seed=3, names=("A1", "D1"))
    a = estep(m, obs, ov)
    assert a[3] == WIDE, a[3]
    b = estep(m, obs, ov, nip_amd.ENGINE_JTREE)
    assert close_cnt(a[0], b[0]), np.abs(a[0] - b[0]).max()
    assert close_ll(a[1], b[1])
    assert np.array_equal(a[2], b[2])


def test_wide_op_estep_two_leaf_factors():
    """A1 and B1 observed with D1 (the estep_opchain_wide request): both
    children are leaf factors of the operators, so the sums are keyed by D1's
    22 operator indices and A1's / B1's counts come from their count rows
    (gamma by code, the missing row weighted by the table) -- against the
    general engine and the oracle."""
    m, ov, obs = demo1_20(30, 21, seed=8, names=("A1", "B1", "D1"))
    obs[5, 7, 1] = m.card(ov[1])                     # an out-of-range leaf state: a zero-mass series
    a = estep(m, obs, ov)
    assert a[3] == WIDE, a[3]
    b = estep(m, obs, ov, nip_amd.ENGINE_JTREE)
    assert close_cnt(a[0], b[0]), np.abs(a[0] - b[0]).max()
    assert close_ll(a[1], b[1])
    assert np.array_equal(a[2], b[2]) and a[2][5] == 3
    # the oracle on live series (its e_step stops counting at a failed one)
    rc, rl, rb = PortOracle(m.desc()).estep(obs[:5], ov, np.ones(m.param_size()))
    c5, l5, s5, _ = estep(m, obs[:5], ov)
    assert np.array_equal(s5 != 0, rb != 0)
    assert close_ll(l5, rl)
    assert close_cnt(c5, rc), np.abs(c5 - rc).max()


def test_wide_op_estep_vs_oracle():
    m, ov, obs = demo1_20(20, 12, seed=4)
    c, ll, st, k = estep(m, obs, ov)
    assert k == WIDE, k
    rc, rl, rb = PortOracle(m.desc()).estep(obs, ov, np.ones(m.param_size()))
    assert np.array_equal(st != 0, rb != 0)
    assert close_ll(ll, rl)
    assert close_cnt(c, rc), np.abs(c - rc).max()


def test_wide_op_estep_zero_mass_sequences():
    m, ov, obs = demo1_20(20, 33, seed=9)
    obs[3, 5, 0] = m.card(ov[0])
    obs[17, 0, 0] = m.card(ov[0]) + 3
    a = estep(m, obs, ov)
    b = estep(m, obs, ov, nip_amd.ENGINE_JTREE)
    assert np.array_equal(a[2], b[2])
    # the two zero-mass series: ZERO_MASS | BAD_LUCK; others may carry the
    # reference's BAD_LUCK verdict on a leading missing run (prefix.cpp)
    assert a[2][3] == 3 and a[2][17] == 3 and set(a[2].tolist()) <= {0, 2, 3} and (a[2] == 3).sum() == 2
    assert close_cnt(a[0], b[0])
    assert close_ll(a[1], b[1])


def test_wide_op_partial_shard_invariant():
    """One slab row per 8 sequences (kOpWideSeqs), power-of-two chunks: four 64-sequence
    shards combine into the 256-sequence partial bit for bit."""
    m, ov, obs = demo1_20(24, 256, seed=2)
    o = torch.from_numpy(obs).cuda().contiguous()
    whole, _, _ = nip_amd.estep_partial(m, o, ov)
    whole = whole.clone()
    assert nip_amd.last_kernel() == WIDE
    again, _, _ = nip_amd.estep_partial(m, o, ov)
    assert torch.equal(whole, again)
    parts = [nip_amd.estep_partial(m, o[k * 64:(k + 1) * 64].contiguous(), ov)[0].clone() for k in range(4)]
    comb = tree_sum(torch.stack(parts))
    body = m.partial_size() - 3
    hdr = 1 + 2 * (3 + 8)
    assert comb[body:body + 3].tolist() == [-4.0, -4.0, -4.0]
    assert torch.equal(comb[body + 3 + hdr:], whole[body + 3 + hdr:])
    c1 = nip_amd.estep_finalize(m, whole, None).cpu().numpy()
    c4 = nip_amd.estep_finalize(m, comb, None).cpu().numpy()
    assert np.array_equal(c1, c4)


def test_wide_op_estep_over_launch_chunks():
    """Several launch chunks per batch (the diagnostics build's lowered message
    budget, _opwide_chunk_worker.py): the chunk trees combine into the batch
    tree bit for bit and the counts match the general engine's."""
    import os
    import subprocess
    import sys
    from nip_amd import build as nb
    here = os.path.dirname(os.path.abspath(__file__))
    r = subprocess.run([sys.executable, os.path.join(here, "_opwide_chunk_worker.py")],
                       env=dict(os.environ, NIPAMD_LIB=nb.DIAG_LIB), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "all passed" in r.stdout


def test_wide_op_em_learn_matches_general_engine():
    """em_learn on demo1 @ 20 with D1 observed runs its e_step on the wide
    operator chain (no join-tree kernel) and follows the general engine's
    curve and parameters within the count tolerance."""
    m1, ov, obs = demo1_20(48, 64, seed=11)
    obs[:, 0, 0] = np.maximum(obs[:, 0, 0], 0)       # see test_op_em_learn_matches_general_engine
    m2 = nip_amd.Model.from_spec(*synth.demo1_spec(20))
    m2.set_engine(nip_amd.ENGINE_JTREE)
    o = torch.from_numpy(obs).cuda()
    c1, c2 = [], []
    assert em_learn(m1, o, ov, 1e-9, c1, seed=5, max_iterations=4) == em_learn(m2, o, ov, 1e-9, c2, seed=5,
                                                                              max_iterations=4)
    l1, l2 = np.asarray(c1), np.asarray(c2)
    assert len(l1) == len(l2) > 1 and np.all(np.abs(l1 - l2) <= 1e-10 * np.maximum(1.0, np.abs(l2)))
    for c in range(nip_amd.lib().nipamd_model_num_cliques(m1._h)):
        assert np.abs(m1.original(c) - m2.original(c)).max() <= 1e-10
    nip_amd.e_step(m1, o, ov)
    assert nip_amd.last_kernel() == WIDE
