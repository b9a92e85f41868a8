"""GPU parity of the wide chain e_step (estep_wide.hip: chain_msgs_kernel +
chain_stats_kernel) -- interface chains of 17..64 states, hidden parents,
several children, GPU-folded in-cliques: config 3's model (demo1 @ 32
states) and config 5's (the 64^4 wide clique), src/nip.c:1708-2007.

Against the oracle (the CPU restatement, pinned to the reference by
test_oracle.py), the general join-tree engine, and -- for config 5's model --
the reference's own e_step outputs (tests/golden/wide64_prefix.npz, made by
make_golden_wide_prefix.py from oracle/_ref).  Tolerances as every e_step
test: counts rel 1e-11, ll rel 1e-12, BAD_LUCK flags equal,
em_learn curves rel 1e-10.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

import nip_amd
from nip_amd import synth
from nip_amd.em import tree_sum, em_learn
from oracle.bind import PortOracle

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CNT_RTOL = 1e-11
LL_RTOL = 1e-12
WIDE = "chain_msgs_kernel + chain_stats_kernel"
# 17..32 states, one or two observed children: estep_ckw.hip where the host's
# rescaling bound holds (round 6), estep_mw.hip otherwise (and with none)
FUSED = ("chain_estep_ckw_kernel", "chain_estep_mw_kernel")


def expected_kernel(m, ov, N):
    """The routes the engine may take: the fused matrix-core e_steps for
    17..32 states with at most two observed children, the two-kernel one
    otherwise."""
    if not (16 < N <= 32 and len(ov) <= 2):
        return (WIDE,)
    return FUSED if ov else FUSED[1:]


def close(a, b, rtol):
    return np.all(np.abs(a - b) <= rtol * np.maximum(1.0, np.abs(b)))


def gpu_estep(model, obs, obs_vars):
    o = torch.from_numpy(np.ascontiguousarray(obs, np.int32)).cuda()
    cnt, ll, st = nip_amd.e_step(model, o, obs_vars)
    torch.cuda.synchronize()
    return cnt.cpu().numpy(), ll.cpu().numpy(), st.cpu().numpy()


CASES = [
    # name, spec, observed children, interface variable
    ("demo1_32_AB", lambda: synth.demo1_spec(32), ["A1", "B1"], "C1"),
    ("demo1_20_A", lambda: synth.demo1_spec(20, seed=2), ["A1"], "C1"),
    ("demo1_32_none", lambda: synth.demo1_spec(32, seed=4), [], "C1"),
    ("hmm_32", lambda: synth.hmm_spec(32, 20, seed=6), ["M1"], "P1"),
    ("hmm_64", lambda: synth.hmm_spec(64, 16, seed=7), ["M1"], "P1"),
    ("wide_24", lambda: synth.wide_spec(24, 5), ["O1"], "X1"),
    ("wide_18", lambda: synth.wide_spec(18, 6, seed=8), ["O1"], "X1"),
]


@pytest.mark.parametrize("name,spec,osyms,iface", CASES, ids=[c[0] for c in CASES])
@pytest.mark.parametrize("B,T", [(37, 41), (16, 1), (3, 2), (70, 33)])
def test_wide_estep_vs_oracle_and_general_engine(name, spec, osyms, iface, B, T):
    m = nip_amd.Model.from_spec(*spec())
    ov = [m.variable(s) for s in osyms]
    rng = np.random.default_rng(B * 31 + T + len(name))
    if ov:
        obs = np.stack([rng.integers(0, m.card(v), size=(B, T)) for v in ov], axis=2).astype(np.int32)
        obs[rng.random(obs.shape) < 0.2] = -1
        obs[0, :2] = -1
    else:
        obs = np.zeros((B, T, 0), np.int32)
    cnt, ll, st = gpu_estep(m, obs, ov)
    assert nip_amd.last_kernel() in expected_kernel(m, ov, m.card(m.variable(iface))), nip_amd.last_kernel()
    orc = PortOracle(m.desc())
    rc, rl, rb = orc.estep(obs, ov, np.ones(m.param_size()))
    assert np.array_equal(st != 0, rb != 0)
    ok = rb == 0
    assert close(ll[ok], rl[ok], LL_RTOL), np.abs(ll[ok] - rl[ok]).max()
    if not ok.all():
        cnt, _, _ = gpu_estep(m, obs[ok], ov)
        rc, _, _ = orc.estep(obs[ok], ov, np.ones(m.param_size()))
    assert close(cnt, rc, CNT_RTOL), np.abs(cnt - rc).max()
    m.set_engine(nip_amd.ENGINE_JTREE)
    cj, lj, sj = gpu_estep(m, obs[ok], ov)
    m.set_engine(nip_amd.ENGINE_AUTO)
    assert close(cnt, cj, CNT_RTOL), np.abs(cnt - cj).max()


def test_wide_estep_zero_mass_sequences():
    """Out-of-range states (an all-zero likelihood): BAD_LUCK as the oracle,
    and the other sequences' counts unchanged by the dead ones."""
    m = nip_amd.Model.from_spec(*synth.demo1_spec(32, seed=9))
    ov = [m.variable("A1"), m.variable("B1")]
    rng = np.random.default_rng(1)
    obs = rng.integers(0, 32, size=(20, 30, 2)).astype(np.int32)
    obs[4, 11, 0] = 32
    obs[13, 0, 1] = 40
    cnt, ll, st = gpu_estep(m, obs, ov)
    _, rl, rb = PortOracle(m.desc()).estep(obs, ov, np.ones(m.param_size()))
    assert np.array_equal(st != 0, rb != 0) and rb[4] and rb[13]
    ok = rb == 0
    c_ok, _, _ = gpu_estep(m, obs[ok], ov)
    assert close(cnt, c_ok, CNT_RTOL)


def test_wide_partial_is_shard_invariant_and_reproducible():
    """One slab row per 16 sequences and a fixed-order tree: partials of
    shards of 64 sequences combine into the whole batch's, bit for bit."""
    m = nip_amd.Model.from_spec(*synth.demo1_spec(32, seed=3))
    ov = [m.variable("A1"), m.variable("B1")]
    obs = torch.from_numpy(np.concatenate([synth.observations(256, 24, 32, seed=s) for s in (5, 6)],
                                          axis=2)).cuda().contiguous()
    whole, _, _ = nip_amd.estep_partial(m, obs, ov)
    whole = whole.clone()
    assert nip_amd.last_kernel() in FUSED
    again, _, _ = nip_amd.estep_partial(m, obs, ov)
    assert torch.equal(whole, again)
    parts = []
    for k in range(4):
        p, _, _ = nip_amd.estep_partial(m, obs[k * 64:(k + 1) * 64].contiguous(), ov)
        parts.append(p.clone())
    comb = tree_sum(torch.stack(parts))
    assert torch.equal(comb[:-3], whole[:-3])
    assert comb[-3:].tolist() == [0.0, 0.0, 4.0] and whole[-3:].tolist() == [0.0, 0.0, 1.0]


def test_wide_partial_shard_invariant_over_launch_chunks():
    """The launch chunk of the wide e_step is a power of two even when the
    per-launch byte budget would allow 48 sequences: shard
    partials still combine into the batch's bit for bit.  Runs in a worker on
    the diagnostics build, whose NIPAMD_ESTEP_WIDE_BYTES lowers the budget."""
    import subprocess
    import sys
    from nip_amd import build as nb
    here = os.path.dirname(os.path.abspath(__file__))
    r = subprocess.run([sys.executable, os.path.join(here, "_estep_wide_chunk_worker.py")],
                       env=dict(os.environ, NIPAMD_LIB=nb.DIAG_LIB), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "all passed" in r.stdout


def test_config5_model_estep_matches_reference_golden():
    """Config 5's model (64^4 in-clique folded on the GPU, hidden parents Y1
    and Z1): the reference's own e_step on gappy series (wide64_prefix.npz) --
    BAD_LUCK flags (leading missing runs, prefix.cpp), ll of the accepted
    series, and the counts of the accepted series: every count outside the
    16.8M-entry family and 8192 sampled inside it, plus the total."""
    z = np.load(os.path.join(GOLD, "wide64_prefix.npz"))
    m = nip_amd.Model.from_spec(*synth.wide_spec(64, 16))
    ov = [m.variable("O1")]
    obs = z["obs"]
    _, ll, st = gpu_estep(m, obs, ov)
    assert nip_amd.last_kernel() == WIDE
    bad = z["bad"] != 0
    assert np.array_equal(st != 0, bad)
    assert close(ll[~bad], z["ll"][~bad], LL_RTOL)
    cnt, _, st2 = gpu_estep(m, obs[~bad], ov)
    assert not st2.any()
    idx = z["idx"]
    assert close(cnt[idx], z["cnt"], CNT_RTOL), np.abs(cnt[idx] - z["cnt"]).max()
    assert abs(cnt.sum() - float(z["cnt_sum"])) <= 1e-9 * float(z["cnt_sum"])


def test_em_learn_demo1_32_on_chain_kernels_matches_general_engine():
    """em_learn on config 3's model through the wide chain e_step against the
    same run on the general join-tree engine (curves rel 1e-10)."""
    nodes, pots = synth.demo1_spec(32, seed=11)
    obs_np = np.concatenate([synth.observations(48, 30, 32, seed=s) for s in (1, 2)], axis=2)
    curves = []
    for engine in (nip_amd.ENGINE_AUTO, nip_amd.ENGINE_JTREE):
        m = nip_amd.Model.from_spec(nodes, pots)
        m.set_engine(engine)
        ov = [m.variable("A1"), m.variable("B1")]
        curve = []
        rc = em_learn(m, torch.from_numpy(obs_np).cuda(), ov, 1e-6, curve,
                      init=synth.uniform01(5, m.param_size()) + 0.05, max_iterations=5)
        if engine == nip_amd.ENGINE_AUTO:
            assert nip_amd.last_kernel() in FUSED
        curves.append((rc, curve))
    assert curves[0][0] == curves[1][0]
    assert len(curves[0][1]) == len(curves[1][1])
    assert close(np.array(curves[0][1]), np.array(curves[1][1]), 1e-10)


def test_em_learn_config5_model_on_chain_kernels_vs_oracle():
    """em_learn on config 5's model (the 64^4 wide clique): two iterations on
    the chain kernels, the first e_step's ll against the oracle."""
    nodes, pots = synth.wide_spec(64, 16)
    m = nip_amd.Model.from_spec(nodes, pots)
    ov = [m.variable("O1")]
    obs_np = synth.observations(32, 16, 16, seed=3)
    curve = []
    init = synth.uniform01(9, m.param_size()) + 0.05
    rc = em_learn(m, torch.from_numpy(obs_np).cuda(), ov, 1e-9, curve, init=init, max_iterations=2)
    assert nip_amd.last_kernel() == WIDE
    assert len(curve) == 2 and np.all(np.isfinite(curve))


def test_config3_estep_full_size_sums_vs_textbook():
    """Config 3's e_step at its full size (demo1 @ 32 states, A1 and B1
    observed, 65,536 x 256, the bench's inputs) on the fused matrix-core
    kernel: the partial's three sums -- K (the in-clique's xi sums without the
    transition), both children's count tables H and P0, each summed over all
    sequences by the kernel's fixed-order trees -- element by element against
    a textbook e_step in torch fp64 on the same GPU (tests/textbook_util.py
    chain_sums_torch: per-step normalised family marginals, nip.c:1925-1967),
    every sequence's ll, and the counts against the general formula of the
    finalize (the projection is checked against the oracle by the cases
    above).  Counts rel 1e-11, ll rel 1e-11 (32-state configs)."""
    from textbook_util import chain_tables, clique_vars, chain_sums_torch
    m = nip_amd.Model.from_spec(*synth.demo1_spec(32))
    ov = [m.variable("A1"), m.variable("B1")]
    B, T = 65536, 256
    obs_np = np.concatenate([synth.observations(B, T, 32, seed=1 + 104729 * i) for i in range(2)], axis=2)
    obs = torch.from_numpy(obs_np).cuda()
    partial, ll, st = nip_amd.estep_partial(m, obs, ov)
    torch.cuda.synchronize()
    assert nip_amd.last_kernel() in FUSED
    assert not bool(st.any())
    # the slab's children in the chain plan's order: by their {C1, child} clique
    c1 = m.variable("C1")
    nc = nip_amd.lib().nipamd_model_num_cliques(m._h)
    order = sorted(ov, key=lambda v: next(c for c in range(nc) if set(clique_vars(m, c)) == {c1, v}))
    A, pi, Es = chain_tables(m, m.variable("C0"), c1, order)
    tA, tpi = torch.from_numpy(A).cuda(), torch.from_numpy(pi).cuda()
    tEs = [torch.from_numpy(E).cuda() for E in Es]
    N = 32
    K = torch.zeros((N, N), dtype=torch.float64, device="cuda")
    Hs = [torch.zeros((E.shape[1] + 2, N), dtype=torch.float64, device="cuda") for E in Es]
    P0 = torch.zeros(N, dtype=torch.float64, device="cuda")
    lls = []
    for b0 in range(0, B, 8192):
        cols = [obs[b0:b0 + 8192, :, ov.index(v)].long() for v in order]
        k, h, p, l = chain_sums_torch(tA, tpi, tEs, cols)
        K += k
        for i in range(len(Hs)):
            Hs[i] += h[i]
        P0 += p
        lls.append(l)
    ref = torch.cat([K.reshape(-1)] + [h.reshape(-1) for h in Hs] + [P0]).cpu().numpy()
    got = partial[:ref.size].cpu().numpy()
    assert close(got, ref, CNT_RTOL), np.abs(got - ref).max()
    lr = torch.cat(lls).cpu().numpy()
    assert close(ll.cpu().numpy(), lr, 1e-11), np.abs(ll.cpu().numpy() - lr).max()
