"""forward_backward_inference on the checkpoint + recompute kernel at 17..32
states (nip_amd/csrc/estep_ckw.hip, chain_fb_ckw_kernel, round 6): config
3's smoothing (demo1 @ 32, A1 and B1 observed) when the host's rescaling bound
holds.  The forward pass keeps every 4th message; the backward pass recomputes
the others a chunk ahead and writes each step's posterior normalised exactly
(nip.c:1103-1315 / 1708-1800: the reference's per-step smoothed marginals).

Against the CPU oracle (pinned to the reference by tests/test_oracle.py) and
the reference's own fixture (fb_demo1.npz at card 4 is the 16-state kernel's;
here 17..32 states): every T mod 4, ragged batches, proper and non-proper
models, missing and out-of-range observations, one and two columns, queries
on the interface and on derived variables (a child, the hidden parent, the
previous slice); the same posteriors as chain_mfma_wide_kernel (diagnostics
build switch).  Tolerances as tests/test_gpu_wide.py: posteriors 1e-12
absolute, ll 1e-11 relative at 32 states.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

import nip_amd
from nip_amd import synth
from oracle.bind import PortOracle

DBL_MAX = np.finfo(np.float64).max
FBCK = "chain_fb_ckw_kernel"


def demo1(card, seed, proper):
    nodes, pots = synth.demo1_spec(card, seed=seed)
    if proper:
        nodes = [nodes[0], nodes[1], nodes[3], nodes[2], nodes[4]]
    return nip_amd.Model.from_spec(nodes, pots)


def gappy(B, T, cards, seed, frac=0.15):
    rng = np.random.default_rng(seed)
    obs = np.stack([rng.integers(0, c, size=(B, T)) for c in cards], axis=2).astype(np.int32)
    obs[rng.random(obs.shape) < frac] = -1
    return obs


def gpu_fb(model, obs, ov, q):
    o = torch.from_numpy(np.ascontiguousarray(obs, np.int32)).cuda()
    post, ll, st = nip_amd.forward_backward_inference(model, o, ov, q)
    torch.cuda.synchronize()
    return post.cpu().numpy(), ll.cpu().numpy(), st.cpu().numpy()


def check_vs_oracle(m, obs, ov, q, kernel=FBCK, ptol=1e-12, ltol=1e-11):
    post, ll, st = gpu_fb(m, obs, ov, q)
    assert nip_amd.last_kernel().startswith(kernel) or kernel in nip_amd.last_kernel(), nip_amd.last_kernel()
    orc = PortOracle(m.desc())
    for b in range(obs.shape[0]):
        rp, rl = orc.fb(obs[b], ov, q)
        if rl == -DBL_MAX:
            assert ll[b] == -DBL_MAX and st[b], b
            continue
        err = np.abs(post[b] - rp).max()
        assert err <= ptol, "sequence %d: posterior error %g" % (b, err)
        assert abs(ll[b] - rl) <= ltol * max(1.0, abs(rl)), (b, ll[b], rl)
        assert st[b] == 0


@pytest.mark.parametrize("proper", [False, True])
@pytest.mark.parametrize("B,T", [(5, 24), (16, 1), (3, 2), (17, 3), (7, 4), (9, 5), (33, 38), (4, 131)])
def test_fb_ckw_two_columns_vs_oracle(B, T, proper):
    m = demo1(32, 500 + T, proper)
    ov = [m.variable("A1"), m.variable("B1")]
    check_vs_oracle(m, gappy(B, T, (32, 32), B * 13 + T), ov, [m.variable("C1")])


@pytest.mark.parametrize("card,B,T", [(32, 6, 21), (20, 5, 30), (17, 9, 8)])
def test_fb_ckw_one_column_vs_oracle(card, B, T):
    m = demo1(card, 60 + card, False)
    ov = [m.variable("B1")]
    check_vs_oracle(m, gappy(B, T, (card,), card * 3 + T), ov, [m.variable("C1")])


@pytest.mark.parametrize("query", ["A1", "D1", "C0"])
def test_fb_ckw_derived_queries_vs_oracle(query):
    """Queries off the interface: the derive kernels read the interface
    marginals this kernel writes (a child, the hidden parent, the previous
    slice's copy)."""
    m = demo1(32, 7, False)
    ov = [m.variable("A1"), m.variable("B1")]
    obs = gappy(6, 19, (32, 32), 11)
    check_vs_oracle(m, obs, ov, [m.variable(query)], kernel="")


def test_fb_ckw_missing_and_invalid_vs_oracle():
    """Whole-sequence and trailing missing runs, out-of-range codes (zero
    mass: ll = -DBL_MAX and the status bit, as the reference)."""
    m = demo1(32, 9, False)
    ov = [m.variable("A1"), m.variable("B1")]
    obs = gappy(12, 29, (32, 32), 4)
    obs[1] = -1
    obs[2, 20:] = -1
    obs[3, 7, 0] = 32
    obs[5, 0, 1] = 77
    obs[8, ::2, 1] = -1
    check_vs_oracle(m, obs, ov, [m.variable("C1")])


def test_fb_ckw_is_the_config3_default_and_rows_sum_to_one():
    m = nip_amd.Model.from_spec(*synth.demo1_spec(32))
    ov = [m.variable("A1"), m.variable("B1")]
    obs = torch.from_numpy(synth.observations(1000, 64, 32, seed=2, n_obs=2)).cuda()
    post, ll, st = nip_amd.forward_backward_inference(m, obs, ov, [m.variable("C1")])
    torch.cuda.synchronize()
    assert nip_amd.last_kernel() == FBCK, nip_amd.last_kernel()
    assert not st.any().item()
    s = post.sum(dim=2)
    assert float((s - 1.0).abs().max()) <= 1e-12


def test_fb_ckw_matches_the_mfma_wide_kernel():
    """The same request on chain_mfma_wide_kernel (NIPAMD_FB_WIDE_KERNEL=mw on
    the diagnostics build, in a child process): posteriors 1e-12, ll 1e-11."""
    from nip_amd import build as nb
    code = (
        "import sys, numpy as np, torch, nip_amd\n"
        "from nip_amd import synth\n"
        "m = nip_amd.Model.from_spec(*synth.demo1_spec(32, seed=5))\n"
        "o = synth.observations(4096, 64, 32, seed=8, n_obs=2)\n"
        "o[5, 10:20, 0] = -1\n"
        "obs = torch.from_numpy(o).cuda()\n"
        "p, l, s = nip_amd.forward_backward_inference(m, obs, [m.variable('A1'), m.variable('B1')], [m.variable('C1')])\n"
        "torch.cuda.synchronize()\n"
        "np.savez(sys.argv[1], p=p.cpu().numpy(), l=l.cpu().numpy(), k=nip_amd.last_kernel())\n")
    outs = []
    for env in ({}, {"NIPAMD_FB_WIDE_KERNEL": "mw", "NIPAMD_LIB": nb.DIAG_LIB}):
        path = os.path.join(os.environ.get("TMPDIR", "/tmp"), "fbckw_%d.npz" % len(outs))
        r = subprocess.run([sys.executable, "-c", code, path], env=dict(os.environ, **env), timeout=300)
        assert r.returncode == 0
        outs.append(np.load(path))
    assert str(outs[0]["k"]) == FBCK and str(outs[1]["k"]).startswith("chain_mfma_wide_kernel")
    assert np.abs(outs[0]["p"] - outs[1]["p"]).max() <= 1e-12
    assert np.all(np.abs(outs[0]["l"] - outs[1]["l"]) <= 1e-11 * np.maximum(1.0, np.abs(outs[1]["l"])))


def test_fb_ckw_several_queries_vs_oracle():
    """The interface and two derived variables in one request: the interface
    rows land inside wider posterior rows (the kernel's strided store path)."""
    m = demo1(32, 13, False)
    ov = [m.variable("A1"), m.variable("B1")]
    obs = gappy(7, 22, (32, 32), 19)
    check_vs_oracle(m, obs, ov, [m.variable("C1"), m.variable("A1"), m.variable("D1")], kernel="")


def test_fb_ckw_interface_not_first_in_the_query():
    """The interface variable after another one: its rows start at an offset."""
    m = demo1(24, 5, True)
    ov = [m.variable("B1")]
    obs = gappy(5, 17, (24,), 23)
    check_vs_oracle(m, obs, ov, [m.variable("D1"), m.variable("C1")], kernel="")
