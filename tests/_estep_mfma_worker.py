"""Worker for tests/test_gpu_estep.py::test_estep_mfma_kernel_in_diagnostics_build:
the matrix-core e_step (NIPAMD_ESTEP_KERNEL=mfma, read per call by the
diagnostics build, NIPAMD_LIB=nip_amd/_lib/diag/libnip_amd_diag.so) against
the oracle and against the default DPP kernel.  Exit code 0 = every check passed.

    NIPAMD_LIB=.../libnip_amd_diag.so python tests/_estep_mfma_worker.py
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

CNT_RTOL = 1e-11
LL_RTOL = 1e-12


def close(a, b, rtol):
    return np.all(np.abs(a - b) <= rtol * np.maximum(1.0, np.abs(b)))


def gpu_estep(model, obs, obs_vars):
    o = torch.from_numpy(np.ascontiguousarray(obs, np.int32)).cuda()
    cnt, ll, st = nip_amd.e_step(model, o, obs_vars)
    torch.cuda.synchronize()
    return cnt.cpu().numpy(), ll.cpu().numpy(), st.cpu().numpy()


def mfma(on):
    if on:
        os.environ["NIPAMD_ESTEP_KERNEL"] = "mfma"
    else:
        os.environ.pop("NIPAMD_ESTEP_KERNEL", None)


def vs_oracle(N, M, B, T):
    mfma(True)
    m = nip_amd.Model.from_spec(*synth.hmm_spec(N, M, seed=N * 7 + M))
    obs = synth.observations(B, T, M, seed=B + T)
    obs[obs.shape[0] // 2, ::3] = -1                  # some missing values
    ov = [m.variable("M1")]
    cnt, ll, st = gpu_estep(m, obs, ov)
    assert nip_amd.last_kernel() == "chain_fb_mfma_kernel<estep>", nip_amd.last_kernel()
    rc, rl, rb = PortOracle(m.desc()).estep(obs, ov, np.ones(m.param_size()))
    assert np.array_equal(st != 0, rb != 0)        # incl. the leading-missing-run verdict
    ok = rb == 0
    assert close(ll[ok], rl[ok], LL_RTOL)
    if ok.all():
        assert close(cnt, rc, CNT_RTOL), np.abs(cnt - rc).max()
    mfma(False)
    cnt2, ll2, _ = gpu_estep(m, obs, ov)
    assert nip_amd.last_kernel() in ("chain_estep16_kernel", "chain_estep_ck_kernel"), nip_amd.last_kernel()
    assert close(cnt, cnt2, CNT_RTOL)
    assert close(ll, ll2, LL_RTOL)
    os.environ["NIPAMD_ESTEP_KERNEL"] = "dpp8"         # the round-2 DPP kernel
    cnt3, ll3, st3 = gpu_estep(m, obs, ov)
    assert nip_amd.last_kernel() == "chain_kernel<true>", nip_amd.last_kernel()
    os.environ.pop("NIPAMD_ESTEP_KERNEL", None)
    assert np.array_equal(st3 != 0, rb != 0)
    assert close(cnt, cnt3, CNT_RTOL)
    assert close(ll, ll3, LL_RTOL)


def missing_and_bad_luck():
    mfma(True)
    m = nip_amd.Model.from_spec(*synth.hmm_spec(16, 16, seed=5))
    rng = np.random.default_rng(3)
    obs = rng.integers(0, 16, size=(20, 30, 1)).astype(np.int32)
    obs[0] = -1                                    # fully missing: ll exactly 0
    obs[2, 7, 0] = 16                              # out of range -> BAD_LUCK
    ov = [m.variable("M1")]
    cnt, ll, st = gpu_estep(m, obs, ov)
    assert ll[0] == 0.0
    _, rl, rb = PortOracle(m.desc()).estep(obs, ov, np.ones(m.param_size()))
    assert (st[2] & nip_amd.STATUS_BAD_LUCK) != 0 and rb[2] != 0
    assert np.array_equal(st != 0, rb != 0)
    good = rb == 0                                 # the sequences the reference accepts
    assert good.sum() >= 17
    cg, _, sg = gpu_estep(m, obs[good], ov)
    rcg, _, _ = PortOracle(m.desc()).estep(obs[good], ov, np.ones(m.param_size()))
    assert not sg.any()
    assert close(cg, rcg, CNT_RTOL), np.abs(cg - rcg).max()


def shard_invariant():
    """Block rows combine like sequence rows: 4 x 64 shards == 256, bit for bit."""
    mfma(True)
    m = nip_amd.Model.from_spec(*synth.hmm_spec(16, 16))
    obs = torch.from_numpy(synth.observations(256, 48, 16, seed=8)).cuda().contiguous()
    ov = [m.variable("M1")]
    whole, _, _ = nip_amd.estep_partial(m, obs, ov)
    whole = whole.clone()
    parts = []
    for k in range(4):
        p, _, _ = nip_amd.estep_partial(m, obs[k * 64:(k + 1) * 64].contiguous(), ov)
        parts.append(p.clone())
    assert torch.equal(tree_sum(torch.stack(parts))[:-3], whole[:-3])


def main():
    cases = [(16, 16, 16, 64), (16, 16, 9, 37), (16, 16, 33, 1), (16, 16, 17, 2), (4, 5, 21, 33),
             (7, 3, 40, 17), (16, 8, 70, 40)]
    for c in cases:
        vs_oracle(*c)
        print("vs_oracle", c, "ok", flush=True)
    missing_and_bad_luck()
    print("missing_and_bad_luck ok", flush=True)
    shard_invariant()
    print("shard_invariant ok", flush=True)
    print("all passed")


if __name__ == "__main__":
    main()
