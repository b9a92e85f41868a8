"""Shared check of an em_learn run against the reference's recorded one
(tests/golden/*.npz: em_init, em_iters, em_curve)."""
import numpy as np

from nip_amd.em import NIP_NO_ERROR, NIP_ERROR_BAD_LUCK


def close(a, b, rtol):
    return np.all(np.abs(a - b) <= rtol * np.maximum(1.0, np.abs(b)))


def check_em_curve(z, rc, curve, rtol):
    """Our em_learn against the reference's recorded run.  Without leading
    missing runs: the same curve and the same stop.  With them, the
    reference's BAD_LUCK verdict on a run (a running ll of pure rounding
    turning > 0, nip.c:1838) depends on the last bits of the tables; a single
    e_step reproduces it exactly (same tables), but after an m_step our
    tables differ from the reference's by rounding (counts summed in another
    order), and 1-ulp changes flip the verdict about half the time
    (DESIGN.md 6).  Then the curves must agree as far as both go, and the run
    that stopped first must have stopped with BAD_LUCK."""
    it = int(z["em_iters"])
    ref_curve = z["em_curve"]
    n = it if it >= 0 else int(np.argmax(np.append(ref_curve, 0.0) == 0.0))
    k = min(n, len(curve))
    assert close(np.array(curve[:k]), ref_curve[:k], rtol)
    lead = bool((z["obs"][:, 0] < 0).all(axis=1).any())
    if not lead or len(curve) == n:
        assert len(curve) == n
        assert rc == (NIP_NO_ERROR if it >= 0 else NIP_ERROR_BAD_LUCK)
    elif len(curve) < n:
        assert rc == NIP_ERROR_BAD_LUCK
    else:
        assert it < 0
