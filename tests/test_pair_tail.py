"""Panel pairs on the TailPair layout (csrc/gpad_panel.hip, GPAD_OPT_PAIR_TAIL): for 192 < n, m <= 200
the last 8 rows of both panels of a pair run as one v_mfma_f32_4x4x1_16b_f32 chain (a relay of four
pieces over the SIMDs) instead of two half-padding 16x16x4 tiles.

Pins: the sixteen-row pair layout (option 0) on the same inputs, bit for bit (z, y, iteration counts,
codes) -- fixed N and to eps (phases, parks, tests, the (A) verification chains), cold and warm
starts (the seed chain u = G_L z_{-1}), KQ = 2 (n = m = 200, 197 with padding rows) and KQ = 1
(n = m = 196, 193) -- and the oracle on a sample of instances.
"""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _solve(qp, B, N, tol, tail, z0=None, plan_twice=False):
    import torch

    import gpad_mpc
    n, m = qp.ML.shape
    dev = torch.device("cuda:0")
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(dev)  # noqa: E731
    M = t(np.asarray(qp.M).reshape(B, n))
    g = t(np.asarray(qp.g).reshape(B, m))
    it = np.zeros(B, np.int32)
    codes = np.zeros(B, np.int32)
    with gpad_mpc.GpadSolver(0) as s:
        s.setup(t(qp.ML), t(qp.G), float(np.float32(qp.L)), n=n, m=m, batch=B, check_every=10)
        s.set_options(pair_tail=int(tail))
        for _ in range(2 if plan_twice else 1):
            z = t(z0) if z0 is not None else torch.zeros(B, n, device=dev)
            y = torch.zeros(B, m, device=dev)
            st = s.run(z, y, M, g, N, tol, iters=it, codes=codes)
    return z.cpu().numpy(), y.cpu().numpy(), it.copy(), codes.copy(), st


@pytest.mark.parametrize("nm", [200, 197, 196, 193])
def test_tail_layout_fixed_n_bitexact(gpu, nm):
    """Fixed N = 60 over 8192 instances (256 pairs: the pair layout on every CU): equal to the
    sixteen-row layout bit for bit."""
    from gpad_mpc import problems
    B = 8192
    qp = problems.synthetic_qp(nm, nm, batch=B, seed=nm)
    a = _solve(qp, B, 60, 0.0, True)
    b = _solve(qp, B, 60, 0.0, False)
    assert a[4]["kernel"] == "panel"
    np.testing.assert_array_equal(a[0], b[0])
    np.testing.assert_array_equal(a[1], b[1])


@pytest.mark.parametrize("nm,warm", [(200, False), (200, True), (197, False), (196, True)])
def test_tail_layout_eps_bitexact(gpu, oracle, nm, warm):
    """To eps = 1e-4 with the phase plan of a previous solve (pairs -> single panels -> finisher):
    counts, codes, z and y equal the sixteen-row layout's; a warm start (non-zero z_{-1}) runs
    the seed chain; a sample equals the oracle."""
    from gpad_mpc import problems
    B = 8192
    qp = problems.synthetic_qp(nm, nm, batch=B, seed=3 * nm + warm)
    z0 = None
    if warm:
        rng = np.random.default_rng(nm)
        z0 = (0.01 * rng.standard_normal((B, nm))).astype(np.float32)
    a = _solve(qp, B, 5000, 1e-4, True, z0=z0, plan_twice=True)
    b = _solve(qp, B, 5000, 1e-4, False, z0=z0, plan_twice=True)
    np.testing.assert_array_equal(a[2], b[2])
    np.testing.assert_array_equal(a[3], b[3])
    np.testing.assert_array_equal(a[0], b[0])
    np.testing.assert_array_equal(a[1], b[1])
    assert (a[3] > 0).all()
    n = m = nm
    M = np.asarray(qp.M).reshape(B, n)
    g = np.asarray(qp.g).reshape(B, m)
    for i in [0, 4097, 8191, int(np.argmax(a[2]))]:
        zi = np.zeros(n, np.float32) if z0 is None else z0[i]
        zo, yo, ito, co = oracle.solve_f32(zi, np.zeros(m), np.asarray(qp.ML), M[i], np.asarray(qp.G), g[i], 5000,
                                           np.float32(qp.L), 1e-4)
        assert (a[2][i], a[3][i]) == (ito, co), i
        np.testing.assert_array_equal(a[0][i], zo)
