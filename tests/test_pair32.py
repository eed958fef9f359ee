"""The W32 pair layout (csrc/gpad_pair32.hip): the C3/C4 shape n = m = 200 in pair phases on
v_mfma_f32_32x32x2_f32 chains (32 instances per chain) with the rows 192..199 on a 16x16x4 chain
per panel and one chain hand-off per SIMD pair.  It must give exactly what the 16x16x4 pair kernel
gives (GPAD_OPT_PAIR32 = 0) -- z, y, iteration counts, termination codes -- which the rest of the
suite pins to the oracle (tests/test_configs.py runs the C3 / C4 sizes through it by default).
"""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _shard(B, seed=0):
    import bench
    ML, G, L, M, g = bench.make_shard(200, 200, B, seed)
    f = lambda a: np.ascontiguousarray(a, np.float32)  # noqa: E731
    return f(ML), f(G), float(np.float32(L)), f(M), f(g)


def _solve(ML, G, L, M, g, N, tol, pair32, *, z0=None, reps=1, K=10):
    import torch

    import gpad_mpc
    B = M.shape[0]
    t = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
    it = np.zeros(B, np.int32)
    codes = np.zeros(B, np.int32)
    with gpad_mpc.GpadSolver(0) as s:
        s.setup(t(ML), t(G), L, n=200, m=200, batch=B, check_every=K)
        s.set_option("pair32", pair32)
        for _ in range(reps):  # later solves follow the plan made from the previous counts
            z = t(z0.copy()) if z0 is not None else torch.zeros(B, 200, device="cuda")
            y = torch.zeros(B, 200, device="cuda")
            st = s.run(z, y, t(M), t(g), N, tol, iters=it, codes=codes)
    return z.cpu().numpy(), y.cpu().numpy(), it.copy(), codes.copy(), st


@pytest.mark.parametrize("B", [8192, 4400, 4401, 8200])
def test_pair32_fixed_n_equals_16x16(gpu, B):
    """Fixed N = 37 (one phase, no test): every instance bit-exact with the 16x16x4 pairs (odd panel
    counts leave the last pair with one panel; 4401 and 8200 end in a partial panel)."""
    ML, G, L, M, g = _shard(B)
    a = _solve(ML, G, L, M, g, 37, 0.0, 1)
    b = _solve(ML, G, L, M, g, 37, 0.0, 0)
    assert a[4]["kernel"] == "panel"
    for x, y_ in zip(a[:4], b[:4]):
        np.testing.assert_array_equal(x, y_)


@pytest.mark.parametrize("B,K", [(8192, 10), (5000, 10), (8192, 1)])
def test_pair32_eps_equals_16x16(gpu, B, K):
    """Algorithm 1 to eps = 1e-4, planned (the second solve follows the first one's counts): phases
    on both layouts, the finisher, every test and verification -- z, y, counts, codes bit-exact."""
    ML, G, L, M, g = _shard(B, seed=3)
    a = _solve(ML, G, L, M, g, 5000, 1e-4, 1, reps=2, K=K)
    b = _solve(ML, G, L, M, g, 5000, 1e-4, 0, reps=2, K=K)
    assert a[4]["converged"] == B
    for x, y_ in zip(a[:4], b[:4]):
        np.testing.assert_array_equal(x, y_)


def test_pair32_warm_start_seed_gemm(gpu, oracle):
    """A non-zero z_{-1} (warm start): the u = G_L z_{-1} seed GEMM on the W32 layout, eps mode,
    bit-exact with the 16x16x4 pairs and, for a sample, with the oracle."""
    B = 8192
    ML, G, L, M, g = _shard(B, seed=5)
    rng = np.random.default_rng(0)
    z0 = (0.05 * rng.standard_normal((B, 200))).astype(np.float32)
    a = _solve(ML, G, L, M, g, 5000, 1e-4, 1, z0=z0)
    b = _solve(ML, G, L, M, g, 5000, 1e-4, 0, z0=z0)
    for x, y_ in zip(a[:4], b[:4]):
        np.testing.assert_array_equal(x, y_)
    for k in (0, 4097, B - 1):
        zo, yo, ito, _ = oracle.solve_f32(z0[k], np.zeros(200), ML, M[k], G, g[k], 5000, np.float32(L), 1e-4)
        assert a[2][k] == ito
        np.testing.assert_array_equal(a[0][k], zo)
        np.testing.assert_array_equal(a[1][k], yo)
