"""One-time QP precompute on the device (acceldualgrad.m:11,20-21):
gpad_precompute computes L = ||H||_F^2, ML = inv(H) A', gP = inv(H) f' in fp64 by Gauss-Jordan
elimination on [H | A' | f'].  The reference forms inv(H) explicitly (MATLAB), so the two agree
to fp64 round-off, not bit for bit: the tolerances below are stated per quantity.  Downstream,
a GPAD solve on the device-precomputed data matches the oracle on the host-precomputed data to
the north-star 1e-6 relative."""
from __future__ import annotations

import numpy as np
import pytest


def _spd(n, rng):
    R = rng.standard_normal((n, n)) / np.sqrt(n)
    return R.T @ R + np.eye(n)


def _rel(a, b):
    return float(np.abs(np.asarray(a) - np.asarray(b)).max() / max(np.abs(np.asarray(b)).max(), 1e-300))


@pytest.mark.gpu
@pytest.mark.parametrize("n,m,batch", [(40, 180, 5), (200, 200, 3), (7, 30, 1), (120, 64, 2300)])
def test_precompute_shared_vs_numpy(gpu, n, m, batch):
    """LTI: one H, one A, a batch of f rows (2300 rows: two elimination chunks)."""
    import gpad_mpc
    rng = np.random.default_rng(n + m)
    H, A, f = _spd(n, rng), rng.standard_normal((m, n)), rng.standard_normal((batch, n))
    s = gpad_mpc.GpadSolver(0)
    ML, gP, L = s.precompute(H, A, f)
    Hi = np.linalg.inv(H)
    assert _rel(ML, Hi @ A.T) < 1e-11
    assert _rel(gP, (Hi @ f.T).T) < 1e-11
    assert abs(L - np.linalg.norm(H, "fro") ** 2) <= 1e-13 * L
    ML2, gP2, L2 = s.precompute(H, A)  # no f: ML and L only
    assert gP2 is None and L2 == L
    np.testing.assert_array_equal(ML2, ML)


@pytest.mark.gpu
def test_precompute_per_instance_and_device_memory(gpu):
    """Distinct H, A per instance (LTV / the C5 shape family), host and torch-device operands."""
    import torch

    import gpad_mpc
    rng = np.random.default_rng(3)
    B, n, m = 6, 64, 96
    H = np.stack([_spd(n, rng) for _ in range(B)])
    A = rng.standard_normal((B, m, n))
    f = rng.standard_normal((B, n))
    s = gpad_mpc.GpadSolver(0)
    ML, gP, L = s.precompute(H, A, f, shared=False)
    t = lambda a: torch.from_numpy(a).to(gpu)  # noqa: E731
    MLd, gPd, Ld = s.precompute(t(H), t(A), t(f), shared=False)
    for b in range(B):
        Hi = np.linalg.inv(H[b])
        assert _rel(ML[b], Hi @ A[b].T) < 1e-11, b
        assert _rel(gP[b], Hi @ f[b]) < 1e-11, b
        assert abs(L[b] - np.linalg.norm(H[b], "fro") ** 2) <= 1e-13 * L[b]
    np.testing.assert_array_equal(MLd.cpu().numpy(), ML)
    np.testing.assert_array_equal(gPd.cpu().numpy(), gP)
    np.testing.assert_array_equal(Ld.cpu().numpy(), L)


@pytest.mark.gpu
def test_precompute_feeds_gpad_battery(gpu, oracle):
    """C1 battery QP (gpad.m construction): device precompute -> gpad_setup/gpad_run, 100
    iterations, vs the oracle on the host (numpy) precompute: within 1e-6 relative."""
    import gpad_mpc
    from gpad_mpc import problems
    qp = problems.battery_mpc(4, 10, seed=0)
    s = gpad_mpc.GpadSolver(0)
    ML, gP, L = s.precompute(qp.H, qp.G, qp.q[None, :])
    assert _rel(ML, qp.ML) < 1e-12 and _rel(gP[0], qp.M) < 1e-12 and abs(L - qp.L) <= 1e-13 * qp.L
    f32 = lambda a: np.ascontiguousarray(np.asarray(a, np.float64).astype(np.float32))  # noqa: E731
    s.setup(f32(ML), f32(qp.G), float(np.float32(L)), n=qp.n, m=qp.m, batch=1)
    z = np.zeros(qp.n, np.float32)
    y = np.zeros(qp.m, np.float32)
    s.run(z, y, f32(gP[0]), f32(qp.g), 100, 0.0)
    zo, yo, _, _ = oracle.solve_f32(np.zeros(qp.n), np.zeros(qp.m), f32(qp.ML), f32(qp.M), f32(qp.G), f32(qp.g),
                                    100, np.float32(qp.L))
    assert _rel(z, zo) < 1e-6 and _rel(y, yo) < 1e-6


@pytest.mark.gpu
@pytest.mark.parametrize("shared", [True, False])
def test_precompute_c5_size_800(gpu, shared):
    """BASELINE C5's shape (N = 200: n = 800, m = 800): the device Gauss-Jordan at the size
    DESIGN.md times, shared (one H, a batch of f rows) and per-instance (3 distinct H, A)."""
    import gpad_mpc
    rng = np.random.default_rng(800)
    n = m = 800
    s = gpad_mpc.GpadSolver(0)
    if shared:
        H, A, f = _spd(n, rng), rng.standard_normal((m, n)), rng.standard_normal((4, n))
        ML, gP, L = s.precompute(H, A, f)
        Hi = np.linalg.inv(H)
        assert _rel(ML, Hi @ A.T) < 1e-10
        assert _rel(gP, (Hi @ f.T).T) < 1e-10
        assert abs(L - np.linalg.norm(H, "fro") ** 2) <= 1e-12 * L
    else:
        B = 3
        H = np.stack([_spd(n, rng) for _ in range(B)])
        A = rng.standard_normal((B, m, n))
        f = rng.standard_normal((B, n))
        ML, gP, L = s.precompute(H, A, f, shared=False)
        for b in range(B):
            Hi = np.linalg.inv(H[b])
            assert _rel(ML[b], Hi @ A[b].T) < 1e-10, b
            assert _rel(gP[b], Hi @ f[b]) < 1e-10, b
            assert abs(L[b] - np.linalg.norm(H[b], "fro") ** 2) <= 1e-12 * L[b]
