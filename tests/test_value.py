"""Algorithm 1 with the value-function branches of acceldualgrad.m:73,76 (the QP Hessian bound
with gpad_setup_hessian).  The reference never runs its termination test (commented out,
acceldualgrad.m:66-79), so the pin is a literal fp64 numpy restatement of that commented test
(tests/matlab_ref.py acceldualgrad_alg1); the oracle's value branches (oracle/gpad_oracle.c
orc_value_branch_*) must reproduce its decisions, and the stream kernel the oracle's, bit for bit
in f32 (iteration counts and termination codes included).

Problems: strictly feasible instances pushed away from the origin (constraints active at an
optimum with a positive objective value), where the relative-gap branch (:73) and the
value-dual branch (:76) decide a share of the instances.
"""
from __future__ import annotations

import numpy as np
import pytest

from matlab_ref import acceldualgrad_alg1


def value_problem(n, m, seed, shift=1.0, qs=0.1, batch=None):
    """H = R'R + I, G ~ N(0, 1/n); b = G z_f + U(0.1, 1), z_f ~ U(shift, shift + 1); q ~ N(0, qs).
    batch: shared H, G (seed) with per-instance z_f, q (seed + 1 + i)."""
    rng = np.random.default_rng(seed)
    R = rng.normal(0, 1 / np.sqrt(n), (n, n))
    H = R.T @ R + np.eye(n)
    G = rng.normal(0, 1 / np.sqrt(n), (m, n))
    Hi = np.linalg.inv(H)
    ML = Hi @ G.T
    L = float(np.linalg.norm(G @ ML, "fro"))

    def draw(r):
        zf = r.uniform(shift, shift + 1, n)
        return r.normal(0, qs, n), G @ zf + r.uniform(0.1, 1.0, m)
    if batch is None:
        q, g = draw(rng)
        return H, ML, Hi @ q, G, g, L, q
    Q = np.empty((batch, n))
    Gv = np.empty((batch, m))
    for i in range(batch):
        Q[i], Gv[i] = draw(np.random.default_rng(seed + 1 + i))
    return H, ML, Q @ Hi.T, G, Gv, L, Q


CASES = [(1.0, 1e-2, 1e-1, 1), (1.0, 1e-3, 1e-2, 1), (3.0, 1e-3, 1e-2, 10), (3.0, 1e-2, 1e-1, 1)]


@pytest.mark.parametrize("shift,tol,tol_gap,K", CASES)
def test_oracle_value_branches_match_literal_matlab(oracle, shift, tol, tol_gap, K):
    """fp64 oracle vs the literal restatement of the commented MATLAB test: same stopping
    iteration and branch on 24 instances; the branches :73 and :76 both occur in the sweep."""
    codes = []
    for seed in range(24):
        H, ML, M, G, g, L, q = value_problem(20, 40, seed, shift)
        z, y, it, c = oracle.solve_value_f64(np.zeros(20), np.zeros(40), ML, M, G, g, H, 5000, L, tol,
                                             check_every=K, tol_gap=tol_gap)
        zr, yr, itr, cr = acceldualgrad_alg1(H, q, G, g, L, tol, tol_gap, 5000, check_every=K)
        assert (it, c) == (itr, cr), (seed, it, c, itr, cr)
        np.testing.assert_allclose(z, zr, rtol=1e-9, atol=1e-12)
        codes.append(c)
    assert set(codes) <= {1, 2, 3, 4}
    TestCoverage.seen.update(codes)


class TestCoverage:
    seen: set = set()

    def test_both_value_branches_exercised(self, oracle):
        if not self.seen:  # run standalone: sweep here
            for case in CASES:
                test_oracle_value_branches_match_literal_matlab(oracle, *case)
        assert {3, 4} <= self.seen, self.seen


def test_oracle_value_f32_without_hessian_is_plain(oracle):
    """With H unbound the f32 value entry is orc_solve_f32 (codes 0..2)."""
    H, ML, M, G, g, L, _ = value_problem(20, 40, 3, 3.0)
    f = lambda a: np.asarray(a, np.float64).astype(np.float32)  # noqa: E731
    z1, y1, it1, c1 = oracle.solve_f32(np.zeros(20), np.zeros(40), f(ML), f(M), f(G), f(g), 5000, np.float32(L),
                                       1e-3, tol_gap=1e-2)
    z2, y2, it2, c2 = oracle.solve_value_f32(np.zeros(20), np.zeros(40), f(ML), f(M), f(G), f(g), f(H), 5000,
                                             np.float32(L), 1e-3, tol_gap=1e-2)
    assert it2 <= it1  # the value branches can only stop earlier
    if c2 <= 2:
        assert it1 == it2 and np.array_equal(z1, z2) and np.array_equal(y1, y2)


def _gpu_batch(n, m, B, seed, shift, dtype, shared=True):
    H, ML, M, G, g, L, Q = value_problem(n, m, seed, shift, batch=B)
    if not shared:  # per-instance copies of the matrices (the distinct-matrix layout)
        H = np.broadcast_to(H, (B, n, n)).copy()
        ML = np.broadcast_to(ML, (B, n, m)).copy()
        G = np.broadcast_to(G, (B, m, n)).copy()
    c = lambda a: np.ascontiguousarray(np.asarray(a, np.float64).astype(dtype))  # noqa: E731
    return c(H), c(ML), c(M), c(G), c(g), L


@pytest.mark.gpu
@pytest.mark.parametrize("shift,tol,tol_gap,K", CASES)
@pytest.mark.parametrize("shared", [True, False])
def test_gpu_value_branches_bitexact_f32(gpu, oracle, shift, tol, tol_gap, K, shared):
    """Stream kernel (f32) with H bound: every instance bit-exact vs the oracle, z, y, iteration
    count and termination code."""
    import gpad_mpc
    n, m, B = 20, 40, 64
    H, ML, M, G, g, L = _gpu_batch(n, m, B, 7, shift, np.float32, shared)
    L32 = np.float32(L)
    z = np.zeros((B, n), np.float32)
    y = np.zeros((B, m), np.float32)
    it = np.zeros(B, np.int32)
    codes = np.zeros(B, np.int32)
    with gpad_mpc.GpadSolver(0) as s:
        s.setup(ML, G, float(L32), n=n, m=m, batch=B, shared=shared, check_every=K, tol_gap=tol_gap)
        s.setup_hessian(H)
        st = s.run(z, y, M, g, 5000, tol, iters=it, codes=codes)
    assert st["kernel"] == "stream"
    for b in range(B):
        Hb, MLb, Gb = (H, ML, G) if shared else (H[b], ML[b], G[b])
        zo, yo, ito, co = oracle.solve_value_f32(np.zeros(n), np.zeros(m), MLb, M[b], Gb, g[b], Hb, 5000, L32, tol,
                                                 check_every=K, tol_gap=tol_gap)
        assert (it[b], codes[b]) == (ito, co), b
        np.testing.assert_array_equal(z[b], zo, err_msg=f"z[{b}]")
        np.testing.assert_array_equal(y[b], yo, err_msg=f"y[{b}]")


@pytest.mark.gpu
def test_gpu_value_branches_f64_and_certified(gpu, oracle):
    """f64 stream kernel with H bound (the reference's own e_g = e_V = 1e-6 regime needs f64):
    iteration counts and codes equal the fp64 oracle's, z within 1e-12; every instance stopped by
    :76 satisfies V(z*) - D(y*) <= e_V max(D(y*), 1) re-evaluated in numpy fp64 on the returned
    point with the exact H and f = H M."""
    import gpad_mpc
    n, m, B = 20, 40, 64
    shift, tol, tol_gap, K = 1.0, 1e-2, 1e-1, 1
    H, ML, M, G, g, L = _gpu_batch(n, m, B, 7, shift, np.float64)
    z = np.zeros((B, n))
    y = np.zeros((B, m))
    it = np.zeros(B, np.int32)
    codes = np.zeros(B, np.int32)
    with gpad_mpc.GpadSolver(0) as s:
        s.setup(ML, G, L, n=n, m=m, batch=B, check_every=K, tol_gap=tol_gap)
        s.setup_hessian(H)
        s.run(z, y, M, g, 5000, tol, iters=it, codes=codes)
    assert {3, 4} & set(codes.tolist()), codes
    Hi = np.linalg.inv(H)
    for b in range(B):
        zo, yo, ito, co = oracle.solve_value_f64(np.zeros(n), np.zeros(m), ML, M[b], G, g[b], H, 5000, L, tol,
                                                 check_every=K, tol_gap=tol_gap)
        assert (it[b], codes[b]) == (ito, co), b
        np.testing.assert_allclose(z[b], zo, rtol=1e-12, atol=1e-14)
        if codes[b] == 4:
            f = H @ M[b]
            V = (0.5 * z[b] @ H + f) @ z[b]
            zy = -Hi @ (f + G.T @ y[b])
            D = (0.5 * zy @ H + f + y[b] @ G) @ zy - y[b] @ g[b]
            # y* is y_{v+1}, the point the test's dualfcn was evaluated at
            assert V - D <= tol_gap * max(D, 1.0) * (1 + 1e-9), (b, V, D)


@pytest.mark.gpu
def test_gpu_value_needs_stream_kernel(gpu):
    import gpad_mpc
    from gpad_mpc import _lib
    H, ML, M, G, g, L = _gpu_batch(20, 40, 4, 1, 1.0, np.float32)
    with gpad_mpc.GpadSolver(0) as s:
        s.setup(ML, G, L, n=20, m=40, batch=4, kernel=_lib.KERNEL_RESIDENT)
        s.setup_hessian(H)
        with pytest.raises(_lib.GpadError) as ei:
            s.run(np.zeros((4, 20), np.float32), np.zeros((4, 40), np.float32), M, g, 100, 1e-3)
        assert ei.value.code == _lib.ERR_UNSUPPORTED
        s.setup_hessian(None)  # unbound: the resident kernel runs again
        st = s.run(np.zeros((4, 20), np.float32), np.zeros((4, 40), np.float32), M, g, 100, 1e-3)
        assert st["kernel"] == "resident"
