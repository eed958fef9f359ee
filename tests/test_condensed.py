"""GPAD_KERNEL_CONDENSED: the opt-in latency kernel on the condensed operator (one m-long chain
per iteration: G_L zhat = H w + c, z = -ML wbar - gP; csrc/gpad_condensed.hip, include/gpad.h).

It is NOT the reference's arithmetic, so parity is two-layered:
  * the HIP kernel is BIT-EXACT against its own restatement, oracle/gpad_oracle.c
    orc_solve_condensed_f32 (same chains, same order) -- the -m gpu tests;
  * that restatement is compared with the reference's fp32 path (orc_solve_f32, pinned to
    seq_functions.cpp) on the CPU: norm-wise relative distance of z and y at most
    max(1e-6, the reference's own fp32-vs-fp64 spread on the same problem), i.e. the condensed
    solve is no further from the reference C++ than the reference C++ is from its MATLAB (fp64)
    path; and to eps it stops at the same iteration with the constraint certified in fp64.
"""
from __future__ import annotations

import numpy as np
import pytest

from test_gpu_parity import assert_bitexact


def _f32(a):
    return np.ascontiguousarray(np.asarray(a, np.float64).astype(np.float32))


def _cases():
    from gpad_mpc import problems
    return {"C2": problems.synthetic_qp(200, 200, seed=11), "C1": problems.battery_mpc(4, 10, seed=0)}


def _inputs(qp):
    ML, G = _f32(qp.ML), _f32(qp.G)
    M, g = _f32(qp.M).reshape(-1, ML.shape[0]), _f32(qp.g).reshape(-1, ML.shape[1])
    return ML, G, M, g, np.float32(qp.L)


def _rel(a, b):
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(np.asarray(a, np.float64) - b) / max(np.linalg.norm(b), 1e-300))


# ---- CPU: the restatement against the reference ----------------------------------------

def test_condense_matches_fp64_product(oracle):
    from gpad_mpc import problems
    qp = problems.synthetic_qp(40, 56, seed=3)
    MGneg, GL, _ = oracle.scale(_f32(qp.ML), _f32(qp.G), _f32(qp.g), np.float32(qp.L))
    H = oracle.condense(GL, MGneg)
    ref = GL.astype(np.float64) @ MGneg.astype(np.float64)
    np.testing.assert_allclose(H, ref.astype(np.float32), rtol=2e-7, atol=1e-7 * np.abs(ref).max())


@pytest.mark.parametrize("name", ["C2", "C1"])
@pytest.mark.parametrize("N", [50, 100])
def test_condensed_within_reference_spread(oracle, name, N):
    """Fixed N: the condensed solve vs the reference's fp32 path, bounded by max(1e-6, the
    reference fp32 path's own distance from its fp64 restatement) -- measured C2/N=100:
    z 1.7e-7, y 4.4e-7 (< 1e-6); C1/N=100: z 3.9e-7, y 2.5e-6 against a spread of 2.7e-6."""
    qp = _cases()[name]
    ML, G, M, g, L = _inputs(qp)
    n, m = ML.shape
    zo, yo, _, _ = oracle.solve_f32(np.zeros(n), np.zeros(m), ML, M[0], G, g[0], N, L)
    zd, yd, _, _ = oracle.solve_f64(np.zeros(n), np.zeros(m), ML.astype(np.float64), M[0].astype(np.float64),
                                    G.astype(np.float64), g[0].astype(np.float64), N, float(L))
    zc, yc, it, _ = oracle.solve_condensed_f32(np.zeros(n), np.zeros(m), ML, M[0], G, g[0], N, L)
    assert it == N
    bz = max(1e-6, _rel(zo, zd))
    by = max(1e-6, _rel(yo, yd))
    assert _rel(zc, zo) <= bz, (_rel(zc, zo), bz)
    assert _rel(yc, yo) <= by, (_rel(yc, yo), by)


@pytest.mark.parametrize("name", ["C2", "C1"])
@pytest.mark.parametrize("tol", [1e-3, 1e-4])
def test_condensed_eps_mode_certified(oracle, name, tol):
    """To eps: same stopping iteration as the reference (within one check period), and the
    returned point satisfies fp64 max(G z - g) <= tol (decided on the direct G_L z)."""
    qp = _cases()[name]
    ML, G, M, g, L = _inputs(qp)
    n, m = ML.shape
    _, _, ito, _ = oracle.solve_f32(np.zeros(n), np.zeros(m), ML, M[0], G, g[0], 5000, L, tol)
    zc, _, itc, cc = oracle.solve_condensed_f32(np.zeros(n), np.zeros(m), ML, M[0], G, g[0], 5000, L, tol)
    assert cc in (1, 2) and abs(itc - ito) <= 10, (itc, ito)
    viol = (G.astype(np.float64) @ zc.astype(np.float64) - g[0].astype(np.float64)).max()
    assert viol <= tol, viol


def test_condensed_ignores_z0_as_the_reference_does(oracle):
    """theta_0 = 1: the reference's first 8c overwrites z0 (z_1 = zhat_1); the condensed form
    never reads it."""
    qp = _cases()["C1"]
    ML, G, M, g, L = _inputs(qp)
    n, m = ML.shape
    a = oracle.solve_condensed_f32(np.zeros(n), np.zeros(m), ML, M[0], G, g[0], 30, L)
    b = oracle.solve_condensed_f32(np.full(n, 7.0), np.zeros(m), ML, M[0], G, g[0], 30, L)
    assert_bitexact(a[0], b[0])
    zr0, _, _, _ = oracle.solve_f32(np.zeros(n), np.zeros(m), ML, M[0], G, g[0], 30, L)
    zr1, _, _, _ = oracle.solve_f32(np.full(n, 7.0), np.zeros(m), ML, M[0], G, g[0], 30, L)
    assert_bitexact(zr0, zr1)


# ---- GPU: the HIP kernel against the restatement, bit for bit ---------------------------

def run_condensed(ML, M, G, g, L, N, tol=0.0, y0=None, shared=True, tol_gap=0.0):
    import gpad_mpc
    from gpad_mpc import _lib
    n, m = ML.shape[-2], ML.shape[-1]
    B = M.shape[0]
    z = np.zeros((B, n), np.float32)
    y = np.zeros((B, m), np.float32) if y0 is None else np.array(y0, np.float32).reshape(B, m)
    it = np.zeros(B, np.int32)
    with gpad_mpc.GpadSolver(0) as s:
        s.setup(ML, G, float(L), n=n, m=m, batch=B, shared=shared, kernel=_lib.KERNEL_CONDENSED,
                tol_gap=tol_gap)
        st = s.run(z, y, M, g, N, tol, iters=it)
    assert st["kernel"] == "condensed"
    return z, y, it, st


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["C2", "C1"])
@pytest.mark.parametrize("N,tol", [(1, 0.0), (100, 0.0), (1000, 0.0), (5000, 1e-3), (5000, 1e-4)])
def test_condensed_kernel_bitexact(gpu, oracle, name, N, tol):
    qp = _cases()[name]
    ML, G, M, g, L = _inputs(qp)
    n, m = ML.shape
    z, y, it, st = run_condensed(ML, M, G, g, L, N, tol)
    zo, yo, ito, co = oracle.solve_condensed_f32(np.zeros(n), np.zeros(m), ML, M[0], G, g[0], N, L, tol)
    assert it[0] == ito and st["converged"] == int(co != 0)
    assert_bitexact(z[0], zo, "z")
    assert_bitexact(y[0], yo, "y")


@pytest.mark.gpu
@pytest.mark.parametrize("nm", [(37, 53), (1, 5), (5, 1), (200, 8), (8, 196), (256, 200), (131, 64), (64, 208)])
def test_condensed_shapes_bitexact(gpu, oracle, nm):
    from gpad_mpc import problems
    n, m = nm
    qp = problems.synthetic_qp(n, m, seed=19)
    ML, G, M, g, L = _inputs(qp)
    for N, tol in ((60, 0.0), (3000, 1e-4)):
        z, y, it, _ = run_condensed(ML, M, G, g, L, N, tol)
        zo, yo, ito, _ = oracle.solve_condensed_f32(np.zeros(n), np.zeros(m), ML, M[0], G, g[0], N, L, tol)
        assert it[0] == ito, (nm, N)
        assert_bitexact(z[0], zo, f"{nm} z")
        assert_bitexact(y[0], yo, f"{nm} y")


@pytest.mark.gpu
@pytest.mark.parametrize("shared", [True, False])
def test_condensed_batch_bitexact(gpu, oracle, shared):
    """Shared and distinct matrices, warm-started y, Algorithm 1 with a separate e_V."""
    from gpad_mpc import problems
    B, n, m = 23, 48, 72
    qp = problems.synthetic_qp(n, m, batch=B, seed=6, shared=shared)
    ML, G = _f32(qp.ML), _f32(qp.G)
    M, g, L = _f32(qp.M).reshape(B, n), _f32(qp.g).reshape(B, m), np.float32(qp.L)
    rng = np.random.default_rng(4)
    y0 = (0.05 * rng.random((B, m))).astype(np.float32)
    z, y, it, _ = run_condensed(ML, M, G, g, L, 3000, 1e-4, y0=y0, shared=shared, tol_gap=3e-4)
    for b in range(B):
        ml, gg = (ML, G) if shared else (ML[b], G[b])
        zo, yo, ito, _ = oracle.solve_condensed_f32(np.zeros(n), y0[b], ml, M[b], gg, g[b], 3000, L, 1e-4,
                                                    tol_gap=3e-4)
        assert it[b] == ito, b
        assert_bitexact(z[b], zo, f"{b} z")
        assert_bitexact(y[b], yo, f"{b} y")


@pytest.mark.gpu
def test_condensed_guards(gpu):
    """Unsupported shapes fail at setup; custom schedules must keep theta_0 = 1."""
    import gpad_mpc
    from gpad_mpc import _lib, problems
    qp = problems.synthetic_qp(40, 300, seed=1)
    ML, G, M, g, L = _inputs(qp)
    with gpad_mpc.GpadSolver(0) as s:
        with pytest.raises(gpad_mpc.GpadError):
            s.setup(ML, G, float(L), n=40, m=300, kernel=_lib.KERNEL_CONDENSED)
    qp = problems.synthetic_qp(40, 60, seed=1)
    ML, G, M, g, L = _inputs(qp)
    with gpad_mpc.GpadSolver(0) as s:
        s.setup(ML, G, float(L), n=40, m=60, kernel=_lib.KERNEL_CONDENSED)
        th, be = gpad_mpc.schedule(20)
        th = th.astype(np.float32)
        be = be.astype(np.float32)
        th[0] = np.float32(0.5)
        with pytest.raises(gpad_mpc.GpadError):
            s.run(np.zeros(40, np.float32), np.zeros(60, np.float32), M, g, 20, 0.0, scaled=True, theta=th,
                  beta=be)


@pytest.mark.gpu
@pytest.mark.parametrize("nm", [(200, 200), (40, 180), (37, 53), (64, 208), (130, 100), (1, 5), (224, 200)])
@pytest.mark.parametrize("N,tol", [(60, 0.0), (4000, 1e-4)])
def test_condensed_panel_batch_bitexact(gpu, oracle, nm, N, tol):
    """Shared-matrix batches beyond 2 per CU run the condensed operator on the MFMA panels
    (gpad_cpanel.hip: one H GEMM per iteration; the tests' direct -ML / G_L GEMMs); a ragged
    last group, warm-started y, a separate e_V; every checked instance bit-exact with its own
    condensed oracle solve, iteration count included.  The same bits with the panels switched off
    (one workgroup per instance), with forced finisher takeovers (the survivors' y, w, wbar, u
    carried to the latency kernel) and with the takeover planned from a previous solve."""
    import gpad_mpc
    from gpad_mpc import _lib, problems
    n, m = nm
    B = 2 * 256 + 37
    qp = problems.synthetic_qp(n, m, batch=B, seed=23)
    ML, G = _f32(qp.ML), _f32(qp.G)
    M, g, L = _f32(qp.M).reshape(B, n), _f32(qp.g).reshape(B, m), np.float32(qp.L)
    y0 = (0.02 * np.random.default_rng(8).random((B, m))).astype(np.float32)
    res = {}
    # panels to the end / panels to a forced takeover then the latency finisher (eps mode) /
    # no panels (one workgroup per instance); then a second solve planned from the first's counts
    for key, opts in (("panel", dict(phased=0)), ("take30", dict(phase_len=30)), ("take150", dict(phase_len=150)),
                      ("latency", dict(condensed_panel=0)), ("planned", {})):
        z = np.zeros((B, n), np.float32)
        y = y0.copy()
        it = np.zeros(B, np.int32)
        with gpad_mpc.GpadSolver(0) as s:
            s.setup(ML, G, float(L), n=n, m=m, batch=B, kernel=_lib.KERNEL_CONDENSED, tol_gap=2e-4)
            s.set_options(**opts)
            for _ in range(2 if key == "planned" else 1):
                z[:] = 0.0
                y[:] = y0
                st = s.run(z, y, M, g, N, tol, iters=it)
        assert st["kernel"] == "condensed"
        res[key] = (z, y, it)
    z, y, it = res["panel"]
    for key in res:
        np.testing.assert_array_equal(res[key][2], it, err_msg=key)
        np.testing.assert_array_equal(res[key][0], z, err_msg=key)
        np.testing.assert_array_equal(res[key][1], y, err_msg=key)
    for b in list(range(0, B, 13)) + [B - 1]:
        zo, yo, ito, _ = oracle.solve_condensed_f32(np.zeros(n), y0[b], ML, M[b], G, g[b], N, L, tol, tol_gap=2e-4)
        assert it[b] == ito, b
        assert_bitexact(z[b], zo, f"{b} z")
        assert_bitexact(y[b], yo, f"{b} y")


@pytest.mark.gpu
@pytest.mark.parametrize("B", [1, 600])
def test_condensed_through_gpad_solve(gpu, oracle, B):
    """The north-star symbol gpad_solve with dims.kernel = GPAD_KERNEL_CONDENSED (host pointers,
    one cached handle): the latency kernel at B = 1, the condensed panels at B = 600 (> 2 per CU),
    each instance bit-exact with its condensed oracle solve; a repeated call (cache hit) too."""
    from test_boundary import c_solve
    from gpad_mpc import _lib, problems
    n, m = 120, 150
    qp = problems.synthetic_qp(n, m, batch=B, seed=31)
    ML, G = _f32(qp.ML), _f32(qp.G)
    M, g, L = _f32(qp.M).reshape(B, n), _f32(qp.g).reshape(B, m), np.float32(qp.L)
    for rep in range(2):
        Z = np.zeros((B, n), np.float32)
        Y = np.zeros((B, m), np.float32)
        it = np.zeros(B, np.int32)
        st = c_solve(Z, Y, ML, M, G, g, 3000, L, 1e-4, batch=B, kernel=_lib.KERNEL_CONDENSED, iters=it)
        assert st.kernel == _lib.KERNEL_CONDENSED
        for b in list(range(0, B, 97)) + [B - 1]:
            zo, yo, ito, _ = oracle.solve_condensed_f32(np.zeros(n), np.zeros(m), ML, M[b], G, g[b], 3000, L, 1e-4)
            assert it[b] == ito, (rep, b)
            assert_bitexact(Z[b], zo, f"{rep} z[{b}]")
            assert_bitexact(Y[b], yo, f"{rep} y[{b}]")


@pytest.mark.gpu
@pytest.mark.parametrize("K", [1, 3])
@pytest.mark.parametrize("B,take", [(4097, 0), (4097, 25), (1100, 7)])
def test_condensed_panel_check_every_and_takeover_edges(gpu, oracle, K, B, take):
    """Edge cases of the condensed panels: a test every iteration (K = 1: slot rewrites in back-to-
    back iterations) or every 3rd, two panels per group just past 16 per CU (B = 4097: a one-column
    last group), takeovers that are not multiples of K, a takeover planned from a first solve;
    checked instances bit-exact with the condensed oracle, iteration counts included."""
    import gpad_mpc
    from gpad_mpc import _lib, problems
    n, m = 48, 64
    qp = problems.synthetic_qp(n, m, batch=1, seed=41)
    rng = np.random.default_rng(K * 1000 + B)
    ML, G, L = _f32(qp.ML), _f32(qp.G), np.float32(qp.L)
    M = (qp.M[None, :] * (1.0 + 0.3 * rng.normal(size=(B, 1)))).astype(np.float32)
    g = (qp.g[None, :] + 0.2 * rng.random((B, m))).astype(np.float32)
    z = np.zeros((B, n), np.float32)
    y = np.zeros((B, m), np.float32)
    it = np.zeros(B, np.int32)
    with gpad_mpc.GpadSolver(0) as s:
        s.setup(ML, G, float(L), n=n, m=m, batch=B, kernel=_lib.KERNEL_CONDENSED, check_every=K)
        s.set_options(phase_len=take)
        for _ in range(2):  # the second solve plans its takeover from the first (take = 0)
            z[:] = 0.0
            y[:] = 0.0
            st = s.run(z, y, M, g, 3000, 1e-4, iters=it)
    assert st["kernel"] == "condensed" and st["converged"] == B
    for b in list(range(0, B, 211)) + [B - 1]:
        zo, yo, ito, _ = oracle.solve_condensed_f32(np.zeros(n), np.zeros(m), ML, M[b], G, g[b], 3000, L, 1e-4,
                                                    check_every=K)
        assert it[b] == ito, b
        assert_bitexact(z[b], zo, f"z[{b}]")
        assert_bitexact(y[b], yo, f"y[{b}]")


@pytest.mark.gpu
@pytest.mark.parametrize("nm", [(200, 200), (150, 207)])
@pytest.mark.parametrize("N,tol,take", [(60, 0.0, 0), (3000, 1e-4, 0), (3000, 1e-4, 40)])
def test_condensed_panel_pairs_handoff_bitexact(gpu, oracle, nm, N, tol, take):
    """Two panels per group at T = 13 (the C4 shape; 16 waves, 7,7,6,6 chains per SIMD), fixed N,
    planned and forced takeovers: instances across the grid bit-exact with the condensed oracle.
    (A chain hand-off as in the bit-exact pairs measured no gain here, profiles/r02_cpanel_handoff_ab.txt:
    a condensed group's iteration is latency-bound, not SIMD-issue-bound.)"""
    import gpad_mpc
    from gpad_mpc import _lib, problems
    n, m = nm
    B = 16 * 256 + 301
    qp = problems.synthetic_qp(n, m, batch=1, seed=43)
    rng = np.random.default_rng(N + n)
    ML, G, L = _f32(qp.ML), _f32(qp.G), np.float32(qp.L)
    M = (qp.M[None, :] * (1.0 + 0.3 * rng.normal(size=(B, 1)))).astype(np.float32)
    g = (qp.g[None, :] + 0.2 * rng.random((B, m))).astype(np.float32)
    z = np.zeros((B, n), np.float32)
    y = np.zeros((B, m), np.float32)
    it = np.zeros(B, np.int32)
    with gpad_mpc.GpadSolver(0) as s:
        s.setup(ML, G, float(L), n=n, m=m, batch=B, kernel=_lib.KERNEL_CONDENSED)
        s.set_options(phase_len=take)
        for _ in range(2):
            z[:] = 0.0
            y[:] = 0.0
            st = s.run(z, y, M, g, N, tol, iters=it)
    assert st["kernel"] == "condensed"
    for b in list(range(0, B, 397)) + [B - 1]:
        zo, yo, ito, _ = oracle.solve_condensed_f32(np.zeros(n), np.zeros(m), ML, M[b], G, g[b], N, L, tol)
        assert it[b] == ito, b
        assert_bitexact(z[b], zo, f"z[{b}]")
        assert_bitexact(y[b], yo, f"y[{b}]")
