"""f64 panels on the f64 MFMA pipe (csrc/gpad_panel64.hip): shared-matrix f64 batches, with the
value-function branches of Algorithm 1 (acceldualgrad.m:30-33, 73, 76) when H is bound -- the
reference's own termination regime e_g = e_V = 1e-6 (acceldualgrad.m:12-13), which lies below the
f32 certification floor.

Pins: (1) the f64 stream kernel on the same inputs, bit for bit (z, y, iteration counts, codes):
v_mfma_f64_16x16x4_f64 is the ascending-k fma chain (profiles/r04_mfma_f64.txt) and the epilogues
are the stream kernel's; (2) the fp64 oracle (orc_solve_value_f64 / orc_solve_f64, the mul/add
order of acceldualgrad.m): iteration counts and termination codes equal, z within 1e-12.  The
oracle itself is pinned to a literal restatement of the commented MATLAB test (test_value.py).
Iteration counts to eps are parity unpinned against the reference, which never runs its test.
"""
from __future__ import annotations

import numpy as np
import pytest

from test_value import value_problem

pytestmark = pytest.mark.gpu


def _run(ML, G, L, M, g, N, tol, *, kernel, H=None, tol_gap=0.0, K=10, dev=True, opts=None, z0=None, y0=None):
    import torch

    import gpad_mpc
    from gpad_mpc import _lib
    B, n = M.shape
    m = g.shape[1]
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float64)).cuda()  # noqa: E731
    z = torch.zeros(B, n, dtype=torch.float64, device="cuda") if z0 is None else t(z0)
    y = torch.zeros(B, m, dtype=torch.float64, device="cuda") if y0 is None else t(y0)
    it = np.zeros(B, np.int32)
    codes = np.full(B, -1, np.int32)
    kern = {"panel": _lib.KERNEL_PANEL, "stream": _lib.KERNEL_STREAM, "auto": _lib.KERNEL_AUTO}[kernel]
    with gpad_mpc.GpadSolver(0) as s:
        s.setup(t(ML), t(G), float(L), n=n, m=m, batch=B, check_every=K, kernel=kern, tol_gap=tol_gap)
        if H is not None:
            s.setup_hessian(t(H))
        s.set_options(**(opts or {}))
        st = s.run(z, y, t(M), t(g), N, tol, iters=it, codes=codes)
    return z.cpu().numpy(), y.cpu().numpy(), it, codes, st


@pytest.mark.parametrize("shift,tol,tol_gap,K", [(1.0, 1e-2, 1e-1, 1), (1.0, 1e-3, 1e-2, 1),
                                                 (3.0, 1e-3, 1e-2, 10), (3.0, 1e-2, 1e-1, 1)])
def test_panel64_value_branches_small(gpu, oracle, shift, tol, tol_gap, K):
    """n = 20, m = 40 (T = 3), 64 instances, H bound: the f64 panel equals the f64 stream kernel bit
    for bit and the fp64 oracle (counts, codes, z to 1e-12); codes 3 / 4 occur in the sweep."""
    B = 64
    H, ML, M, G, g, L = (np.asarray(a) for a in value_problem(20, 40, 7, shift, batch=B)[:6])
    zp, yp, itp, cp, stp = _run(ML, G, L, M, g, 5000, tol, kernel="panel", H=H, tol_gap=tol_gap, K=K)
    zs, ys, its, cs, sts = _run(ML, G, L, M, g, 5000, tol, kernel="stream", H=H, tol_gap=tol_gap, K=K)
    assert stp["kernel"] == "panel" and sts["kernel"] == "stream"
    np.testing.assert_array_equal(itp, its)
    np.testing.assert_array_equal(cp, cs)
    np.testing.assert_array_equal(zp, zs)
    np.testing.assert_array_equal(yp, ys)
    for b in range(B):
        zo, yo, ito, co = oracle.solve_value_f64(np.zeros(20), np.zeros(40), ML, M[b], G, g[b], H, 5000, L, tol,
                                                 check_every=K, tol_gap=tol_gap)
        assert (itp[b], cp[b]) == (ito, co), b
        np.testing.assert_allclose(zp[b], zo, rtol=1e-12, atol=1e-14)
    TestCodes.seen.update(cp.tolist())


class TestCodes:
    seen: set = set()

    def test_value_codes_exercised(self, gpu, oracle):
        if not self.seen:
            for case in [(1.0, 1e-2, 1e-1, 1), (3.0, 1e-2, 1e-1, 1)]:
                test_panel64_value_branches_small(gpu, oracle, *case)
        assert {3, 4} & self.seen, self.seen


@pytest.mark.parametrize("relay", [1, 0])
def test_panel64_reference_tolerance_c4_shape(gpu, oracle, relay):
    """C4 shape (n = m = 200, T = 13), the reference's e_g = e_V = 1e-6 with H bound, 512 instances
    (value problems: constraints active at an optimum with a positive objective): bit-exact with the
    f64 stream kernel on every instance, and a spread sample equal to the fp64 oracle (counts,
    codes, z to 1e-12); every instance converged (codes 2 / 3).  relay = 1: the 16-wave layout
    (tile 12's chain cut over four waves, round 5), 0: one wave per tile."""
    B, tol = 512, 1e-6
    H, ML, M, G, g, L = (np.asarray(a) for a in value_problem(200, 200, 7, 1.0, batch=B)[:6])
    zp, yp, itp, cp, stp = _run(ML, G, L, M, g, 20000, tol, kernel="panel", H=H, tol_gap=tol,
                                opts={"p64_relay": relay})
    zs, ys, its, cs, _ = _run(ML, G, L, M, g, 20000, tol, kernel="stream", H=H, tol_gap=tol)
    assert stp["kernel"] == "panel" and stp["converged"] == B
    np.testing.assert_array_equal(itp, its)
    np.testing.assert_array_equal(cp, cs)
    np.testing.assert_array_equal(zp, zs)
    np.testing.assert_array_equal(yp, ys)
    assert 3 in set(cp.tolist())
    for b in list(range(0, B, 37)) + [int(np.argmax(itp))]:
        zo, yo, ito, co = oracle.solve_value_f64(np.zeros(200), np.zeros(200), ML, M[b], G, g[b], H, 20000, L, tol,
                                                 tol_gap=tol)
        assert (itp[b], cp[b]) == (ito, co), b
        np.testing.assert_allclose(zp[b], zo, rtol=1e-12, atol=1e-14)


@pytest.mark.parametrize("n,m,B", [(37, 53, 40), (200, 180, 40), (256, 256, 40), (5, 129, 40), (160, 200, 40),
                                   (144, 144, 40), (130, 137, 40), (200, 193, 40), (40, 53, 4100), (16, 16, 5000)])
def test_panel64_fixed_n_ragged(gpu, n, m, B):
    """Fixed N = 60 (no test) and eps = 1e-6 without H on ragged shapes: bit-exact with the f64
    stream kernel (zero-padded k-steps and skipped tiles).  (144, 144), (130, 137), (200, 193): the
    relay layout at T = 9 / 13; (40, 53) and (16, 16) at thousands of instances: several small
    workgroups per CU (the occupancy-sized grid)."""
    from gpad_mpc import problems
    qp = problems.synthetic_qp(n, m, batch=B, seed=n + m)
    ML, G = np.asarray(qp.ML), np.asarray(qp.G)
    M, g = np.asarray(qp.M).reshape(B, n), np.asarray(qp.g).reshape(B, m)
    for N, tol in ((60, 0.0), (3000, 1e-6)):
        a = _run(ML, G, qp.L, M, g, N, tol, kernel="panel")
        if n > 128:  # the relay and the one-wave-per-tile layout agree bit for bit too
            c = _run(ML, G, qp.L, M, g, N, tol, kernel="panel", opts={"p64_relay": 0})
            for x, y_ in zip(a[:4], c[:4]):
                np.testing.assert_array_equal(x, y_)
        b = _run(ML, G, qp.L, M, g, N, tol, kernel="stream")
        assert a[4]["kernel"] == "panel"
        for x, y_ in zip(a[:4], b[:4]):
            np.testing.assert_array_equal(x, y_)


def test_panel64_auto_c4_batch_certified(gpu, oracle):
    """AUTO picks the f64 panels for a C4-generator batch of 8192 in f64 at eps = 1e-6 (the f32 path's
    floor is ~2^-20 max|g|): every instance converges with fp64 max(G z* - g) <= eps on the returned
    z*; a sample and the longest instances equal the fp64 oracle (counts, z to 1e-12)."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    n = m = 200
    B, tol = 8192, 1e-6
    ML, G, L, M, g = bench.make_shard(n, m, B, 0)
    z, y, it, codes, st = _run(ML, G, L, M, g, 20000, tol, kernel="auto", tol_gap=tol)
    assert st["kernel"] == "panel" and st["converged"] == B
    viol = (z @ G.T - g).max(axis=1)
    assert viol.max() <= tol, (viol.max(), int(viol.argmax()))
    for b in list(range(0, B, 1021)) + [int(i) for i in np.argsort(-it, kind="stable")[:4]]:
        zo, yo, ito, co = oracle.solve_f64(np.zeros(n), np.zeros(m), ML, M[b], G, g[b], 20000, L, tol, tol_gap=tol)
        assert it[b] == ito and co and codes[b] in (1, 2), b
        np.testing.assert_allclose(z[b], zo, rtol=1e-12, atol=1e-14)


@pytest.mark.parametrize("shift,tol,tol_gap,K", [(1.0, 1e-5, 1e-5, 10), (3.0, 1e-3, 1e-2, 1)])
def test_panel64_value_branches_relay_t9(gpu, shift, tol, tol_gap, K):
    """n = m = 140 (T = 9): the relay layout with the value branches (H bound) equals the f64 stream
    kernel bit for bit -- counts and codes included -- and the one-wave-per-tile layout."""
    B = 256
    H, ML, M, G, g, L = (np.asarray(a) for a in value_problem(140, 140, 5, shift, batch=B)[:6])
    a = _run(ML, G, L, M, g, 20000, tol, kernel="panel", H=H, tol_gap=tol_gap, K=K)
    b = _run(ML, G, L, M, g, 20000, tol, kernel="stream", H=H, tol_gap=tol_gap, K=K)
    c = _run(ML, G, L, M, g, 20000, tol, kernel="panel", H=H, tol_gap=tol_gap, K=K, opts={"p64_relay": 0})
    assert a[4]["kernel"] == "panel" and a[4]["converged"] == B
    for x, y_, w in zip(a[:4], b[:4], c[:4]):
        np.testing.assert_array_equal(x, y_)
        np.testing.assert_array_equal(x, w)
    assert set(a[3].tolist()) & {3, 4}


@pytest.mark.parametrize("K", [10, 1])
def test_panel64_refill_bitexact(gpu, K):
    """More panels than workgroups at the C4 shape (4608 value problems, n = m = 200: 288 panels on
    at most 256 one-panel workgroups) with e_g = e_V = 1e-6 and H bound: finished columns take the
    next instances (column refills, round 5).  Bit-identical to the run without refills and to the
    f64 stream kernel -- z, y, counts and codes."""
    B, tol = 4608, 1e-6
    H, ML, M, G, g, L = (np.asarray(a) for a in value_problem(200, 200, 7, 1.0, batch=B)[:6])
    N = 20000 if K == 10 else 19999  # K = 1: every N is a test event
    a = _run(ML, G, L, M, g, N, tol, kernel="panel", H=H, tol_gap=tol, K=K)
    b = _run(ML, G, L, M, g, N, tol, kernel="panel", H=H, tol_gap=tol, K=K, opts={"p64_refill": 0})
    c = _run(ML, G, L, M, g, N, tol, kernel="stream", H=H, tol_gap=tol, K=K)
    assert a[4]["kernel"] == "panel" and a[4]["converged"] == B
    for x, y_, w in zip(a[:4], b[:4], c[:4]):
        np.testing.assert_array_equal(x, y_)
        np.testing.assert_array_equal(x, w)


@pytest.mark.parametrize("hessian", [True, False])
def test_panel64_refill_warm_start(gpu, oracle, hessian):
    """Column refills from a non-zero warm start: every instance starts from its own
    z_{-1} != 0 and y_0 >= 0, so a refilled column seeds u = G_L z_{-1} with the GEMM over the new
    columns while the other columns' state sits in the operand tile, and w_0 = y_0.  4608 instances
    (more panels than workgroups): bit-identical to the run without refills and to the f64 stream
    kernel (z, y, counts, codes), and a sample equal to the fp64 oracle's warm-started solve."""
    B, tol = 4608, 1e-6
    H, ML, M, G, g, L = (np.asarray(a) for a in value_problem(200, 200, 7, 1.0, batch=B)[:6])
    rng = np.random.default_rng(11)
    z0 = 0.05 * rng.normal(size=(B, 200))
    y0 = 0.01 * np.abs(rng.normal(size=(B, 200)))
    Hb = H if hessian else None
    a = _run(ML, G, L, M, g, 20000, tol, kernel="panel", H=Hb, tol_gap=tol, z0=z0, y0=y0)
    b = _run(ML, G, L, M, g, 20000, tol, kernel="panel", H=Hb, tol_gap=tol, z0=z0, y0=y0, opts={"p64_refill": 0})
    c = _run(ML, G, L, M, g, 20000, tol, kernel="stream", H=Hb, tol_gap=tol, z0=z0, y0=y0)
    assert a[4]["kernel"] == "panel" and a[4]["converged"] == B
    for x, y_, w in zip(a[:4], b[:4], c[:4]):
        np.testing.assert_array_equal(x, y_)
        np.testing.assert_array_equal(x, w)
    for i in (0, B // 2 + 1, B - 1, int(np.argmax(a[2]))):
        if hessian:  # (the value oracle returns the termination code, solve_f64 whether it converged)
            zo, yo, ito, co = oracle.solve_value_f64(z0[i], y0[i], ML, M[i], G, g[i], H, 20000, L, tol, tol_gap=tol)
            assert (a[2][i], a[3][i]) == (ito, co), i
        else:
            zo, yo, ito, co = oracle.solve_f64(z0[i], y0[i], ML, M[i], G, g[i], 20000, L, tol, tol_gap=tol)
            assert a[2][i] == ito and bool(co) and a[3][i] in (1, 2), i
        np.testing.assert_allclose(a[0][i], zo, rtol=1e-12, atol=1e-14)


def test_panel64_refill_max_iterations(gpu):
    """Refills with columns that stop at N (N a multiple of the test period, tolerance out of reach
    for some): the counts and codes (0 = ran to N) equal the run without refills."""
    from gpad_mpc import problems
    B, n, m = 4200, 200, 200
    qp = problems.synthetic_qp(n, m, batch=B, seed=5)
    ML, G = np.asarray(qp.ML), np.asarray(qp.G)
    M, g = np.asarray(qp.M).reshape(B, n), np.asarray(qp.g).reshape(B, m)
    a = _run(ML, G, qp.L, M, g, 120, 1e-12, kernel="panel")
    b = _run(ML, G, qp.L, M, g, 120, 1e-12, kernel="panel", opts={"p64_refill": 0})
    for x, y_ in zip(a[:4], b[:4]):
        np.testing.assert_array_equal(x, y_)
    assert (a[3] == 0).any() and (a[2] <= 120).all()


@pytest.mark.parametrize("hessian", [True, False])
def test_panel64_lpt_order_bitexact(gpu, hessian):
    """an f64 panel solve with column refills starts its instances longest-
    predicted-first (the handle's previous counts, GPAD_OPT_LPT) so each column's instances end
    together.  Three solves of one batch on one handle (the second and third follow the first's /
    second's counts; a warm start on the third) equal, bit for bit, the same solves with lpt = 0 and
    the f64 stream kernel -- z, y, counts and codes."""
    import torch

    import gpad_mpc
    from gpad_mpc import _lib
    B, tol = 4608, 1e-6
    H, ML, M, G, g, L = (np.asarray(a) for a in value_problem(200, 200, 7, 1.0, batch=B)[:6])
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float64)).cuda()  # noqa: E731
    rng = np.random.default_rng(3)
    starts = [(np.zeros((B, 200)), np.zeros((B, 200)))] * 2 + [(0.02 * rng.normal(size=(B, 200)),
                                                                0.01 * np.abs(rng.normal(size=(B, 200))))]
    res = {}
    for name, kern, opts in (("lpt", _lib.KERNEL_PANEL, {}), ("plain", _lib.KERNEL_PANEL, {"lpt": 0}),
                             ("stream", _lib.KERNEL_STREAM, {})):
        out = []
        with gpad_mpc.GpadSolver(0) as s:
            s.setup(t(ML), t(G), float(L), n=200, m=200, batch=B, check_every=10, kernel=kern, tol_gap=tol)
            if hessian:
                s.setup_hessian(t(H))
            s.set_options(**opts)
            for z0, y0 in starts:
                z, y = t(z0), t(y0)
                it = np.zeros(B, np.int32)
                codes = np.full(B, -1, np.int32)
                st = s.run(z, y, t(M), t(g), 20000, tol, iters=it, codes=codes)
                assert st["converged"] == B
                out.append((z.cpu().numpy(), y.cpu().numpy(), it, codes))
        res[name] = out
    for k in range(len(starts)):
        for x, y_, w in zip(res["lpt"][k], res["plain"][k], res["stream"][k]):
            np.testing.assert_array_equal(x, y_)
            np.testing.assert_array_equal(x, w)
