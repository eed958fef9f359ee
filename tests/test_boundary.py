"""The north-star boundary as shipped: the C symbol ``gpad_solve(z0, y0, ML, M, G, g, N, L, tol,
dims, stats)`` (include/gpad.h) called directly through ctypes, and by a plain-C caller
(apps/gpad_main.c --one-shot), against the oracle (bit-exact, iteration counts included).

gpad_solve keeps one handle per thread and device between calls (csrc/gpad_host.cpp): repeated
calls with changing shapes, batches, memory kinds and dtypes, and with host matrices rewritten in
place under the same pointers, must each solve exactly the problem they were given.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, PKG

pytestmark = pytest.mark.gpu


def _problem(n, m, batch, seed, shared=True):
    from gpad_mpc import problems
    qp = problems.synthetic_qp(n, m, batch=batch, seed=seed)
    f = lambda a: np.ascontiguousarray(np.asarray(a, np.float64).astype(np.float32))  # noqa: E731
    ML, G = f(qp.ML), f(qp.G)
    if not shared:  # distinct matrices: perturb each instance's copy
        rng = np.random.default_rng(seed + 100)
        ML = f(ML[None] * (1.0 + 0.01 * rng.random((batch, 1, 1))))
        G = f(G[None] * (1.0 + 0.01 * rng.random((batch, 1, 1))))
    M = f(qp.M).reshape(batch, n)
    g = f(qp.g).reshape(batch, m)
    return ML, M, G, g, np.float32(qp.L)


def c_solve(z, y, ML, M, G, g, N, L, tol, *, batch, shared=True, memory=0, dtype=0, kernel=0, iters=None):
    """One direct call of the exported C symbol; numpy -> host pointers, torch -> device."""
    from gpad_mpc import _lib
    lib = _lib.load()
    ptr = (lambda a: C.c_void_p(a.data_ptr())) if memory else (lambda a: C.c_void_p(a.ctypes.data))
    n, m = ML.shape[-2], ML.shape[-1]
    d = _lib.Dims(n=n, m=m, batch=batch, shared=int(shared), dtype=dtype, memory=memory,
                  schedule=_lib.SCHEDULE_MATLAB, check_every=10, kernel=kernel)
    st = _lib.Stats()
    if iters is not None:
        st.iters = iters.ctypes.data_as(C.POINTER(C.c_int))
    rc = lib.gpad_solve(ptr(z), ptr(y), ptr(ML), ptr(M), ptr(G), ptr(g), int(N), float(L), float(tol),
                        C.byref(d), C.byref(st))
    _lib.check(rc, "gpad_solve")
    return st


def check_vs_oracle(oracle, Z, Y, it, ML, M, G, g, L, N, tol, shared=True):
    batch = M.shape[0]
    for b in range(batch):
        ml = ML if shared else ML[b]
        gg = G if shared else G[b]
        zo, yo, ito, _ = oracle.solve_f32(np.zeros(ml.shape[0]), np.zeros(ml.shape[1]), ml, M[b], gg, g[b],
                                          N, L, tol)
        assert it[b] == ito, (b, it[b], ito)
        np.testing.assert_array_equal(Z[b], zo, err_msg=f"z[{b}]")
        np.testing.assert_array_equal(Y[b], yo, err_msg=f"y[{b}]")


@pytest.mark.parametrize("memory", [0, 1])
def test_gpad_solve_symbol_bitexact(gpu, oracle, memory):
    """gpad_solve through ctypes: C2 batch 1 (fixed N, then to eps), a shared batch of 37, a
    panel-sized shared batch of 300 to eps, distinct matrices, then a shape change and back --
    one cached handle serves them all, every result exact."""
    import torch
    cases = [  # (n, m, batch, N, tol, shared)
        (200, 200, 1, 60, 0.0, True),
        (200, 200, 1, 3000, 1e-4, True),
        (64, 96, 37, 2000, 1e-4, True),
        (40, 72, 300, 3000, 1e-4, True),
        (50, 40, 5, 200, 1e-4, False),
        (200, 200, 1, 60, 0.0, True),   # back to the first shape
    ]
    for k, (n, m, B, N, tol, shared) in enumerate(cases):
        ML, M, G, g, L = _problem(n, m, B, seed=40 + k, shared=shared)
        Z = np.zeros((B, n), np.float32)
        Y = np.zeros((B, m), np.float32)
        it = np.zeros(B, np.int32)
        if memory:
            t = lambda a: torch.from_numpy(a).to(gpu)  # noqa: E731
            dZ, dY = t(Z), t(Y)
            st = c_solve(dZ, dY, t(ML), t(M), t(G), t(g), N, L, tol, batch=B, shared=shared, memory=1,
                         iters=it)
            Z, Y = dZ.cpu().numpy(), dY.cpu().numpy()
        else:
            st = c_solve(Z, Y, ML, M, G, g, N, L, tol, batch=B, shared=shared, iters=it)
        assert st.total_iterations == int(it.sum())
        check_vs_oracle(oracle, Z, Y, it, ML, M, G, g, L, N, tol, shared)


def test_gpad_solve_rewritten_host_matrices(gpu, oracle):
    """The one-shot cache must not trust pointers: the same host buffers, rewritten in place
    between calls, and a changed L, are solved as the new problem."""
    n, m, B, N = 60, 80, 3, 150
    ML, M, G, g, L = _problem(n, m, B, seed=7)
    for k in range(4):
        if k == 1:
            ML[3, 5] += np.float32(0.25)       # same pointer, new contents
        elif k == 2:
            G[:, 0] *= np.float32(1.5)
        elif k == 3:
            L = np.float32(L * 1.25)           # same matrices, new Lipschitz constant
        Z = np.zeros((B, n), np.float32)
        Y = np.zeros((B, m), np.float32)
        it = np.zeros(B, np.int32)
        c_solve(Z, Y, ML, M, G, g, N, L, 0.0, batch=B, iters=it)
        check_vs_oracle(oracle, Z, Y, it, ML, M, G, g, L, N, 0.0)
        # repeated identical call (cache hit) gives the identical answer
        Z2 = np.zeros((B, n), np.float32)
        Y2 = np.zeros((B, m), np.float32)
        c_solve(Z2, Y2, ML, M, G, g, N, L, 0.0, batch=B)
        np.testing.assert_array_equal(Z2, Z)
        np.testing.assert_array_equal(Y2, Y)


def test_gpad_solve_f64_matches_oracle(gpu, oracle):
    """dtype f64 through the one-shot symbol (stream kernel): within 1e-12 of the fp64 oracle."""
    from gpad_mpc import _lib, problems
    qp = problems.synthetic_qp(48, 64, batch=1, seed=3)
    ML, G = np.ascontiguousarray(qp.ML), np.ascontiguousarray(qp.G)
    M, g = np.ascontiguousarray(qp.M).reshape(1, -1), np.ascontiguousarray(qp.g).reshape(1, -1)
    Z = np.zeros((1, 48))
    Y = np.zeros((1, 64))
    c_solve(Z, Y, ML, M, G, g, 300, qp.L, 0.0, batch=1, dtype=_lib.DTYPE_F64)
    zo, yo, _, _ = oracle.solve_f64(np.zeros(48), np.zeros(64), ML, M[0], G, g[0], 300, qp.L)
    np.testing.assert_allclose(Z[0], zo, rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(Y[0], yo, rtol=1e-12, atol=1e-12)


def test_c_app_one_shot_bitexact(gpu, oracle):
    """apps/gpad_main.c --one-shot: a plain-C caller of gpad_solve on the data file's problem
    (ML = -M_G, G = L G_L, g = -L p_D), 100 iterations, then 50 repeated calls (cache hits,
    each checked equal to the first by the app); bit-exact vs the oracle on the same unscaled
    inputs; prints the per-call latency."""
    from gpad_mpc import datafile
    app = os.path.join(PKG, "gpad_mpc", "gpad_main")
    path = os.path.join(GOLDEN, "datafile_battery_3x4.txt")
    r = subprocess.run([app, path, "--one-shot", "--repeat", "50"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    lines = {ln.split()[0]: ln.split()[1:] for ln in r.stdout.splitlines()}
    z = np.array([np.float32(v) for v in lines["z"]], np.float32)
    y = np.array([np.float32(v) for v in lines["y"]], np.float32)
    d = datafile.read(path, 0)
    L = np.float32(d.L)
    ML = (-d.M_G).astype(np.float32)
    G = (np.float64(L) * d.G_L.astype(np.float64)).astype(np.float32)
    g = (-np.float64(L) * d.p_D.astype(np.float64)).astype(np.float32)
    zo, yo, ito, _ = oracle.solve_f32(np.zeros(d.n), np.zeros(d.m), ML, d.g_P, G, g, 100, L)
    np.testing.assert_array_equal(z, zo)
    np.testing.assert_array_equal(y, yo)
    assert lines["iterations"][0] == "100"
    print("gpad_solve one-shot latency (us/call, battery 3x4, 100 iterations):", lines["solve_us"][0])


def test_fresh_handle_follows_shape_prior(gpu, oracle):
    """a handle with no plan of its own plans its first phased solve from the
    shape's prior -- the last plan any handle of the process made for the same (n, m, batch, K, N)
    (csrc/gpad_host.cpp plan_for).  Handle A solves batch 1 (its plan then becomes the prior); a new
    handle B solves batch 2 following that prior: the same phases and survivor counts as A solving
    batch 2 with its own plan (made from the same counts), bit-identical results.  Then the north-star
    gpad_solve, from a freshly created cached handle, equals the oracle on batch 3."""
    import torch

    import bench
    import gpad_mpc
    n = m = 200
    B, N, tol = 2048, 5000, 1e-4
    ML, G, L, M1, g1 = bench.make_shard(n, m, B, 0)
    (M2, g2), (M3, g3) = bench.make_stream(n, m, B, 2, 0)
    f = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(gpu)  # noqa: E731
    L32 = float(np.float32(L))
    dML, dG = f(ML), f(G)

    def solve(s, M, g):
        z = torch.zeros(B, n, device=gpu)
        y = torch.zeros(B, m, device=gpu)
        it = np.zeros(B, np.int32)
        s.run(z, y, f(M), f(g), N, tol, iters=it)
        return z.cpu().numpy(), y.cpu().numpy(), it, s.last_phases()

    with gpad_mpc.GpadSolver(0) as a, gpad_mpc.GpadSolver(0) as b:
        for s in (a, b):
            s.setup(dML, dG, L32, n=n, m=m, batch=B, shared=True, check_every=10)
        solve(a, M1, g1)
        zb, yb, itb, pb = solve(b, M2, g2)
        za, ya, ita, pa2 = solve(a, M2, g2)
    assert pb["prior"] and not pa2["prior"]
    assert pb["ends"] == pa2["ends"] and pb["fins"] == pa2["fins"] and pb["counts"] == pa2["counts"]
    assert len(pb["ends"]) <= 6, pb  # planned: a few phases, not the default 40-iteration run-up
    np.testing.assert_array_equal(itb, ita)
    np.testing.assert_array_equal(zb, za)
    np.testing.assert_array_equal(yb, ya)
    # gpad_solve: its cached handle is new after gpad_release_cached, so it follows the prior
    from gpad_mpc import _lib
    _lib.load().gpad_release_cached()
    M3f, g3f = np.ascontiguousarray(M3, np.float32), np.ascontiguousarray(g3, np.float32)
    MLf, Gf = np.ascontiguousarray(ML, np.float32), np.ascontiguousarray(G, np.float32)
    Z = np.zeros((B, n), np.float32)
    Y = np.zeros((B, m), np.float32)
    it3 = np.zeros(B, np.int32)
    st = c_solve(Z, Y, MLf, M3f, Gf, g3f, N, np.float32(L), tol, batch=B, iters=it3)
    assert st.converged == B
    for k in (0, 1, B // 2, B - 1, int(np.argmax(it3))):
        zo, yo, ito, _ = oracle.solve_f32(np.zeros(n), np.zeros(m), MLf, M3f[k], Gf, g3f[k], N, np.float32(L), tol)
        assert it3[k] == ito, k
        np.testing.assert_array_equal(Z[k], zo)
        np.testing.assert_array_equal(Y[k], yo)
