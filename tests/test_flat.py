"""Flat battery path: the reference's structure-exploiting steps
StepTwoGPADFlatSequential / StepFourGPADFlatSequential (seq_functions.cpp:5-43) for equal cell
capacities, and libgpad's gpad_setup_flat + flat kernel + per-step flat entry points.

Parity pins: the golden end states come from the reference's OWN flat steps compiled from
/root/reference (oracle/_ref, main_prof.cu loop order; tests/golden/make_golden.py).  The oracle's
flat restatement must match them bit for bit (CPU), and the HIP path must match both (GPU).
"""
from __future__ import annotations

import os

import numpy as np
import pytest

from conftest import GOLDEN, load_golden

FLAT_SETS = ["battery_flat_4x10", "battery_flat_3x4"]


# ---------------------------------------------------------------------------------- CPU
@pytest.mark.parametrize("name", FLAT_SETS)
def test_oracle_flat_matches_reference_steps(oracle, name):
    gd = load_golden(name)
    n_u = int(gd["n_u"])
    n, m = gd["gP"].size, gd["pD"].size
    for K in (1, 10, 100):
        z, y, it, _ = oracle.solve_flat_f32(np.zeros(n), np.zeros(m), gd["MGf"], gd["gP"], gd["GLf"],
                                            gd["pD"], n_u, K, gd["L"], theta=gd["theta100"],
                                            beta=gd["beta100"])
        assert it == K
        np.testing.assert_array_equal(z, gd[f"ref_z_{K}"])
        np.testing.assert_array_equal(y, gd[f"ref_y_{K}"])
    np.testing.assert_array_equal(oracle.step2_flat(gd["MGf"], gd["kat_w"], gd["gP"], n_u), gd["kat_zhat"])
    np.testing.assert_array_equal(oracle.step4_flat(gd["GLf"], gd["kat_w"], gd["pD"], gd["kat_zh_in"], n_u),
                                  gd["kat_yp1"])


def test_flatten_is_exact_for_equal_cells():
    """The flat data reproduces the full battery matrices (gpad.m, equal capacities) to fp64
    round-off: the structural zeros are zeros and the coupling columns are cell-independent."""
    from gpad_mpc import problems
    n_u, N = 4, 10
    qp = problems.battery_mpc(n_u, N, seed=0)
    MGf, GLf, L = problems.flatten_battery(qp, n_u, N)
    n, m, mc = qp.n, qp.m, 4 * n_u * N
    ML = np.zeros((n, m))
    G = np.zeros((m, n))
    for i in range(N):
        for j in range(n_u):
            for k in range(m):
                if k >= mc or k % n_u == j:
                    ML[i * n_u + j, k] = -MGf[i, k]
    for r in range(m):
        for t in range(N):
            for c in range(n_u):
                if r >= mc or r % n_u == c:
                    G[r, t * n_u + c] = GLf[r, t] * L
    assert np.abs(ML - qp.ML).max() <= 1e-15 * np.abs(qp.ML).max()
    assert np.abs(G - qp.G).max() <= 1e-15 * np.abs(qp.G).max()


def test_flat_solution_close_to_full(oracle):
    """Flat and full fp32 paths solve the same QP; they differ only by rounding (the flat step 4
    adds (s + w) + p_D where the full one adds (w + p_D) + s)."""
    gd = load_golden("battery_flat_4x10")
    full = load_golden("battery_c1")
    rel = lambda a, b: np.abs(a - b).max() / np.abs(b).max()  # noqa: E731
    assert rel(gd["ref_z_100"], full["ref_z_100"]) < 1e-5
    assert rel(gd["ref_y_100"], full["ref_y_100"]) < 1e-5
    assert int(gd["tol_iters"]) == int(full["tol_iters"])


def test_flat_datafile_reads(tmp_path):
    """ENABLE_FLATTEN_MATRICES files (main.cu:39-56): M_G N x m, G_L m x N; a write/read round trip
    is exact and the numpy-written fixture reads at its print precision."""
    from gpad_mpc import datafile
    gd = load_golden("battery_flat_3x4")
    d = datafile.read(os.path.join(GOLDEN, "datafile_battery_flat_3x4.txt"), datafile.FILE_FLAT)
    assert d.M_G.shape == (4, 56) and d.G_L.shape == (56, 4) and d.n == 12
    np.testing.assert_allclose(d.M_G, gd["MGf"], rtol=1e-7, atol=1e-12)
    np.testing.assert_allclose(d.G_L, gd["GLf"], rtol=1e-7, atol=1e-12)
    p = str(tmp_path / "flat.txt")
    datafile.write(p, d, datafile.FILE_FLAT)
    r = datafile.read(p, datafile.FILE_FLAT)
    for k in ("M_G", "g_P", "G_L", "p_D", "theta", "beta"):
        np.testing.assert_array_equal(getattr(r, k), getattr(d, k), err_msg=k)


# ---------------------------------------------------------------------------------- GPU
VARIANTS = [0, 1]  # KERNEL_AUTO: register-resident flat chains; KERNEL_STREAM: the LDS flat kernel


def _flat_solver(gd, batch=1, kernel=0):
    import gpad_mpc
    s = gpad_mpc.GpadSolver(0)
    s.setup_flat(gd["MGf"], gd["GLf"], float(gd["L"]), n_u=int(gd["n_u"]), batch=batch, kernel=kernel)
    return s


@pytest.mark.gpu
@pytest.mark.parametrize("name", FLAT_SETS)
@pytest.mark.parametrize("kernel", VARIANTS)
def test_flat_kernel_matches_reference_steps(gpu, name, kernel):
    """Fixed N = 1, 10, 100 with the reference's θ/β: bit-exact with its own flat steps."""
    gd = load_golden(name)
    s = _flat_solver(gd, kernel=kernel)
    n, m = gd["gP"].size, gd["pD"].size
    for K in (1, 10, 100):
        z = np.zeros(n, np.float32)
        y = np.zeros(m, np.float32)
        st = s.run(z, y, gd["gP"], gd["pD"], K, 0.0, scaled=True, theta=gd["theta100"],
                   beta=gd["beta100"])
        assert st["kernel"] == "flat"
        np.testing.assert_array_equal(z, gd[f"ref_z_{K}"])
        np.testing.assert_array_equal(y, gd[f"ref_y_{K}"])


@pytest.mark.gpu
@pytest.mark.parametrize("name", FLAT_SETS)
@pytest.mark.parametrize("kernel", VARIANTS)
def test_flat_kernel_algorithm1(gpu, name, kernel):
    gd = load_golden(name)
    s = _flat_solver(gd, kernel=kernel)
    n, m = gd["gP"].size, gd["pD"].size
    z = np.zeros(n, np.float32)
    y = np.zeros(m, np.float32)
    st = s.run(z, y, gd["gP"], gd["pD"], 5000, 1e-4, scaled=True)
    assert st["iterations"] == int(gd["tol_iters"]) and st["converged"] == (1 if gd["tol_conv"] else 0)
    np.testing.assert_array_equal(z, gd["tol_z"])
    np.testing.assert_array_equal(y, gd["tol_y"])


@pytest.mark.gpu
@pytest.mark.parametrize("tol,N", [(0.0, 150), (1e-4, 4000)])
@pytest.mark.parametrize("kernel", VARIANTS)
@pytest.mark.parametrize("cells", [(4, 10), (3, 17), (5, 6)])
def test_flat_batch_bitexact(gpu, oracle, tol, N, kernel, cells):
    """A battery-scenario batch (one plant, per-state g_P, p_D) on the flat kernel vs the
    oracle's flat solve per instance."""
    from gpad_mpc import problems
    (n_u, Nh), B = cells, 48
    qp = problems.battery_scenarios(n_u, Nh, B, seed=4)
    MGf, GLf, L = problems.flatten_battery(qp, n_u, Nh)
    f32 = lambda a: np.ascontiguousarray(np.asarray(a, np.float64).astype(np.float32))  # noqa: E731
    L32 = np.float32(L)
    MGf32, GLf32 = f32(MGf), f32(GLf)
    GP = f32(qp.M)
    PD = oracle.scale_vec(f32(qp.g), L32)
    import gpad_mpc
    s = gpad_mpc.GpadSolver(0)
    s.setup_flat(MGf32, GLf32, float(L32), n_u=n_u, batch=B, kernel=kernel)
    Z = np.zeros((B, qp.n), np.float32)
    Y = np.zeros((B, qp.m), np.float32)
    it = np.zeros(B, np.int32)
    s.run(Z, Y, GP, np.ascontiguousarray(PD), N, tol, scaled=True, iters=it)
    for b in range(B):
        z, y, its, _ = oracle.solve_flat_f32(np.zeros(qp.n), np.zeros(qp.m), MGf32, GP[b], GLf32, PD[b],
                                             n_u, N, L32, tol)
        assert it[b] == its, b
        np.testing.assert_array_equal(Z[b], z, err_msg=f"z[{b}]")
        np.testing.assert_array_equal(Y[b], y, err_msg=f"y[{b}]")


@pytest.mark.gpu
@pytest.mark.parametrize("tol,N", [(0.0, 120), (1e-4, 4000)])
@pytest.mark.parametrize("cells,B,P", [((4, 10), 40, 1), ((3, 17), 33, 1), ((5, 6), 16 * 3 + 1, 1),
                                       ((4, 50), 24, 1), ((2, 30), 20, 1), ((4, 10), 16 * 5 + 3, 4),
                                       ((4, 10), 16 * 3 + 7, 2), ((3, 17), 16 * 4 + 9, 3), ((5, 6), 16 * 2 + 1, 4),
                                       ((4, 50), 1, 1), ((3, 17), 5, 1), ((4, 10), 16 * 3 + 5, 8),
                                       ((3, 17), 16 * 2 + 3, 8), ((5, 6), 16 * 4 + 1, 8)])
def test_flat_panel_bitexact(gpu, oracle, tol, N, cells, B, P):
    """The flat MFMA panel kernel (gpad_flatpanel.hip, forced with KERNEL_PANEL): per-cell
    skinny GEMMs over 16-instance panels, P panels per workgroup (ragged last panel, partly
    empty last group), vs the oracle's flat solve."""
    from gpad_mpc import problems
    import gpad_mpc
    n_u, Nh = cells
    qp = problems.battery_scenarios(n_u, Nh, B, seed=11)
    MGf, GLf, L = problems.flatten_battery(qp, n_u, Nh)
    f32 = lambda a: np.ascontiguousarray(np.asarray(a, np.float64).astype(np.float32))  # noqa: E731
    L32 = np.float32(L)
    MGf32, GLf32 = f32(MGf), f32(GLf)
    GP = f32(qp.M)
    PD = np.ascontiguousarray(oracle.scale_vec(f32(qp.g), L32))
    s = gpad_mpc.GpadSolver(0)
    s.setup_flat(MGf32, GLf32, float(L32), n_u=n_u, batch=B, kernel=gpad_mpc.KERNEL_PANEL)
    if P == 8:  # 8-wave workgroups, two per CU
        s.set_option("flat_waves", 8)
    else:
        s.set_option("flat_panels", P)
    Z = np.zeros((B, qp.n), np.float32)
    Y = np.zeros((B, qp.m), np.float32)
    it = np.zeros(B, np.int32)
    st = s.run(Z, Y, GP, PD, N, tol, scaled=True, iters=it)
    assert st["kernel"] == "flat"
    for b in range(B):
        z, y, its, _ = oracle.solve_flat_f32(np.zeros(qp.n), np.zeros(qp.m), MGf32, GP[b], GLf32, PD[b],
                                             n_u, N, L32, tol)
        assert it[b] == its, b
        np.testing.assert_array_equal(Z[b], z, err_msg=f"z[{b}]")
        np.testing.assert_array_equal(Y[b], y, err_msg=f"y[{b}]")


@pytest.mark.gpu
@pytest.mark.parametrize("phase_len,phased,P", [(10, 2, 1), (30, 2, 2), (0, 2, 4), (0, 0, 1), (10, 2, 8),
                                                 (20, 2, 3)])
@pytest.mark.parametrize("cells,B", [((4, 10), 16 * 6 + 5), ((3, 17), 16 * 4 + 9)])
def test_flat_panel_phased_bitexact(gpu, oracle, phase_len, phased, P, cells, B):
    """Phased compaction on the flat panels (tol mode): survivors of each phase are parked
    (z, y in place; w, u carried) and re-packed into new groups (other columns, panels and
    workgroups) for the next phase; warm-started y.  Every instance must equal its own oracle
    flat solve, iteration count included.  phased=2 forces phases at this small batch (the
    default starts at 4 panels per CU); phased=0: one launch, groups run to their last column."""
    from gpad_mpc import problems
    import gpad_mpc
    n_u, Nh = cells
    qp = problems.battery_scenarios(n_u, Nh, B, seed=13)
    MGf, GLf, L = problems.flatten_battery(qp, n_u, Nh)
    f32 = lambda a: np.ascontiguousarray(np.asarray(a, np.float64).astype(np.float32))  # noqa: E731
    L32 = np.float32(L)
    MGf32, GLf32, GP = f32(MGf), f32(GLf), f32(qp.M)
    PD = np.ascontiguousarray(oracle.scale_vec(f32(qp.g), L32))
    Y0 = (0.02 * np.random.default_rng(3).random((B, qp.m))).astype(np.float32)
    s = gpad_mpc.GpadSolver(0)
    s.setup_flat(MGf32, GLf32, float(L32), n_u=n_u, batch=B, kernel=gpad_mpc.KERNEL_PANEL)
    if P == 8:
        s.set_option("flat_waves", 8)
    else:
        s.set_option("flat_panels", P)
    s.set_options(phase_len=phase_len, phased=phased)
    for rnd, tol in enumerate((1e-3, 1e-4)):  # the second solve's phases end at the first's last iteration
        Z = np.zeros((B, qp.n), np.float32)
        Y = Y0.copy()
        it = np.zeros(B, np.int32)
        st = s.run(Z, Y, GP, PD, 4000, tol, scaled=True, iters=it)
        assert st["kernel"] == "flat" and st["converged"] == B
        assert it.max() > it.min() + 40  # the batch spans several phases
        for b in range(B):
            z, y, its, _ = oracle.solve_flat_f32(np.zeros(qp.n), Y0[b], MGf32, GP[b], GLf32, PD[b], n_u, 4000,
                                                 L32, tol)
            assert it[b] == its, (rnd, b)
            np.testing.assert_array_equal(Z[b], z, err_msg=f"{rnd} z[{b}]")
            np.testing.assert_array_equal(Y[b], y, err_msg=f"{rnd} y[{b}]")


@pytest.mark.gpu
@pytest.mark.parametrize("name", FLAT_SETS)
def test_flat_step_entry_points(gpu, name):
    """gpad_step2_primal_flat / gpad_step4_project_flat vs the reference's flat step KATs."""
    import torch

    import gpad_mpc
    gd = load_golden(name)
    n_u = int(gd["n_u"])
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(gpu)  # noqa: E731
    s = gpad_mpc.GpadSolver(0)
    zh = torch.empty(gd["gP"].size, device=gpu)
    s.step2_flat(t(gd["MGf"]), t(gd["kat_w"]), t(gd["gP"]), zh, n_u)
    yp = torch.empty(gd["pD"].size, device=gpu)
    s.step4_flat(t(gd["GLf"]), yp, t(gd["kat_w"]), t(gd["pD"]), t(gd["kat_zh_in"]), n_u)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(zh.cpu().numpy(), gd["kat_zhat"])
    np.testing.assert_array_equal(yp.cpu().numpy(), gd["kat_yp1"])


@pytest.mark.gpu
def test_flat_datafile_run(gpu, oracle):
    """ENABLE_FLATTEN_MATRICES data file -> gpad_setup_flat -> 100 iterations with the file's θ/β:
    bit-exact with the oracle's flat solve on the values read."""
    from gpad_mpc import datafile
    d = datafile.read(os.path.join(GOLDEN, "datafile_battery_flat_3x4.txt"), datafile.FILE_FLAT)
    import gpad_mpc
    s = gpad_mpc.GpadSolver(0)
    s.setup_flat(d.M_G, d.G_L, float(d.L), n_u=d.n_u)
    z = np.zeros(d.n, np.float32)
    y = np.zeros(d.m, np.float32)
    s.run(z, y, d.g_P, d.p_D, 100, 0.0, scaled=True, theta=d.theta, beta=d.beta)
    zo, yo, _, _ = oracle.solve_flat_f32(np.zeros(d.n), np.zeros(d.m), d.M_G, d.g_P, d.G_L, d.p_D, d.n_u,
                                         100, np.float32(d.L), theta=d.theta, beta=d.beta)
    np.testing.assert_array_equal(z, zo)
    np.testing.assert_array_equal(y, yo)


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", [0, 3])  # AUTO (register flat chains at this batch) / forced flat panels
@pytest.mark.parametrize("tol", [0.0, 1e-4])
def test_flat_closed_loop_bitexact(gpu, oracle, kernel, tol):
    """gpad.m:79-95 on flat battery data: gpad_setup_flat + gpad_setup_plant + gpad_closed_loop
    (per-state g_P, b on the device, the flat solve, x+ = A x + B u), cold start, 3 MPC steps,
    vs the oracle composed step by step (affine maps, flat solve, plant update) per pack."""
    import gpad_mpc
    from gpad_mpc import problems
    n_u, Nh, B, steps, N = 4, 10, 20, 3, 100
    qp, pl = problems.battery_plant(n_u, Nh)
    MGf, GLf, L = problems.flatten_battery(qp, n_u, Nh)
    c = lambda a: np.ascontiguousarray(np.asarray(a, np.float64).astype(np.float32))  # noqa: E731
    MGf32, GLf32, L32 = c(MGf), c(GLf), np.float32(L)
    PM, Pg, g0, A, Bm = c(pl.PM), c(pl.Pg), c(pl.g0), c(pl.A), c(pl.B)
    X0 = c(np.random.default_rng(7).random((B, n_u)) - 0.5)
    s = gpad_mpc.GpadSolver(0)
    s.setup_flat(MGf32, GLf32, float(L32), n_u=n_u, batch=B, kernel=kernel)
    s.setup_plant(PM, Pg, g0=g0, A=A, B=Bm)
    X = X0.copy()
    Z = np.zeros((B, qp.n), np.float32)
    Y = np.zeros((B, qp.m), np.float32)
    xs = np.zeros((steps, B, n_u), np.float32)
    us = np.zeros((steps, B, n_u), np.float32)
    it = np.zeros(steps * B, np.int32)
    s.closed_loop(X, Z, Y, steps, N, tol, xs=xs, us=us, iters=it)
    ninv = -1.0 / np.float64(L32)
    for b in range(B):
        x = X0[b].copy()
        for t in range(steps):
            gP = oracle.affine(PM, None, x)
            g = oracle.affine(Pg, g0, x)
            pD = (ninv * g.astype(np.float64)).astype(np.float32)
            z, y, its, _ = oracle.solve_flat_f32(np.zeros(qp.n), np.zeros(qp.m), MGf32, gP, GLf32, pD, n_u, N,
                                                 L32, tol)
            np.testing.assert_array_equal(xs[t, b], x, err_msg=f"x[{t}][{b}]")
            np.testing.assert_array_equal(us[t, b], z[:n_u], err_msg=f"u[{t}][{b}]")
            assert it[t * B + b] == its, (t, b)
            xn = np.zeros(n_u, np.float32)
            oracle.lib.orc_plant_step_f32(*(a.ctypes.data_as(oracle_fp()) for a in (A, Bm, x, z[:n_u].copy(), xn)),
                                          n_u, n_u)
            x = xn
        np.testing.assert_array_equal(X[b], x, err_msg=f"x_T[{b}]")
        np.testing.assert_array_equal(Z[b], z, err_msg=f"z[{b}]")
        np.testing.assert_array_equal(Y[b], y, err_msg=f"y[{b}]")


def oracle_fp():
    import ctypes
    return ctypes.POINTER(ctypes.c_float)


@pytest.mark.gpu
def test_flat_panel_grid_stride_large_batch(gpu, oracle):
    """40000 C1 packs on the flat panels (AUTO: 4 panels per workgroup, more groups than
    workgroups, so each workgroup loops over groups reusing its LDS), ragged last group; a
    sample of instances vs the oracle's flat solve, bit for bit."""
    import torch

    import gpad_mpc
    from gpad_mpc import problems
    n_u, Nh, B, N = 4, 10, 40000 + 7, 60
    qp = problems.battery_scenarios(n_u, Nh, B, seed=21)
    MGf, GLf, L = problems.flatten_battery(qp, n_u, Nh)
    f32 = lambda a: np.ascontiguousarray(np.asarray(a, np.float64).astype(np.float32))  # noqa: E731
    L32 = np.float32(L)
    MGf32, GLf32, GP = f32(MGf), f32(GLf), f32(qp.M)
    PD = np.ascontiguousarray(oracle.scale_vec(f32(qp.g), L32))
    t = lambda a: torch.from_numpy(a).to(gpu)  # noqa: E731
    s = gpad_mpc.GpadSolver(0)
    s.setup_flat(t(MGf32), t(GLf32), float(L32), n_u=n_u, batch=B)
    Z = torch.zeros(B, qp.n, device=gpu)
    Y = torch.zeros(B, qp.m, device=gpu)
    st = s.run(Z, Y, t(GP), t(PD), N, 0.0, scaled=True)
    assert st["kernel"] == "flat"
    Zc, Yc = Z.cpu().numpy(), Y.cpu().numpy()
    for b in list(range(0, B, 2311)) + [B - 1, B - 7]:
        z, y, _, _ = oracle.solve_flat_f32(np.zeros(qp.n), np.zeros(qp.m), MGf32, GP[b], GLf32, PD[b], n_u, N, L32)
        np.testing.assert_array_equal(Zc[b], z, err_msg=f"z[{b}]")
        np.testing.assert_array_equal(Yc[b], y, err_msg=f"y[{b}]")


@pytest.mark.gpu
@pytest.mark.parametrize("K,phase_len", [(1, 10), (3, 10), (7, 20)])
def test_flat_panel_phased_check_every(gpu, oracle, K, phase_len):
    """Flat-panel phases whose boundaries do not fall on the test grid (phase lengths that are not
    multiples of K, K = 1 testing every iteration): every instance bit-exact with the oracle."""
    from gpad_mpc import problems
    import gpad_mpc
    n_u, Nh, B = 4, 10, 16 * 5 + 3
    qp = problems.battery_scenarios(n_u, Nh, B, seed=17)
    MGf, GLf, L = problems.flatten_battery(qp, n_u, Nh)
    f32 = lambda a: np.ascontiguousarray(np.asarray(a, np.float64).astype(np.float32))  # noqa: E731
    L32 = np.float32(L)
    MGf32, GLf32, GP = f32(MGf), f32(GLf), f32(qp.M)
    PD = np.ascontiguousarray(oracle.scale_vec(f32(qp.g), L32))
    s = gpad_mpc.GpadSolver(0)
    s.setup_flat(MGf32, GLf32, float(L32), n_u=n_u, batch=B, kernel=gpad_mpc.KERNEL_PANEL, check_every=K)
    s.set_options(phase_len=phase_len, phased=2)
    Z = np.zeros((B, qp.n), np.float32)
    Y = np.zeros((B, qp.m), np.float32)
    it = np.zeros(B, np.int32)
    st = s.run(Z, Y, GP, PD, 4000, 1e-4, scaled=True, iters=it)
    assert st["kernel"] == "flat" and st["converged"] == B
    for b in range(0, B, 3):
        z, y, its, _ = oracle.solve_flat_f32(np.zeros(qp.n), np.zeros(qp.m), MGf32, GP[b], GLf32, PD[b], n_u, 4000,
                                             L32, 1e-4, check_every=K)
        assert it[b] == its, b
        np.testing.assert_array_equal(Z[b], z, err_msg=f"z[{b}]")
        np.testing.assert_array_equal(Y[b], y, err_msg=f"y[{b}]")
