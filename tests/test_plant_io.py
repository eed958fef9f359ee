"""Per-state QP data, closed-loop MPC and the reference data-file boundary (SURVEY.md §8f
rows 1 and 3; include/gpad.h gpad_setup_plant / gpad_run_state / gpad_closed_loop /
gpad_datafile_*).

CPU tests pin the oracle's closed loop against the fp64 restatement of gpad.m:79-95 and test
the data-file reader/writer (host code in libgpad, no GPU call).  GPU tests compare the HIP
path with the oracle bit for bit (fp32) and with the MATLAB restatement (fp64, 1e-9).
"""
from __future__ import annotations

import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, PKG, load_golden

F32 = lambda a: np.ascontiguousarray(np.asarray(a, np.float64).astype(np.float32))  # noqa: E731


def battery(n_u=3, N=4):
    from gpad_mpc import problems
    return problems.battery_plant(n_u, N)


# ---------------------------------------------------------------------------------- CPU
def test_oracle_closed_loop_vs_matlab_restatement(oracle):
    """fp32 oracle closed loop (gpad_closed_loop semantics) tracks the fp64 restatement of
    gpad.m:79-95 (golden) over 40 MPC steps.  Tolerance: 2e-6 absolute on the state of
    charge / 2e-5 on the currents (fp32 rounding of 100 GPAD iterations per step)."""
    gd = load_golden("closed_loop_battery_3x4")
    qp, pl = battery(3, 4)
    L = np.float32(qp.L)
    MGneg, GL, _ = oracle.scale(F32(qp.ML), F32(qp.G), F32(qp.g), L)
    steps = gd["xs"].shape[0]
    x, z, y, xs, us, iters = oracle.closed_loop_f32(gd["x0"], MGneg, GL, L, pl.PM, pl.Pg, pl.A, pl.B,
                                                    steps, 100, g0=pl.g0)
    assert (iters == 100).all()
    np.testing.assert_allclose(xs, gd["xs"], atol=2e-6, rtol=0)
    np.testing.assert_allclose(us, gd["us"], atol=2e-5, rtol=0)
    np.testing.assert_allclose(x, gd["x_final"], atol=2e-6, rtol=0)


def test_battery_plant_reproduces_per_state_qp():
    """M(x) = PM x and g(x) = g0 + Pg x equal gpad.m:81-85 + acceldualgrad.m:21 for any x."""
    from gpad_mpc import problems
    qp, pl = battery(4, 10)
    x = np.array([0.3, -0.2, 0.1, -0.4])
    ref = problems.battery_mpc(4, 10, x0=x)
    np.testing.assert_allclose(pl.PM @ x, ref.M, rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(pl.g0 + pl.Pg @ x, ref.g, rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(qp.ML, ref.ML, rtol=1e-12, atol=1e-15)
    assert qp.L == ref.L


@pytest.mark.parametrize("layout,fname", [(0, "datafile_battery_3x4.txt"),
                                          (1, "datafile_battery_3x4_flipped.txt")])
def test_datafile_reads_reference_format(layout, fname):
    """A main.cu:29-67 file written by plain numpy formatting reads back to the values fscanf
    would produce, in both matrix layouts."""
    from gpad_mpc import datafile
    gd = load_golden("datafile_battery_3x4")
    d = datafile.read(os.path.join(GOLDEN, fname), layout)
    assert (d.n_u, d.N, d.m, d.num_iterations) == (3, 4, 56, 120)
    assert np.float32(d.L) == gd["L"]
    for k in ("M_G", "g_P", "G_L", "p_D", "theta", "beta"):
        np.testing.assert_array_equal(getattr(d, k), gd[k], err_msg=k)


@pytest.mark.parametrize("layout", [0, 1])
def test_datafile_write_read_roundtrip_exact(tmp_path, layout):
    from gpad_mpc import datafile, problems
    qp = problems.battery_mpc(4, 10, seed=0)
    d = datafile.from_qp(qp, 4, 10, num_iterations=100)
    p = str(tmp_path / "input.txt")
    datafile.write(p, d, layout)
    r = datafile.read(p, layout)
    for k in ("M_G", "g_P", "G_L", "p_D", "theta", "beta"):
        np.testing.assert_array_equal(getattr(r, k), getattr(d, k), err_msg=k)
    assert np.float32(r.L) == np.float32(d.L)


def test_datafile_errors(tmp_path):
    from gpad_mpc import datafile
    from gpad_mpc._lib import GpadError
    with pytest.raises(GpadError):
        datafile.read(str(tmp_path / "missing.txt"))
    full = open(os.path.join(GOLDEN, "datafile_battery_3x4.txt")).read()
    (tmp_path / "trunc.txt").write_text(full[: len(full) // 2])
    with pytest.raises(GpadError, match="truncated"):
        datafile.read(str(tmp_path / "trunc.txt"))
    (tmp_path / "hdr.txt").write_text("3 4 x 100 1.0\n")
    with pytest.raises(GpadError, match="header"):
        datafile.read(str(tmp_path / "hdr.txt"))
    (tmp_path / "neg.txt").write_text("0 4 5 100 1.0\n")
    with pytest.raises(GpadError):
        datafile.read(str(tmp_path / "neg.txt"))


def test_driver_app_is_built():
    app = os.path.join(PKG, "gpad_mpc", "gpad_main")
    if not os.path.exists(app):
        subprocess.run(["make", "-s", "-C", PKG], check=True)
    assert os.access(app, os.X_OK)
    r = subprocess.run([app], capture_output=True, text=True)
    assert r.returncode == 2 and "usage" in r.stderr


# ---------------------------------------------------------------------------------- GPU
def _solver(qp, batch, kernel=None, dtype=np.float32):
    import gpad_mpc
    from gpad_mpc import _lib
    s = gpad_mpc.GpadSolver(0)
    c = (lambda a: np.ascontiguousarray(a, np.float64)) if dtype == np.float64 else F32
    L = float(qp.L) if dtype == np.float64 else float(np.float32(qp.L))
    s.setup(c(qp.ML), c(qp.G), L, n=qp.n, m=qp.m, batch=batch, shared=True,
            kernel=_lib.KERNEL_AUTO if kernel is None else kernel)
    return s, c


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [1, 5, 96])
@pytest.mark.parametrize("tol", [0.0, 1e-4])
def test_run_state_bitexact(gpu, oracle, batch, tol):
    """gpad_run_state == oracle(affine precompute + solve) for every instance (fp32)."""
    qp, pl = battery(4, 10)
    s, c = _solver(qp, batch)
    s.setup_plant(c(pl.PM), c(pl.Pg), g0=c(pl.g0))
    rng = np.random.default_rng(3)
    X = rng.uniform(-0.45, 0.45, (batch, 4)).astype(np.float32)
    Z = np.zeros((batch, qp.n), np.float32)
    Y = np.zeros((batch, qp.m), np.float32)
    it = np.zeros(batch, np.int32)
    st = s.run_state(X, Z, Y, 3000 if tol else 100, tol)
    s.last_stats(iters=it)
    L = np.float32(qp.L)
    MGneg, GL, _ = oracle.scale(F32(qp.ML), F32(qp.G), F32(qp.g), L)
    for b in range(batch):
        gP = oracle.affine(pl.PM, None, X[b])
        g = oracle.affine(pl.Pg, pl.g0, X[b])
        pD = oracle.scale_vec(g, L)
        z, y, its, conv = oracle.solve_scaled_f32(np.zeros(qp.n), np.zeros(qp.m), MGneg, gP, GL, pD,
                                                  3000 if tol else 100, L, tol)
        np.testing.assert_array_equal(Z[b], z, err_msg=f"z[{b}]")
        np.testing.assert_array_equal(Y[b], y, err_msg=f"y[{b}]")
        assert it[b] == its
    assert st["total_iterations"] == it.sum()


@pytest.mark.gpu
@pytest.mark.parametrize("batch,warm,tol,kernel", [(1, False, 0.0, None), (1, True, 1e-4, None),
                                                   (80, False, 1e-4, None), (80, True, 0.0, None),
                                                   (3, False, 1e-4, None), (80, False, 1e-4, 3),
                                                   (80, True, 1e-4, 3), (80, False, 0.0, 3)])
def test_closed_loop_bitexact(gpu, oracle, batch, warm, tol, kernel):
    """gpad_closed_loop (gpad.m:79-95 on the device) == the oracle's closed loop, every
    trajectory value and every per-step iteration count bit for bit (kernel 3 = panel)."""
    qp, pl = battery(3, 4)
    s, c = _solver(qp, batch, kernel=kernel)
    s.setup_plant(c(pl.PM), c(pl.Pg), g0=c(pl.g0), A=c(pl.A), B=c(pl.B))
    steps, N = 12, (2000 if tol else 100)
    rng = np.random.default_rng(batch)
    X0 = (rng.random((batch, 3)) - 0.5).astype(np.float32)
    X = X0.copy()
    Z = np.zeros((batch, qp.n), np.float32)
    Y = np.zeros((batch, qp.m), np.float32)
    XS = np.zeros((steps, batch, 3), np.float32)
    US = np.zeros((steps, batch, 3), np.float32)
    IT = np.zeros(steps * batch, np.int32)
    # codes are [steps][batch] like iters (a [batch]-sized array overflowed); a guard
    # tail past steps * batch must stay untouched
    CD = np.full(steps * batch + 16, -7, np.int32)
    st = s.closed_loop(X, Z, Y, steps, N, tol, warm=warm, xs=XS, us=US, iters=IT, codes=CD)
    assert (CD[steps * batch:] == -7).all()
    CD = CD[:steps * batch].reshape(steps, batch)
    assert ((CD > 0).sum() == st["converged"]) and (CD >= 0).all()
    if tol <= 0:
        assert (CD == 0).all()
    else:  # converged exactly where the step stopped before N
        np.testing.assert_array_equal(CD > 0, IT.reshape(steps, batch) < N)
    IT = IT.reshape(steps, batch)
    L = np.float32(qp.L)
    MGneg, GL, _ = oracle.scale(F32(qp.ML), F32(qp.G), F32(qp.g), L)
    for b in range(batch):
        x, z, y, xs, us, its = oracle.closed_loop_f32(X0[b], MGneg, GL, L, pl.PM, pl.Pg, pl.A, pl.B,
                                                      steps, N, tol, g0=pl.g0, warm=warm)
        np.testing.assert_array_equal(XS[:, b], xs, err_msg=f"xs[{b}]")
        np.testing.assert_array_equal(US[:, b], us, err_msg=f"us[{b}]")
        np.testing.assert_array_equal(X[b], x)
        np.testing.assert_array_equal(Z[b], z)
        np.testing.assert_array_equal(Y[b], y)
        np.testing.assert_array_equal(IT[:, b], its)
    assert st["total_iterations"] == IT.sum()


@pytest.mark.gpu
def test_closed_loop_f64_vs_matlab(gpu):
    """fp64 closed loop on the device vs the fp64 restatement of gpad.m (golden), 1e-9 abs."""
    gd = load_golden("closed_loop_battery_3x4")
    qp, pl = battery(3, 4)
    s, c = _solver(qp, 1, dtype=np.float64)
    s.setup_plant(c(pl.PM), c(pl.Pg), g0=c(pl.g0), A=c(pl.A), B=c(pl.B))
    steps = gd["xs"].shape[0]
    X = gd["x0"].reshape(1, 3).astype(np.float64).copy()
    Z = np.zeros((1, qp.n))
    Y = np.zeros((1, qp.m))
    XS = np.zeros((steps, 1, 3))
    US = np.zeros((steps, 1, 3))
    s.closed_loop(X, Z, Y, steps, 100, 0.0, xs=XS, us=US)
    np.testing.assert_allclose(XS[:, 0], gd["xs"], atol=1e-9, rtol=0)
    np.testing.assert_allclose(US[:, 0], gd["us"], atol=1e-9, rtol=0)
    np.testing.assert_allclose(X[0], gd["x_final"], atol=1e-9, rtol=0)


@pytest.mark.gpu
def test_closed_loop_device_memory(gpu, oracle):
    """Device-tensor closed loop (no host round trip, trajectories on the device)."""
    import torch
    import gpad_mpc
    from gpad_mpc import _lib
    qp, pl = battery(3, 4)
    batch, steps = 64, 6
    t = lambda a: torch.from_numpy(F32(a)).to(gpu)  # noqa: E731
    s = gpad_mpc.GpadSolver(0)
    s.setup(t(qp.ML), t(qp.G), float(np.float32(qp.L)), n=qp.n, m=qp.m, batch=batch)
    s.setup_plant(t(pl.PM), t(pl.Pg), g0=t(pl.g0), A=t(pl.A), B=t(pl.B))
    X0 = (np.random.default_rng(2).random((batch, 3)) - 0.5).astype(np.float32)
    X = torch.from_numpy(X0).to(gpu)
    Z = torch.zeros(batch, qp.n, device=gpu)
    Y = torch.zeros(batch, qp.m, device=gpu)
    XS = torch.zeros(steps, batch, 3, device=gpu)
    st = s.closed_loop(X, Z, Y, steps, 100, 0.0, xs=XS)
    # 64 packs: the latency kernel (AUTO picks panels above 4 instances per CU)
    assert st["kernel"] in ("resident", "panel") and st["total_iterations"] == 100 * steps * batch
    L = np.float32(qp.L)
    MGneg, GL, _ = oracle.scale(F32(qp.ML), F32(qp.G), F32(qp.g), L)
    for b in (0, 17, 63):
        x, z, y, xs, us, its = oracle.closed_loop_f32(X0[b], MGneg, GL, L, pl.PM, pl.Pg, pl.A, pl.B,
                                                      steps, 100, g0=pl.g0)
        np.testing.assert_array_equal(X[b].cpu().numpy(), x)
        np.testing.assert_array_equal(XS[:, b].cpu().numpy(), xs)


@pytest.mark.gpu
def test_plant_errors(gpu):
    import gpad_mpc
    from gpad_mpc._lib import GpadError
    qp, pl = battery(3, 4)
    s, c = _solver(qp, 1)
    X = np.zeros((1, 3), np.float32)
    Z = np.zeros((1, qp.n), np.float32)
    Y = np.zeros((1, qp.m), np.float32)
    with pytest.raises(GpadError, match="setup_plant"):
        s.run_state(X, Z, Y, 10)
    s.setup_plant(c(pl.PM), c(pl.Pg), g0=c(pl.g0))  # no dynamics
    s.run_state(X, Z, Y, 10)
    with pytest.raises(GpadError, match="without A, B"):
        s.closed_loop(X, Z, Y, 3, 10)
    s2 = gpad_mpc.GpadSolver(0)
    with pytest.raises(GpadError):
        s2.setup_plant(c(pl.PM), c(pl.Pg))  # before gpad_setup


@pytest.mark.gpu
@pytest.mark.parametrize("layout,fname", [(0, "datafile_battery_3x4.txt"),
                                          (1, "datafile_battery_3x4_flipped.txt")])
def test_datafile_run_matches_reference_steps(gpu, layout, fname):
    """File -> gpad_setup_scaled/run_scaled with the file's theta/beta, 100 iterations:
    bit-exact against the reference's own seq_functions.cpp run on the same values (golden)."""
    import gpad_mpc
    from gpad_mpc import datafile
    gd = load_golden("datafile_battery_3x4")
    d = datafile.read(os.path.join(GOLDEN, fname), layout)
    s = gpad_mpc.GpadSolver(0)
    s.setup(d.M_G, d.G_L, float(d.L), n=d.n, m=d.m, scaled=True)
    z = np.zeros(d.n, np.float32)
    y = np.zeros(d.m, np.float32)
    s.run(z, y, d.g_P, d.p_D, 100, 0.0, scaled=True, theta=d.theta, beta=d.beta)
    np.testing.assert_array_equal(z, gd["ref_z_100"])
    np.testing.assert_array_equal(y, gd["ref_y_100"])


@pytest.mark.gpu
def test_driver_app_matches_reference_steps(gpu):
    """apps/gpad_main.c (main.cu on the C-ABI) prints the reference's 100-iteration result."""
    app = os.path.join(PKG, "gpad_mpc", "gpad_main")
    gd = load_golden("datafile_battery_3x4")
    for flag in ([], ["--flipped"]):
        fname = "datafile_battery_3x4_flipped.txt" if flag else "datafile_battery_3x4.txt"
        r = subprocess.run([app, os.path.join(GOLDEN, fname), *flag], capture_output=True, text=True,
                           timeout=120)
        assert r.returncode == 0, r.stderr
        lines = {ln.split()[0]: ln.split()[1:] for ln in r.stdout.splitlines()}
        z = np.array([np.float32(v) for v in lines["z"]], np.float32)
        y = np.array([np.float32(v) for v in lines["y"]], np.float32)
        np.testing.assert_array_equal(z, gd["ref_z_100"])
        np.testing.assert_array_equal(y, gd["ref_y_100"])
        assert lines["iterations"][0] == "100"
