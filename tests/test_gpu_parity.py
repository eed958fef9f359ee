"""GPU parity tests: the HIP path (libgpad.so, called through its C-ABI) against the oracle.

Bar: fp32 results are BIT-EXACT with the reference CPU arithmetic (every kernel computes one
sequential fmaf chain per row, as seq_functions.cpp does under FMA contraction); fp64 results
match the fp64 oracle / MATLAB restatement within 1e-12 relative (elementwise op order of
acceldualgrad.m vs seq_functions.cpp differs in the last bit).
"""
from __future__ import annotations

import numpy as np
import pytest

from conftest import GOLDEN_SETS, f32_inputs, load_golden

pytestmark = pytest.mark.gpu

KERNELS = ["stream", "resident", "panel"]


def kcode(name):
    from gpad_mpc import _lib
    return {"auto": _lib.KERNEL_AUTO, "stream": _lib.KERNEL_STREAM, "resident": _lib.KERNEL_RESIDENT,
            "panel": _lib.KERNEL_PANEL}[name]


def run_gpu(ML, M, G, g, L, N, tol=0.0, z0=None, y0=None, kernel="auto", shared=True,
            schedule=0, check_every=10, opts=None, tol_gap=0.0):
    import gpad_mpc
    n, m = ML.shape[-2], ML.shape[-1]
    batch = M.shape[0] if M.ndim == 2 else 1
    z = np.zeros((batch, n) if batch > 1 else n, ML.dtype) if z0 is None else np.array(z0, ML.dtype)
    y = np.zeros((batch, m) if batch > 1 else m, ML.dtype) if y0 is None else np.array(y0, ML.dtype)
    iters = np.zeros(batch, np.int32)
    with gpad_mpc.GpadSolver(0) as s:
        s.setup(np.ascontiguousarray(ML), np.ascontiguousarray(G), float(L), n=n, m=m, batch=batch,
                shared=shared, kernel=kcode(kernel), schedule=schedule, check_every=check_every,
                tol_gap=tol_gap)
        s.set_options(**(opts or {}))
        st = s.run(z, y, np.ascontiguousarray(M), np.ascontiguousarray(g), N, tol, iters=iters)
    return z, y, st, iters


def assert_bitexact(a, b, what=""):
    a = np.asarray(a)
    b = np.asarray(b)
    assert a.shape == b.shape, what
    if not np.array_equal(a, b):
        d = np.abs(a.astype(np.float64) - b.astype(np.float64))
        i = int(np.argmax(d))
        raise AssertionError(f"{what}: {int((d > 0).sum())} of {a.size} differ, max |d| = {d.max():.3g}"
                             f" at {i} ({a.flat[i]!r} vs {b.flat[i]!r})")


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("name", GOLDEN_SETS)
@pytest.mark.parametrize("K", [1, 10, 100])
def test_fixed_iterations_bitexact_vs_reference(gpu, kernel, name, K):
    gd = load_golden(name)
    ML, M, G, g, L = f32_inputs(gd)
    z, y, st, _ = run_gpu(ML, M, G, g, L, K, kernel=kernel)
    assert st["kernel"] == kernel and st["iterations"] == K
    assert_bitexact(z, gd[f"ref_z_{K}"], f"{name} z K={K}")
    assert_bitexact(y, gd[f"ref_y_{K}"], f"{name} y K={K}")


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("name", GOLDEN_SETS)
def test_warm_start_bitexact(gpu, kernel, name):
    gd = load_golden(name)
    ML, M, G, g, L = f32_inputs(gd)
    z, y, _, _ = run_gpu(ML, M, G, g, L, 50, z0=gd["warm_z0"], y0=gd["warm_y0"], kernel=kernel)
    assert_bitexact(z, gd["ref_warm_z_50"], "warm z")
    assert_bitexact(y, gd["ref_warm_y_50"], "warm y")


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("name", GOLDEN_SETS)
def test_algorithm1_termination_bitexact(gpu, kernel, name):
    gd = load_golden(name)
    ML, M, G, g, L = f32_inputs(gd)
    z, y, st, iters = run_gpu(ML, M, G, g, L, 5000, tol=1e-4, kernel=kernel)
    assert st["converged"] == 1 and st["iterations"] == int(gd["tol_iters"])
    assert_bitexact(z, gd["tol_z"], "tol z")
    assert_bitexact(y, gd["tol_y"], "tol y")


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("nm", [(200, 200), (37, 53), (1, 5), (5, 1), (64, 64), (65, 129), (208, 180),
                                (256, 250), (144, 129), (193, 201), (201, 193), (199, 200), (192, 200),
                                (200, 8), (8, 196)])
def test_shapes_bitexact_vs_oracle(gpu, oracle, kernel, nm):
    """C2 (200 x 200) and ragged shapes (not multiples of 4 / 64, single row or column)."""
    from gpad_mpc import problems
    n, m = nm
    if kernel == "resident" and max(n, m) > 208:
        pytest.skip("resident kernel holds at most 208 rows per lane chain")
    qp = problems.synthetic_qp(n, m, seed=11)
    ML, M, G, g = (qp.ML.astype(np.float32), qp.M.astype(np.float32), qp.G.astype(np.float32),
                   qp.g.astype(np.float32))
    L = np.float32(qp.L)
    zo, yo, _, _ = oracle.solve_f32(np.zeros(n), np.zeros(m), ML, M, G, g, 100, L)
    z, y, st, _ = run_gpu(ML, M, G, g, L, 100, kernel=kernel)
    assert_bitexact(z, zo, f"{nm} z")
    assert_bitexact(y, yo, f"{nm} y")


@pytest.mark.parametrize("nm", [(800, 800), (300, 1000), (1500, 257)])
def test_large_shapes_stream_bitexact(gpu, oracle, nm):
    """C5-sized instances (n = m = 800) and beyond the resident kernel's register budget."""
    from gpad_mpc import problems
    n, m = nm
    qp = problems.synthetic_qp(n, m, seed=5)
    ML, M, G, g = (qp.ML.astype(np.float32), qp.M.astype(np.float32), qp.G.astype(np.float32),
                   qp.g.astype(np.float32))
    L = np.float32(qp.L)
    zo, yo, _, _ = oracle.solve_f32(np.zeros(n), np.zeros(m), ML, M, G, g, 20, L)
    z, y, st, _ = run_gpu(ML, M, G, g, L, 20, kernel="auto")
    assert st["kernel"] == "stream"
    assert_bitexact(z, zo, "z")
    assert_bitexact(y, yo, "y")


@pytest.mark.parametrize("kernel", ["auto", "stream", "resident", "panel"])
def test_shared_batch_bitexact_per_instance(gpu, oracle, kernel):
    """A battery-scenario-style batch: shared ML/G, per-instance M and g, Algorithm 1."""
    from gpad_mpc import problems
    B, n, m = 37, 40, 64
    qp = problems.synthetic_qp(n, m, batch=B, seed=2)
    ML, G = qp.ML.astype(np.float32), qp.G.astype(np.float32)
    M, g = qp.M.astype(np.float32), qp.g.astype(np.float32)
    L = np.float32(qp.L)
    z, y, st, iters = run_gpu(ML, M, G, g, L, 3000, tol=1e-4, kernel=kernel)
    for b in range(B):
        zo, yo, it, conv = oracle.solve_f32(np.zeros(n), np.zeros(m), ML, M[b], G, g[b], 3000, L, 1e-4)
        assert iters[b] == it
        assert_bitexact(z[b], zo, f"instance {b} z")
        assert_bitexact(y[b], yo, f"instance {b} y")
    assert st["converged"] == B and st["total_iterations"] == int(iters.sum())


@pytest.mark.parametrize("kernel", ["stream", "resident"])
def test_distinct_batch_bitexact(gpu, oracle, kernel):
    from gpad_mpc import problems
    B, n, m = 9, 48, 72
    qp = problems.synthetic_qp(n, m, batch=B, seed=4, shared=False)
    f = lambda a: np.ascontiguousarray(a.astype(np.float32))  # noqa: E731
    ML, G, M, g, L = f(qp.ML), f(qp.G), f(qp.M), f(qp.g), np.float32(qp.L)
    z, y, st, iters = run_gpu(ML, M, G, g, L, 60, kernel=kernel, shared=False)
    for b in range(B):
        zo, yo, _, _ = oracle.solve_f32(np.zeros(n), np.zeros(m), ML[b], M[b], G[b], g[b], 60, L)
        assert_bitexact(z[b], zo, f"instance {b} z")
        assert_bitexact(y[b], yo, f"instance {b} y")


@pytest.mark.parametrize("nm", [(40, 64), (200, 200)])
def test_panel_two_wave_panels_large_batch(gpu, oracle, nm):
    """>= 512 panels selects 2-wave panels; spot-check instances across the whole grid."""
    from gpad_mpc import problems
    n, m = nm
    B = 8192 + 5  # ragged last panel
    base = problems.synthetic_qp(n, m, batch=1, seed=21)
    rng = np.random.default_rng(0)
    M = (base.M[None, :] * (1.0 + 0.3 * rng.normal(size=(B, 1)))).astype(np.float32)
    g = (base.g[None, :] + 0.2 * rng.random((B, m))).astype(np.float32)
    ML, G, L = base.ML.astype(np.float32), base.G.astype(np.float32), np.float32(base.L)
    z, y, st, iters = run_gpu(ML, M, G, g, L, 2000, tol=1e-4, kernel="panel")
    assert st["kernel"] == "panel"
    for b in list(range(0, B, 257)) + [B - 1]:
        zo, yo, it, _ = oracle.solve_f32(np.zeros(n), np.zeros(m), ML, M[b], G, g[b], 2000, L, 1e-4)
        assert iters[b] == it, b
        assert_bitexact(z[b], zo, f"instance {b} z")
        assert_bitexact(y[b], yo, f"instance {b} y")


@pytest.mark.parametrize("grid,phase,fin", [(1, 0, None), (3, 0, 0), (0, 10, 0), (3, 20, 24),
                                            (0, 0, None), (0, 10, 24)])
@pytest.mark.parametrize("tol,N", [(1e-4, 3000), (0.0, 57)])
@pytest.mark.parametrize("nm,B", [((40, 72), 150), ((150, 130), 40), ((131, 256), 37), ((200, 200), 120),
                                  ((193, 207), 101), ((207, 194), 70), ((140, 135), 90), ((170, 176), 80)])
def test_panel_phased_compaction_bitexact(gpu, oracle, grid, phase, fin, tol, N, nm, B):
    """Phased compaction + grid-stride panels (+ panel pairs for T > 8 when panels outnumber
    workgroups) + the resident finisher for the tail (fin = its threshold; 0 disables it);
    n, m in (192, 208], (160, 176] and (128, 144] run the panel pairs' chain hand-off (T = 13, 11,
    9, gpad_panel.hip Handoff; one-panel relays at T = 13, 9) with the receiver's last k-block at
    every kq:
    survivors of each phase are re-packed into new panels (different columns, workgroups,
    pairs and phases) or finished one per workgroup; every instance must still match its own
    oracle solve exactly, including its iteration count."""
    from gpad_mpc import problems
    opts = dict(panel_max_grid=grid, phase_len=phase, finish_thresh=-1 if fin is None else fin)
    n, m = nm
    qp = problems.synthetic_qp(n, m, batch=B, seed=8)
    ML, G = qp.ML.astype(np.float32), qp.G.astype(np.float32)
    M, g = qp.M.astype(np.float32), qp.g.astype(np.float32)
    L = np.float32(qp.L)
    rng = np.random.default_rng(1)
    z0 = (0.1 * rng.normal(size=(B, n))).astype(np.float32)  # warm starts: exercises the u seed
    y0 = np.abs(0.1 * rng.normal(size=(B, m))).astype(np.float32)  # and every state load per instance
    z, y, st, iters = run_gpu(ML, M, G, g, L, N, tol=tol, kernel="panel", z0=z0, y0=y0, opts=opts)
    assert st["kernel"] == "panel"
    for b in range(B):
        zo, yo, it, _ = oracle.solve_f32(z0[b], y0[b], ML, M[b], G, g[b], N, L, tol)
        assert iters[b] == it, b
        assert_bitexact(z[b], zo, f"instance {b} z")
        assert_bitexact(y[b], yo, f"instance {b} y")


@pytest.mark.parametrize("tol,N", [(1e-4, 2000), (0.0, 37)])
@pytest.mark.parametrize("nm,B", [((200, 900), 40), ((300, 300), 20), ((257, 130), 33), ((520, 600), 17), ((1000, 300), 9)])
@pytest.mark.parametrize("grid,phase", [(0, 0), (2, 20)])
def test_bigpanel_bitexact(gpu, oracle, tol, N, nm, B, grid, phase):
    """Shared matrices beyond 256 rows on the big-panel MFMA kernel (gpad_bigpanel.hip): GEMMs of
    different tile counts, up to 4 row tiles per wave, grid-stride panels and phases; every
    instance must match its own oracle solve exactly, iteration count included."""
    from gpad_mpc import problems
    opts = dict(panel_max_grid=grid, phase_len=phase)
    n, m = nm
    qp = problems.synthetic_qp(n, m, batch=B, seed=17)
    ML, G = qp.ML.astype(np.float32), qp.G.astype(np.float32)
    M, g = qp.M.astype(np.float32), qp.g.astype(np.float32)
    L = np.float32(qp.L)
    rng = np.random.default_rng(3)
    z0 = (0.1 * rng.normal(size=(B, n))).astype(np.float32)
    z, y, st, iters = run_gpu(ML, M, G, g, L, N, tol=tol, kernel="panel", z0=z0, opts=opts)
    assert st["kernel"] == "panel"
    for b in range(B):
        zo, yo, it, _ = oracle.solve_f32(z0[b], np.zeros(m), ML, M[b], G, g[b], N, L, tol)
        assert iters[b] == it, b
        assert_bitexact(z[b], zo, f"instance {b} z")
        assert_bitexact(y[b], yo, f"instance {b} y")


@pytest.mark.parametrize("grid", [1, 3, 5, 0])
@pytest.mark.parametrize("nm,B,z0s", [((200, 200), 120, 0.0), ((40, 180), 200, 0.1), ((131, 64), 97, 0.1)])
def test_finisher_queue_bitexact(gpu, oracle, grid, nm, B, z0s):
    """The tail of a phased panel solve on the duo finisher (two instances per workgroup in
    ping-pong, slots refilled from the survivor list through a device counter; grid capped to 1, 3
    or 5 workgroups to force many claims).  The finisher takes over after the first 10-iteration
    phase, so nearly the whole solve runs there; every instance must match its own oracle solve,
    iteration count included."""
    from gpad_mpc import problems
    opts = dict(phase_len=10, finish_thresh=100000, duo_max_grid=grid)
    n, m = nm
    qp = problems.synthetic_qp(n, m, batch=B, seed=12)
    ML, G = qp.ML.astype(np.float32), qp.G.astype(np.float32)
    M, g = qp.M.astype(np.float32), qp.g.astype(np.float32)
    L = np.float32(qp.L)
    rng = np.random.default_rng(2)
    z0 = (z0s * rng.normal(size=(B, n))).astype(np.float32)
    N = 1500
    z, y, st, iters = run_gpu(ML, M, G, g, L, N, tol=1e-4, kernel="panel", z0=z0, opts=opts)
    assert st["kernel"] == "panel"
    assert iters.min() > 10  # the finisher ran every instance's tail
    for b in range(B):
        zo, yo, it, _ = oracle.solve_f32(z0[b], np.zeros(m), ML, M[b], G, g[b], N, L, 1e-4)
        assert iters[b] == it, b
        assert_bitexact(z[b], zo, f"instance {b} z")
        assert_bitexact(y[b], yo, f"instance {b} y")


@pytest.mark.parametrize("fin", [None, 0])
def test_panel_phase_plan_reuse_bitexact(gpu, oracle, fin):
    """A handle plans its phases from the previous solve's iteration counts (csrc/gpad_panel.hip
    panel_plan); a later solve that needs more (or fewer) iterations than the plan expects must
    still be exact -- the plan moves launch boundaries and the finisher takeover only."""
    import gpad_mpc
    from gpad_mpc import problems
    n, m, B = 40, 72, 300
    qp = problems.synthetic_qp(n, m, batch=B, seed=31)
    ML, G = qp.ML.astype(np.float32), qp.G.astype(np.float32)
    L = np.float32(qp.L)
    rng = np.random.default_rng(5)
    with gpad_mpc.GpadSolver(0) as s:
        s.setup(ML, G, float(L), n=n, m=m, batch=B, kernel=kcode("panel"))
        s.set_options(phase_len=10, finish_thresh=-1 if fin is None else fin)
        for scale, tol in ((1.0, 1e-3), (3.0, 1e-5), (1.0, 1e-4)):  # easy, harder, middle
            M = (qp.M * scale).astype(np.float32)
            g = (qp.g + 0.1 * rng.random((B, m))).astype(np.float32)
            z = np.zeros((B, n), np.float32)
            y = np.zeros((B, m), np.float32)
            it = np.zeros(B, np.int32)
            plan = s.phase_plan()
            st = s.run(z, y, M, g, 4000, tol, iters=it)
            assert st["kernel"] == "panel"
            if scale != 1.0 or tol != 1e-3:  # planned from the previous solve
                assert plan["ends"] and plan["ends"][-1] == 4000, plan
            for b in range(0, B, 7):
                zo, yo, ito, _ = oracle.solve_f32(np.zeros(n), np.zeros(m), ML, M[b], G, g[b], 4000, L, tol)
                assert it[b] == ito, (scale, b)
                assert_bitexact(z[b], zo, f"{scale} z[{b}]")
                assert_bitexact(y[b], yo, f"{scale} y[{b}]")


def test_async_runs_plan_from_previous_solve(gpu, oracle):
    """Asynchronous solves (device tensors, stats=False) never sync for counts: each phased solve
    copies its counts to pinned host memory behind it and the next run plans from them once they
    landed (csrc/gpad_host.cpp run_typed).  The plan appears without any stats call, and the
    planned solve of a different batch is still exact."""
    import torch
    import gpad_mpc
    from gpad_mpc import problems
    n, m, B, N, tol = 40, 72, 300, 4000, 1e-4
    qp = problems.synthetic_qp(n, m, batch=B, seed=33)
    ML, G = qp.ML.astype(np.float32), qp.G.astype(np.float32)
    L = np.float32(qp.L)
    rng = np.random.default_rng(9)
    with gpad_mpc.GpadSolver(0) as s:
        s.setup(torch.from_numpy(ML).to(gpu), torch.from_numpy(G).to(gpu), float(L), n=n, m=m, batch=B,
                kernel=kcode("panel"))
        s.set_options(phase_len=10)
        assert s.phase_plan()["ends"] == []
        for k in range(3):
            M = (qp.M * (1.0 + 0.5 * k)).astype(np.float32)
            g = (qp.g + 0.1 * rng.random((B, m))).astype(np.float32)
            dz = torch.zeros((B, n), device=gpu)
            dy = torch.zeros((B, m), device=gpu)
            assert s.run(dz, dy, torch.from_numpy(M).to(gpu), torch.from_numpy(g).to(gpu), N, tol,
                         stats=False) is None
            plan = s.phase_plan()
            if k > 0:  # the previous solve finished (synchronised below) -> its counts planned this one
                assert plan["ends"] and plan["ends"][-1] == N, plan
            torch.cuda.synchronize()
            z, y = dz.cpu().numpy(), dy.cpu().numpy()
            for b in range(0, B, 11):
                zo, yo, _, _ = oracle.solve_f32(np.zeros(n), np.zeros(m), ML, M[b], G, g[b], N, L, tol)
                assert_bitexact(z[b], zo, f"{k} z[{b}]")
                assert_bitexact(y[b], yo, f"{k} y[{b}]")


def test_paper_schedule_bitexact(gpu, oracle):
    gd = load_golden("battery_c1")
    ML, M, G, g, L = f32_inputs(gd)
    n, m = ML.shape
    zo, yo, _, _ = oracle.solve_f32(np.zeros(n), np.zeros(m), ML, M, G, g, 100, L, schedule=1)
    for k in KERNELS:
        z, y, _, _ = run_gpu(ML, M, G, g, L, 100, kernel=k, schedule=1)
        assert_bitexact(z, zo, k)
        assert_bitexact(y, yo, k)


@pytest.mark.parametrize("name", GOLDEN_SETS)
def test_f64_vs_matlab_restatement(gpu, oracle, name):
    gd = load_golden(name)
    n, m = gd["ML"].shape
    z, y, st, _ = run_gpu(gd["ML"], gd["M"], gd["G"], gd["g"], float(gd["L"]), 100)
    assert st["kernel"] == "stream"
    rel = lambda a, b: np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)  # noqa: E731
    assert rel(z, gd["matlab_z_100"]) < 1e-12 and rel(y, gd["matlab_y_100"]) < 1e-12
    zo, yo, _, _ = oracle.solve_f64(np.zeros(n), np.zeros(m), gd["ML"], gd["M"], gd["G"], gd["g"],
                                    100, float(gd["L"]))
    assert rel(z, zo) < 1e-12 and rel(y, yo) < 1e-12


def test_zero_iterations_returns_inputs(gpu):
    gd = load_golden("synth_small")
    ML, M, G, g, L = f32_inputs(gd)
    z0 = np.linspace(-1, 1, ML.shape[0]).astype(np.float32)
    y0 = np.linspace(0, 1, ML.shape[1]).astype(np.float32)
    for k in KERNELS:
        z, y, st, _ = run_gpu(ML, M, G, g, L, 0, z0=z0, y0=y0, kernel=k)
        assert st["iterations"] == 0
        assert_bitexact(z, z0)
        assert_bitexact(y, y0)


def test_step_entry_points_vs_kats(gpu, oracle):
    """gpad_step1..4 (the kernel_functions.h mirror) on device tensors vs the reference KATs."""
    import torch
    import gpad_mpc
    gd = load_golden("battery_c1")
    ML, M, G, g, L = f32_inputs(gd)
    MGneg, GL, pD = oracle.scale(ML, G, g, L)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(gpu)  # noqa: E731
    n, m = MGneg.shape
    y, ym1, zm1 = t(gd["kat_y"]), t(gd["kat_ym1"]), t(gd["kat_zm1"])
    w, zh, z, yp = (torch.empty(m, device=gpu), torch.empty(n, device=gpu), torch.empty(n, device=gpu),
                    torch.empty(m, device=gpu))
    with gpad_mpc.GpadSolver(0) as s:
        s.step1(y, ym1, w, float(gd["kat_beta"]))
        s.step2(t(MGneg), w, t(M), zh)
        s.step3(float(gd["kat_theta"]), zm1, zh, z)
        s.step4(t(GL), yp, w, t(pD), zh)
        s.sync()
    assert_bitexact(w.cpu().numpy(), gd["kat_w"], "8a")
    assert_bitexact(zh.cpu().numpy(), gd["kat_zhat"], "8b")
    assert_bitexact(z.cpu().numpy(), gd["kat_z"], "8c")
    assert_bitexact(yp.cpu().numpy(), gd["kat_yp1"], "8d")


@pytest.mark.parametrize("k", [1, 2, 3, 4, 5])
def test_step3_reference_fixtures_on_gpu(gpu, oracle, k):
    import torch
    import gpad_mpc
    from test_oracle import read_step3
    n_u, N, m, theta, zm1, zhat, out = read_step3(k)
    z = torch.empty(zm1.size, device=gpu)
    with gpad_mpc.GpadSolver(0) as s:
        s.step3(float(theta), torch.from_numpy(zm1).to(gpu), torch.from_numpy(zhat).to(gpu), z)
        s.sync()
    zz = z.cpu().numpy()
    assert_bitexact(zz, oracle.step3(theta, zm1, zhat))
    assert np.max(np.abs(zz - out)) <= 1e-6 * max(1.0, float(np.max(np.abs(out))))


def test_device_memory_async_and_one_shot_solve(gpu, oracle):
    """Device tensors (MEM_DEVICE, async launch + last_stats) and the one-shot gpad_solve."""
    import torch
    import gpad_mpc
    from gpad_mpc import problems
    B, n, m = 20, 56, 88
    qp = problems.synthetic_qp(n, m, batch=B, seed=9)
    f = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(gpu)  # noqa: E731
    ML, G, M, g = f(qp.ML), f(qp.G), f(qp.M), f(qp.g)
    z = torch.zeros(B, n, device=gpu)
    y = torch.zeros(B, m, device=gpu)
    with gpad_mpc.GpadSolver(0) as s:
        s.setup(ML, G, float(np.float32(qp.L)), n=n, m=m, batch=B)
        assert s.run(z, y, M, g, 500, 1e-4, stats=False) is None
        s.sync()
        st = s.last_stats()
    zo, yo, it, _ = oracle.solve_f32(np.zeros(n), np.zeros(m), qp.ML.astype(np.float32),
                                     qp.M[3].astype(np.float32), qp.G.astype(np.float32),
                                     qp.g[3].astype(np.float32), 500, np.float32(qp.L), 1e-4)
    assert_bitexact(z[3].cpu().numpy(), zo)
    assert_bitexact(y[3].cpu().numpy(), yo)
    assert st["iterations"] >= it and st["kernel_ms"] > 0
    z2, y2, st2 = gpad_mpc.solve(np.zeros((B, n)), np.zeros((B, m)), qp.ML.astype(np.float32),
                                 qp.M.astype(np.float32), qp.G.astype(np.float32),
                                 qp.g.astype(np.float32), 500, float(np.float32(qp.L)), 1e-4)
    assert_bitexact(z2, z.cpu().numpy())


@pytest.mark.parametrize("kernel", ["panel", "resident", "stream"])
def test_async_runs_ordered_after_torch_work(gpu, oracle, kernel):
    """Back-to-back asynchronous runs on torch's current stream with torch ops in between (no
    host sync): every run must see the zeroed state (regression: a private stream raced)."""
    import torch
    import gpad_mpc
    from gpad_mpc import problems
    B, n, m = 300, 48, 80
    qp = problems.synthetic_qp(n, m, batch=B, seed=31)
    f = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(gpu)  # noqa: E731
    ML, G, M, g = f(qp.ML), f(qp.G), f(qp.M), f(qp.g)
    z = torch.empty(B, n, device=gpu)
    y = torch.empty(B, m, device=gpu)
    with gpad_mpc.GpadSolver(0) as s:
        s.setup(ML, G, float(np.float32(qp.L)), n=n, m=m, batch=B, kernel=kcode(kernel))
        for _ in range(4):
            z.fill_(7.0)
            y.fill_(3.0)
            z.zero_()
            y.zero_()
            s.run(z, y, M, g, 3000, 1e-4, stats=False)
        iters = np.zeros(B, np.int32)
        s.last_stats(iters=iters)
    for b in (0, 57, B - 1):
        zo, yo, it, _ = oracle.solve_f32(np.zeros(n), np.zeros(m), qp.ML.astype(np.float32),
                                         qp.M[b].astype(np.float32), qp.G.astype(np.float32),
                                         qp.g[b].astype(np.float32), 3000, np.float32(qp.L), 1e-4)
        assert iters[b] == it
        assert_bitexact(z[b].cpu().numpy(), zo)
        assert_bitexact(y[b].cpu().numpy(), yo)


def test_error_paths(gpu):
    import gpad_mpc
    from gpad_mpc import _lib
    s = gpad_mpc.GpadSolver(0)
    z = np.zeros(4, np.float32)
    with pytest.raises(gpad_mpc.GpadError) as e:
        s.run(z, z, z, z, 10, 0.0)
    assert e.value.code == _lib.ERR_NOT_SETUP
    big = np.zeros((300, 300), np.float32)
    s.setup(big, big, 1.0, n=300, m=300, kernel=_lib.KERNEL_RESIDENT)
    with pytest.raises(gpad_mpc.GpadError) as e:
        s.run(np.zeros(300, np.float32), np.zeros(300, np.float32), np.zeros(300, np.float32),
              np.zeros(300, np.float32), 10, 0.0)
    assert e.value.code == _lib.ERR_UNSUPPORTED
    for name, bad in (("lpt", 2), (99, 1)) + tuple((r, 0) for r in _lib.OPT_RETIRED):
        with pytest.raises(gpad_mpc.GpadError) as e:  # out of range / unknown / retired
            s.set_option(name, bad)
        assert e.value.code == _lib.ERR_INVALID
    s.set_option("lpt", _lib.OPT_DEFAULT)
    with pytest.raises(gpad_mpc.GpadError) as e:  # the removed condensed operator (0.4)
        s.setup(np.zeros((8, 8), np.float32), np.zeros((8, 8), np.float32), 1.0, n=8, m=8, kernel=5)
    assert e.value.code == _lib.ERR_INVALID
    s.close()


def test_acceldualgrad_mirror(gpu):
    """The MATLAB-signature mirror returns u = z(1:n_u) of the fp64 path."""
    import gpad_mpc
    gd = load_golden("battery_10x4")
    u, z, y = gpad_mpc.acceldualgrad(gd["H"], gd["q"], gd["G"], gd["g"], None, None, 10)
    assert np.allclose(u, gd["matlab_z_100"][:10], rtol=1e-12, atol=1e-14)


@pytest.mark.gpu
def test_accumulate_iterations_matches_stats(gpu):
    """gpad_accumulate_iterations (bench.py's sync-free work count) equals the per-instance counts
    the stats path reports, summed over back-to-back asynchronous runs (phased panel solves)."""
    import torch

    import bench
    import gpad_mpc
    n, m, B = 200, 200, 1500
    ML, G, L, M, g = bench.make_shard(n, m, B, 0)
    f32 = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(gpu)  # noqa: E731
    dML, dG, dM, dg = f32(ML), f32(G), f32(M), f32(g)
    z = torch.zeros(B, n, device=gpu)
    y = torch.zeros(B, m, device=gpu)
    s = gpad_mpc.GpadSolver(0)
    s.setup(dML, dG, float(np.float32(L)), n=n, m=m, batch=B, shared=True)
    acc = torch.zeros(1, dtype=torch.int64, device=gpu)
    for _ in range(3):
        s.run(z.zero_(), y.zero_(), dM, dg, 5000, 1e-4, stats=False)
        s.accumulate_iterations(acc)
    it = np.zeros(B, np.int32)
    st = s.last_stats(iters=it)
    assert int(acc.item()) == 3 * int(it.sum()) == 3 * st["total_iterations"]


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("tol,tol_gap", [(1e-4, 1e-2), (1e-3, 1e-7)])
def test_separate_gap_tolerance_bitexact(gpu, oracle, kernel, tol, tol_gap):
    """e_g and e_V (acceldualgrad.m:12-13) as separate tolerances: tol bounds the constraint
    violation of both tests, tol_gap the duality-gap term of test (B); every kernel family
    stops at the oracle's iteration with the oracle's z*, y* and convergence code."""
    from gpad_mpc import problems
    B = 300 if kernel == "panel" else 24
    qp = problems.synthetic_qp(64, 96, batch=B, seed=21)
    ML, G = qp.ML.astype(np.float32), qp.G.astype(np.float32)
    M, g = qp.M.astype(np.float32), qp.g.astype(np.float32)
    L = np.float32(qp.L)
    z, y, st, iters = run_gpu(ML, M, G, g, L, 4000, tol=tol, kernel=kernel, tol_gap=tol_gap)
    assert st["kernel"] == kernel
    for b in range(0, B, 7 if kernel == "panel" else 1):
        zo, yo, it, _ = oracle.solve_f32(np.zeros(64), np.zeros(96), ML, M[b], G, g[b], 4000, L, tol,
                                         tol_gap=tol_gap)
        assert iters[b] == it, b
        assert_bitexact(z[b], zo, f"{b} z")
        assert_bitexact(y[b], yo, f"{b} y")


def test_panel_phased_beyond_lds_compaction_bitexact(gpu, oracle):
    """A phased solve whose first boundary lists more panels than the compaction keeps in LDS
    (> kCompactMaxPanels = 8192, i.e. > 131072 instances; > 8 panels per compaction thread): the
    global-memory compaction path.  Two solves on one handle (default schedule, then planned);
    a sample of instances, the ragged last panel included, must match the oracle exactly, counts
    included, and every instance must converge."""
    import gpad_mpc
    from gpad_mpc import problems
    n = m = 136  # T = 9 panel pairs
    B = 140003
    base = problems.synthetic_qp(n, m, batch=1, seed=21)
    ML, G = base.ML.astype(np.float32), base.G.astype(np.float32)
    L = np.float32(base.L)
    rng = np.random.default_rng(22)
    Hinv = np.linalg.inv(base.H)
    M = (rng.normal(0.0, 1.0, size=(B, n)) @ Hinv.T).astype(np.float32)
    zf = rng.uniform(-0.5, 0.5, size=(B, n))
    g = (zf @ base.G.T + rng.uniform(0.1, 1.0, size=(B, m))).astype(np.float32)
    sample = np.unique(np.concatenate([rng.choice(B, 40, replace=False), np.arange(B - 8, B)]))
    import torch
    dev = torch.device("cuda:0")
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    dM, dg = t(M), t(g)
    with gpad_mpc.GpadSolver(0) as s:
        s.setup(t(ML), t(G), float(L), n=n, m=m, batch=B)
        for _ in range(2):
            z = torch.zeros(B, n, device=dev)
            y = torch.zeros(B, m, device=dev)
            iters = np.zeros(B, np.int32)
            st = s.run(z, y, dM, dg, 3000, 1e-4, iters=iters)
            assert st["kernel"] == "panel" and st["converged"] == B, st
            zh, yh = z.cpu().numpy(), y.cpu().numpy()
            for b in sample:
                zo, yo, it, _ = oracle.solve_f32(np.zeros(n), np.zeros(m), ML, M[b], G, g[b], 3000, L, 1e-4)
                assert iters[b] == it, b
                assert_bitexact(zh[b], zo, f"instance {b} z")
                assert_bitexact(yh[b], yo, f"instance {b} y")
