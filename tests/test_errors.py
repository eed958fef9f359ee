"""Failure reporting of the C-ABI (include/gpad.h): a device-side failure of a run surfaces as
GPAD_ERR_DEVICE, never as GPAD_OK with wrong results, and a tolerance below the f32 certification
floor is flagged in the stats.  The reference reports nothing (main.cu:34-37 perror()s a failed
read and continues; no cudaGetLastError anywhere), which is the pattern the boundary must not
repeat.
"""
from __future__ import annotations

import numpy as np
import pytest

from test_gpu_parity import assert_bitexact

pytestmark = pytest.mark.gpu


def _shard(batch, seed=0):
    import bench
    ML, G, L, M, g = bench.make_shard(200, 200, batch, seed)
    f = lambda a: np.ascontiguousarray(a, np.float32)  # noqa: E731
    return f(ML), f(G), float(np.float32(L)), f(M), f(g)


@pytest.mark.parametrize("batch", [64, 4400])  # one panel per workgroup (relay), panel pairs
def test_dropped_handoff_fails_the_run(gpu, oracle, batch):
    """A chain hand-off that never arrives (fault injection GPAD_OPT_DEBUG_DROP_HANDOFF) ends the
    run in GPAD_ERR_DEVICE -- with stats, at gpad_sync for an asynchronous run -- and the handle
    is usable again afterwards (bit-exact once the injection is off)."""
    import torch

    import gpad_mpc
    from gpad_mpc import _lib
    ML, G, L, M, g = _shard(batch)
    dev = torch.device("cuda:0")
    t = lambda a: torch.from_numpy(a).to(dev)  # noqa: E731
    with gpad_mpc.GpadSolver(0) as s:
        s.setup(t(ML), t(G), L, n=200, m=200, batch=batch, kernel=_lib.KERNEL_PANEL)
        z = torch.zeros(batch, 200, device=dev)
        y = torch.zeros(batch, 200, device=dev)
        s.set_option("debug_drop_handoff", 1)
        with pytest.raises(_lib.GpadError) as ei:
            s.run(z, y, t(M), t(g), 20, 0.0)
        assert ei.value.code == _lib.ERR_DEVICE
        assert "hand-off" in str(ei.value)
        z.zero_()
        y.zero_()
        s.run(z, y, t(M), t(g), 20, 0.0, stats=False)  # asynchronous: reported at the sync
        with pytest.raises(_lib.GpadError) as ei:
            s.sync()
        assert ei.value.code == _lib.ERR_DEVICE
        s.set_option("debug_drop_handoff", 0)
        z.zero_()
        y.zero_()
        st = s.run(z, y, t(M), t(g), 20, 0.0)
        assert st["kernel"] == "panel"
        s.sync()
    k = [0, batch // 2, batch - 1]
    for b in k:
        zo, yo, _, _ = oracle.solve_f32(np.zeros(200), np.zeros(200), ML, M[b], G, g[b], 20, np.float32(L))
        assert_bitexact(z[b].cpu().numpy(), zo, f"z[{b}]")
        assert_bitexact(y[b].cpu().numpy(), yo, f"y[{b}]")


def test_device_error_is_sticky_across_async_runs(gpu):
    """a faulty asynchronous run followed by a clean one, then one gpad_sync: the sync
    reports the first run's GPAD_ERR_DEVICE (the second run's status reset must not wipe it); every
    later sync / stats call keeps reporting it (gpad_last_stats after the failing sync
    must not return GPAD_OK) until the next run starts."""
    import torch

    import gpad_mpc
    from gpad_mpc import _lib
    ML, G, L, M, g = _shard(64)
    dev = torch.device("cuda:0")
    t = lambda a: torch.from_numpy(a).to(dev)  # noqa: E731
    with gpad_mpc.GpadSolver(0) as s:
        s.setup(t(ML), t(G), L, n=200, m=200, batch=64, kernel=_lib.KERNEL_PANEL)
        z = torch.zeros(64, 200, device=dev)
        y = torch.zeros(64, 200, device=dev)
        dM, dg = t(M), t(g)
        s.set_option("debug_drop_handoff", 1)
        s.run(z, y, dM, dg, 20, 0.0, stats=False)          # faulty, asynchronous
        s.set_option("debug_drop_handoff", 0)
        s.run(z.zero_(), y.zero_(), dM, dg, 20, 0.0, stats=False)  # clean, queued behind it
        with pytest.raises(_lib.GpadError) as ei:
            s.sync()
        assert ei.value.code == _lib.ERR_DEVICE
        for call in (s.sync, s.last_stats):  # still failed: the results are invalid
            with pytest.raises(_lib.GpadError) as ei:
                call()
            assert ei.value.code == _lib.ERR_DEVICE
        st = s.run(z.zero_(), y.zero_(), dM, dg, 20, 0.0)
        assert st["kernel"] == "panel"


@pytest.mark.parametrize("bad", [np.nan, np.inf])
def test_nonfinite_g_is_flagged(gpu, bad):
    """max |g| of the certification floor keeps a NaN / infinity of g (panel pairs fold
    it into their loads, every other path runs the absmax kernel): the stats flag it."""
    import gpad_mpc
    for batch in (8, 4400):  # resident kernel + absmax launch; panel pairs' folded max
        ML, G, L, M, g = _shard(batch)
        g[batch // 2, 7] = bad
        with gpad_mpc.GpadSolver(0) as s:
            s.setup(ML, G, L, n=200, m=200, batch=batch)
            z = np.zeros((batch, 200), np.float32)
            y = np.zeros((batch, 200), np.float32)
            st = s.run(z, y, M, g, 60, 1e-4)
        assert st["nonfinite_g"] and st["below_tol_floor"], (batch, st)
        assert (np.isnan(st["tol_floor"]) if np.isnan(bad) else np.isinf(st["tol_floor"])), st


def test_dropped_handoff_fails_host_memory_run(gpu):
    """Host-memory runs synchronise inside gpad_run: the error comes back from gpad_run itself,
    with or without a stats struct."""
    import gpad_mpc
    from gpad_mpc import _lib
    ML, G, L, M, g = _shard(64)
    with gpad_mpc.GpadSolver(0) as s:
        s.setup(ML, G, L, n=200, m=200, batch=64, kernel=_lib.KERNEL_PANEL)
        s.set_option("debug_drop_handoff", 1)
        for stats in (True, False):
            z = np.zeros((64, 200), np.float32)
            y = np.zeros((64, 200), np.float32)
            with pytest.raises(_lib.GpadError) as ei:
                s.run(z, y, M, g, 20, 0.0, stats=stats)
            assert ei.value.code == _lib.ERR_DEVICE


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_tol_below_certification_floor_is_flagged(gpu, dtype):
    """tol_floor = margin * max|g| (2^-20 f32, 2^-49 f64); below it the stats carry
    GPAD_FLAG_TOL_FLOOR (and, f32 at the reference's e_g = 1e-6 scale, nothing certifies)."""
    import gpad_mpc
    from gpad_mpc import _lib
    ML, G, L, M, g = _shard(8)
    ML, G, M, g = (a.astype(dtype) for a in (ML, G, M, g))
    margin = 2.0 ** -20 if dtype == np.float32 else 2.0 ** -49
    floor = margin * float(np.abs(g.astype(np.float64)).max())
    with gpad_mpc.GpadSolver(0) as s:
        s.setup(ML, G, L, n=200, m=200, batch=8)
        for tol, below in [(1e-4, False), (floor * 0.5, True)]:
            z = np.zeros((8, 200), dtype)
            y = np.zeros((8, 200), dtype)
            st = s.run(z, y, M, g, 300, tol)
            assert st["tol_floor"] == pytest.approx(floor, rel=1e-6)
            assert st["below_tol_floor"] is below, (tol, st)
            if below and dtype == np.float32:
                assert st["converged"] == 0 and st["iterations"] == 300
        z = np.zeros((8, 200), dtype)
        y = np.zeros((8, 200), dtype)
        st = s.run(z, y, M, g, 30, 0.0)  # fixed N: no floor
        assert st["tol_floor"] == 0.0 and not st["below_tol_floor"]


def test_tol_floor_is_the_current_runs(gpu):
    """The per-workgroup max |g| slots are not zeroed before a run: its first writer (the panel
    pairs' first launch, or the absmax kernel) stores them and zeroes the rest.  On one handle, a
    run with a large |g| followed by smaller ones -- a phased panel solve, then a smaller grid on
    the absmax path -- must report each run's own floor, never a stale slot."""
    import gpad_mpc
    margin = 2.0 ** -20
    with gpad_mpc.GpadSolver(0) as s:
        for batch, scale in [(4400, 100.0), (4400, 1.0), (8, 1.0), (4400, 0.5), (8, 3.0)]:
            ML, G, L, M, g = _shard(batch)
            g = (g * np.float32(scale)).astype(np.float32)
            s.setup(ML, G, L, n=200, m=200, batch=batch)
            z = np.zeros((batch, 200), np.float32)
            y = np.zeros((batch, 200), np.float32)
            st = s.run(z, y, M, g, 300, 1e-4)
            floor = margin * float(np.abs(g.astype(np.float64)).max())
            assert st["tol_floor"] == pytest.approx(floor, rel=1e-6), (batch, scale, st["tol_floor"], floor)


def test_dims_reserved_must_be_zero(gpu):
    import ctypes as C

    from gpad_mpc import _lib
    L = _lib.load()
    h = C.c_void_p()
    _lib.check(L.gpad_create(C.byref(h), 0, None), "gpad_create")
    try:
        ML = np.eye(4, dtype=np.float32)
        d = _lib.Dims(n=4, m=4, batch=1, shared=1, dtype=0, memory=0, schedule=0, check_every=10,
                      kernel=0, reserved=7, tol_gap=0.0)
        rc = L.gpad_setup(h, C.byref(d), ML.ctypes.data, ML.ctypes.data, 1.0)
        assert rc == _lib.ERR_INVALID
        assert b"reserved" in L.gpad_last_error()
    finally:
        L.gpad_destroy(h)
