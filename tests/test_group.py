"""Multi-device C-ABI (include/gpad.h gpad_group_*, gpad_solve_sharded): instance shards over
several devices of one process, RCCL scatter/gather to the root for device memory.

On the 1-GPU box: devices [0] is a one-rank RCCL clique (every code path of the RCCL transport
but the sends, which a single rank does not need); devices [0, 0, 0] stand three shards on one
GPU with the peer-copy transport (the same scatter/gather moves, by hipMemcpyPeerAsync).  Every
shard layout must give exactly the single-handle (oracle-pinned) results -- the 8-GPU timing is
the driver's SCALE run.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _qp(n, m, B, seed, shared=True):
    from gpad_mpc import problems
    qp = problems.synthetic_qp(n, m, batch=B, seed=seed)
    f = lambda a: np.ascontiguousarray(np.asarray(a, np.float64).astype(np.float32))  # noqa: E731
    ML, G = f(qp.ML), f(qp.G)
    if not shared:
        rng = np.random.default_rng(seed)
        ML = f(ML[None] * (1 + 0.02 * rng.random((B, 1, 1))))
        G = f(G[None] * (1 + 0.02 * rng.random((B, 1, 1))))
    return ML, f(qp.M).reshape(B, n), G, f(qp.g).reshape(B, m), np.float32(qp.L)


def _single(ML, M, G, g, L, N, tol, shared, codes=None):
    import gpad_mpc
    B, n = M.shape
    m = g.shape[1]
    z = np.zeros((B, n), np.float32)
    y = np.zeros((B, m), np.float32)
    it = np.zeros(B, np.int32)
    with gpad_mpc.GpadSolver(0) as s:
        s.setup(ML, G, float(L), n=n, m=m, batch=B, shared=shared)
        s.run(z, y, M, g, N, tol, iters=it, codes=codes)
    return z, y, it


@pytest.mark.parametrize("devices,transport", [([0], "rccl"), ([0, 0, 0], "peer"), ([0, 0], "peer")])
@pytest.mark.parametrize("memory", ["host", "device"])
@pytest.mark.parametrize("shared,B,N,tol", [(True, 300, 3000, 1e-4), (True, 37, 60, 0.0), (False, 7, 2000, 1e-4),
                                            (True, 2, 500, 1e-4)])
def test_group_shards_equal_single_handle(gpu, devices, transport, memory, shared, B, N, tol):
    import torch

    import gpad_mpc
    n, m = 40, 72
    ML, M, G, g, L = _qp(n, m, B, seed=B + 3, shared=shared)
    cr = np.full(B, -1, np.int32)
    zr, yr, itr = _single(ML, M, G, g, L, N, tol, shared, codes=cr)
    Z = np.zeros((B, n), np.float32)
    Y = np.zeros((B, m), np.float32)
    it = np.zeros(B, np.int32)
    codes = np.full(B, -1, np.int32)  # the group forwards st->codes to every shard
    with gpad_mpc.GpadGroup(devices) as grp:
        assert grp.transport == transport
        if memory == "device":
            t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(gpu)  # noqa: E731
            dZ, dY = t(Z), t(Y)
            grp.setup(t(ML), t(G), float(L), n=n, m=m, batch=B, shared=shared)
            st = grp.run(dZ, dY, t(M), t(g), N, tol, iters=it, codes=codes)
            Z, Y = dZ.cpu().numpy(), dY.cpu().numpy()
        else:
            grp.setup(ML, G, float(L), n=n, m=m, batch=B, shared=shared)
            st = grp.run(Z, Y, M, g, N, tol, iters=it, codes=codes)
    np.testing.assert_array_equal(it, itr)
    np.testing.assert_array_equal(codes, cr)
    assert (cr >= 0).all() and ((cr > 0).sum() == st["converged"])
    np.testing.assert_array_equal(Z, zr)
    np.testing.assert_array_equal(Y, yr)
    assert st["total_iterations"] == int(itr.sum()) and st["iterations"] == int(itr.max())


@pytest.mark.parametrize("devices", [[0], [0, 0, 0, 0]])
def test_solve_sharded_one_shot(gpu, oracle, devices):
    """gpad_solve_sharded(ndev, devices, z0, y0, ML, M, G, g, N, L, tol, dims, stats) through ctypes,
    called three times (the cached group re-binds the matrices; before the third call
    gpad_release_cached frees the group, which is then rebuilt) -- bit-exact vs the oracle."""
    from gpad_mpc import _lib
    lib = _lib.load()
    n, m, B, N, tol = 64, 96, 50, 3000, 1e-4
    for seed in (1, 2, 3):
        if seed == 3:
            lib.gpad_release_cached()
        ML, M, G, g, L = _qp(n, m, B, seed)
        Z = np.zeros((B, n), np.float32)
        Y = np.zeros((B, m), np.float32)
        it = np.zeros(B, np.int32)
        d = _lib.Dims(n=n, m=m, batch=B, shared=1, dtype=_lib.DTYPE_F32, memory=_lib.MEM_HOST,
                      schedule=_lib.SCHEDULE_MATLAB, check_every=10, kernel=_lib.KERNEL_AUTO)
        st = _lib.Stats()
        st.iters = it.ctypes.data_as(C.POINTER(C.c_int))
        devs = (C.c_int * len(devices))(*devices)
        p = lambda a: C.c_void_p(a.ctypes.data)  # noqa: E731
        _lib.check(lib.gpad_solve_sharded(len(devices), devs, p(Z), p(Y), p(ML), p(M), p(G), p(g), N, float(L), tol,
                                          C.byref(d), C.byref(st)), "gpad_solve_sharded")
        for b in range(0, B, 5):
            zo, yo, ito, _ = oracle.solve_f32(np.zeros(n), np.zeros(m), ML, M[b], G, g[b], N, L, tol)
            assert it[b] == ito
            np.testing.assert_array_equal(Z[b], zo)
            np.testing.assert_array_equal(Y[b], yo)


@pytest.mark.gpu
@pytest.mark.parametrize("tol", [0.0, 1e-4])
def test_c_app_scenarios_over_devices(gpu, tol):
    """apps/gpad_main.c --scenarios: the main.cu-shaped C caller solving a battery-scenario batch
    over several devices with gpad_solve_sharded (no Python in the loop).  On this one-GPU box
    the device lists 1, "0,0" and "0,0,0" shard the batch differently (peer copies when a device
    repeats); every layout must give the bits of one handle solving the whole batch."""
    import os
    import subprocess

    import gpad_mpc
    from conftest import GOLDEN, PKG
    from gpad_mpc import _lib, datafile
    app = os.path.join(PKG, "gpad_mpc", "gpad_main")
    path = os.path.join(GOLDEN, "datafile_battery_3x4.txt")
    B, N = 600, 100
    out = {}
    for devs in ("1", "0,0", "0,0,0"):
        r = subprocess.run([app, path, "--scenarios", str(B), "--devices", devs, "--iters", str(N), "--tol", str(tol)],
                           capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        out[devs] = {ln.split()[0]: ln.split()[1:] for ln in r.stdout.splitlines()}
    assert out["1"]["hash"] == out["0,0"]["hash"] == out["0,0,0"]["hash"]
    assert out["1"]["total_iterations"] == out["0,0,0"]["total_iterations"]
    # the same batch through one handle (gpad_mpc.solve), hashed the app's way (FNV-1a of z*, y*)
    d = datafile.read(path, 0)
    n, m = d.n, d.m
    L = np.float32(d.L)
    ML = (-d.M_G).astype(np.float32)
    G = (np.float64(L) * d.G_L.astype(np.float64)).astype(np.float32)
    g1 = (-np.float64(L) * d.p_D.astype(np.float64)).astype(np.float32)
    bi, ii = np.meshgrid(np.arange(B), np.arange(n), indexing="ij")
    M = (d.g_P.astype(np.float64)[None, :] * (1.0 + 1e-3 * ((31 * bi + ii) % 17))).astype(np.float32)
    g = np.repeat(g1[None, :], B, axis=0)
    Z = np.zeros((B, n), np.float32)
    Y = np.zeros((B, m), np.float32)
    with gpad_mpc.GpadSolver(0) as s:
        s.setup(ML, G, float(L), n=n, m=m, batch=B, kernel=_lib.KERNEL_AUTO)
        st = s.run(Z, Y, M, g, N, tol)
    h = 1469598103934665603
    for byte in Z.tobytes() + Y.tobytes():
        h = ((h ^ byte) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    assert out["1"]["hash"][0] == f"{h:016x}"
    assert int(out["1"]["total_iterations"][0]) == st["total_iterations"]


# ---- the RCCL transport with several ranks on one GPU ----------------------
# tests/rccl_stub: the eight RCCL entry points libgpad binds, implemented with HIP copies and
# accepting a repeated device; gpad_group_rccl_library(stub, force_rccl = 1) points the groups at it,
# so the grouped ncclSend / ncclRecv scatter and gather of ragged shards and the ncclBroadcast of the
# shared matrices run through csrc/gpad_group.cpp's RCCL branch over 2 and 3 "ranks".
def _stub_path():
    import os
    import subprocess
    d = os.path.join(os.path.dirname(os.path.abspath(__file__)), "rccl_stub")
    so = os.path.join(d, "librccl_stub.so")
    if not os.path.exists(so):  # (normally built by __graft_entry__.build())
        subprocess.run(["make", "-s", "-C", d], check=True, timeout=120)
    return so


@pytest.fixture
def rccl_stub():
    from gpad_mpc import _lib
    lib = _lib.load()
    so = _stub_path()
    _lib.check(lib.gpad_group_rccl_library(so.encode(), 1), "gpad_group_rccl_library")
    stub = C.CDLL(so)
    stub.rccl_stub_moves.restype = C.c_longlong
    try:
        yield stub
    finally:
        lib.gpad_release_cached()  # (a cached sharded group made with the stub)
        lib.gpad_group_rccl_library(None, 0)


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0]])
@pytest.mark.parametrize("memory", ["host", "device"])
@pytest.mark.parametrize("shared,B,N,tol", [(True, 301, 3000, 1e-4), (True, 37, 60, 0.0), (False, 8, 2000, 1e-4)])
def test_group_rccl_transport_ranks(gpu, rccl_stub, devices, memory, shared, B, N, tol):
    """gpad_group_* with the RCCL transport over 2 and 3 ranks (one GPU standing in for each, through
    the stub): ragged shards (sizes differing by one), host and device memory, shared and per-instance
    matrices -- z*, y*, counts and codes bit-identical to one handle; with device memory the stub
    performed the broadcast / scatter / gather moves (so the RCCL branch really ran)."""
    import torch

    import gpad_mpc
    n, m = 40, 72
    ML, M, G, g, L = _qp(n, m, B, seed=B + 11, shared=shared)
    cr = np.full(B, -1, np.int32)
    zr, yr, itr = _single(ML, M, G, g, L, N, tol, shared, codes=cr)
    Z = np.zeros((B, n), np.float32)
    Y = np.zeros((B, m), np.float32)
    it = np.zeros(B, np.int32)
    codes = np.full(B, -1, np.int32)
    moves0 = rccl_stub.rccl_stub_moves()
    with gpad_mpc.GpadGroup(devices) as grp:
        assert grp.transport == "rccl"
        if memory == "device":
            t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(gpu)  # noqa: E731
            dZ, dY = t(Z), t(Y)
            grp.setup(t(ML), t(G), float(L), n=n, m=m, batch=B, shared=shared)
            st = grp.run(dZ, dY, t(M), t(g), N, tol, iters=it, codes=codes)
            Z, Y = dZ.cpu().numpy(), dY.cpu().numpy()
        else:
            grp.setup(ML, G, float(L), n=n, m=m, batch=B, shared=shared)
            st = grp.run(Z, Y, M, g, N, tol, iters=it, codes=codes)
    moved = rccl_stub.rccl_stub_moves() - moves0
    k = len(devices) - 1  # non-root ranks
    if memory == "device":  # setup: 2 matrices per rank (broadcast or sends); run: 4 vectors out, 2 back
        assert moved == 2 * k + 6 * k, moved
    else:
        assert moved == 0, moved
    np.testing.assert_array_equal(it, itr)
    np.testing.assert_array_equal(codes, cr)
    np.testing.assert_array_equal(Z, zr)
    np.testing.assert_array_equal(Y, yr)
    assert st["total_iterations"] == int(itr.sum()) and st["iterations"] == int(itr.max())


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0]])
def test_solve_sharded_rccl_transport_ranks(gpu, oracle, rccl_stub, devices):
    """gpad_solve_sharded (device memory) over 2 and 3 RCCL ranks through the stub: the cached group
    is rebuilt for the new RCCL configuration, ragged shards (B = 50 over 3: 17, 17, 16), every
    instance equal to one handle and a sample to the oracle; the stub moved the bytes."""
    import torch

    from gpad_mpc import _lib
    lib = _lib.load()
    n, m, B, N, tol = 64, 96, 50, 3000, 1e-4
    ML, M, G, g, L = _qp(n, m, B, 21)
    zr, yr, itr = _single(ML, M, G, g, L, N, tol, True)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(gpu)  # noqa: E731
    dZ, dY = t(np.zeros((B, n), np.float32)), t(np.zeros((B, m), np.float32))
    dML, dM, dG, dg = t(ML), t(M), t(G), t(g)
    torch.cuda.synchronize()
    it = np.zeros(B, np.int32)
    d = _lib.Dims(n=n, m=m, batch=B, shared=1, dtype=_lib.DTYPE_F32, memory=_lib.MEM_DEVICE,
                  schedule=_lib.SCHEDULE_MATLAB, check_every=10, kernel=_lib.KERNEL_AUTO)
    st = _lib.Stats()
    st.iters = it.ctypes.data_as(C.POINTER(C.c_int))
    devs = (C.c_int * len(devices))(*devices)
    p = lambda a: C.c_void_p(a.data_ptr())  # noqa: E731
    moves0 = rccl_stub.rccl_stub_moves()
    _lib.check(lib.gpad_solve_sharded(len(devices), devs, p(dZ), p(dY), p(dML), p(dM), p(dG), p(dg), N, float(L),
                                      tol, C.byref(d), C.byref(st)), "gpad_solve_sharded")
    assert rccl_stub.rccl_stub_moves() - moves0 == 8 * (len(devices) - 1)
    np.testing.assert_array_equal(it, itr)
    np.testing.assert_array_equal(dZ.cpu().numpy(), zr)
    np.testing.assert_array_equal(dY.cpu().numpy(), yr)
    for b in (0, B // 2, B - 1):
        zo, yo, ito, _ = oracle.solve_f32(np.zeros(n), np.zeros(m), ML, M[b], G, g[b], N, L, tol)
        assert itr[b] == ito
        np.testing.assert_array_equal(zr[b], zo)


def test_unloadable_rccl_falls_back_to_peer_copies(gpu):
    """An RCCL library that cannot be loaded: gpad_group_rccl_library reports GPAD_ERR_UNSUPPORTED and
    groups -- even over distinct devices, here the one-rank clique [0] -- use the peer copies, with
    the same results; restoring the default brings the RCCL clique back."""
    import gpad_mpc
    from gpad_mpc import _lib
    lib = _lib.load()
    try:
        assert lib.gpad_group_rccl_library(b"/nonexistent/librccl_missing.so", 1) == _lib.ERR_UNSUPPORTED
        n, m, B, N, tol = 40, 72, 33, 2000, 1e-4
        ML, M, G, g, L = _qp(n, m, B, 5)
        zr, yr, itr = _single(ML, M, G, g, L, N, tol, True)
        with gpad_mpc.GpadGroup([0]) as grp:
            assert grp.transport == "peer"
            Z, Y = np.zeros((B, n), np.float32), np.zeros((B, m), np.float32)
            it = np.zeros(B, np.int32)
            grp.setup(ML, G, float(L), n=n, m=m, batch=B)
            grp.run(Z, Y, M, g, N, tol, iters=it)
        np.testing.assert_array_equal(it, itr)
        np.testing.assert_array_equal(Z, zr)
        np.testing.assert_array_equal(Y, yr)
    finally:
        rc = lib.gpad_group_rccl_library(None, 0)
    assert rc == _lib.GPAD_OK
    with gpad_mpc.GpadGroup([0]) as grp:
        assert grp.transport == "rccl"
