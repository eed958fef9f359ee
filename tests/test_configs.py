"""BASELINE.json configs at their full size on the GPU, checked against the oracle.

C5: long horizon N = 200 (n = 800), m = 800, batch 1024 with DISTINCT per-instance matrices
(5.2 GB of ML/G, streamed from HBM by the stream kernel), 20 iterations; instances spread over
the grid (first, last and strides between) bit-exact vs the oracle's solve of that instance.
"""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_c5_batch1024_distinct_800x800_bitexact(gpu, oracle):
    import torch

    import gpad_mpc
    B, n, m, N = 1024, 800, 800, 20
    g0 = torch.Generator(device=gpu).manual_seed(5)
    ML = torch.randn(B, n, m, device=gpu, generator=g0) * (0.1 / np.sqrt(m))
    G = torch.randn(B, m, n, device=gpu, generator=g0) / np.sqrt(n)
    M = torch.randn(B, n, device=gpu, generator=g0)
    g = torch.rand(B, m, device=gpu, generator=g0) + 0.1
    L = 10.0
    z = torch.zeros(B, n, device=gpu)
    y = torch.zeros(B, m, device=gpu)
    with gpad_mpc.GpadSolver(0) as s:
        s.setup(ML, G, L, n=n, m=m, batch=B, shared=False)
        st = s.run(z, y, M, g, N, 0.0)
    assert st["kernel"] == "stream" and st["iterations"] == N
    Z, Y = z.cpu().numpy(), y.cpu().numpy()
    for b in (0, 1, 257, 514, 771, 1000, 1023):
        zo, yo, it, _ = oracle.solve_f32(np.zeros(n), np.zeros(m), ML[b].cpu().numpy(), M[b].cpu().numpy(),
                                         G[b].cpu().numpy(), g[b].cpu().numpy(), N, np.float32(L))
        assert it == N
        np.testing.assert_array_equal(Z[b], zo, err_msg=f"z[{b}]")
        np.testing.assert_array_equal(Y[b], yo, err_msg=f"y[{b}]")


def test_c4_shard_certified_on_the_constraint(gpu, oracle):
    """C4 shard (bench.py's workload: 8192 instances sharing ML/G, eps = 1e-4, phased panel
    solve + finisher): every instance reported converged satisfies max(G z* - g) <= 1e-4
    evaluated exactly (fp64) on the returned z* and the caller's f32 G, g; iteration counts
    of a spread sample and of the 12 longest solves (the finisher's) equal the oracle's.  The
    second solve of the handle runs the phase plan made from the first one's counts, as in the
    bench."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    import torch

    import gpad_mpc
    n = m = 200
    B, tol, N = 8192, 1e-4, 5000
    ML, G, L, M, g = bench.make_shard(n, m, B, 0)
    f32 = np.float32
    ML32, G32, M32, g32, L32 = ML.astype(f32), G.astype(f32), M.astype(f32), g.astype(f32), f32(L)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(gpu)  # noqa: E731
    z = torch.zeros(B, n, device=gpu)
    y = torch.zeros(B, m, device=gpu)
    it = np.zeros(B, np.int32)
    with gpad_mpc.GpadSolver(0) as s:
        s.setup(t(ML32), t(G32), float(L32), n=n, m=m, batch=B, check_every=10)
        for _ in range(2):  # the second solve is planned from the first one's counts
            z.zero_()
            y.zero_()
            st = s.run(z, y, t(M32), t(g32), N, tol, iters=it)
    assert st["kernel"] == "panel" and st["converged"] == B
    Z = z.cpu().numpy().astype(np.float64)
    viol = (Z @ G32.astype(np.float64).T - g32.astype(np.float64)).max(axis=1)
    assert viol.max() <= tol, (viol.max(), int(viol.argmax()))
    for b in list(range(0, B, 257)) + [int(i) for i in np.argsort(-it, kind="stable")[:12]]:
        zo, yo, ito, _ = oracle.solve_f32(np.zeros(n), np.zeros(m), ML32, M32[b], G32, g32[b], N, L32, tol)
        assert it[b] == ito, b
        np.testing.assert_array_equal(Z[b].astype(np.float32), zo)


def test_c3_batch4096_bitexact(gpu, oracle):
    """C3 at its full size (BASELINE.json configs[2]): 4096 instances sharing ML/G, N = 50
    (n = 200), m = 200, eps = 1e-4 -- one panel per workgroup (256 panels = 256 CUs, tile 12 as
    the 3-hop relay), phased with the finisher.  Run twice so the second solve follows the plan
    made from the first one's counts (the default path of a repeated caller); every 257th instance
    bit-exact against the oracle, iteration count included, and every instance certified in fp64
    on the returned z*."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    import torch

    import gpad_mpc
    n = m = 200
    B, tol, N = 4096, 1e-4, 5000
    ML, G, L, M, g = bench.make_shard(n, m, B, 0)
    f32 = np.float32
    ML32, G32, M32, g32, L32 = ML.astype(f32), G.astype(f32), M.astype(f32), g.astype(f32), f32(L)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(gpu)  # noqa: E731
    it = np.zeros(B, np.int32)
    with gpad_mpc.GpadSolver(0) as s:
        s.setup(t(ML32), t(G32), float(L32), n=n, m=m, batch=B, check_every=10)
        for rep in range(2):
            z = torch.zeros(B, n, device=gpu)
            y = torch.zeros(B, m, device=gpu)
            st = s.run(z, y, t(M32), t(g32), N, tol, iters=it)
            assert st["kernel"] == "panel" and st["converged"] == B
        plan = s.phase_plan()
    assert plan["ends"], "the second solve follows a plan"
    Z, Y = z.cpu().numpy(), y.cpu().numpy()
    viol = (Z.astype(np.float64) @ G32.astype(np.float64).T - g32.astype(np.float64)).max(axis=1)
    assert viol.max() <= tol, (viol.max(), int(viol.argmax()))
    for b in list(range(0, B, 257)) + [B - 1]:
        zo, yo, ito, _ = oracle.solve_f32(np.zeros(n), np.zeros(m), ML32, M32[b], G32, g32[b], N, L32, tol)
        assert it[b] == ito, b
        np.testing.assert_array_equal(Z[b], zo, err_msg=f"z[{b}]")
        np.testing.assert_array_equal(Y[b], yo, err_msg=f"y[{b}]")


def test_c4_global_65536(gpu, oracle):
    """C4 at its own size (BASELINE.json configs[3]): 65536 instances sharing ML/G, N = 50 (n = 200),
    m = 200, eps = 1e-4, through the C-ABI multi-device entry gpad_solve_sharded over devices
    [0] * 8 -- eight 8192-instance shards, the shard layout of the 8-GPU run, with the same scatter
    of M, g, z0, y0 and gather of (z*, y*) into the root buffers (peer copies: the device repeats;
    distinct devices use the RCCL clique, gpad_group.cpp).  Every instance converges and is
    certified in fp64 on the returned z*; the counts equal ONE handle solving all 65536 at once
    (planned twice, as the bench runs it); a spread sample and the 12 longest instances are
    bit-exact against the oracle.  The reference solves one problem per process
    (Code/CUDA/FinalProject/main.cu:106-108); this is the batch row the build adds on top."""
    import ctypes as C
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    import torch

    import gpad_mpc
    from gpad_mpc import _lib
    lib = _lib.load()
    n = m = 200
    B, tol, N, shards = 65536, 1e-4, 5000, 8
    ML, G, L, M, g = bench.make_shard(n, m, B, 0)
    f32 = np.float32
    ML32, G32, M32, g32, L32 = ML.astype(f32), G.astype(f32), M.astype(f32), g.astype(f32), f32(L)
    del ML, G, M, g
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(gpu)  # noqa: E731
    dML, dG, dM, dg = t(ML32), t(G32), t(M32), t(g32)
    # one handle, the whole batch (the strong-scaling anchor of bench.py's c4_global_1gpu leg)
    it1 = np.zeros(B, np.int32)
    with gpad_mpc.GpadSolver(0) as s:
        s.setup(dML, dG, float(L32), n=n, m=m, batch=B, check_every=10)
        for _ in range(2):
            z1 = torch.zeros(B, n, device=gpu)
            y1 = torch.zeros(B, m, device=gpu)
            st1 = s.run(z1, y1, dM, dg, N, tol, iters=it1)
    assert st1["kernel"] == "panel" and st1["converged"] == B
    # eight shards on device 0 through gpad_solve_sharded (device memory on the root)
    z = torch.zeros(B, n, device=gpu)
    y = torch.zeros(B, m, device=gpu)
    it = np.zeros(B, np.int32)
    codes = np.full(B, -1, np.int32)
    d = _lib.Dims(n=n, m=m, batch=B, shared=1, dtype=_lib.DTYPE_F32, memory=_lib.MEM_DEVICE,
                  schedule=_lib.SCHEDULE_MATLAB, check_every=10, kernel=_lib.KERNEL_AUTO)
    st = _lib.Stats()
    st.iters = it.ctypes.data_as(C.POINTER(C.c_int))
    st.codes = codes.ctypes.data_as(C.POINTER(C.c_int))
    devs = (C.c_int * shards)(*([0] * shards))
    p = lambda a: C.c_void_p(a.data_ptr())  # noqa: E731
    torch.cuda.synchronize()
    _lib.check(lib.gpad_solve_sharded(shards, devs, p(z), p(y), p(dML), p(dM), p(dG), p(dg), N, float(L32), tol,
                                      C.byref(d), C.byref(st)), "gpad_solve_sharded")
    lib.gpad_release_cached()
    assert st.converged == B and st.kernel == _lib.KERNEL_PANEL
    assert (codes > 0).all()
    np.testing.assert_array_equal(it, it1)
    assert st.total_iterations == int(it1.sum()) and st.iterations == int(it1.max())
    Z, Y = z.cpu().numpy(), y.cpu().numpy()
    np.testing.assert_array_equal(Z, z1.cpu().numpy())
    np.testing.assert_array_equal(Y, y1.cpu().numpy())
    viol = (Z.astype(np.float64) @ G32.astype(np.float64).T - g32.astype(np.float64)).max(axis=1)
    assert viol.max() <= tol, (viol.max(), int(viol.argmax()))
    sample = list(range(0, B, 4099)) + [B - 1] + [int(i) for i in np.argsort(-it, kind="stable")[:12]]
    for b in sample:
        zo, yo, ito, _ = oracle.solve_f32(np.zeros(n), np.zeros(m), ML32, M32[b], G32, g32[b], N, L32, tol)
        assert it[b] == ito, b
        np.testing.assert_array_equal(Z[b], zo, err_msg=f"z[{b}]")
        np.testing.assert_array_equal(Y[b], yo, err_msg=f"y[{b}]")
