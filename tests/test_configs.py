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
