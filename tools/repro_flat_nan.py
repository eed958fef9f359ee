"""Repro of a fuzz finding (profiles/r06_fuzz_parity.txt): a diverging (infeasible, horizon-1) flat
battery case whose second warm-started solve ends with NaN where the oracle has +inf."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, ROOT + "/gpu-dualgradient-mpc_amd", ROOT + "/oracle", ROOT + "/tests"):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import gpad_mpc  # noqa: E402
import pyoracle  # noqa: E402
from gpad_mpc import _lib, problems  # noqa: E402

O = pyoracle.Oracle()
n_u, Nh, B, S, seed, K, N, tol = 8, 1, 17, 2, 956118523, 10, 3000, 1e-3
rng = np.random.default_rng(seed)
qp = problems.battery_scenarios(n_u, Nh, B * S, seed=seed)
MGf, GLf, L = problems.flatten_battery(qp, n_u, Nh)
f32 = lambda a: np.ascontiguousarray(np.asarray(a, np.float64).astype(np.float32))  # noqa: E731
L32 = np.float32(L)
MGf32, GLf32 = f32(MGf), f32(GLf)
GPall = f32(qp.M).reshape(B * S, -1)
PDall = np.ascontiguousarray(O.scale_vec(f32(qp.g).reshape(B * S, -1), L32))
n, m = GPall.shape[1], PDall.shape[1]
inputs = []
for k in range(S):
    z0 = rng.uniform(-0.5, 0.5, (B, n)).astype(np.float32)
    y0 = np.maximum(rng.normal(0.0, 0.3, (B, m)), 0.0).astype(np.float32)
    inputs.append((np.ascontiguousarray(GPall[k * B:(k + 1) * B]), np.ascontiguousarray(PDall[k * B:(k + 1) * B]), z0, y0))


def gpu(kernel, k, handle=None, opts=None, NN=N):
    GP, PD, z0, y0 = inputs[k]
    s = handle or gpad_mpc.GpadSolver(0)
    if handle is None:
        s.setup_flat(MGf32, GLf32, float(L32), n_u=n_u, batch=B, kernel=kernel, check_every=K)
        s.set_options(**(opts or {}))
    z, y = z0.copy(), y0.copy()
    it = np.zeros(B, np.int32)
    st = s.run(z, y, GP, PD, NN, tol, scaled=True, iters=it)
    return z, y, it, st["kernel"], s


def orc(k, b, NN=N):
    GP, PD, z0, y0 = inputs[k]
    return O.solve_flat_f32(z0[b], y0[b], MGf32, GP[b], GLf32, PD[b], n_u, NN, L32, tol, K)


def cmp(tag, z, y, it, k, NN=N):
    bad = []
    for b in range(B):
        zo, yo, ito, _ = orc(k, b, NN)
        ok = it[b] == ito and np.array_equal(z[b], zo, equal_nan=True) and np.array_equal(y[b], yo, equal_nan=True)
        if not ok:
            bad.append(b)
    print(tag, "mismatching instances:", bad[:8], len(bad), flush=True)
    return bad


for name, kern in (("auto", _lib.KERNEL_AUTO), ("stream", _lib.KERNEL_STREAM), ("panel", _lib.KERNEL_PANEL)):
    for k in range(S):
        z, y, it, kn, _ = gpu(kern, k, opts={"phased": 0, "phase_len": 30})
        cmp(f"{name}/{kn} fresh handle solve {k}", z, y, it, k)
    z, y, it, kn, s = gpu(kern, 0, opts={"phased": 0, "phase_len": 30})
    z, y, it, kn, _ = gpu(kern, 1, handle=s)
    cmp(f"{name}/{kn} same handle solve 1", z, y, it, 1)
# where does it start: fixed iteration counts, fresh handle, auto
GP, PD, z0, y0 = inputs[1]
for NN in (10, 50, 100, 200, 400, 800, 1600):
    z, y, it, kn, _ = gpu(_lib.KERNEL_AUTO, 1, NN=NN)
    zo, yo, ito, _ = orc(1, 0, NN)
    print(NN, "it", it[0], ito, "y gpu", y[0][:3], "orc", yo[:3], "nan gpu/orc", int(np.isnan(y[0]).sum()), int(np.isnan(yo).sum()),
          "inf", int(np.isinf(y[0]).sum()), int(np.isinf(yo).sum()), flush=True)
