"""Per-iteration cost of each GPAD kernel family (fixed N iterations, no termination test).

Prints one JSON line per case: kernel, shape, batch, us/iteration (per launch), instance-it/s,
fp32 TFLOP/s (F = 4nm + 5m + 4n per instance-iteration) and algorithmic GB/s.
Usage (GPU box):  python tools/microbench.py [--quick]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-dualgradient-mpc_amd"))


def case(kernel, n, m, batch, N, shared=True, reps=3, tol=0.0, check_every=10):
    import torch
    import gpad_mpc
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import tune_env  # noqa: F401  (legacy GPAD_* env -> gpad_set_option)
    from gpad_mpc import _lib, problems
    dev = torch.device("cuda:0")
    kc = {"stream": _lib.KERNEL_STREAM, "resident": _lib.KERNEL_RESIDENT, "panel": _lib.KERNEL_PANEL,
          "auto": _lib.KERNEL_AUTO}[kernel]
    rng = np.random.default_rng(0)
    if shared:
        base = problems.synthetic_qp(n, m, batch=1, seed=1)
        ML = torch.from_numpy(base.ML.astype(np.float32)).to(dev)
        G = torch.from_numpy(base.G.astype(np.float32)).to(dev)
    else:
        # distinct matrices: random but well scaled, generated on the device
        ML = (torch.randn(batch, n, m, device=dev) / np.sqrt(m)).float()
        G = (torch.randn(batch, m, n, device=dev) / np.sqrt(n)).float()
        base = problems.synthetic_qp(n, m, batch=1, seed=1)
    L = float(np.float32(base.L))
    M = torch.from_numpy((base.M[None, :] * (1 + 0.1 * rng.normal(size=(batch, 1)))).astype(np.float32)).to(dev)
    g = torch.from_numpy((base.g[None, :] + 0.1 * rng.random((batch, m))).astype(np.float32)).to(dev)
    z = torch.zeros(batch, n, device=dev)
    y = torch.zeros(batch, m, device=dev)
    with gpad_mpc.GpadSolver(0) as s:
        s.setup(ML, G, L, n=n, m=m, batch=batch, shared=shared, kernel=kc, check_every=check_every)
        s.run(z, y, M, g, N, tol)
        best = 1e30
        for _ in range(reps):
            z.zero_()
            y.zero_()
            st = s.run(z, y, M, g, N, tol)
            best = min(best, st["kernel_ms"])
    us_it = best * 1e3 / N
    F = 4 * n * m + 5 * m + 4 * n
    B = 4 * (2 * n * m + 4 * m + 3 * n) if not shared else 4 * (2 * n * m / batch + 4 * m + 3 * n)
    rate = batch * N / (best / 1e3)
    return dict(kernel=st["kernel"], n=n, m=m, batch=batch, shared=shared, N=N, tol=tol,
                us_per_iter=round(us_it, 3), inst_it_per_s=rate, tflops=rate * F / 1e12,
                alg_gbs=rate * B / 1e9)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--only", default="")
    ap.add_argument("--batch", type=int, default=0, help="only cases of this batch size")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--case", action="append", default=[],
                    help="kernel,n,m,batch,N (repeatable): run these instead of the default list")
    ap.add_argument("--check-every", type=int, default=10)
    ap.add_argument("--tol", type=float, default=0.0,
                    help="> 0: run the Algorithm-1 test path (tiny tol: never converges, N its)")
    args = ap.parse_args()
    cases = [
        ("resident", 40, 180, 1, 2000, True),
        ("resident", 200, 200, 1, 2000, True),
        ("stream", 200, 200, 1, 500, True),
        ("panel", 200, 200, 16, 500, True),
        ("panel", 200, 200, 4096, 300, True),
        ("panel", 200, 200, 8192, 300, True),
        ("panel", 200, 200, 16384, 200, True),
        ("resident", 200, 200, 8192, 100, True),
        ("stream", 800, 800, 1024, 20, False),
        ("stream", 200, 200, 8192, 50, False),
        ("resident", 200, 200, 8192, 100, False),
    ]
    if args.quick:
        cases = cases[:6]
    if args.case:
        cases = [(k, int(n), int(m), int(b), int(N), True) for k, n, m, b, N in (c.split(",") for c in args.case)]
    for c in cases:
        if args.only and args.only not in c[0]:
            continue
        if args.batch and c[3] != args.batch:
            continue
        print(json.dumps(case(*c, reps=args.reps, tol=args.tol, check_every=args.check_every)), flush=True)


if __name__ == "__main__":
    main()
