"""A/B of the f64 panel layouts (csrc/gpad_panel64.hip) on bench.py's f64 value leg: 8192 C4-shaped
value problems, H bound, e_g = e_V = 1e-6; options interleaved over rounds on one handle each
(relay+refill+lpt: refills in longest-predicted-first order from the handle's previous counts, r06).

  python tools/p64_ab.py [--rounds 3] [--batch 8192] [--small]
--small adds the ADVICE r04 small-shape check: n = 40, m = 53 at 4096 instances (f64, no H, eps
1e-8), the f64 panels (occupancy-sized grid) against the f64 stream kernel.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpu-dualgradient-mpc_amd"), os.path.join(ROOT, "tests")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--small", action="store_true")
    ap.add_argument("--only", nargs="*", default=None, help="variant names to run")
    args = ap.parse_args()
    import torch

    import gpad_mpc
    from gpad_mpc import _lib, problems
    from test_value import value_problem
    dev = torch.device("cuda:0")
    n = m = 200
    B, tol = args.batch, 1e-6
    H, ML, M, G, g, L, _ = value_problem(n, m, 7, 1.0, batch=B)
    f64 = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float64)).to(dev)  # noqa: E731
    dH, dML, dG, dM, dg = f64(H), f64(ML), f64(G), f64(M), f64(g)
    z = torch.zeros(B, n, dtype=torch.float64, device=dev)
    y = torch.zeros(B, m, dtype=torch.float64, device=dev)
    variants = {"relay+refill+lpt": {"p64_relay": 1, "p64_refill": 1, "lpt": 1},
                "relay+refill": {"p64_relay": 1, "p64_refill": 1, "lpt": 0},
                "relay": {"p64_relay": 1, "p64_refill": 0}, "tiles": {"p64_relay": 0, "p64_refill": 0}}
    if args.only:
        variants = {k: v for k, v in variants.items() if k in args.only}
    solvers = {}
    for name, opts in variants.items():
        s = gpad_mpc.GpadSolver(0)
        s.setup(dML, dG, float(L), n=n, m=m, batch=B, shared=True, check_every=10, kernel=_lib.KERNEL_PANEL,
                tol_gap=tol)
        s.setup_hessian(dH)
        s.set_options(**opts)
        s.run(z.zero_(), y.zero_(), dM, dg, 20000, tol)  # warm-up
        solvers[name] = s
    res = {k: [] for k in variants}
    for _ in range(args.rounds):
        for name, s in solvers.items():
            st = s.run(z.zero_(), y.zero_(), dM, dg, 20000, tol)
            res[name].append(st["kernel_ms"])
            tot = st["total_iterations"]
    for name in variants:
        best = min(res[name])
        tf = tot * 4.0 * n * m / (best / 1e3) / 1e12
        print(json.dumps({"variant": name, "ms": [round(x, 3) for x in res[name]], "best_ms": round(best, 3),
                          "iters_per_s": tot / (best / 1e3), "tflops_2matvec": round(tf, 2),
                          "frac_of_78.6": round(tf / 78.6, 4)}))
    # fixed N = 400 (no test, every column busy): the layout's panel-iteration time
    fixed = {k: [] for k in variants}
    for _ in range(args.rounds):
        for name, s in solvers.items():
            st = s.run(z.zero_(), y.zero_(), dM, dg, 400, 0.0)
            fixed[name].append(st["kernel_ms"])
    panels = (B + 15) // 16
    for name in variants:
        best = min(fixed[name])
        print(json.dumps({"variant": name, "fixed_N": 400, "best_ms": round(best, 3),
                          "us_per_panel_iteration_per_cu": round(best * 1e3 / 400 / (panels / 256), 3),
                          "tflops_2matvec": round(B * 400 * 4.0 * n * m / (best / 1e3) / 1e12, 2)}))
    for s in solvers.values():
        s.close()
    if args.small:
        ns, ms_, Bs = 40, 53, 4096
        qp = problems.synthetic_qp(ns, ms_, batch=Bs, seed=3)
        a = [f64(np.asarray(x)) for x in (qp.ML, qp.G, np.asarray(qp.M).reshape(Bs, ns), np.asarray(qp.g).reshape(Bs, ms_))]
        out = {}
        for name, kern in (("panel64", _lib.KERNEL_PANEL), ("stream", _lib.KERNEL_STREAM)):
            zz = torch.zeros(Bs, ns, dtype=torch.float64, device=dev)
            yy = torch.zeros(Bs, ms_, dtype=torch.float64, device=dev)
            with gpad_mpc.GpadSolver(0) as s:
                s.setup(a[0], a[1], float(qp.L), n=ns, m=ms_, batch=Bs, shared=True, kernel=kern)
                s.run(zz.zero_(), yy.zero_(), a[2], a[3], 2000, 1e-8)
                t = []
                for _ in range(3):
                    st = s.run(zz.zero_(), yy.zero_(), a[2], a[3], 2000, 1e-8)
                    t.append(st["kernel_ms"])
            out[name] = {"best_ms": round(min(t), 4), "iters_per_s": st["total_iterations"] / (min(t) / 1e3),
                         "mean_iters": st["total_iterations"] / Bs}
        print(json.dumps({"small_shape": f"n={ns} m={ms_} batch={Bs} f64 eps=1e-8", **out}))


if __name__ == "__main__":
    main()
