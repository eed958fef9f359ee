"""f64 value problems (bench.py f64_value_leg): the per-instance iteration distribution and the
latency of the f64 stream kernel at one instance per CU -- the inputs of a tail-finisher estimate.
  python3 tools/f64_tail.py [--batch 8192]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpu-dualgradient-mpc_amd"), os.path.join(ROOT, "tests")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8192)
    args = ap.parse_args()
    import torch

    import gpad_mpc
    from gpad_mpc import _lib
    from test_value import value_problem
    dev = torch.device("cuda:0")
    n = m = 200
    B, tol = args.batch, 1e-6
    H, ML, M, G, g, L, _ = value_problem(n, m, 7, 1.0, batch=B)
    f64 = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float64)).to(dev)  # noqa: E731
    dH, dML, dG, dM, dg = f64(H), f64(ML), f64(G), f64(M), f64(g)
    z = torch.zeros(B, n, dtype=torch.float64, device=dev)
    y = torch.zeros(B, m, dtype=torch.float64, device=dev)
    iters = np.zeros(B, np.int32)
    with gpad_mpc.GpadSolver(0) as s:
        s.setup(dML, dG, float(L), n=n, m=m, batch=B, shared=True, check_every=10, kernel=_lib.KERNEL_PANEL,
                tol_gap=tol)
        s.setup_hessian(dH)
        s.run(z.zero_(), y.zero_(), dM, dg, 20000, tol)
        st = s.run(z.zero_(), y.zero_(), dM, dg, 20000, tol, iters=iters)
    q = np.percentile(iters, [0, 10, 25, 50, 75, 90, 99, 100])
    cols = 256 * 16
    lb_mean = iters.sum() / cols
    print(json.dumps({"batch": B, "panel_ms": st["kernel_ms"], "mean": float(iters.mean()),
                      "quantiles_0_10_25_50_75_90_99_100": [int(x) for x in q],
                      "lower_bound_iterations_per_column_mean": float(lb_mean), "max": int(iters.max()),
                      "utilisation_vs_mean_bound": float(lb_mean * 12.8e-3 / st["kernel_ms"])}), flush=True)
    # latency mode: the f64 stream kernel, the 256 longest instances, one per CU
    order = np.argsort(-iters)[:256]
    idx = torch.from_numpy(order.astype(np.int64)).to(dev)
    for kname, kern in (("stream", _lib.KERNEL_STREAM),):
        z2 = torch.zeros(256, n, dtype=torch.float64, device=dev)
        y2 = torch.zeros(256, m, dtype=torch.float64, device=dev)
        it2 = np.zeros(256, np.int32)
        with gpad_mpc.GpadSolver(0) as s:
            s.setup(dML, dG, float(L), n=n, m=m, batch=256, shared=True, check_every=10, kernel=kern,
                    tol_gap=tol)
            s.setup_hessian(dH)
            s.run(z2, y2, dM[idx].contiguous(), dg[idx].contiguous(), 20000, tol)
            st2 = s.run(z2.zero_(), y2.zero_(), dM[idx].contiguous(), dg[idx].contiguous(), 20000, tol, iters=it2)
        print(json.dumps({"latency_kernel": kname, "instances": 256, "ms": st2["kernel_ms"], "max_iters": int(it2.max()),
                          "us_per_iteration_of_longest": st2["kernel_ms"] * 1e3 / max(1, int(it2.max()))}), flush=True)


if __name__ == "__main__":
    main()
