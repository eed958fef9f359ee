"""Per-launch cost of the panel solve: fixed-N solves (one launch, no test) at several N; the
intercept of time vs N is the launch's fixed cost, the slope the iteration time.
  python3 tools/launch_cost.py [--batch 4096 8192]"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpu-dualgradient-mpc_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, nargs="+", default=[4096, 8192])
    ap.add_argument("--tol", type=float, default=0.0)
    args = ap.parse_args()
    import torch

    import bench
    import gpad_mpc
    dev = torch.device("cuda:0")
    n = m = 200
    ML, G, L, _, _ = bench.make_shard(n, m, 1, 0)
    f32 = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(dev)  # noqa: E731
    for B in args.batch:
        Mv, gv = [f32(x) for x in bench.make_stream(n, m, B, 1, 0)[0]]
        z = torch.zeros(B, n, device=dev)
        y = torch.zeros(B, m, device=dev)
        rows = []
        with gpad_mpc.GpadSolver(0) as s:
            s.setup(f32(ML), f32(G), float(np.float32(L)), n=n, m=m, batch=B, check_every=10)
            s.set_options(phased=0)
            for N in (1, 2, 10, 20, 40, 80, 160):
                t = []
                for _ in range(5):
                    st = s.run(z.zero_(), y.zero_(), Mv, gv, N, args.tol)
                    t.append(st["kernel_ms"] * 1e3)
                rows.append((N, min(t)))
        Ns = np.array([r[0] for r in rows if r[0] >= 10], float)
        ts = np.array([r[1] for r in rows if r[0] >= 10], float)
        slope, icpt = np.polyfit(Ns, ts, 1)
        print(json.dumps({"batch": B, "tol": args.tol, "us_by_N": {str(a): round(b, 2) for a, b in rows},
                          "fit_us_per_iteration": round(slope, 3), "fit_launch_us": round(icpt, 2)}))


if __name__ == "__main__":
    main()
