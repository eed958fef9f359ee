"""Why does a panel-pair iteration get cheaper as a solve goes on (profiles/r05_launch_cost_vecio.txt:
11.3 us per iteration over the first 10 at 8192 instances, 9.4 us between iterations 80 and 160)?
The work per iteration is fixed, so either the clock or the operand data changes.  Fixed-N solves of
N iterations (one launch, no test) at the C4 shape from different starting states:
  cold      : z = y = 0 (as every solve starts)
  warm@K    : (z, y) after K cold iterations (later-iteration operand data, same schedule restart)
  zeros     : M = g = 0 and z = y = 0: every operand of every MFMA stays exactly 0
Reports us per solve (best of reps) and us per iteration.
  python3 tools/iter_trend.py [--batch 8192] [--N 40] [--reps 5]"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpu-dualgradient-mpc_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--N", type=int, default=40)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--warm", type=int, nargs="+", default=[40, 160, 300])
    args = ap.parse_args()
    import torch

    import bench
    import gpad_mpc
    dev = torch.device("cuda:0")
    n = m = 200
    B, N = args.batch, args.N
    ML, G, L, _, _ = bench.make_shard(n, m, 1, 0)
    f32 = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(dev)  # noqa: E731
    Mv, gv = [f32(x) for x in bench.make_stream(n, m, B, 1, 0)[0]]
    with gpad_mpc.GpadSolver(0) as s:
        s.setup(f32(ML), f32(G), float(np.float32(L)), n=n, m=m, batch=B, check_every=10)
        s.set_options(phased=0)
        starts = {"cold": (torch.zeros(B, n, device=dev), torch.zeros(B, m, device=dev), Mv, gv)}
        for K in args.warm:
            z = torch.zeros(B, n, device=dev)
            y = torch.zeros(B, m, device=dev)
            s.run(z, y, Mv, gv, K, 0.0)
            starts[f"warm@{K}"] = (z, y, Mv, gv)
        starts["zeros"] = (torch.zeros(B, n, device=dev), torch.zeros(B, m, device=dev), torch.zeros_like(Mv),
                           torch.zeros_like(gv))
        out = {}
        for rep in range(args.reps):  # interleaved: the clock's history is the same for every start
            for name, (z0, y0, M, g) in starts.items():
                z, y = z0.clone(), y0.clone()
                torch.cuda.synchronize()
                st = s.run(z, y, M, g, N, 0.0)
                out.setdefault(name, []).append(st["kernel_ms"] * 1e3)
        for name, t in out.items():
            print(json.dumps({"batch": B, "N": N, "start": name, "us_best": round(min(t), 2),
                              "us_median": round(float(np.median(t)), 2),
                              "us_per_iteration_best": round(min(t) / N, 3)}))


if __name__ == "__main__":
    main()
