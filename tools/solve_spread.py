"""Per-solve spread of the fresh-input C4 step: for each of R fresh batches (bench.make_stream, the
bench's own inputs), the solve's device time (HIP events) and the phases it launched with the
survivors each boundary handed on (gpad_last_phases) -- which solves are slow, and where.
  python3 tools/solve_spread.py [--reps 20] [--batch 8192]"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpu-dualgradient-mpc_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--opt", nargs="*", default=[], help="handle options name=value")
    args = ap.parse_args()
    import torch

    import bench
    import gpad_mpc
    dev = torch.device("cuda:0")
    n = m = 200
    B = args.batch
    ML, G, L, _, _ = bench.make_shard(n, m, 1, 0)
    f32 = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(dev)  # noqa: E731
    stream = [(f32(a), f32(b)) for a, b in bench.make_stream(n, m, B, args.warmup + args.reps, 0)]
    z = torch.zeros(B, n, device=dev)
    y = torch.zeros(B, m, device=dev)
    rows = []
    with gpad_mpc.GpadSolver(0) as s:
        s.setup(f32(ML), f32(G), float(np.float32(L)), n=n, m=m, batch=B, shared=True, check_every=10)
        s.set_options(**{k: int(v) for k, v in (o.split("=") for o in args.opt)})
        for k, (Mv, gv) in enumerate(stream):
            it = np.zeros(B, np.int32)
            st = s.run(z.zero_(), y.zero_(), Mv, gv, 5000, 1e-4, iters=it)
            ph = s.last_phases()
            if k >= args.warmup:
                rows.append({"solve": k, "ms": round(st["kernel_ms"], 4), "ends": ph["ends"], "counts": ph["counts"],
                             "fins": ph["fins"], "takeover": ph["takeover"], "max_iter": int(it.max()),
                             "iters": int(it.sum())})
                print(json.dumps(rows[-1]), flush=True)
    ms = np.array([r["ms"] for r in rows])
    print(json.dumps({"mean_ms": round(float(ms.mean()), 4), "median_ms": round(float(np.median(ms)), 4),
                      "min_ms": round(float(ms.min()), 4), "max_ms": round(float(ms.max()), 4),
                      "opts": args.opt}))


if __name__ == "__main__":
    main()
