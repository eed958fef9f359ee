"""A fresh handle's first phased solve: in a warm process where another handle
has solved the shape, a new handle follows the shape's plan prior (csrc/gpad_host.cpp plan_for)
instead of the default schedule.  Fresh C4-shard inputs every solve (bench.make_stream):
  A        : 4 solves on one handle (its plans become the shape's prior)
  B first  : a new handle's first solve (prior)            B planned : its next 4 (own plans)
  C first  : a new handle with GPAD_OPT_PLAN = 0 (the default schedule a first solve ran before r06)
Rounds interleave B / C handles; device ms per solve (HIP events), best and median.
  python3 tools/first_solve.py [--rounds 4] [--batch 8192]"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpu-dualgradient-mpc_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--batch", type=int, default=8192)
    args = ap.parse_args()
    import torch

    import bench
    import gpad_mpc
    dev = torch.device("cuda:0")
    n = m = 200
    B = args.batch
    ML, G, L, _, _ = bench.make_shard(n, m, 1, 0)
    f32 = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(dev)  # noqa: E731
    dML, dG, L32 = f32(ML), f32(G), float(np.float32(L))
    stream = [(f32(a), f32(b)) for a, b in bench.make_stream(n, m, B, 4 + 6 * args.rounds, 0)]
    z = torch.zeros(B, n, device=dev)
    y = torch.zeros(B, m, device=dev)
    k = 0

    def solve(s):
        nonlocal k
        Mv, gv = stream[k % len(stream)]
        k += 1
        st = s.run(z.zero_(), y.zero_(), Mv, gv, 5000, 1e-4, iters=np.zeros(B, np.int32))
        return st["kernel_ms"], s.last_phases()

    def handle(plan=1):
        s = gpad_mpc.GpadSolver(0)
        s.setup(dML, dG, L32, n=n, m=m, batch=B, shared=True, check_every=10)
        if not plan:
            s.set_options(plan=0)
        return s

    a = handle()
    for _ in range(4):
        solve(a)
    res = {"B_first": [], "B_planned": [], "C_first_default": []}
    prior_used = []
    for _ in range(args.rounds):
        b = handle()
        ms, ph = solve(b)
        res["B_first"].append(ms)
        prior_used.append(ph["prior"])
        for _ in range(4):
            res["B_planned"].append(solve(b)[0])
        b.close()
        c = handle(plan=0)
        res["C_first_default"].append(solve(c)[0])
        c.close()
    a.close()
    out = {k2: {"best_ms": round(min(v), 4), "median_ms": round(float(np.median(v)), 4), "n": len(v)}
           for k2, v in res.items()}
    out["prior_followed"] = prior_used
    out["B_first_over_planned_median"] = round(float(np.median(res["B_first"]) / np.median(res["B_planned"])), 4)
    out["C_first_over_planned_median"] = round(float(np.median(res["C_first_default"]) / np.median(res["B_planned"])), 4)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
