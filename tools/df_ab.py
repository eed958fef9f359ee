"""A/B of the dataflow GEMM boundaries (GPAD_OPT_PANEL_DATAFLOW, csrc/gpad_panel.hip DfWait):
fixed-N panel iterations (one launch, no test) and to-eps solves as bench.py's legs run them, each
variant on its own handle, interleaved over rounds; z*, y* and the counts of every variant must be
bit-identical to dataflow off.
  python3 tools/df_ab.py [--rounds 5] [--variants 0 1 5] [--pairs 0 2]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpu-dualgradient-mpc_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--variants", type=int, nargs="+", default=[0, 1, 5])  # one-panel bits (C3, 4096)
    ap.add_argument("--pairs", type=int, nargs="+", default=[0, 2, 3, 7])  # C4 shard (8192) bits
    ap.add_argument("--fixed-n", type=int, default=160)
    args = ap.parse_args()
    import torch

    import bench
    import gpad_mpc
    dev = torch.device("cuda:0")
    n = m = 200
    ML, G, L, _, _ = bench.make_shard(n, m, 1, 0)
    f32 = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(dev)  # noqa: E731
    L32 = float(np.float32(L))

    def case(name, B, variants, N, tol, phased):
        Mv, gv = [f32(x) for x in bench.make_stream(n, m, B, 1, 0)[0]]
        solvers, res, outs = {}, {}, {}
        for v in variants:
            s = gpad_mpc.GpadSolver(0)
            s.setup(f32(ML), f32(G), L32, n=n, m=m, batch=B, shared=True, check_every=10)
            s.set_options(phased=phased, panel_dataflow=v)
            z = torch.zeros(B, n, device=dev)
            y = torch.zeros(B, m, device=dev)
            for _ in range(2):  # warm-up; the second solve plans from the first
                s.run(z.zero_(), y.zero_(), Mv, gv, N, tol)
            solvers[v], res[v], outs[v] = (s, z, y), [], None
        for _ in range(args.rounds):
            for v, (s, z, y) in solvers.items():
                st = s.run(z.zero_(), y.zero_(), Mv, gv, N, tol)
                res[v].append(st["kernel_ms"])
                outs[v] = (z.cpu().numpy().copy(), y.cpu().numpy().copy(), st["total_iterations"])
        z0, y0, t0 = outs[variants[0]]
        for v in variants:
            z1, y1, t1 = outs[v]
            ms = res[v]
            print(json.dumps({"case": name, "batch": B, "N": N, "tol": tol, "dataflow": v,
                              "ms": [round(x, 4) for x in ms], "best_ms": round(min(ms), 4),
                              "median_ms": round(float(np.median(ms)), 4),
                              "us_per_iteration": round(min(ms) * 1e3 / N, 3) if tol == 0 else None,
                              "total_iterations": t1,
                              "bitexact_vs_first": bool(np.array_equal(z0, z1) and np.array_equal(y0, y1)
                                                        and t0 == t1)}), flush=True)
        for s, _, _ in solvers.values():
            s.close()

    case("one-panel fixed N", 4096, args.variants, args.fixed_n, 0.0, 0)
    case("C3 to eps", 4096, args.variants, 5000, 1e-4, 1)
    case("pairs fixed N", 8192, args.pairs, args.fixed_n, 0.0, 0)
    case("C4 shard to eps", 8192, args.pairs, 5000, 1e-4, 1)


if __name__ == "__main__":
    main()
