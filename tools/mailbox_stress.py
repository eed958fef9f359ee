"""Mailbox stress (tools; GPU box): fresh C4-generator batches solved with and without the finisher's
slot hand-off (GPAD_OPT_DUO_MAILBOX), results compared bit for bit, counts included -- the hand-off's
interleavings differ from solve to solve, its results must not.
  python3 tools/mailbox_stress.py [--rounds 6] [--batch 8192 4096]
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
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--batch", type=int, nargs="+", default=[8192, 4096])
    args = ap.parse_args()
    import torch

    import bench
    import gpad_mpc
    dev = torch.device("cuda:0")
    n = m = 200
    ML, G, L, _, _ = bench.make_shard(n, m, 1, 0)
    f32 = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(dev)  # noqa: E731
    for B in args.batch:
        draws = [(f32(a), f32(b)) for a, b in bench.make_stream(n, m, B, args.rounds, 5)]
        sol = {}
        for mb in (0, 1):
            s = gpad_mpc.GpadSolver(0)
            s.setup(f32(ML), f32(G), float(np.float32(L)), n=n, m=m, batch=B, shared=True, check_every=10)
            s.set_options(duo_mailbox=mb)
            sol[mb] = s
        bad = 0
        for k, (Mv, gv) in enumerate(draws):
            out = {}
            for mb, s in sol.items():
                z = torch.zeros(B, n, device=dev)
                y = torch.zeros(B, m, device=dev)
                it = np.zeros(B, np.int32)
                st = s.run(z, y, Mv, gv, 5000, 1e-4, iters=it)
                out[mb] = (z.cpu().numpy(), y.cpu().numpy(), it, st["kernel_ms"])
            same = all(np.array_equal(out[0][i], out[1][i]) for i in range(3))
            bad += not same
            print(json.dumps({"batch": B, "round": k, "bitexact": same, "ms_off": round(out[0][3], 3),
                              "ms_mailbox": round(out[1][3], 3)}), flush=True)
        for s in sol.values():
            s.close()
        assert bad == 0, f"{bad} rounds differ at batch {B}"


if __name__ == "__main__":
    main()
