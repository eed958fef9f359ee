"""Condensed C4 shard: solve time vs the finisher takeover iteration (GPAD_OPT_PHASE_LEN forces it;
0 = planned from the previous solve's counts).  One JSON line per setting."""
from __future__ import annotations

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "gpu-dualgradient-mpc_amd"))


def main():
    import numpy as np
    import torch

    import bench
    import gpad_mpc
    from gpad_mpc import _lib
    dev = torch.device("cuda:0")
    n, m, B = 200, 200, 8192
    ML, G, L, M, g = bench.make_shard(n, m, B, 0)
    f32 = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(dev)  # noqa: E731
    dML, dG, dM, dg = f32(ML), f32(G), f32(M), f32(g)
    z = torch.zeros(B, n, device=dev)
    y = torch.zeros(B, m, device=dev)
    for take in (290, 300, 0, 5000, 0):
        with gpad_mpc.GpadSolver(0, stream=torch.cuda.current_stream(dev).cuda_stream) as s:
            s.setup(dML, dG, float(np.float32(L)), n=n, m=m, batch=B, kernel=_lib.KERNEL_CONDENSED)
            s.set_option("phase_len", take if take < 5000 else 0)
            if take >= 5000:
                s.set_option("phased", 0)
            t = []
            it = np.zeros(B, np.int32)
            for k in range(6):
                st = s.run(z.zero_(), y.zero_(), dM, dg, 5000, 1e-4, iters=it)
                if k >= 2:
                    t.append(st["kernel_ms"])
        surv = int((it > take).sum()) if take < 5000 else 0
        if take == 0:  # the host model (gpad_cpanel.hip cpanel_takeover) on these counts
            T = 13
            tp = ((2 * T + 3) // 4) * T * 4 * 32 / 2.2e3 + 1.5
            tl = 1.6
            cost = {}
            for v in range(10, int(it.max()) + 1, 10):
                r = np.maximum(it.astype(np.int64) - v, 0)
                cost[v] = v * tp + 25.0 + max(int(r.max()) * tl, float(r.sum()) * tl / 256)
            vbest = min(cost, key=cost.get)
            print(json.dumps({"model_takeover": vbest, "model_us": {k: round(c) for k, c in cost.items() if k >= 240}}),
                  flush=True)
        print(json.dumps({"takeover": take or "planned", "best_ms": round(min(t), 4), "median_ms": round(sorted(t)[2], 4),
                          "survivors_at_takeover": surv, "max_iters": int(it.max())}), flush=True)


if __name__ == "__main__":
    main()
