"""C4 shard on the opt-in condensed operator: best / median solve ms over --reps solves after two
warm-ups (the first plans the takeover), fresh inputs per solve (bench.make_stream).  A/B with
GPAD_LIB=<build>."""
from __future__ import annotations

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "gpu-dualgradient-mpc_amd"))


def main(reps=10):
    import numpy as np
    import torch

    import bench
    import gpad_mpc
    from gpad_mpc import _lib
    dev = torch.device("cuda:0")
    n, m, B = 200, 200, 8192
    ML, G, L, M, g = bench.make_shard(n, m, B, 0)
    f32 = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(dev)  # noqa: E731
    stream = [(f32(a), f32(b)) for a, b in bench.make_stream(n, m, B, reps + 2, 0)]
    z = torch.zeros(B, n, device=dev)
    y = torch.zeros(B, m, device=dev)
    t = []
    with gpad_mpc.GpadSolver(0) as s:
        s.setup(f32(ML), f32(G), float(np.float32(L)), n=n, m=m, batch=B, kernel=_lib.KERNEL_CONDENSED)
        for i in range(reps + 2):
            st = s.run(z.zero_(), y.zero_(), *stream[i], 5000, 1e-4)
            if i >= 2:
                t.append(st["kernel_ms"])
    t.sort()
    print(json.dumps({"lib": os.path.basename(os.environ.get("GPAD_LIB", "libgpad.so")),
                      "best_ms": round(t[0], 4), "median_ms": round(t[len(t) // 2], 4)}), flush=True)


if __name__ == "__main__":
    main()
