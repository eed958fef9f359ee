"""C4 shard on the opt-in condensed operator (GPAD_KERNEL_CONDENSED), for rocprofv3:
  PROFILE_SCRIPT=tools/cond_run.py bash tools/profile.sh r02_cond
Solves the bench's C4 shard to eps 1e-4 (--steps + --warmup times; the first plans the takeover);
unknown bench-style arguments are ignored."""
from __future__ import annotations

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "gpu-dualgradient-mpc_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--warmup", type=int, default=1)
    args, _ = ap.parse_known_args()
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
    with gpad_mpc.GpadSolver(0, stream=torch.cuda.current_stream(dev).cuda_stream) as s:
        s.setup(dML, dG, float(np.float32(L)), n=n, m=m, batch=B, kernel=_lib.KERNEL_CONDENSED)
        for _ in range(args.steps + args.warmup):
            st = s.run(z.zero_(), y.zero_(), dM, dg, 5000, 1e-4)
    print("condensed C4 solve ms", st["kernel_ms"], "iterations", st["total_iterations"])


if __name__ == "__main__":
    main()
