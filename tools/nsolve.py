"""Fixed-N panel solves of the C4-generator shard, for PMC passes (tools only):
  python3 tools/nsolve.py --batch 4096 --N 1 --reps 4"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpu-dualgradient-mpc_amd")]

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=4096)
ap.add_argument("--N", type=int, default=1)
ap.add_argument("--reps", type=int, default=4)
args = ap.parse_args()
import torch  # noqa: E402

import bench  # noqa: E402
import gpad_mpc  # noqa: E402
dev = torch.device("cuda:0")
n = m = 200
B = args.batch
ML, G, L, _, _ = bench.make_shard(n, m, 1, 0)
f32 = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(dev)  # noqa: E731
Mv, gv = [f32(x) for x in bench.make_stream(n, m, B, 1, 0)[0]]
z = torch.zeros(B, n, device=dev)
y = torch.zeros(B, m, device=dev)
with gpad_mpc.GpadSolver(0) as s:
    s.setup(f32(ML), f32(G), float(np.float32(L)), n=n, m=m, batch=B, check_every=10)
    s.set_options(phased=0)
    for _ in range(args.reps):
        st = s.run(z.zero_(), y.zero_(), Mv, gv, args.N, 0.0)
print("last kernel_ms", st["kernel_ms"])
