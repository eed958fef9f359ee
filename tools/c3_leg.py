"""bench.py's C3 leg alone (4096 instances sharing ML/G to eps, best of 3 after 2 planning solves):
  python3 tools/c3_leg.py  -> one JSON line (GPAD_LIB / GPAD_LIB_TOLERANT select an A/B build)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpu-dualgradient-mpc_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

out = bench.c3_leg(torch.device("cuda:0"))
print(json.dumps({k: out[k] for k in ("iters_per_s", "solve_ms", "mean_iters_to_eps")}))
