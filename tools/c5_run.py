"""C5 alone (1024 distinct 800x800 instances, HBM-streaming kernel) for a PMC cross-check of the
bench leg's algorithmic GB/s:  PROFILE_SCRIPT=tools/c5_run.py bash tools/profile.sh r01_c5 --steps 2
(--steps = timed launches after one warm-up; each launch runs 20 iterations)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "gpu-dualgradient-mpc_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-extra", action="store_true")
    args = ap.parse_args()
    import torch

    import bench
    dev = torch.device("cuda:0")
    out = [bench.hbm_leg(dev) for _ in range(args.steps)]
    print(json.dumps(out[-1]), flush=True)


if __name__ == "__main__":
    main()
