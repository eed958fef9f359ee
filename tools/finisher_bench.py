"""Latency-kernel finishers of a phased panel solve, head to head (GPU box).

The finisher takes every survivor after the first 10-iteration panel phase
(GPAD_PANEL_PHASE=10, GPAD_FINISH_THRESH large) and runs it to N with a tolerance nothing meets,
so the solve is ~N iterations of the finisher over the whole batch.  Prints one JSON line per
(finisher, batch): solve ms, us per instance-iteration and per slot-iteration.
  python tools/finisher_bench.py [--n 200 --m 200 --N 1000]
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-dualgradient-mpc_amd"))


def one(args):
    import numpy as np
    import torch

    import gpad_mpc
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import tune_env  # noqa: F401  (legacy GPAD_* env -> gpad_set_option)
    from gpad_mpc import _lib, problems
    dev = torch.device("cuda:0")
    n, m, B, N = args.n, args.m, args.batch, args.N
    qp = problems.synthetic_qp(n, m, batch=1, seed=1)
    ML = torch.from_numpy(qp.ML.astype(np.float32)).to(dev)
    G = torch.from_numpy(qp.G.astype(np.float32)).to(dev)
    rng = np.random.default_rng(0)
    M = torch.from_numpy((qp.M[None, :] * (1 + 0.1 * rng.normal(size=(B, 1)))).astype(np.float32)).to(dev)
    g = torch.from_numpy((qp.g[None, :] + 0.1 * rng.random((B, m))).astype(np.float32)).to(dev)
    z = torch.zeros(B, n, device=dev)
    y = torch.zeros(B, m, device=dev)
    best = 1e30
    with gpad_mpc.GpadSolver(0) as s:
        s.setup(ML, G, float(np.float32(qp.L)), n=n, m=m, batch=B, shared=True, kernel=_lib.KERNEL_PANEL)
        for _ in range(4):
            z.zero_()
            y.zero_()
            st = s.run(z, y, M, g, N, 1e-30)
            best = min(best, st["kernel_ms"])
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    slots = min(B, 2 * ncu) if os.environ.get("GPAD_FINISHER", "duo") == "duo" else min(B, ncu)
    print(json.dumps(dict(finisher=os.environ.get("GPAD_FINISHER", "duo"), n=n, m=m, batch=B, N=N,
                          ms=round(best, 3), us_per_inst_iter=round(best * 1e3 / (B * N), 5),
                          us_per_slot_iter=round(best * 1e3 * slots / (B * N), 4))), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=200)
    ap.add_argument("--m", type=int, default=200)
    ap.add_argument("--N", type=int, default=1000)
    ap.add_argument("--batch", type=int, default=0)
    args = ap.parse_args()
    if args.batch:
        one(args)
        return
    for fin in ("duo", "resident"):
        for B in (1, 256, 512, 1024, 2048):
            env = dict(os.environ, GPAD_FINISHER=fin, GPAD_PANEL_PHASE="10", GPAD_FINISH_THRESH="1000000",
                       GPAD_PANEL_NOPLAN="1")
            subprocess.run([sys.executable, __file__, "--n", str(args.n), "--m", str(args.m), "--N", str(args.N),
                            "--batch", str(B)], env=env, check=True)


if __name__ == "__main__":
    main()
