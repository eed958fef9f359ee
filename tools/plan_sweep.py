"""Phase schedule sweep for the C4 shard (GPU box): solve time of the planned schedule vs
unplanned uniform phases x finisher thresholds, one subprocess per setting.

  python3 tools/plan_sweep.py [--reps 6] [--batch 8192] [--fresh] [--takeover]
--takeover: the planned schedule vs one panel phase to iteration T, then the finisher (T = 230..310;
C3's shape of schedule at 4096 instances).
Prints one JSON line per setting: best / median solve ms over the reps (after two warm-up solves).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def one(reps, fresh=False, B=8192):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "gpu-dualgradient-mpc_amd"))
    import numpy as np
    import torch

    import bench
    import gpad_mpc
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import tune_env  # noqa: F401  (legacy GPAD_* env -> gpad_set_option)
    dev = torch.device("cuda:0")
    n, m = 200, 200
    ML, G, L, M, g = bench.make_shard(n, m, B, 0)
    f32 = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(dev)  # noqa: E731
    dML, dG, dM, dg = f32(ML), f32(G), f32(M), f32(g)
    # --fresh: a new batch every solve (bench.make_stream, the bench's honest mode)
    stream = [(f32(a), f32(b)) for a, b in bench.make_stream(n, m, B, reps + 2, 0)] if fresh else None
    z = torch.zeros(B, n, device=dev)
    y = torch.zeros(B, m, device=dev)
    s = gpad_mpc.GpadSolver(0)
    s.setup(dML, dG, float(np.float32(L)), n=n, m=m, batch=B, shared=True, check_every=10)
    t = []
    for i in range(reps + 2):
        z.zero_()
        y.zero_()
        Mv, gv = stream[i] if fresh else (dM, dg)
        s.run(z, y, Mv, gv, 5000, 1e-4, stats=False)
        st = s.last_stats()
        if i >= 2:
            t.append(st["kernel_ms"])
    t.sort()
    plan = s.phase_plan()
    print(json.dumps({"fresh": fresh, "env": {k: v for k, v in os.environ.items() if k.startswith("GPAD_")},
                      "best_ms": round(t[0], 4), "median_ms": round(t[len(t) // 2], 4),
                      "plan": plan}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--one", action="store_true")
    ap.add_argument("--fresh", action="store_true")
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--takeover", action="store_true")
    args = ap.parse_args()
    if args.one:
        one(args.reps, args.fresh, args.batch)
        return
    settings = [{}, {"GPAD_NO_LPT": "1"}]
    if args.takeover:
        for ph in range(230, 320, 10):
            settings.append({"GPAD_PANEL_NOPLAN": "1", "GPAD_PANEL_PHASE": str(ph), "GPAD_FINISH_THRESH": str(args.batch)})
    else:
        for ph in (20, 40, 80, 260):
            for fin in (512, 1024, 2048, 4096):
                settings.append({"GPAD_PANEL_NOPLAN": "1", "GPAD_PANEL_PHASE": str(ph), "GPAD_FINISH_THRESH": str(fin)})
    for st in settings:
        env = {k: v for k, v in os.environ.items() if not k.startswith("GPAD_")}
        env.update(st)
        cmd = [sys.executable, __file__, "--one", "--reps", str(args.reps), "--batch", str(args.batch)] + \
            (["--fresh"] if args.fresh else [])
        subprocess.run(cmd, env=env, check=True)


if __name__ == "__main__":
    main()
