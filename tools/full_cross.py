"""Shared full matrices beyond the register budget (battery N=50: n=200, m=900): big panel vs
stream kernel by batch.  GPU box: python tools/full_cross.py"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-dualgradient-mpc_amd"))


def main():
    import torch

    import gpad_mpc
    from gpad_mpc import _lib, problems
    dev = torch.device("cuda:0")
    for batch in (1, 4, 16, 32, 64, 128):
        qp = problems.battery_scenarios(4, 50, batch, seed=9)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(np.asarray(a, np.float64).astype(np.float32))).to(dev)  # noqa: E731
        L32 = float(np.float32(qp.L))
        GP = t(qp.M).reshape(batch, -1)
        PD = (t(qp.g).reshape(batch, -1) * np.float32(-1.0 / np.float64(np.float32(qp.L)))).contiguous()
        row = {"batch": batch}
        for name, k in (("panel", _lib.KERNEL_PANEL), ("stream", _lib.KERNEL_STREAM)):
            s = gpad_mpc.GpadSolver(0)
            s.setup(-t(qp.ML), t(qp.G) / np.float32(L32), L32, n=qp.n, m=qp.m, batch=batch, scaled=True, kernel=k)
            Z = torch.zeros(batch, qp.n, device=dev)
            Y = torch.zeros(batch, qp.m, device=dev)
            s.run(Z, Y, GP, PD, 200, 0.0, scaled=True)
            best = min(s.run(Z.zero_(), Y.zero_(), GP, PD, 200, 0.0, scaled=True)["kernel_ms"] for _ in range(3))
            row[name] = {"kernel": s.last_stats()["kernel"], "us_per_iter": round(best * 1e3 / 200, 3)}
            s.close()
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
