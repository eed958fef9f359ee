"""Flat panel sweep: panels per workgroup (GPAD_FLAT_PANELS) x batch, C1 packs, fixed N.
GPU box: python tools/fp_sweep.py  (one subprocess per setting)"""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def one(n_u, Nh, batch, N):
    sys.path.insert(0, os.path.join(ROOT, "gpu-dualgradient-mpc_amd"))
    import torch

    import gpad_mpc
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import tune_env  # noqa: F401  (legacy GPAD_* env -> gpad_set_option)
    from gpad_mpc import problems
    dev = torch.device("cuda:0")
    qp = problems.battery_scenarios(n_u, Nh, batch, seed=9)
    MGf, GLf, L = problems.flatten_battery(qp, n_u, Nh)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(np.asarray(a, np.float64).astype(np.float32))).to(dev)  # noqa: E731
    L32 = float(np.float32(L))
    GP = t(qp.M).reshape(batch, -1)
    PD = (t(qp.g).reshape(batch, -1) * np.float32(-1.0 / np.float64(np.float32(L)))).contiguous()
    s = gpad_mpc.GpadSolver(0)
    s.setup_flat(t(MGf), t(GLf), L32, n_u=n_u, batch=batch, kernel=gpad_mpc.KERNEL_PANEL)
    Z = torch.zeros(batch, qp.n, device=dev)
    Y = torch.zeros(batch, qp.m, device=dev)
    s.run(Z, Y, GP, PD, N, 0.0, scaled=True)
    best = min(s.run(Z.zero_(), Y.zero_(), GP, PD, N, 0.0, scaled=True)["kernel_ms"] for _ in range(3))
    print(json.dumps({"n_u": n_u, "N": Nh, "batch": batch, "P": os.environ.get("GPAD_FLAT_PANELS"),
                      "alds": "GPAD_FLAT_NO_ALDS" not in os.environ, "us_per_iter": round(best * 1e3 / N, 3),
                      "iters_per_s": batch * N / (best / 1e3)}), flush=True)


def main():
    if len(sys.argv) > 1:
        one(*(int(x) for x in sys.argv[1:5]))
        return
    for batch in (8192, 16384):
        for P in ("1", "2", "3", "4"):
            for alds in (True, False):
                env = {k: v for k, v in os.environ.items() if not k.startswith("GPAD_")}
                env["GPAD_FLAT_PANELS"] = P
                if not alds:
                    env["GPAD_FLAT_NO_ALDS"] = "1"
                subprocess.run([sys.executable, __file__, "4", "10", str(batch), "200"], env=env, check=True)


if __name__ == "__main__":
    main()
