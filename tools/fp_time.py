"""Per-phase cycle split of the flat panel kernel (build with -DFP_TIMING into tools/fpt/fptime.so):
GPAD_LIB=tools/fpt/fptime.so python tools/fp_time.py N_u N batch iters"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-dualgradient-mpc_amd"))


def main():
    import torch

    import gpad_mpc
    from gpad_mpc import problems
    n_u, Nh, batch, N = (int(x) for x in sys.argv[1:5])
    dev = torch.device("cuda:0")
    qp = problems.battery_scenarios(n_u, Nh, batch, seed=9)
    MGf, GLf, L = problems.flatten_battery(qp, n_u, Nh)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(np.asarray(a, np.float64).astype(np.float32))).to(dev)  # noqa: E731
    L32 = float(np.float32(L))
    GP = t(qp.M).reshape(batch, -1)
    PD = (t(qp.g).reshape(batch, -1) * np.float32(-1.0 / np.float64(np.float32(L)))).contiguous()
    s = gpad_mpc.GpadSolver(0)
    s.setup_flat(t(MGf), t(GLf), L32, n_u=n_u, batch=batch)
    Z = torch.zeros(batch, qp.n, device=dev)
    Y = torch.zeros(batch, qp.m, device=dev)
    st = s.run(Z, Y, GP, PD, N, 0.0, scaled=True)
    print("kernel_ms", st["kernel_ms"], "us/iter", st["kernel_ms"] * 1e3 / N, flush=True)


if __name__ == "__main__":
    main()
