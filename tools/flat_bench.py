"""Flat vs full battery path, per-iteration cost (fixed N), single instance and batches.
Usage (GPU box): python tools/flat_bench.py"""
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
    for n_u, Nh in ((4, 10), (4, 50)):
        for batch, N in ((1, 2000), (8192, 100)):
            qp = problems.battery_scenarios(n_u, Nh, batch, seed=9)
            MGf, GLf, L = problems.flatten_battery(qp, n_u, Nh)
            t = lambda a: torch.from_numpy(np.ascontiguousarray(np.asarray(a, np.float64).astype(np.float32))).to(dev)  # noqa: E731
            L32 = float(np.float32(L))
            GP = t(qp.M).reshape(batch, -1)
            PD = (t(qp.g).reshape(batch, -1) * np.float32(-1.0 / np.float64(np.float32(L)))).contiguous()
            row = {"n_u": n_u, "N": Nh, "n": qp.n, "m": qp.m, "batch": batch}
            for name in ("flat", "flat_chains", "full"):
                s = gpad_mpc.GpadSolver(0)
                if name == "flat":  # auto: the MFMA flat panels at large batches
                    s.setup_flat(t(MGf), t(GLf), L32, n_u=n_u, batch=batch)
                elif name == "flat_chains":  # the per-instance flat kernels (register / LDS chains)
                    s.setup_flat(t(MGf), t(GLf), L32, n_u=n_u, batch=batch, kernel=_lib.KERNEL_RESIDENT)
                else:
                    s.setup(-t(qp.ML), t(qp.G) / np.float32(L32), L32, n=qp.n, m=qp.m, batch=batch,
                            scaled=True)
                Z = torch.zeros(batch, qp.n, device=dev)
                Y = torch.zeros(batch, qp.m, device=dev)
                s.run(Z, Y, GP, PD, N, 0.0, scaled=True)
                best = min(s.run(Z.zero_(), Y.zero_(), GP, PD, N, 0.0, scaled=True)["kernel_ms"] for _ in range(3))
                st = s.last_stats()
                row[name] = {"kernel": st["kernel"], "us_per_iter": round(best * 1e3 / N, 3),
                             "iters_per_s": batch * N / (best / 1e3)}
                s.close()
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
