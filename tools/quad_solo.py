"""Per-iteration cost of the finisher kernels on ONE workgroup (tools; GPU box):
  python3 tools/quad_solo.py
duo with 1 / 2 live instances, quad with 1..8 (slot 0 fills first: 4 = one full MFMA slot, 5 = a
full slot beside a DPP slot, 8 = two full MFMA slots).  Tol mode with a tolerance no instance
meets (every 10th iteration runs the test); us per slot-iteration from the N = 210 / 1010 difference."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "gpu-dualgradient-mpc_amd"))


def main():
    import torch

    import bench
    import gpad_mpc
    from gpad_mpc import _lib
    dev = torch.device("cuda:0")
    ML, G, L, M, g = bench.make_shard(200, 200, 8, 0)
    f32 = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(dev)  # noqa: E731
    dML, dG, dM, dg = f32(ML), f32(G), f32(M), f32(g)
    out = {}
    cases = [("duo", 1, 0), ("duo", 2, 0)] + [("quad", b, 1) for b in (1, 2, 4, 5, 8)]
    for name, B, quad in cases:
        with gpad_mpc.GpadSolver(0) as s:
            s.setup(dML, dG, float(np.float32(L)), n=200, m=200, batch=B, kernel=_lib.KERNEL_PANEL)
            s.set_options(phase_len=10, finish_thresh=100000, duo_max_grid=1, quad_finisher=quad)
            best = {}
            for N in (210, 1010):
                t = []
                for _ in range(4):
                    z = torch.zeros(B, 200, device=dev)
                    y = torch.zeros(B, 200, device=dev)
                    st = s.run(z, y, dM[:B], dg[:B], N, 1e-12)
                    t.append(st["kernel_ms"])
                best[N] = min(t)
            out[f"{name}_{B}"] = round((best[1010] - best[210]) / 800 * 1e3, 4)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
