"""Per-iteration cost of the duo finisher when one slot is live (the end of every solve tail)
against the resident kernel on the same instance (tools; GPU box):
  python3 tools/duo_solo.py
Both in tol mode with a tolerance no instance meets (every 10th iteration runs the test)."""
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
    ML, G, L, M, g = bench.make_shard(200, 200, 2, 0)
    f32 = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(dev)  # noqa: E731
    dML, dG, dM, dg = f32(ML), f32(G), f32(M), f32(g)
    out = {}
    for name, B, kern, opts in (("resident", 1, _lib.KERNEL_RESIDENT, {}),
                                ("duo_one_slot", 1, _lib.KERNEL_PANEL, dict(phase_len=10, finish_thresh=100000)),
                                ("duo_two_slots", 2, _lib.KERNEL_PANEL, dict(phase_len=10, finish_thresh=100000,
                                                                            duo_max_grid=1))):
        with gpad_mpc.GpadSolver(0) as s:
            s.setup(dML, dG, float(np.float32(L)), n=200, m=200, batch=B, kernel=kern)
            s.set_options(**opts)
            best = {}
            for N in (210, 1010):
                t = []
                for _ in range(4):
                    z = torch.zeros(B, 200, device=dev)
                    y = torch.zeros(B, 200, device=dev)
                    st = s.run(z, y, dM[:B], dg[:B], N, 1e-12)
                    t.append(st["kernel_ms"])
                best[N] = min(t)
            out[name] = {"us_per_iter": round((best[1010] - best[210]) / 800 * 1e3, 4), "kernel": st["kernel"]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
