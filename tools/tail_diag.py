"""Diagnostic (GPU box): the TailPair layout against the sixteen-row pairs after N = 1, 2, 3 fixed
iterations of the C4-shaped synthetic batch -- where (rows, instances) the results first differ."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-dualgradient-mpc_amd"))


def main():
    import torch

    import gpad_mpc
    from gpad_mpc import problems
    B, nm = 8192, 200
    qp = problems.synthetic_qp(nm, nm, batch=B, seed=7)
    dev = torch.device("cuda:0")
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(dev)  # noqa: E731
    M = t(np.asarray(qp.M).reshape(B, nm))
    g = t(np.asarray(qp.g).reshape(B, nm))
    for N in (1, 2, 3):
        out = []
        for tail in (1, 0):
            with gpad_mpc.GpadSolver(0) as s:
                s.setup(t(qp.ML), t(qp.G), float(np.float32(qp.L)), n=nm, m=nm, batch=B)
                s.set_options(pair_tail=tail)
                z = torch.zeros(B, nm, device=dev)
                y = torch.zeros(B, nm, device=dev)
                st = s.run(z, y, M, g, N, 0.0)
            out.append((z.cpu().numpy(), y.cpu().numpy()))
        for name, k in (("z", 0), ("y", 1)):
            d = np.abs(out[0][k] - out[1][k])
            rows = np.nonzero(d.max(axis=0) > 0)[0]
            inst = np.nonzero(d.max(axis=1) > 0)[0]
            print(f"N={N} {name}: max diff {d.max():.3e}; differing rows {len(rows)} "
                  f"(first {rows[:12].tolist()}), instances {len(inst)} (first {inst[:8].tolist()})")
            if len(rows):
                r = rows[0]
                i = inst[0]
                print(f"   e.g. [{i},{r}] tail {out[0][k][i, r]:.6g} rows16 {out[1][k][i, r]:.6g}; "
                      f"tail rows 192..199 of inst {i}: {np.round(out[0][k][i, 192:], 5).tolist()} vs "
                      f"{np.round(out[1][k][i, 192:], 5).tolist()}")


if __name__ == "__main__":
    main()
