"""Where do the panel kernel's HBM writes come from (WRITE_SIZE per solve ~2x
the state it parks)?  One C4 shard (8192 x 200 x 200) solve per process, after a warm-up, in one of
three modes; run each under `rocprofv3 --pmc WRITE_SIZE` and compare the panel launches' bytes with
the algorithmic stores printed here:
  fixed : N = 100, tol = 0: one launch, every column stores z*, y* once at the end
  notest: N = 100, tol = 1e-30: tests every 10 iterations, nothing converges (one launch: plan off,
          one phase), stores as fixed -- any excess over `fixed` is the test path's scratch traffic
  tol   : N = 5000, tol = 1e-4, the planned phases: parked state + results
  python3 tools/write_probe.py run <mode>      (under rocprofv3)
  python3 tools/write_probe.py parse <dir>     (per-dispatch WRITE_SIZE of the panel kernel)"""
import csv
import glob
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpu-dualgradient-mpc_amd")]


def run(mode):
    import torch

    import bench
    import gpad_mpc
    dev = torch.device("cuda:0")
    n = m = 200
    B = 8192
    ML, G, L, M, g = bench.make_shard(n, m, B, 0)
    f32 = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(dev)  # noqa: E731
    dM, dg = f32(M), f32(g)
    z = torch.zeros(B, n, device=dev)
    y = torch.zeros(B, m, device=dev)
    N, tol = {"fixed": (100, 0.0), "notest": (100, 1e-30), "tol": (5000, 1e-4)}[mode]
    with gpad_mpc.GpadSolver(0) as s:
        s.setup(f32(ML), f32(G), float(np.float32(L)), n=n, m=m, batch=B, shared=True, check_every=10)
        if mode != "tol":
            s.set_options(phased=0)
        it = np.zeros(B, np.int32)
        for _ in range(2):
            st = s.run(z.zero_(), y.zero_(), dM, dg, N, tol, iters=it)
        ph = s.last_phases() if mode == "tol" else None
    out = {"mode": mode, "results_bytes": B * (n + m) * 4, "kernel_ms": st["kernel_ms"]}
    if ph:  # parked state per boundary: survivors x (z, y, w, u)
        out["phases"] = ph
        out["parked_bytes"] = [c * (n + 3 * m) * 4 for c in ph["counts"][:-1]]
    print(json.dumps(out))


def parse(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows += [r for r in csv.DictReader(open(f)) if r["Counter_Name"] == "WRITE_SIZE"]
    rows.sort(key=lambda r: int(r.get("Dispatch_Id", 0) or 0))
    for r in rows:
        k = r["Kernel_Name"].split("(")[0]
        if "gpad" in k:
            print(f"{k[-40:]:<40} WRITE_SIZE {float(r['Counter_Value']) * 1024 / 1e6:10.3f} MB")


if __name__ == "__main__":
    {"run": lambda: run(sys.argv[2]), "parse": lambda: parse(sys.argv[2])}[sys.argv[1]]()
