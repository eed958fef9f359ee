"""Anatomy of one phase of a phased panel solve (diagnostic build: GPAD_LIB=<stamped libgpad>).

  GPAD_LIB=tools/abx/libgpad_stamp.so GPAD_LIB_TOLERANT=1 python3 tools/phase_stamps.py --batch 4096
Solves fresh C4-generator batches with uniform 20-iteration phases and no finisher (plan off), then
reads workgroup 0's stamps of the phase [100, 120) (gpad_panel.hip GPAD_PSTAMP): kernel entry,
(--plan V: the default planned solve instead, the library built with -DGPAD_STAMP_PHASE_V=V
-DGPAD_STAMP_V0=V+1, e.g. the C4 shard's second phase at V = 260)
state loaded, after the load barrier, loop exit, survivors parked, after the closing barrier --
and of its iterations 101..104 (GPAD_STAMP_AT) for the per-iteration scale.
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpu-dualgradient-mpc_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--plan", type=int, default=0, help="planned solve; the stamped phase starts at this v")
    args = ap.parse_args()
    import torch

    import bench
    import gpad_mpc
    from gpad_mpc import _lib
    dev = torch.device("cuda:0")
    n = m = 200
    B = args.batch
    ML, G, L, _, _ = bench.make_shard(n, m, 1, 0)
    f32 = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(dev)  # noqa: E731
    draws = [(f32(a), f32(b)) for a, b in bench.make_stream(n, m, B, 4, 0)]
    z = torch.zeros(B, n, device=dev)
    y = torch.zeros(B, m, device=dev)
    with gpad_mpc.GpadSolver(0) as s:
        s.setup(f32(ML), f32(G), float(np.float32(L)), n=n, m=m, batch=B, check_every=10)
        if not args.plan:
            s.set_options(plan=0, phase_len=20, finish_thresh=0)
        for Mv, gv in draws:
            st = s.run(z.zero_(), y.zero_(), Mv, gv, 5000, 1e-4)
            if args.plan:
                print(f"solve {st['kernel_ms']:.3f} ms", flush=True)
    lib = _lib.load()
    f = lib.gpad_debug_stamps
    f.argtypes = [C.c_void_p, C.c_size_t]
    n_it = 16 * 4 * 8
    buf = (C.c_ulonglong * (n_it + 16 * 10))()
    assert f(buf, C.sizeof(buf)) == 0
    a = np.array(buf, dtype=np.float64)
    it = a[:n_it].reshape(16, 4, 8)
    ph = a[n_it:].reshape(16, 10)
    ph[ph == 0] = np.nan
    t0 = np.nanmin(ph[:, 0])
    names = ["entry", "loaded", "loadbar", "loopexit", "parked", "endbar", "lasttest", "voted", "verified",
             "out"]
    v0 = args.plan or 100
    print(f"batch {B}: {st['kernel']} solve {st['kernel_ms']:.3f} ms (last, stamped build); phase from {v0}, WG 0")
    print("wave  " + " ".join(f"{x:>9s}" for x in names) + "   (cycles after the earliest entry)")
    for w in range(16):
        print(f"{w:4d}  " + " ".join("        -" if np.isnan(x) else f"{int(x - t0):9d}" for x in ph[w]))
    if args.plan:  # per stamped iteration: the earliest / latest wave at each point, after the entry
        it[it == 0] = np.nan
        for k in range(4):
            lo = np.nanmin(it[:, k, :6], axis=0) - t0
            hi = np.nanmax(it[:, k, :6], axis=0) - t0
            print(f"iteration +{k}: " + " ".join(f"{int(a_)}/{int(b_)}" for a_, b_ in zip(lo, hi)))
        it = np.nan_to_num(it)
    itv = it[:, :, 0]
    itv = itv[itv > 0]
    if itv.size:
        per = (np.max(it[:, 3, 0]) - np.max(it[:, 0, 0])) / 3 if (it[:, 3, 0] > 0).any() else float("nan")
        print(f"iteration {v0 + 1}..{v0 + 4} loop tops: {per:.0f} cycles per iteration; phase span "
              f"{np.nanmax(ph[:, 5]) - t0:.0f} cycles = {20} iterations + prologue {np.nanmax(ph[:, 2]) - t0:.0f} "
              f"+ epilogue {np.nanmax(ph[:, 5]) - np.nanmin(ph[:, 3]):.0f}")


if __name__ == "__main__":
    main()
