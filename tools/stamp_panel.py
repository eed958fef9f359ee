"""Phase anatomy of the panel kernels from in-kernel shader-clock stamps (diagnostic build only).

  GPAD_LIB=tools/abl/stamp.so python3 tools/stamp_panel.py --batch 8192
(the library built with EXTRA=-DGPAD_STAMP; the product build has no stamps).  Runs the C4-shape
panel solve for a fixed N, reads workgroup 0's stamps (gpad_panel.hip GPAD_STAMP_AT) and prints,
per wave and averaged over the stamped iterations, the cycles of: GEMM-1 issue, its epilogue, the
wait at its barrier, GEMM-2 issue, its epilogue, the wait at the closing barrier.
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-dualgradient-mpc_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--N", type=int, default=110)
    args = ap.parse_args()
    import microbench
    r = microbench.case("panel", 200, 200, args.batch, args.N, reps=1)
    from gpad_mpc import _lib
    L = _lib.load()
    ITS, PTS = 4, 6
    buf = (C.c_ulonglong * (16 * ITS * PTS))()
    f = L._lib.gpad_debug_stamps if hasattr(L, "_lib") else L.gpad_debug_stamps
    f.argtypes = [C.c_void_p, C.c_size_t]
    assert f(buf, C.sizeof(buf)) == 0
    st = np.array(buf, dtype=np.int64).reshape(16, ITS, PTS)
    names = ["gemm1", "epi1", "bar1", "gemm2", "epi2", "bar2"]
    print(f"batch {args.batch}: {r['us_per_iter']} us/iteration (stamped build)")
    pair = (args.batch + 15) // 16 > 256
    per_iter = []
    for w in range(16):
        # the role this wave plays (gpad_panel2_kernel: one panel -> 15 - w; pairs -> the receiver swap)
        role = ((w + 4) if (w >> 1) == 4 else ((w - 4) if (w >> 1) == 6 else w)) if pair else 15 - w
        d = np.zeros(PTS)
        ok = np.ones(PTS, bool)
        for i in range(ITS - 1):
            s_ = st[w, i]
            nxt = st[w, i + 1, 0]
            pts = list(s_) + [nxt]
            for k in range(PTS):
                if pts[k] == 0 or pts[k + 1] == 0:
                    ok[k] = False
                else:
                    d[k] += pts[k + 1] - pts[k]
        d /= ITS - 1
        it = (st[w, ITS - 1, 0] - st[w, 0, 0]) / (ITS - 1)
        per_iter.append(it)
        # relay waves (no GEMM-issue stamps): merge the issue and epilogue segments
        if not ok[1] or not ok[0]:
            seg = f"piece1+epi1 {int(st[w, :ITS - 1, 2].astype(float).mean() - st[w, :ITS - 1, 0].astype(float).mean()):6d}"
        else:
            seg = f"{names[0]} {int(d[0]):6d}  {names[1]} {int(d[1]):6d}"
        rest = "  ".join(f"{n} {int(x):6d}" if ok[k] else f"{n}      -" for k, (n, x) in enumerate(zip(names, d)) if k >= 2)
        print(f"wave {w:2d} SIMD {w % 4} role {role:2d}: {seg}  {rest}  | iter {int(it)}")
    t0 = st[:, :, 0]
    print("loop-top skew across waves (cycles):", int(t0[:, 1].max() - t0[:, 1].min()))
    cyc = float(np.mean(per_iter))
    print(f"cycles per iteration {cyc:.0f}; implied clock {cyc / r['us_per_iter'] / 1e3:.2f} GHz "
          f"(stamps from a stamped build, whose iteration may differ from the product's)")


if __name__ == "__main__":
    main()
