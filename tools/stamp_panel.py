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
    tot = []
    for w in range(16):
        d = np.zeros(PTS)
        for i in range(ITS - 1):
            s = st[w, i]
            nxt = st[w, i + 1, 0]
            seg = [s[1] - s[0], s[2] - s[1], s[3] - s[2], s[4] - s[3], s[5] - s[4], nxt - s[5]]
            d += np.array(seg)
        d /= ITS - 1
        tot.append(d.sum())
        print(f"wave {w:2d} SIMD {w % 4}: " + "  ".join(f"{n} {int(x):6d}" for n, x in zip(names, d)) +
              f"  | iter {int(d.sum())}")
    t0 = st[:, :, 0]
    print("loop-top skew across waves (cycles):", int(t0[:, 1].max() - t0[:, 1].min()))


if __name__ == "__main__":
    main()
