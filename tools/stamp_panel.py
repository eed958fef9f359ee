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
    ITS, PTS = 4, 8
    buf = (C.c_ulonglong * (16 * ITS * PTS))()
    f = L._lib.gpad_debug_stamps if hasattr(L, "_lib") else L.gpad_debug_stamps
    f.argtypes = [C.c_void_p, C.c_size_t]
    assert f(buf, C.sizeof(buf)) == 0
    st = np.array(buf, dtype=np.int64).reshape(16, ITS, PTS).astype(np.float64)
    st[st == 0] = np.nan
    print(f"batch {args.batch}: {r['us_per_iter']} us/iteration (stamped build)")
    pair = (args.batch + 15) // 16 > 256
    # times relative to each iteration's loop-top release (min over waves of stamp 0), averaged
    # over the stamped iterations; columns in program order
    cols = [(0, "top"), (6, "wait1"), (1, "gemm1"), (2, "prebar1"), (3, "bar1"), (7, "wait2"), (4, "gemm2"),
            (5, "prebar2")]
    ref = np.nanmin(st[:, :, 0], axis=0)  # [ITS]
    nxt = np.nanmin(st[:, 1:, 0], axis=0)  # next iteration's release
    print("cycles after the iteration's loop-top release (min over waves of stamp 0); '-' = no stamp:")
    print("wave SIMD role " + " ".join(f"{n:>8s}" for _, n in cols))
    for w in range(16):
        role = ((w + 4) if (w >> 1) == 4 else ((w - 4) if (w >> 1) == 6 else w)) if pair else 15 - w
        vals = []
        for k, _ in cols:
            x = st[w, :, k] - ref
            m = np.nanmean(x[:ITS - 1]) if np.isfinite(x[:ITS - 1]).any() else np.nan
            vals.append("       -" if np.isnan(m) else f"{int(m):8d}")
        print(f"{w:4d} {w % 4:4d} {role:4d} " + " ".join(vals))
    it = float(np.nanmean(nxt - ref[:ITS - 1]))
    print(f"iteration (release to release): {it:.0f} cycles; implied clock {it / r['us_per_iter'] / 1e3:.2f} GHz "
          f"(stamped build)")
    bar1 = np.nanmin(st[:, :, 3] - ref, axis=0)[:ITS - 1].mean()
    print(f"barrier-1 release at {bar1:.0f}; GEMM-2 phase {it - bar1:.0f}")


if __name__ == "__main__":
    main()
