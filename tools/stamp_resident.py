"""Iteration anatomy of the resident (latency) kernel from in-kernel shader-clock stamps
(diagnostic build only: GPAD_LIB=tools/abl/stamp.so, the library built with EXTRA=-DGPAD_STAMP).

  GPAD_LIB=tools/abl/stamp.so python3 tools/stamp_resident.py
C2 single instance (n = m = 200), 200 fixed iterations; prints, per wave of workgroup 0 and
averaged over the stamped iterations, the cycles of: the 8b chain (A waves), the A epilogue + first
barrier, the 8d chain (B waves), its epilogue, the second barrier -- the breakdown of the bit-exact
latency bound.
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-dualgradient-mpc_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main():
    import microbench
    r = microbench.case("resident", 200, 200, 1, 200, reps=1)
    from gpad_mpc import _lib
    L = _lib.load()
    buf = (C.c_ulonglong * (8 * 4 * 6))()
    f = L._lib.gpad_debug_res_stamps if hasattr(L, "_lib") else L.gpad_debug_res_stamps
    f.argtypes = [C.c_void_p, C.c_size_t]
    assert f(buf, C.sizeof(buf)) == 0
    st = np.array(buf, dtype=np.int64).reshape(8, 4, 6)
    print(f"C2 single instance: {r['us_per_iter']} us/iteration (stamped build)")
    # A waves 0-3 stamp 0,1,2,4,5 (no 3); B waves 4-7 stamp 0,2,3,4,5 (no 1)
    for w in range(8):
        isA = w < 4
        d = []
        for i in range(3):
            s = st[w, i]
            nxt = st[w, i + 1, 0]
            if isA:
                d.append([s[1] - s[0], s[2] - s[1], s[4] - s[2], s[5] - s[4], nxt - s[5]])
            else:
                d.append([s[2] - s[0], s[3] - s[2], s[4] - s[3], s[5] - s[4], nxt - s[5]])
        d = np.mean(d, axis=0)
        names = (["8b chain", "epi+barrier1", "idle (8d)", "barrier2", "loop"] if isA else
                 ["idle (8b)+barrier1", "8d chain", "epilogue", "barrier2", "loop"])
        print(f"wave {w} ({'A' if isA else 'B'}): " + "  ".join(f"{n} {int(x)}" for n, x in zip(names, d)) +
              f"  | iteration {int(d.sum())} cycles")


if __name__ == "__main__":
    main()
