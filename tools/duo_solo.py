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
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import tune_env  # noqa: E402,F401  (GPAD_* env -> handle options)


def stamps(two=False):
    """Step anatomy of the duo (diagnostic build: GPAD_LIB=tools/abl/stamp.so): one live slot, or
    two (--two); steps 200..207 of workgroup 0, per wave: chain, epilogue, barrier wait, post-barrier
    bookkeeping, gap to the next step (cycles of the shader clock)."""
    import ctypes as C

    import torch

    import bench
    import gpad_mpc
    from gpad_mpc import _lib
    dev = torch.device("cuda:0")
    B = 2 if two else 1
    ML, G, L, M, g = bench.make_shard(200, 200, B, 0)
    f32 = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(dev)  # noqa: E731
    with gpad_mpc.GpadSolver(0) as s:
        s.setup(f32(ML), f32(G), float(np.float32(L)), n=200, m=200, batch=B, kernel=_lib.KERNEL_PANEL)
        s.set_options(phase_len=10, finish_thresh=100000, **({"duo_max_grid": 1} if two else {}))
        z = torch.zeros(B, 200, device=dev)
        y = torch.zeros(B, 200, device=dev)
        s.run(z, y, f32(M), f32(g), 300, 1e-12)
    L_ = _lib.load()
    buf = (C.c_ulonglong * (8 * 8 * 5))()
    f = L_._lib.gpad_debug_duo_stamps if hasattr(L_, "_lib") else L_.gpad_debug_duo_stamps
    f.argtypes = [C.c_void_p, C.c_size_t]
    assert f(buf, C.sizeof(buf)) == 0
    st = np.array(buf, dtype=np.int64).reshape(8, 8, 5)
    print(f"duo, {'two live slots' if two else 'one live slot'}: steps 200..206, cycles (shader clock)")
    for w in range(8):
        rows = []
        for i in range(7):
            x = st[w, i].copy()
            if x[1] == 0:  # no chain on this wave this step
                x[1] = x[0]
            rows.append([x[1] - x[0], x[2] - x[1], x[3] - x[2], x[4] - x[3], st[w, i + 1, 0] - x[4],
                         st[w, i + 1, 0] - x[0]])
        rows = np.array(rows)
        for par in (0, 1):
            d = rows[par::2].mean(axis=0).astype(int)
            print(f"wave {w} ({'B' if w < 4 else 'A'}) steps {'even' if par == 0 else 'odd '}: chain {d[0]:5d} "
                  f"epi {d[1]:4d} bar {d[2]:5d} post {d[3]:4d} gap {d[4]:4d} | step {d[5]}")


def main():
    if "--stamps" in sys.argv:
        stamps(two="--two" in sys.argv)
        return
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
