"""Tail schedule model (tools, CPU): list-scheduling simulation of a C4 solve's tail on persistent
finisher engines, from per-instance iteration counts (numpy fp32 restatement of the C4 shard,
not bit-exact -- counts within a few of the GPU's, the survival curve is the same).

  python3 tools/tail_model.py [seed]

Engines: per CU two slots in ping-pong; a half-step runs the 8b chain of one slot beside the 8d
chain of the other.  Half-step = chain cycles (table, measured: DPP 6.7 cyc/step alone, 10.2 with
a partner; 4x4x1 MFMA 14.6 alone, 20.7 with a partner -- tools/lat/dpp_chain.hip, quad_bcast.hip)
+ OV cycles of exchange/epilogue, at 2.36 GHz.  duo = one instance per slot; quad = four columns
per slot on MFMA, a slot's last column on DPP.  The current C4 plan is phase 2 on single panels
(260 -> 290, 6.9 us per iteration) then the duo.  Prints the tail length (us) per scheme; the
measured duo is ~10-20 % above the model (its step overhead is larger than OV), the measured quad
far above (profiles/r03_quad_finisher.txt: 1.1-3.5k cycles of step overhead, not 850).
Round 4 (profiles/r04_duo_solo.txt): two live slots 2.27 us per slot-iteration, one live slot (solo
mode) 1.63, the resident kernel 1.31-1.33 in tol mode; a per-CU simulation with those speeds gives
solo mode -8 to -10 us over the old one-slot speed (1.80) and migrating a busy CU's second slot to an
idle CU once the queue drains -3 to -27 us (seeds 0, 1).
"""
import heapq
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "gpu-dualgradient-mpc_amd"))
CLK, OV = 2360.0, 850.0
CH = {("n", "n"): 0, ("d", "n"): 1340, ("m", "n"): 2920, ("d", "d"): 2040, ("m", "m"): 4150, ("m", "d"): 4050}


def counts(seed, B=8192, N=600, tol=1e-4):
    import bench
    ML, G, L, M, g = bench.make_shard(200, 200, B, seed * 100000)
    f = lambda a: np.ascontiguousarray(a, np.float32)  # noqa: E731
    MLn, GL, pD, gP, Gf, gf = f(-ML), f(G / np.float32(L)), f(-g / np.float32(L)), f(M), f(G), f(g)
    th, be = np.empty(N), np.empty(N)
    t, tm1, b = 1.0, 1.0, 0.0
    for v in range(N):
        tn = (np.sqrt(t ** 4 + 4 * t ** 2) - t ** 2) / 2
        th[v], be[v] = t, b
        b = t * (1 / tm1 - 1)
        tm1, t = t, tn
    th, be = th.astype(np.float32), be.astype(np.float32)
    y = np.zeros((B, 200), np.float32)
    yp, z = y.copy(), np.zeros((B, 200), np.float32)
    done, iters = np.zeros(B, bool), np.full(B, N)
    for v in range(N):
        w = y + be[v] * (y - yp)
        zh = w @ MLn.T - gP
        z = (1 - th[v]) * z + th[v] * zh
        yp, y = y, np.maximum(w + zh @ GL.T + pD, 0)
        if (v + 1) % 10 == 0:
            r, rh = z @ Gf.T - gf, zh @ Gf.T - gf
            ok = (r.max(1) <= tol) | ((rh.max(1) <= tol) & (w.min(1) >= 0) & (-(w * rh).sum(1) <= tol))
            nw = ~done & ok
            iters[nw], done = v + 1, done | nw
            if done.all():
                break
    return iters


def chain(a, b):
    return CH[tuple(sorted((a, b), key="mdn".index))]


def run(rem, ncol, dpp_fallback, seed=0, ncu=256, lpt=False):
    rng = np.random.default_rng(seed)
    q = list(np.sort(rem)[::-1] if lpt else rng.permutation(rem))
    qi = 0
    cus = [[[0] * ncol for _ in range(2)] for _ in range(ncu)]
    for s in range(2):
        for j in range(ncol):
            for c in range(ncu):
                if qi < len(q):
                    cus[c][s][j] = q[qi]
                    qi += 1
    h = [(0.0, c) for c in range(ncu)]
    heapq.heapify(h)
    end = 0.0
    while h:
        t, c = heapq.heappop(h)
        live = [sum(1 for x in s if x > 0) for s in cus[c]]
        if sum(live) == 0:
            end = max(end, t)
            continue
        modes = ["n" if k == 0 else ("d" if ncol == 1 or (k == 1 and dpp_fallback) else "m") for k in live]
        heapq.heappush(h, (t + 2 * (chain(*modes) + OV) / CLK, c))
        for s in cus[c]:
            for j in range(ncol):
                if s[j] > 0:
                    s[j] -= 1
                    if s[j] == 0 and qi < len(q):
                        s[j] = q[qi]
                        qi += 1
    return end


def main():
    seed = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    it = counts(seed)
    surv = lambda v: it[it > v] - v  # noqa: E731
    print(f"seed {seed}: mean {it.mean():.1f}, max {it.max()}; survivors past 260/290: {(it > 260).sum()}/{(it > 290).sum()}")
    print(f"  current: phase 2 260->290 on single panels + duo from 290: {30 * 6.9 + run(surv(290), 1, False, seed):.0f} us"
          f" (duo with a perfect longest-first queue: {30 * 6.9 + run(surv(290), 1, False, seed, lpt=True):.0f})")
    for T0 in (260, 270, 280, 290):
        extra = (T0 - 260) * 6.9
        print(f"  quad from {T0} (+ single panels 260->{T0}): {extra + run(surv(T0), 4, True, seed):.0f} us")
    print(f"  lower bound (longest instance at the resident kernel's 1.36 us/iteration from 260): {(it.max() - 260) * 1.36:.0f} us")


if __name__ == "__main__":
    main()
