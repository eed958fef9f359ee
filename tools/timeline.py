"""Per-launch timeline of one C4 solve (phase launches, finisher launches, gaps).

  run   : python3 tools/timeline.py run [--reps R]     -- the bench's C4 shard, R solves
  parse : python3 tools/timeline.py parse <rocprof dir> [--iters file.npy]

On the GPU box:
  rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl -o run -- python3 tools/timeline.py run
  python3 tools/timeline.py parse gpurun_out/tl
prints, for the last solve, each launch's kernel, grid, duration and the idle gap before it,
and (with the iteration counts the run step saves) the survivors each phase starts with.
"""
from __future__ import annotations

import argparse
import csv
import glob
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def run(args):
    import torch

    import bench
    import gpad_mpc
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import tune_env  # noqa: F401  (GPAD_* env -> gpad_set_option)
    dev = torch.device("cuda:0")
    n, m, B = 200, 200, args.batch
    ML, G, L, M, g = bench.make_shard(n, m, B, 0)
    f32 = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(dev)  # noqa: E731
    dML, dG, dM, dg = f32(ML), f32(G), f32(M), f32(g)
    fresh = [(f32(a), f32(b)) for a, b in bench.make_stream(n, m, B, args.reps, 0)] if args.fresh else None
    z = torch.zeros(B, n, device=dev)
    y = torch.zeros(B, m, device=dev)
    s = gpad_mpc.GpadSolver(0)
    s.setup(dML, dG, float(np.float32(L)), n=n, m=m, batch=B, shared=True, check_every=10)
    it = np.zeros(B, np.int32)
    prev = np.zeros(B, np.int32)
    for r in range(args.reps):
        z.zero_()
        y.zero_()
        Mv, gv = fresh[r] if fresh else (dM, dg)
        prev[:] = it
        plan = s.phase_plan()
        s.run(z, y, Mv, gv, 5000, 1e-4, stats=False)
        st = s.last_stats(iters=it)
        print(f"rep {r}: plan ends {plan['ends']} fins {plan['fins']} -> survivors after each phase "
              f"{s.phase_counts()}; past 260: {int((it > 260).sum())}")
    torch.cuda.synchronize()
    np.save(args.out, it)
    np.save(args.out.replace(".npy", "_prev.npy"), prev)
    print(f"kernel {st['kernel']} kernel_ms {st['kernel_ms']:.4f} mean_iters {it.mean():.1f} "
          f"min {it.min()} max {it.max()}")


def parse(args):
    files = glob.glob(os.path.join(args.dir, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        sys.exit(f"no kernel_trace.csv under {args.dir}")
    rows = []
    with open(files[0]) as f:
        for r in csv.DictReader(f):
            rows.append(r)
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    gpad = [r for r in rows if "gpad" in r["Kernel_Name"] and "pack" not in r["Kernel_Name"]]
    # the last solve: launches after the last gap > 200 us
    starts = [int(r["Start_Timestamp"]) for r in gpad]
    ends = [int(r["End_Timestamp"]) for r in gpad]
    cut = 0
    for i in range(1, len(gpad)):
        if starts[i] - ends[i - 1] > 200_000:
            cut = i
    last = gpad[cut:]
    t0 = int(last[0]["Start_Timestamp"])
    print(f"{'#':>3} {'kernel':<34} {'grid':>8} {'start_us':>9} {'dur_us':>9} {'gap_us':>7}")
    prev = None
    busy = 0
    for i, r in enumerate(last):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev) / 1e3 if prev is not None else 0.0
        name = r["Kernel_Name"].split("(")[0][-34:]
        grid = r.get("Grid_Size_X") or r.get("Grid_Size") or "?"
        print(f"{i:>3} {name:<34} {grid:>8} {(s - t0) / 1e3:>9.1f} {(e - s) / 1e3:>9.1f} {gap:>7.1f}")
        prev = e
        busy += e - s
    span = (ends[-1] - t0) / 1e3
    print(f"solve span {span:.1f} us, busy {busy / 1e3:.1f} us, launches {len(last)}")
    if args.iters and os.path.exists(args.iters):
        it = np.load(args.iters)
        for v in (0, 40, 80, 160, 170, 200, 240, 280, 320, 360, 380):
            print(f"survivors past iteration {v:>4}: {(it > v).sum()}")


def solves(args):
    """One line per solve of the trace: every launch's kernel (short name) and duration, in order --
    to line up with the run step's per-rep survivor counts (which solves are slow, in which phase)."""
    files = glob.glob(os.path.join(args.dir, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        sys.exit(f"no kernel_trace.csv under {args.dir}")
    with open(files[0]) as f:
        rows = sorted(csv.DictReader(f), key=lambda r: int(r["Start_Timestamp"]))
    gpad = [r for r in rows if "gpad" in r["Kernel_Name"] and "pack" not in r["Kernel_Name"]
            and "accumulate" not in r["Kernel_Name"]]
    out, cur = [], []
    for r in gpad:
        if cur and int(r["Start_Timestamp"]) - int(cur[-1]["End_Timestamp"]) > 200_000:
            out.append(cur)
            cur = []
        cur.append(r)
    out.append(cur)
    short = lambda k: ("panel" if "panel2" in k else "duo" if "duo" in k else "cmp" if "compact" in k  # noqa: E731
                       else k.split("(")[0][-12:])
    for i, sv in enumerate(out):
        span = (int(sv[-1]["End_Timestamp"]) - int(sv[0]["Start_Timestamp"])) / 1e3
        seq = " ".join(f"{short(r['Kernel_Name'])}:{(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3:.1f}"
                       for r in sv)
        print(f"solve {i}: span {span:8.1f} us | {seq}")


def stats(args):
    """Per-kernel durations over every solve of the trace, and the solve spans (A/B of a phase)."""
    files = glob.glob(os.path.join(args.dir, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        sys.exit(f"no kernel_trace.csv under {args.dir}")
    with open(files[0]) as f:
        rows = sorted(csv.DictReader(f), key=lambda r: int(r["Start_Timestamp"]))
    gpad = [r for r in rows if "gpad" in r["Kernel_Name"] and "pack" not in r["Kernel_Name"]]
    solves, cur = [], []
    for r in gpad:
        if cur and int(r["Start_Timestamp"]) - int(cur[-1]["End_Timestamp"]) > 200_000:
            solves.append(cur)
            cur = []
        cur.append(r)
    solves.append(cur)
    solves = solves[1:]  # (the first solve warms up)
    spans = [(int(s[-1]["End_Timestamp"]) - int(s[0]["Start_Timestamp"])) / 1e3 for s in solves]
    per = {}
    for s in solves:
        for r in s:
            k = r["Kernel_Name"].split("(")[0][-34:]
            per.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(f"{args.label} solves {len(solves)}: span mean {np.mean(spans):.1f} median {np.median(spans):.1f} "
          f"min {np.min(spans):.1f} us")
    for k, d in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        print(f"{args.label}   {k:<34} n {len(d):>3} per solve {sum(d) / len(solves):8.1f} us  "
              f"mean {np.mean(d):7.1f}  min {np.min(d):7.1f}")


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    a = sub.add_parser("run")
    a.add_argument("--reps", type=int, default=5)
    a.add_argument("--batch", type=int, default=8192)
    a.add_argument("--out", default="gpurun_out/tl_iters.npy")
    a.add_argument("--fresh", action="store_true", help="new q/b draws every solve (bench default)")
    b = sub.add_parser("parse")
    b.add_argument("dir")
    b.add_argument("--iters", default="gpurun_out/tl_iters.npy")
    d = sub.add_parser("solves")
    d.add_argument("dir")
    c = sub.add_parser("stats")
    c.add_argument("dir")
    c.add_argument("--label", default="")
    args = ap.parse_args()
    {"run": run, "parse": parse, "stats": stats, "solves": solves}[args.cmd](args)


if __name__ == "__main__":
    main()
