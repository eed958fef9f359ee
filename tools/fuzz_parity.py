"""Randomised parity campaign on the GPU box (tests/fuzz_util.py): R random configurations
from seed S, each solved through the C-ABI and checked bit for bit against the oracle on a
sample of instances; one JSON line per case, a summary line last.
  python3 tools/fuzz_parity.py [--seed S] [--cases R] [--sample K] [--budget-s T] [--rccl-stub]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "gpu-dualgradient-mpc_amd"), os.path.join(ROOT, "oracle"),
          os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import fuzz_util  # noqa: E402
import pyoracle  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--seed", type=int, default=1)
ap.add_argument("--cases", type=int, default=200)
ap.add_argument("--sample", type=int, default=24)
ap.add_argument("--budget-s", type=float, default=400.0)
ap.add_argument("--flat", type=float, default=0.25, help="share of flat battery cases")
ap.add_argument("--value", type=float, default=0.0, help="share of value-branch (H bound) cases")
ap.add_argument("--loop", type=float, default=0.0, help="share of closed-loop (gpad_closed_loop) cases")
ap.add_argument("--heavy", type=float, default=0.0, help="share of C3/C4-shaped phased solves")
ap.add_argument("--steps", type=float, default=0.0, help="share of per-step entry point cases")
ap.add_argument("--rccl-stub", action="store_true",
                help="group cases through the RCCL transport (tests/rccl_stub, one GPU standing in for each rank)")
args = ap.parse_args()
if args.rccl_stub:
    from gpad_mpc import _lib
    so = os.path.join(ROOT, "tests", "rccl_stub", "librccl_stub.so")
    _lib.check(_lib.load().gpad_group_rccl_library(so.encode(), 1), "gpad_group_rccl_library")
if not os.path.exists(pyoracle.LIB):
    pyoracle.build(ref=False)
O = pyoracle.Oracle()
t0, fails, done, checked = time.time(), 0, 0, 0
for i in range(args.cases):
    if time.time() - t0 > args.budget_s:
        break
    rng = np.random.default_rng(args.seed + i)
    u = rng.random()
    edges = np.cumsum([args.flat, args.value, args.loop, args.heavy, args.steps])
    kind = ("flat" if u < edges[0] else "value" if u < edges[1] else "loop" if u < edges[2] else
            "heavy" if u < edges[3] else "steps" if u < edges[4] else "full")
    cfg = {"flat": fuzz_util.draw_flat_case, "value": fuzz_util.draw_value_case, "loop": fuzz_util.draw_loop_case,
           "heavy": fuzz_util.draw_heavy_case, "full": fuzz_util.draw_case,
           "steps": lambda r: {"steps_seed": int(r.integers(1 << 30))}}[kind](rng)
    t = time.time()
    try:
        if kind == "flat":
            r = fuzz_util.run_flat_case(cfg, O, sample=min(args.sample, 16))
        elif kind == "steps":
            r = fuzz_util.run_steps_case(cfg["steps_seed"], O)
        elif kind == "loop":
            r = fuzz_util.run_loop_case(cfg, O)
        elif kind == "value":
            r = fuzz_util.run_value_case(cfg, O, sample=min(args.sample, 16))
        else:
            r = fuzz_util.run_case(cfg, O, sample=args.sample, threads=16)
    except Exception as e:  # a library error is a finding too
        r = dict(ok=False, checked=0, why=f"{type(e).__name__}: {e}")
    done += 1
    checked += r["checked"]
    fails += not r["ok"]
    print(json.dumps(dict(case=i, s=round(time.time() - t, 2), cfg=cfg, **r)), flush=True)
print(json.dumps(dict(summary=True, seed=args.seed, rccl_stub=args.rccl_stub, cases=done, failed=fails, instances_checked=checked,
                      seconds=round(time.time() - t0, 1))), flush=True)
