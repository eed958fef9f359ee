"""bench.py -- GPAD inner-loop throughput on MI355X (BASELINE.json metric).

Workload (default, ``--workload c4``): the C4 shard -- 8192 independent MPC QP instances per GPU
(weak scaling), horizon N = 50 with n_u = 4 (n = 200 primal variables), m = 200 constraints,
shared ML/G (one plant) and per-instance M/g (seeded synthetic generator of SURVEY.md §8d),
solved to eps = 1e-4 with Algorithm 1 (check every 10 iterations, at most 5000 iterations).
One step = reset z, y -> one gpad_run over the local shard -> RCCL gather of (z*, y*, iters) to
rank 0.  ``value`` = GPAD iterations/s (instance-iterations actually executed, summed over all
ranks) / max-over-ranks step time.

Also reported on rank 0: QP-solves/s, the C2 single-instance iteration rate, the roofline of
the dominant kernel (HIP events on the solve stream) and the reference's own CPU GPAD timed on
this host (cpu_baseline).

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W]
        torchrun --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gpu-dualgradient-mpc_amd"))

FP32_PEAK_TFLOPS = 157.3   # MI355X dense fp32 (VALU = f32 MFMA rate), MI355X_MICROARCH.md
FP64_MFMA_PEAK_TFLOPS = 78.6  # MI355X f64 matrix (spec; measured 70 TF/s back-to-back, profiles/r04_mfma_f64.txt)
HBM_PEAK_GBS = 8000.0


def flops_per_iter(n, m):
    """F = 4nm + 5m + 4n per instance-iteration."""
    return 4 * n * m + 5 * m + 4 * n


def bytes_per_iter_shared(n, m, batch):
    """shared ML/G: 4 (2nm + B (4m + 3n)) per batch-iteration."""
    return 4 * (2 * n * m + batch * (4 * m + 3 * n))


def make_shard(n, m, batch, start, seed=0):
    """Shared (ML, G, L) from ``seed``; instance i (global index) draws q, b from seed + 1 + i."""
    from gpad_mpc import problems
    base = problems.synthetic_qp(n, m, batch=1, seed=seed)
    G, H = base.G, base.H
    Hinv = np.linalg.inv(H)
    Q = np.empty((batch, n))
    Bv = np.empty((batch, m))
    for j in range(batch):
        rng = np.random.default_rng(seed + 1 + start + j)
        zf = rng.uniform(-0.5, 0.5, size=n)
        Bv[j] = G @ zf + rng.uniform(0.1, 1.0, size=m)
        Q[j] = rng.normal(0.0, 1.0, size=n)
    M = Q @ Hinv.T
    return base.ML, G, base.L, M, Bv


def host_info():
    """The host this run's CPU numbers come from: CPU model, the cores in this process's
    affinity mask, the cgroup CPU quota (the GPU box grants a share of a larger machine) and
    the thread count the CPU legs use = the quota when one is set, else the affinity count."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        pass
    model = None
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    threads = min(aff, quota) if quota else aff
    return {"cpu_model": model, "nproc_affinity": aff, "cgroup_cpu_quota": quota, "threads": threads}


class CpuRef:
    """The reference's own seq_functions.cpp (oracle/_ref/libref_seq_o3.so: -O3 -march=x86-64-v3,
    the timing build) in main.cu:160-175 loop order, OpenMP over instances (oracle/ref_driver.c);
    the oracle's C port when the reference build is absent.  Test/measurement infrastructure:
    only this CPU leg uses it, never the timed GPU region."""

    def __init__(self):
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import pyoracle
        self.O = pyoracle.Oracle()
        path = pyoracle.REF_O3 if os.path.exists(pyoracle.REF_O3) else pyoracle.REF
        self.R = pyoracle.RefSeq(path) if os.path.exists(path) else None
        self.kind = "reference" if self.R is not None else "port"
        self.info = host_info()

    def _run(self, MGneg, GP, GL, PD, N, shared, threads):
        th, be = self.O.schedule_f32(N)
        count, n = GP.shape
        m = PD.shape[1]
        Z = np.zeros((count, n), np.float32)
        Y = np.zeros((count, m), np.float32)
        t0 = time.perf_counter()
        if self.R is not None:
            self.R.solve_batch_c(Z, Y, MGneg, GP, GL, PD, th, be, N, shared=shared, threads=threads)
        else:
            self.O.solve_batch_f32(Z, Y, MGneg, GP, GL, PD, N, 1.0, 0.0, shared=shared, threads=threads)
        return time.perf_counter() - t0

    def rate(self, MGneg, GP, GL, PD, N, shared=True, threads=None, budget_s=3.0, what=""):
        """Instance-iterations/s of N fixed iterations over a bounded sample: instances are taken
        cyclically from the given ones (shared: GP/PD rows; distinct: whole instances) until the
        sample costs about ``budget_s``."""
        threads = threads or self.info["threads"]
        pool = GP.shape[0]

        def take(k):
            idx = np.arange(k) % pool
            if shared:
                return MGneg, GP[idx], GL, PD[idx]
            return MGneg[idx], GP[idx], GL[idx], PD[idx]

        k0 = max(1, min(threads, 64))
        probe = self._run(*take(k0), N, shared, threads)
        per = probe / k0 * min(threads, k0)  # seconds per instance on one thread
        count = int(max(threads, min(1 << 20, budget_s * threads / max(per, 1e-9))))
        count = max(threads, (count // threads) * threads) if threads > 1 else max(1, count)
        dt = self._run(*take(count), N, shared, threads)
        return {"value": count * N / dt, "unit": "GPAD iterations/s", "cores": threads, "kind": self.kind,
                "sample": f"{count} instances x {N} iterations{', ' + what if what else ''}, fp32, "
                          f"{'OpenMP over instances' if threads > 1 else 'one thread'}",
                "seconds": round(dt, 3), **{k: v for k, v in self.info.items() if k != "threads"}}


def cpu_baseline(n, m, ML, G, L, M, g, iters_per_instance, budget_s=12.0, ref=None):
    """Headline CPU baseline: the C4 workload (shared ML/G, this rank's q/b draws) for the mean
    GPU iteration count to eps, all granted host cores; plus the single-thread rate."""
    ref = ref or CpuRef()
    O = ref.O
    ML32, G32, L32 = ML.astype(np.float32), G.astype(np.float32), np.float32(L)
    MGneg, GL, _ = O.scale(ML32, G32, g[0].astype(np.float32), L32)
    N = max(1, int(round(iters_per_instance)))
    GP = M.astype(np.float32)
    PD = O.scale_vec(g.astype(np.float32), L32)
    out = ref.rate(MGneg, GP, GL, PD, N, shared=True, budget_s=budget_s,
                   what=f"C4 instances (shared ML/G), N = mean GPU iterations to eps")
    one = ref.rate(MGneg, GP[:64], GL, PD[:64], N, shared=True, threads=1, budget_s=1.5)
    out["single_thread_value"] = one["value"]
    return out


def phase_schedule(N, K=10, plan=None, fin=512):
    """The phase boundaries a phased panel solve follows (csrc/gpad_panel.hip launch_panel_t):
    the handle's plan (gpad_phase_plan: made from the previous solve's iteration counts), or
    without one the default phases of 4K iterations, doubling after the 10th.  Returns
    [(v0, v1, finisher threshold at v0)]."""
    out, v0, ph = [], 0, 0
    ends = plan["ends"] if plan and plan.get("ends") else []
    fins = plan["fins"] if ends else []
    while v0 < N:
        plen = 4 * K if ph < 10 else (4 * K) << min(ph - 9, 20)
        f = fin
        if ph < len(ends):
            plen, f = ends[ph] - v0, (fins[ph] if ph else fin)
        v1 = N if N - v0 <= plen else v0 + plen
        out.append((v0, v1, f))
        v0, ph = v1, ph + 1
    return out


def phase_util(iters, N, K=10, plan=None, fin=512):
    """Column utilisation of phased compaction, estimated from the per-instance iteration
    counts: a phase [v0, v1) packs its survivors (iters > v0) into 16-column panels that run
    until v1 or their last column's end, until the survivors fit the resident finisher (one
    instance per workgroup, no idle columns); useful = sum of iterations.  Also the phase
    launches per solve."""
    it = iters.astype(np.int64)  # survivors keep (roughly) index order in the kernel's lists
    executed = 0
    phases = phase_schedule(N, K, plan, fin)
    takeover = None
    for v0, v1, f in phases:
        surv = it[it > v0]
        if surv.size == 0:
            continue
        if v0 > 0 and surv.size <= f:  # the finisher runs them to the end
            executed += int((surv - v0).sum())
            takeover = v0
            break
        for i in range(0, surv.size, 16):
            executed += 16 * (min(v1, int(surv[i:i + 16].max())) - v0)
    return {"column_util_est": float(it.sum() / executed) if executed else None,
            "launches_per_solve": len(phases), "phase_ends": [p[1] for p in phases],
            "finisher_takeover": takeover, "planned": bool(plan and plan.get("ends")),
            "plan_model_us": plan.get("cost_us") if plan else None,
            "min_iters": int(it.min()), "max_iters": int(it.max())}


def traffic_from_profile(kernel_name):
    """HBM bytes per solve of the dominant kernel from the committed PMC profile of this same
    bench command (tools/profile.sh -> the newest profiles/rNN_bench_summary.json; FETCH_SIZE x2 +
    WRITE_SIZE, MI355X_MICROARCH.md §HBM): the kernel's bytes summed over every launch of the
    profiled run / the C4 solves that run made (2 x (--warmup + --steps): the fresh-input and the
    repeated-input loops; the side legs launch other kernel instantiations).  ``kernel_name`` is
    a prefix: every instantiation of that kernel family and tile count is summed (the T = 13 pairs
    are compiled per last-block length, gpad_panel2_kernel<13, KQ>).  None when absent."""
    import glob
    found = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_bench_summary.json")))
    if not found:
        return None, None
    path = found[-1]
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return None, None
    args = d.get("bench_args", "").split()
    try:
        solves = 2 * (int(args[args.index("--steps") + 1]) + int(args[args.index("--warmup") + 1]))
    except (ValueError, IndexError):
        return None, None
    names = kernel_name if isinstance(kernel_name, (list, tuple)) else [kernel_name]
    tot = [v["hbm_bytes_total"] for k, v in d.get("pmc_per_launch", {}).items()
           if any(k == kn or (kn.endswith(">") and k.startswith(kn[:-1] + ", ")) for kn in names)
           and "hbm_bytes_total" in v]
    if not tot or solves <= 0:
        return None, None
    return sum(tot) / solves, os.path.relpath(path, ROOT)


def kernel_ms_from_profile(kernel_prefix):
    """Device time per C4 solve of one kernel family from the committed kernel trace of this same
    bench command (the newest profiles/rNN_bench_summary.json, `kernels` = rocprofv3 --stats): the
    total of every instantiation whose name starts with ``kernel_prefix`` / the profiled run's
    solves (2 x (--warmup + --steps), as traffic_from_profile).  (None, None) when absent."""
    import glob
    found = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_bench_summary.json")))
    if not found:
        return None, None
    try:
        d = json.load(open(found[-1]))
        args = d.get("bench_args", "").split()
        solves = 2 * (int(args[args.index("--steps") + 1]) + int(args[args.index("--warmup") + 1]))
    except (OSError, ValueError, IndexError):
        return None, None
    tot = sum(v["total_ns"] for k, v in d.get("kernels", {}).items() if k.startswith(kernel_prefix))
    if not tot or solves <= 0:
        return None, None
    return tot / solves / 1e6, os.path.relpath(found[-1], ROOT)


def panel_share(iters, phases):
    """Instance-iterations of one phased solve that ran on the panels: everything up to the
    finisher's takeover (gpad_last_phases: the first phase whose input the duo took), the rest on
    the finisher."""
    it = np.asarray(iters, np.int64)
    take = phases.get("takeover") if phases else None
    if not take:
        return int(it.sum()), 0, None
    v = int(take["iteration"])
    pan = int(np.minimum(it, v).sum())
    return pan, int(it.sum()) - pan, v


def hbm_leg(dev, batch=1024, n=800, m=800, N=20, ref=None):
    """C5: long horizon (N = 200 -> n = 800), m = 800, 1024 instances with DISTINCT matrices:
    the matrices cannot stay on chip, so every iteration streams 5.1 MB per instance from HBM
    (stream kernel).  Returns achieved algorithmic GB/s vs the 8 TB/s roofline."""
    import torch

    import gpad_mpc
    g = torch.Generator(device=dev).manual_seed(0)
    R = torch.randn(batch, n, n, device=dev, generator=g) / np.sqrt(n)
    H = R.transpose(1, 2) @ R + torch.eye(n, device=dev)
    G = torch.randn(batch, m, n, device=dev, generator=g) / np.sqrt(n)
    Hi = torch.cholesky_inverse(torch.linalg.cholesky(H))
    ML = (Hi @ G.transpose(1, 2)).contiguous()
    L = float(torch.linalg.matrix_norm(G @ ML, "fro").max())
    zf = torch.rand(batch, n, device=dev, generator=g) - 0.5
    gv = (G @ zf.unsqueeze(2)).squeeze(2) + 0.1 + 0.9 * torch.rand(batch, m, device=dev, generator=g)
    M = (Hi @ torch.randn(batch, n, 1, device=dev, generator=g)).squeeze(2).contiguous()
    del R, H, Hi
    z = torch.zeros(batch, n, device=dev)
    y = torch.zeros(batch, m, device=dev)
    with gpad_mpc.GpadSolver(dev.index or 0, stream=torch.cuda.current_stream(dev).cuda_stream) as s:
        s.setup(ML, G.contiguous(), L, n=n, m=m, batch=batch, shared=False)
        s.run(z, y, M, gv, N, 0.0)
        best = 1e30
        for _ in range(3):
            st = s.run(z.zero_(), y.zero_(), M, gv, N, 0.0)
            best = min(best, st["kernel_ms"])
    per_it = 4 * (2 * n * m + 4 * m + 3 * n)
    gbs = batch * N * per_it / (best / 1e3) / 1e9
    out = {"config": f"C5: {batch} distinct instances, N=200 (n={n}), m={m}, {N} iterations",
           "kernel": st["kernel"], "iters_per_s": batch * N / (best / 1e3),
           "achieved_GBs": gbs, "peak_GBs": HBM_PEAK_GBS, "frac": gbs / HBM_PEAK_GBS,
           "bytes_per_instance_iter": per_it}
    if ref is not None:  # the reference's CPU steps on a pool of these distinct instances
        k = min(batch, 2 * ref.info["threads"])
        L32 = np.float32(L)
        MGneg = (-ML[:k]).cpu().numpy()
        GL = (G[:k].double() * (1.0 / float(L32))).float().cpu().numpy()
        PD = (gv[:k].double() * (-1.0 / float(L32))).float().cpu().numpy()
        out["cpu_baseline"] = ref.rate(MGneg, M[:k].cpu().numpy(), GL, PD, N, shared=False,
                                       what=f"C5 distinct 800x800 instances (pool of {k})")
    return out


def distinct_leg(dev, n, m, batch=8192, N=100, ref=None):
    """C2-shape instances with distinct matrices, register-resident (resident kernel)."""
    import torch

    import gpad_mpc
    g = torch.Generator(device=dev).manual_seed(1)
    ML = (torch.randn(batch, n, m, device=dev, generator=g) / np.sqrt(m) * 0.1).contiguous()
    G = (torch.randn(batch, m, n, device=dev, generator=g) / np.sqrt(n)).contiguous()
    M = torch.randn(batch, n, device=dev, generator=g)
    gv = torch.rand(batch, m, device=dev, generator=g) + 0.1
    z = torch.zeros(batch, n, device=dev)
    y = torch.zeros(batch, m, device=dev)
    with gpad_mpc.GpadSolver(dev.index or 0, stream=torch.cuda.current_stream(dev).cuda_stream) as s:
        s.setup(ML, G, 10.0, n=n, m=m, batch=batch, shared=False)
        s.run(z, y, M, gv, N, 0.0)
        st = s.run(z.zero_(), y.zero_(), M, gv, N, 0.0)
    ips = batch * N / (st["kernel_ms"] / 1e3)
    alg = ips * 4.0 * (2 * n * m + 4 * m + 3 * n) / 1e9  # SURVEY §8d distinct-matrix bytes per iteration
    out = {"config": f"{batch} distinct {n}x{m} instances, {N} iterations", "kernel": st["kernel"],
           "iters_per_s": ips, "algorithmic_gbs": alg, "algorithmic_over_hbm_peak": alg / HBM_PEAK_GBS,
           "note": "SURVEY §8d's distinct-matrix bytes 4 (2nm + 4m + 3n) per instance-iteration: what a kernel "
                   "streaming each instance's ML and G every iteration would move; the resident kernel loads "
                   "them into VGPRs once per solve (HBM sees ~1/N of it), so the algorithmic rate exceeds the "
                   "8 TB/s roofline -- the N = 50, m = 200 distinct batch is not HBM-bound on this design"}
    if ref is not None:
        k = min(batch, 4 * ref.info["threads"])
        GL = (G[:k].double() * 0.1).float().cpu().numpy()
        PD = (gv[:k].double() * -0.1).float().cpu().numpy()
        out["cpu_baseline"] = ref.rate((-ML[:k]).cpu().numpy(), M[:k].cpu().numpy(), GL, PD, N, shared=False,
                                       what=f"distinct {n}x{m} instances (pool of {k})")
    return out


def c3_leg(dev, n=200, m=200, batch=4096, reps=3, max_iters=5000, tol=1e-4, ref=None):
    """BASELINE config C3: 4096 instances sharing ML/G (N = 50: n = 200), m = 200, solved to
    eps = 1e-4 (Algorithm 1, K = 10) on the panel kernels -- the same generator as the headline
    shard, half its size (one panel per workgroup instead of pairs: 256 panels = 256 CUs)."""
    import torch

    import gpad_mpc
    ML, G, L, M, g = make_shard(n, m, batch, 0)
    f32 = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(dev)  # noqa: E731
    dML, dG, dM, dg = f32(ML), f32(G), f32(M), f32(g)
    z = torch.zeros(batch, n, device=dev)
    y = torch.zeros(batch, m, device=dev)
    with gpad_mpc.GpadSolver(dev.index or 0, stream=torch.cuda.current_stream(dev).cuda_stream) as s:
        s.setup(dML, dG, float(np.float32(L)), n=n, m=m, batch=batch, shared=True, check_every=10)
        best, st = 1e30, None
        for _ in range(reps + 2):  # the first two solves build the phase plan
            r = s.run(z.zero_(), y.zero_(), dM, dg, max_iters, tol)
            if r["kernel_ms"] < best:
                best, st = r["kernel_ms"], r
    out = {"config": f"C3: {batch} instances sharing ML/G, n={n}, m={m}, eps={tol}", "kernel": st["kernel"],
           "iters_per_s": st["total_iterations"] / (best / 1e3), "qp_solves_per_s": batch / (best / 1e3),
           "mean_iters_to_eps": st["total_iterations"] / batch, "solve_ms": best}
    if ref is not None:
        N = max(1, int(round(st["total_iterations"] / batch)))
        O = ref.O
        L32 = np.float32(L)
        MGneg, GL, _ = O.scale(ML.astype(np.float32), G.astype(np.float32), g[0].astype(np.float32), L32)
        c = ref.rate(MGneg, M.astype(np.float32), GL, O.scale_vec(g.astype(np.float32), L32), N, shared=True,
                     what="C3 instances (shared ML/G), N = mean GPU iterations to eps")
        c["qp_solves_per_s"] = c["value"] / N
        out["cpu_baseline"] = c
    return out


def c4_global_leg(dev, n=200, m=200, batch=65536, steps=6, warmup=2, max_iters=5000, tol=1e-4, ref=None):
    """BASELINE config C4 at its global size on ONE GPU: all 65536 instances (the batch the 8-GPU
    run shards 8 x 8192) as one gpad_run per step, FRESH q/b every step as in the headline, steps
    enqueued back to back (no host sync, work summed on the device), HIP events around them.  The
    strong-scaling anchor for the driver's 1/2/4/8-GPU curve of the sharded batch (the headline
    itself is weak scaling: 8192 per GPU).  tests/test_configs.py::test_c4_global_65536 checks the
    same batch through gpad_solve_sharded over 8 shards against one handle and the oracle."""
    import torch

    import gpad_mpc
    ML, G, L, _, _ = make_shard(n, m, 1, 0)
    f32 = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(dev)  # noqa: E731
    draws = make_stream(n, m, batch, warmup + steps, 99)
    fresh = [(f32(a), f32(b)) for a, b in draws]
    dML, dG = f32(ML), f32(G)
    z = torch.zeros(batch, n, device=dev)
    y = torch.zeros(batch, m, device=dev)
    stream = torch.cuda.current_stream(dev)
    with gpad_mpc.GpadSolver(dev.index or 0, stream=stream.cuda_stream) as s:
        s.setup(dML, dG, float(np.float32(L)), n=n, m=m, batch=batch, shared=True, check_every=10)
        for k in range(warmup):
            s.run(z.zero_(), y.zero_(), *fresh[k], max_iters, tol, stats=False)
        torch.cuda.synchronize(dev)
        acc = torch.zeros(1, dtype=torch.int64, device=dev)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        ev0.record(stream)
        for k in range(steps):
            s.run(z.zero_(), y.zero_(), *fresh[warmup + k], max_iters, tol, stats=False)
            s.accumulate_iterations(acc)
        ev1.record(stream)
        torch.cuda.synchronize(dev)
        dt = time.perf_counter() - t0
        dev_ms = ev0.elapsed_time(ev1) / steps
        st = s.last_stats()
        total = int(acc.item())
    out = {"config": f"C4 global batch on one GPU: {batch} instances sharing ML/G, n={n}, m={m}, eps={tol}, "
                     f"fresh q/b every step ({steps} timed after {warmup})",
           "kernel": st["kernel"], "converged_last": st["converged"],
           "iters_per_s": total / dt, "qp_solves_per_s": batch * steps / dt, "ms_per_solve": dt / steps * 1e3,
           "device_ms_per_solve": dev_ms, "mean_iters_to_eps": total / (batch * steps),
           "achieved_tflops": total / steps * flops_per_iter(n, m) / (dev_ms / 1e3) / 1e12}
    if ref is not None:
        N = max(1, int(round(out["mean_iters_to_eps"])))
        O = ref.O
        L32 = np.float32(L)
        k = min(batch, 64 * ref.info["threads"])
        Mv, gv = (a[:k].astype(np.float32) for a in draws[-1])
        MGneg, GL, _ = O.scale(ML.astype(np.float32), G.astype(np.float32), gv[0], L32)
        c = ref.rate(MGneg, Mv, GL, O.scale_vec(gv, L32), N, shared=True,
                     what=f"C4 instances (pool of {k}, shared ML/G), N = mean GPU iterations to eps")
        c["qp_solves_per_s"] = c["value"] / N
        out["cpu_baseline"] = c
    return out


def f64_value_leg(dev, n=200, m=200, batch=8192, tol=1e-6, max_iters=20000, ref=None):
    """The reference's own termination regime (acceldualgrad.m:12-13: e_g = e_V = 1e-6, below the
    f32 certification floor, so f64) with the QP Hessian bound -- Algorithm 1's value-function
    branches (:73, :76) evaluated -- on C4-shaped value problems (n = m = 200 sharing H, ML, G;
    constraints active at optima with positive objective values: tests/test_value.py's generator):
    the f64 MFMA panels (gpad_panel64.hip) beside the one-instance-per-workgroup f64 stream kernel
    on the same batch (bit-identical results, tests/test_panel64.py).  CPU: the oracle's fp64
    restatement of acceldualgrad.m (the reference's f64 path is MATLAB, not runnable here)."""
    import torch

    import gpad_mpc
    from gpad_mpc import _lib
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_value import value_problem
    H, ML, M, G, g, L, _ = value_problem(n, m, 7, 1.0, batch=batch)
    f64 = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float64)).to(dev)  # noqa: E731
    dH, dML, dG, dM, dg = f64(H), f64(ML), f64(G), f64(M), f64(g)
    out = {"config": f"{batch} value problems sharing H, ML, G, n={n}, m={m}, f64, e_g = e_V = {tol}, "
                     "H bound (value-function branches)"}
    for name, kern in (("panel64", _lib.KERNEL_PANEL), ("stream", _lib.KERNEL_STREAM)):
        z = torch.zeros(batch, n, dtype=torch.float64, device=dev)
        y = torch.zeros(batch, m, dtype=torch.float64, device=dev)
        codes = np.zeros(batch, np.int32)
        with gpad_mpc.GpadSolver(dev.index or 0, stream=torch.cuda.current_stream(dev).cuda_stream) as s:
            s.setup(dML, dG, float(L), n=n, m=m, batch=batch, shared=True, check_every=10, kernel=kern,
                    tol_gap=tol)
            s.setup_hessian(dH)
            s.run(z.zero_(), y.zero_(), dM, dg, max_iters, tol)  # untimed warm-up, both kernels alike
            best, st = 1e30, None
            for _ in range(2):
                r = s.run(z.zero_(), y.zero_(), dM, dg, max_iters, tol, codes=codes)
                if r["kernel_ms"] < best:
                    best, st = r["kernel_ms"], r
        out[name] = {"kernel": st["kernel"], "iters_per_s": st["total_iterations"] / (best / 1e3),
                     "qp_solves_per_s": batch / (best / 1e3), "solve_ms": best,
                     "mean_iters_to_eps": st["total_iterations"] / batch, "converged": st["converged"],
                     "codes": {str(k): int((codes == k).sum()) for k in range(5) if (codes == k).any()}}
    out["speedup_vs_stream"] = out["panel64"]["iters_per_s"] / out["stream"]["iters_per_s"]
    # the same problems at 4x the batch (8 instances per panel column): the regime where column
    # refills (gpad_panel64.hip REFILL) pay -- a finished column takes the next instance at its test
    B4 = 4 * batch
    H4, ML4, M4, G4, g4, L4, _ = value_problem(n, m, 7, 1.0, batch=B4)
    dM4, dg4 = f64(M4), f64(g4)
    z4 = torch.zeros(B4, n, dtype=torch.float64, device=dev)
    y4 = torch.zeros(B4, m, dtype=torch.float64, device=dev)
    with gpad_mpc.GpadSolver(dev.index or 0, stream=torch.cuda.current_stream(dev).cuda_stream) as s:
        s.setup(dML, dG, float(L), n=n, m=m, batch=B4, shared=True, check_every=10, kernel=_lib.KERNEL_PANEL,
                tol_gap=tol)
        s.setup_hessian(dH)
        s.run(z4.zero_(), y4.zero_(), dM4, dg4, max_iters, tol)
        best4, st4 = 1e30, None
        for _ in range(2):
            r = s.run(z4.zero_(), y4.zero_(), dM4, dg4, max_iters, tol)
            if r["kernel_ms"] < best4:
                best4, st4 = r["kernel_ms"], r
    it4 = st4["total_iterations"] / (best4 / 1e3)
    out[f"panel64_batch{B4}"] = {"iters_per_s": it4, "solve_ms": best4, "converged": st4["converged"],
                                 "mean_iters_to_eps": st4["total_iterations"] / B4,
                                 "frac_of_f64_peak": it4 * 4.0 * n * m / 1e12 / FP64_MFMA_PEAK_TFLOPS}
    del dM4, dg4, z4, y4
    achieved = out["panel64"]["iters_per_s"] * 4.0 * n * m / 1e12
    out["roofline"] = {"bound": "mfma", "achieved": achieved, "peak": FP64_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                       "frac": achieved / FP64_MFMA_PEAK_TFLOPS,
                       "note": "4nm flop per instance-iteration (the two mat-vecs); peak = f64 MFMA spec"}
    if ref is not None:  # the oracle's fp64 solve (acceldualgrad.m order) on a bounded sample, one thread
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import pyoracle
        O = pyoracle.Oracle()
        t0, its, k = time.perf_counter(), 0, 0
        while time.perf_counter() - t0 < 3.0 and k < batch:
            _, _, it, _ = O.solve_value_f64(np.zeros(n), np.zeros(m), ML, M[k], G, g[k], H, max_iters, L, tol,
                                            tol_gap=tol)
            its += it
            k += 1
        dt = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": its / dt, "unit": "GPAD iterations/s", "cores": 1, "kind": "port",
                               "sample": f"{k} instances to e_g = e_V = {tol} (value branches), fp64 oracle "
                                         "(acceldualgrad.m order), one thread", "seconds": round(dt, 3)}
    return out


def flat_leg(dev, batch=8192, N=100, horizon=10, ref=None):
    """the flat (equal-cell) battery path vs the full-matrix path on the
    same battery packs (n_u = 4; horizon 10: n = 40, m = 180 = C1; horizon 50: n = 200, m = 900,
    the full path then on the big-panel kernel), fixed N iterations, fp32."""
    import torch

    import gpad_mpc
    from gpad_mpc import problems
    qp = problems.battery_scenarios(4, horizon, batch, seed=9)
    MGf, GLf, L = problems.flatten_battery(qp, 4, horizon)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(np.asarray(a, np.float64).astype(np.float32))).to(dev)  # noqa: E731
    L32 = float(np.float32(L))
    GP, G = t(qp.M), t(qp.g)
    PD = (G * np.float32(-1.0 / np.float64(np.float32(L)))).contiguous()
    out = {"config": f"{batch} battery packs (n_u=4, N={horizon}: n={qp.n}, m={qp.m}), {N} iterations"}
    stream = torch.cuda.current_stream(dev).cuda_stream
    for name in ("flat", "full"):
        with gpad_mpc.GpadSolver(dev.index or 0, stream=stream) as s:
            if name == "flat":
                s.setup_flat(t(MGf), t(GLf), L32, n_u=4, batch=batch)
            else:
                s.setup(-t(qp.ML), t(qp.G) / np.float32(L32), L32, n=qp.n, m=qp.m, batch=batch,
                        scaled=True)
            Z = torch.zeros(batch, qp.n, device=dev)
            Y = torch.zeros(batch, qp.m, device=dev)
            s.run(Z, Y, GP, PD, N, 0.0, scaled=True)
            best = 1e30
            for _ in range(3):
                st = s.run(Z.zero_(), Y.zero_(), GP, PD, N, 0.0, scaled=True)
                best = min(best, st["kernel_ms"])
        out[name] = {"kernel": st["kernel"], "iters_per_s": batch * N / (best / 1e3)}
    if ref is not None and ref.R is not None:  # the reference's own flat steps, one thread
        th, be = ref.O.schedule_f32(N)
        MGf32 = np.ascontiguousarray(np.asarray(MGf, np.float64).astype(np.float32))
        GLf32 = np.ascontiguousarray(np.asarray(GLf, np.float64).astype(np.float32))
        GPh, PDh = GP.cpu().numpy(), PD.cpu().numpy()
        k, t0 = 0, time.perf_counter()
        while k < batch and time.perf_counter() - t0 < 2.0:
            ref.R.solve_flat_c(np.zeros(qp.n, np.float32), np.zeros(qp.m, np.float32), MGf32, GPh[k], GLf32,
                               PDh[k], 4, th, be, N)
            k += 1
        dt = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": k * N / dt, "unit": "GPAD iterations/s", "cores": 1, "kind": "reference",
                               "sample": f"{k} packs x {N} iterations, the reference's flat steps "
                                         "(StepTwo/FourGPADFlatSequential), one thread"}
    return out


def flat_phase_schedule(N, K=10, base=0, vpred=0):
    """csrc/gpad_flatpanel.hip flat_phase_len: 2K, then a quarter of the iterations done; past
    the previous solve's last iteration vpred one phase to N."""
    out, v0 = [], 0
    while v0 < N:
        plen = max(base or 2 * K, (v0 // 4) // K * K)
        if vpred and v0 >= vpred:
            plen = N
        v1 = N if N - v0 <= plen else v0 + plen
        out.append((v0, v1))
        v0 = v1
    return out


def flat_util(iters, N, width, phased=True, K=10, vpred=0):
    """Column utilisation of the flat panels: useful instance-iterations / column-iterations
    issued.  A group of `width` columns runs until the phase end or its last column's end;
    phased=False: one phase (a group runs until its slowest column)."""
    it = iters.astype(np.int64)
    phases = flat_phase_schedule(N, K, vpred=vpred) if phased else [(0, N)]
    executed = 0
    for v0, v1 in phases:
        surv = it[it > v0]
        for i in range(0, surv.size, width):
            executed += width * (min(v1, int(surv[i:i + width].max())) - v0)
    return float(it.sum() / executed) if executed else None, len(phases)


def flat_tol_leg(dev, batch=8192, horizon=10, tol=1e-4, N=5000):
    """§8 f4 in tol mode: the flat panels with phased compaction vs one launch (groups run to
    their slowest column); column utilisation estimated from the per-instance counts.  The
    timed solves repeat one batch, so the phase schedule's end (the previous solve's last
    iteration) is exact here."""
    import torch

    import gpad_mpc
    from gpad_mpc import problems
    qp = problems.battery_scenarios(4, horizon, batch, seed=9)
    MGf, GLf, L = problems.flatten_battery(qp, 4, horizon)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(np.asarray(a, np.float64).astype(np.float32))).to(dev)  # noqa: E731
    L32 = float(np.float32(L))
    GP, G = t(qp.M), t(qp.g)
    PD = (G * np.float32(-1.0 / np.float64(np.float32(L)))).contiguous()
    out = {"config": f"{batch} battery packs (n_u=4, N={horizon}: n={qp.n}, m={qp.m}), flat data, eps={tol}"}
    stream = torch.cuda.current_stream(dev).cuda_stream
    for phased in (2, 0):  # forced phases / one launch (the default picks phases from 4 panels per CU)
        with gpad_mpc.GpadSolver(dev.index or 0, stream=stream) as s:
            s.setup_flat(t(MGf), t(GLf), L32, n_u=4, batch=batch)
            s.set_option("phased", phased)
            Z = torch.zeros(batch, qp.n, device=dev)
            Y = torch.zeros(batch, qp.m, device=dev)
            it = np.zeros(batch, np.int32)
            s.run(Z, Y, GP, PD, N, tol, scaled=True)
            best = 1e30
            for _ in range(3):
                st = s.run(Z.zero_(), Y.zero_(), GP, PD, N, tol, scaled=True, iters=it)
                best = min(best, st["kernel_ms"])
        vp = int(it.max())  # the timed solves re-solve the same batch: predicted = last max
        u16, launches = flat_util(it, N, 16, bool(phased), vpred=vp)
        u32, _ = flat_util(it, N, 32, bool(phased), vpred=vp)
        out["phased" if phased else "one_launch"] = {
            "kernel": st["kernel"], "iters_per_s": float(it.sum()) / (best / 1e3),
            "qp_solves_per_s": batch / (best / 1e3), "solve_ms": best, "converged": st["converged"],
            "mean_iters": float(it.mean()), "max_iters": int(it.max()),
            "column_util_est": {"P1_16_columns": u16, "P2_32_columns": u32}, "launches": launches}
    return out


def closed_loop_leg(dev, batch=8192, steps=20, N=100, cpu=True, flat=False):
    """gpad.m:79-95 closed loop on the device for a batch of battery
    packs (C1 plant: n_u = 4 cells, horizon 10 -> n = 40, m = 180), each MPC step = per-state
    QP data + 100 GPAD iterations (acceldualgrad's fixed count) + plant update.  MPC steps/s
    (all packs) and GPAD iterations/s; CPU: the oracle's closed loop (fp32 port, 1 thread) on
    a bounded sample of packs."""
    import torch

    import gpad_mpc
    from gpad_mpc import problems
    qp, pl = problems.battery_plant(4, 10)
    f32 = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(dev)  # noqa: E731
    L32 = float(np.float32(qp.L))
    X0 = (np.random.default_rng(3).random((batch, 4)) - 0.5).astype(np.float32)
    with gpad_mpc.GpadSolver(dev.index or 0, stream=torch.cuda.current_stream(dev).cuda_stream) as s:
        if flat:  # the same packs on the reference's flat data (equal cells; §8f row 4)
            MGf, GLf, Lf = problems.flatten_battery(qp, 4, 10)
            s.setup_flat(f32(MGf), f32(GLf), float(np.float32(Lf)), n_u=4, batch=batch)
        else:
            s.setup(f32(qp.ML), f32(qp.G), L32, n=qp.n, m=qp.m, batch=batch)
        s.setup_plant(f32(pl.PM), f32(pl.Pg), g0=f32(pl.g0), A=f32(pl.A), B=f32(pl.B))
        X = torch.from_numpy(X0).to(dev)
        Z = torch.zeros(batch, qp.n, device=dev)
        Y = torch.zeros(batch, qp.m, device=dev)
        s.closed_loop(X, Z, Y, steps, N, 0.0)
        X.copy_(torch.from_numpy(X0))
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        s.closed_loop(X, Z, Y, steps, N, 0.0, stats=False)  # asynchronous: no per-step counters copy
        torch.cuda.synchronize(dev)
        wall = time.perf_counter() - t0
        st = s.last_stats()
    out = {"config": f"{batch} battery packs (n_u=4, N=10: n={qp.n}, m={qp.m}), {steps} MPC steps "
                     f"x {N} GPAD iterations, cold start (gpad.m)", "kernel": st["kernel"],
           "mpc_steps_per_s": batch * steps / wall, "iters_per_s": st["total_iterations"] / wall,
           "device_ms": st["kernel_ms"], "wall_ms": wall * 1e3}
    if flat:
        out["config"] += ", flat battery data (gpad_setup_flat)"
    if cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import pyoracle
        O = pyoracle.Oracle()
        MGneg, GL, _ = O.scale(np.float32(qp.ML), np.float32(qp.G), np.float32(qp.g), np.float32(L32))
        k, t0 = 0, time.perf_counter()
        while k < 64 and time.perf_counter() - t0 < 3.0:
            O.closed_loop_f32(X0[k], MGneg, GL, L32, pl.PM, pl.Pg, pl.A, pl.B, steps, N, g0=pl.g0)
            k += 1
        dt = time.perf_counter() - t0
        out["cpu_baseline"] = {"mpc_steps_per_s": k * steps / dt, "cores": 1, "kind": "port",
                               "sample": f"{k} packs x {steps} steps (oracle closed loop, fp32)"}
    return out


def sharded_leg(dev, ndev, n=200, m=200, batch=65536, steps=6, warmup=2, max_iters=5000, tol=1e-4, devices=None):
    """BASELINE config C4 through the library's own multi-device entry (include/gpad.h
    gpad_group_*, the path gpad_solve_sharded caches): the 65536-instance batch resident on device
    0, scattered to devices 0..ndev-1 by the group's RCCL clique (ncclBroadcast of the shared
    matrices at setup, grouped ncclSend/Recv of M, g, z0, y0 per run), one shard solved per device,
    (z*, y*) gathered back -- FRESH q/b every run, each run synchronous (wall clock around it).
    The same inputs then go through ONE handle on device 0 (device-event time per solve): the
    ratio is the strong-scaling speedup of the global batch, and the last run's iteration counts,
    z* and y* must be bit-identical between the two (the shards are independent instances).
    Run on rank 0 after every rank's timed region; skipped with fewer than 2 distinct devices
    (``devices`` overrides the list: tests run it over [0, 0] on the peer-copy transport).
    The reference solves one problem per process (Code/CUDA/FinalProject/main.cu:106-108)."""
    import torch

    import gpad_mpc
    ML, G, L, _, _ = make_shard(n, m, 1, 0)
    L32 = float(np.float32(L))
    f32 = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(dev)  # noqa: E731
    fresh = [(f32(a), f32(b)) for a, b in make_stream(n, m, batch, warmup + steps, 99)]
    dML, dG = f32(ML), f32(G)
    z = torch.zeros(batch, n, device=dev)
    y = torch.zeros(batch, m, device=dev)
    devices = list(devices) if devices is not None else list(range(ndev))
    it_g = np.zeros(batch, np.int32)
    torch.cuda.synchronize(dev)
    with gpad_mpc.GpadGroup(devices) as grp:
        transport = grp.transport
        grp.setup(dML, dG, L32, n=n, m=m, batch=batch, shared=True, check_every=10)
        t = []
        for k in range(warmup + steps):
            z.zero_()
            y.zero_()
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            st = grp.run(z, y, *fresh[k], max_iters, tol, iters=it_g)
            t.append(time.perf_counter() - t0)
        zg, yg = z.clone(), y.clone()
    group_s = sum(t[warmup:])
    it_1 = np.zeros(batch, np.int32)
    stream = torch.cuda.current_stream(dev)
    with gpad_mpc.GpadSolver(dev.index or 0, stream=stream.cuda_stream) as s:
        s.setup(dML, dG, L32, n=n, m=m, batch=batch, shared=True, check_every=10)
        for k in range(warmup):
            s.run(z.zero_(), y.zero_(), *fresh[k], max_iters, tol, stats=False)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for k in range(warmup, warmup + steps):
            st1 = s.run(z.zero_(), y.zero_(), *fresh[k], max_iters, tol, iters=it_1)
        one_s = time.perf_counter() - t0
    same = bool(np.array_equal(it_g, it_1) and torch.equal(zg, z) and torch.equal(yg, y))
    total = int(it_g.sum())
    return {"config": f"C4 global batch: {batch} instances sharing ML/G, n={n}, m={m}, eps={tol}, resident on "
                      f"device 0, gpad_group over devices {devices} ({transport}), fresh q/b every run "
                      f"({steps} timed after {warmup})",
            "n_devices": len(devices), "transport": transport, "kernel": st["kernel"],
            "ms_per_solve": group_s / steps * 1e3, "qp_solves_per_s": batch * steps / group_s,
            "last_run_iters_per_s": total / t[-1], "converged_last": st["converged"],
            "one_gpu_ms_per_solve": one_s / steps * 1e3, "strong_scaling_speedup": one_s / group_s,
            "bitexact_vs_one_handle": same,
            "note": "ms_per_solve includes the scatter of M, g, z0, y0 and the gather of (z*, y*) over the "
                    "group's transport; one_gpu_ms_per_solve is the same batches on one handle (host clock, "
                    "stats copied each run); bitexact_vs_one_handle compares the last run's counts, z*, y*"}


def guarded(fn, timeout_s, what):
    """Run fn() in a daemon thread; past timeout_s return a "skipped" record instead of its result,
    so a hung multi-device leg cannot take the bench's JSON line with it (rank 0 then prints the
    line and leaves with os._exit, the other ranks' final barrier fails and they exit cleanly)."""
    import threading
    box = {}

    def run():
        try:
            box["r"] = fn()
        except Exception as e:  # reported in the line, not raised: the timed results stand
            box["r"] = {"skipped": f"{what} failed: {type(e).__name__}: {e}"}
    th = threading.Thread(target=run, daemon=True)
    th.start()
    th.join(timeout_s)
    if th.is_alive():
        return {"skipped": f"{what} did not finish in {timeout_s} s"}, True
    return box["r"], False


def launch_ranks(gpus, argv):
    """``python bench.py --gpus N`` without a launcher: start the N ranks as ONE child process
    (torch.distributed.run, one rank per GPU, rendezvous on 127.0.0.1) and return its exit status.
    Runs before this process imports torch or touches the GPU; rank 0's JSON line reaches stdout
    through the inherited file descriptors.  The parent never execs itself."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *argv]
    sys.stdout.flush()
    return subprocess.call(cmd)


def make_stream(n, m, batch, count, rank, seed=0):
    """``count`` independent draws of this rank's shard for the timed steps: every step solves
    NEW problems (q, b of the SURVEY §8d generator, fresh per instance and per step), so the
    phase plan and the finisher's longest-first queue -- both built from the previous solve's
    iteration counts -- predict from a different problem, as in an MPC stream.  Vectorised
    numpy draws (one generator per rank and step), shared matrices from ``seed``."""
    from gpad_mpc import problems
    base = problems.synthetic_qp(n, m, batch=1, seed=seed)
    G, Hinv = base.G, np.linalg.inv(base.H)
    out = []
    for k in range(count):
        rng = np.random.default_rng([seed, 7919, rank, k])
        zf = rng.uniform(-0.5, 0.5, size=(batch, n))
        Bv = zf @ G.T + rng.uniform(0.1, 1.0, size=(batch, m))
        M = rng.normal(0.0, 1.0, size=(batch, n)) @ Hinv.T
        out.append((M, Bv))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    # untimed: the shader clock ramps over the first ~10 solves after an idle box (3.0 -> 3.2 ms per
    # fresh-input C4 solve, profiles/r06_timeline_fresh_solves.txt); the timed steps are steady state
    ap.add_argument("--warmup", type=int, default=12)
    ap.add_argument("--batch", type=int, default=8192, help="instances per GPU")
    ap.add_argument("--horizon", type=int, default=50)
    ap.add_argument("--nu", type=int, default=4)
    ap.add_argument("--m", type=int, default=200)
    ap.add_argument("--tol", type=float, default=1e-4)
    ap.add_argument("--max-iters", type=int, default=5000)
    ap.add_argument("--kernel", default="auto", choices=["auto", "stream", "resident", "panel"])
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip the C2/C5 side legs")
    ap.add_argument("--repeat-inputs", action="store_true",
                    help="headline on the SAME inputs every step (the planner then sees its own future); "
                         "default: fresh inputs per step, the repeated-input rate reported beside it")
    ap.add_argument("--no-sharded", action="store_true",
                    help="N > 1: skip rank 0's gpad_group leg over devices 0..N-1 after the timed region")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL) for real runs; gloo to rehearse ranks sharing one GPU")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:  # no launcher: start the ranks ourselves
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if env_world is not None and int(env_world) != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={env_world}: the launcher started a different "
              "number of ranks than the run was asked for", file=sys.stderr)
        sys.exit(2)

    import torch
    import torch.distributed as dist

    import gpad_mpc
    from gpad_mpc import _lib

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU; --dist-backend gloo only to rehearse several ranks on one GPU
    ndev = torch.cuda.device_count()
    dev = torch.device("cuda", local % max(ndev, 1))
    torch.cuda.set_device(dev)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    # a host-side group for the end-of-run barrier: the other ranks wait off the GPU while rank 0
    # runs its post-timing legs (the sharded leg drives every rank's device)
    host_pg = dist.new_group(backend="gloo") if world > 1 else None
    comm_dev = dev if args.dist_backend == "nccl" else torch.device("cpu")
    stream = torch.cuda.current_stream(dev)

    n, m, B = args.nu * args.horizon, args.m, args.batch
    ML, G, L, M, g = make_shard(n, m, B, rank * B)
    f32 = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(dev)  # noqa: E731
    dML, dG, dM, dg = f32(ML), f32(G), f32(M), f32(g)
    # fresh problems for every warm-up and timed step, resident in HBM before timing
    fresh = [(f32(a), f32(b)) for a, b in make_stream(n, m, B, args.warmup + args.steps, rank)]
    # z and y back to back in one buffer, so the cold start of every step is one fill
    zy = torch.zeros(B * (n + m), device=dev)
    z, y = zy[: B * n].view(B, n), zy[B * n:].view(B, m)
    kern = {"auto": _lib.KERNEL_AUTO, "stream": _lib.KERNEL_STREAM, "resident": _lib.KERNEL_RESIDENT,
            "panel": _lib.KERNEL_PANEL}[args.kernel]
    solver = gpad_mpc.GpadSolver(dev.index, stream=stream.cuda_stream)
    L32 = float(np.float32(L))
    solver.setup(dML, dG, L32, n=n, m=m, batch=B, shared=True, check_every=10, kernel=kern)
    # one gather of (z*, y*) to rank 0 per step, asynchronous and double buffered: the gather of
    # step k (RCCL on its own stream, ordered after the copy into its buffer) may overlap the
    # solve of step k + 1; a buffer is reused only after its gather two steps back completed,
    # and every gather is waited for inside the timed region (drain)
    slots = []
    if world > 1:
        for _ in range(2):
            pk = torch.empty(B, n + m, device=comm_dev)
            slots.append({"packed": pk, "work": None,
                          "gl": [torch.empty_like(pk) for _ in range(world)] if rank == 0 else None})
    nstep = [0]

    def step(Mv, gv):
        zy.zero_()  # z0 = 0, y0 = 0
        solver.run(z, y, Mv, gv, args.max_iters, args.tol, stats=False)
        if world > 1:
            sl = slots[nstep[0] % 2]
            nstep[0] += 1
            if sl["work"] is not None:
                sl["work"].wait()
            sl["packed"][:, :n] = z
            sl["packed"][:, n:] = y
            sl["work"] = dist.gather(sl["packed"], sl["gl"], dst=0, async_op=True)

    def drain():
        for sl in slots:
            if sl["work"] is not None:
                sl["work"].wait()
                sl["work"] = None

    def timed(inputs):
        """W warm-up steps, then K timed steps enqueued back to back with no host
        synchronisation: each step's work (the sum of its per-instance iteration counts) is
        accumulated on the device after its solve; HIP events on the solve stream bracket the
        K steps (device time of the solves plus the z/y resets, a few us per step).
        inputs(k) -> (M, g) of step k (k < W: warm-up)."""
        for k in range(args.warmup):
            step(*inputs(k))
        drain()
        torch.cuda.synchronize(dev)
        acc = torch.zeros(1, dtype=torch.int64, device=dev)
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        ev0.record(stream)
        ev_solved = torch.cuda.Event(enable_timing=True)
        for k in range(args.steps):
            step(*inputs(args.warmup + k))
            solver.accumulate_iterations(acc)
        ev_solved.record(stream)  # every solve enqueued; the last gathers may still be in flight
        drain()
        ev1.record(stream)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        dt = time.perf_counter() - t0
        kern_ms = ev0.elapsed_time(ev1)
        # the drain: from the last solve's end to the last gather's completion, on the solve stream
        drain_ms = ev_solved.elapsed_time(ev1)
        total_iters = int(acc.item())
        iters_host = np.zeros(B, np.int32)
        st = solver.last_stats(iters=iters_host)  # the last step's counters, outside the timed region
        # max time over ranks, sum of work over ranks
        stats = torch.tensor([dt, float(total_iters), kern_ms, float(st["converged"])], dtype=torch.float64,
                             device=comm_dev)
        if world > 1:
            tmax = stats[0:1].clone()
            dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
            work = stats[1:4].clone()
            dist.all_reduce(work, op=dist.ReduceOp.SUM)
            dt_all, iters_all, conv_all = float(tmax.item()), float(work[0].item()), float(work[2].item())
        else:
            dt_all, iters_all, conv_all = dt, float(total_iters), float(st["converged"])
        per_rank = None
        if world > 1:  # per-rank step time, device time and drain, for attributing a scaling loss
            mine = torch.tensor([dt / args.steps * 1e3, kern_ms / args.steps, drain_ms], dtype=torch.float64,
                                device=comm_dev)
            allr = [torch.empty_like(mine) for _ in range(world)]
            dist.all_gather(allr, mine)
            per_rank = [[float(v) for v in t.cpu()] for t in allr]
        return dict(dt=dt_all, iters_all=iters_all, converged_all=conv_all, total_iters=total_iters,
                    kern_ms=kern_ms, st=st, iters_host=iters_host, plan=solver.phase_plan(),
                    phases=last_phases(), drain_ms=drain_ms, per_rank=per_rank)

    def last_phases():
        try:
            return solver.last_phases()
        except gpad_mpc.GpadError:  # (an A/B build older than gpad_last_phases, GPAD_LIB_TOLERANT)
            return None

    def gather_ms(reps=3):
        """One step's gather of (z*, y*) to rank 0 on its own: barrier, blocking gather, device
        sync; the best of ``reps`` (after the timed regions; max over ranks)."""
        sl = slots[0]
        best = 1e30
        for _ in range(reps):
            dist.barrier()
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            dist.gather(sl["packed"], sl["gl"], dst=0)
            torch.cuda.synchronize(dev)
            best = min(best, (time.perf_counter() - t0) * 1e3)
        t = torch.tensor([best], dtype=torch.float64, device=comm_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    fresh_run = timed(lambda k: fresh[k])
    repeat_run = timed(lambda k: (dM, dg))
    head = repeat_run if args.repeat_inputs else fresh_run
    side = fresh_run if args.repeat_inputs else repeat_run
    multi = None
    if world > 1:
        pr = head["per_rank"]
        multi = {
            "per_rank_step_ms": [r[0] for r in pr],
            "per_rank_kernel_ms": [r[1] for r in pr],
            "solve_ms_min": min(r[1] for r in pr), "solve_ms_max": max(r[1] for r in pr),
            "drain_ms_max": max(r[2] for r in pr),
            "gather_ms": gather_ms(),
            "gather_bytes_per_rank": B * (n + m) * 4,
            "backend": args.dist_backend,
            "note": "per_rank_kernel_ms: device time per step on each rank's solve stream (solve + "
                    "resets + gather copies); drain_ms: last solve's end to the last gather's completion; "
                    "gather_ms: one blocking gather of a step's (z*, y*) measured alone after the timed "
                    "regions (max over ranks)"}

    # the C-ABI multi-device path on rank 0 (every rank's timed region is over, the barrier above;
    # the other ranks wait on host_pg): the global batch over devices 0..N-1 through gpad_group
    ndist = min(world, ndev)
    hung = False
    if multi is not None:
        if rank == 0 and ndist >= 2 and not args.no_sharded:
            multi["sharded_c4_global"], hung = guarded(lambda: sharded_leg(dev, ndist, n, m), 240,
                                                       "sharded_leg")
        else:
            multi["sharded_c4_global"] = {"skipped": f"{ndist} distinct device(s) visible" if ndist < 2 else
                                          "--no-sharded"}

    # CPU reference on rank 0 (all ranks' timed regions are over: the barrier above)
    ref = None
    if rank == 0 and not args.no_cpu:
        ref = CpuRef()

    if rank == 0:
        dt, st, total_iters, kern_ms = head["dt"], head["st"], head["total_iters"], head["kern_ms"]
        ms_per_step = dt / args.steps * 1e3
        value = head["iters_all"] / dt
        solves = B * world * args.steps / dt
        avg_kernel_s = kern_ms / args.steps / 1e3
        iters_per_launch = total_iters / args.steps
        F = flops_per_iter(n, m)
        achieved_tf = iters_per_launch * F / avg_kernel_s / 1e12
        hbm_alg_gbs = bytes_per_iter_shared(n, m, B) * (iters_per_launch / B) / (ms_per_step / 1e3) / 1e9
        mean_iters = iters_per_launch / B
        util = phase_util(head["iters_host"], args.max_iters, 10, head["plan"])
        T = (max(n, m) + 15) // 16
        kname = (f"gpad::gpad_panel2_kernel<{T}>" if T > 8 else f"gpad::gpad_panel_kernel<{T}>") \
            if st["kernel"] == "panel" else f"gpad::gpad_{st['kernel']}_kernel"
        traffic, traffic_src = traffic_from_profile(kname)
        launches = util["launches_per_solve"] if st["kernel"] == "panel" else 1
        # the dominant kernel alone: useful flops the panels did in the last
        # fresh-input solve (its counts up to the finisher's takeover) / the panel kernel's rocprof
        # time per solve from the committed profile of this bench command
        pan_iters, fin_iters, v_take = panel_share(head["iters_host"], head["phases"])
        pan_ms, pan_src = kernel_ms_from_profile(kname[:-1] + ", " if kname.endswith(">") else kname)
        kernel_frac = (pan_iters * F / (pan_ms * 1e-3) / 1e12 / FP32_PEAK_TFLOPS) if pan_ms else None
        # single instances (configs C1 and C2): latency kernels, fixed iteration counts
        singles = {}
        from gpad_mpc import problems
        qp1 = problems.battery_mpc(4, 10, seed=0)
        c1 = [np.ascontiguousarray(np.asarray(a, np.float64).astype(np.float32))
              for a in (qp1.ML, qp1.G, qp1.M, qp1.g)]
        for name, (mML, mG, mM, mg_, mL, iters) in {
                "c2": (dML, dG, dM[:1], dg[:1], L32, 1000),
                "c1": (*[f32(a) for a in c1[:2]], f32(c1[2]).reshape(1, -1), f32(c1[3]).reshape(1, -1),
                       float(np.float32(qp1.L)), 1000)}.items():
            nn, mm = mML.shape
            with gpad_mpc.GpadSolver(dev.index, stream=stream.cuda_stream) as s1:
                s1.setup(mML, mG, mL, n=nn, m=mm, batch=1)
                z1 = torch.zeros(1, nn, device=dev)
                y1 = torch.zeros(1, mm, device=dev)
                s1.run(z1, y1, mM, mg_, iters, 0.0)
                t = []
                for _ in range(5):
                    st1 = s1.run(z1.zero_(), y1.zero_(), mM, mg_, iters, 0.0)
                    t.append(st1["kernel_ms"])
            kb = (st1["kernel"], iters / (min(t) / 1e3))
            singles[name] = {"config": ("C2 single instance n=200 m=200" if name == "c2" else
                                        f"C1 single instance: battery n_u=4, N=10 (n={nn}, m={mm})"),
                             "kernel": kb[0], "iters_per_s": kb[1]}
            if ref is not None:  # the reference's CPU steps on the same instance, one thread
                O = ref.O
                hm = [a.cpu().numpy() for a in (mML, mG, mM, mg_)]
                MGneg, GLh, _ = O.scale(hm[0], hm[1], hm[3][0], np.float32(mL))
                singles[name]["cpu_baseline"] = ref.rate(
                    MGneg, hm[2], GLh, O.scale_vec(hm[3], np.float32(mL)), iters,
                    shared=True, threads=1, budget_s=1.5, what=singles[name]["config"])
        cpu = None
        if ref is not None:
            cpu = cpu_baseline(n, m, ML, G, L, M, g, mean_iters, ref=ref)
            cpu["qp_solves_per_s"] = cpu["value"] / max(1, int(round(mean_iters)))
        extra = {}
        if not args.no_extra and world == 1:
            extra["hbm_bound_c5"] = hbm_leg(dev, ref=ref)
            extra["distinct_c2_batch"] = distinct_leg(dev, n, m, ref=ref)
            extra["c3_batch4096"] = c3_leg(dev, n, m, ref=ref)
            extra["c4_global_1gpu"] = c4_global_leg(dev, n, m, ref=ref)
            extra["f64_value_c4"] = f64_value_leg(dev, n, m, ref=ref)
            extra["closed_loop_battery"] = closed_loop_leg(dev, cpu=not args.no_cpu)
            extra["closed_loop_battery_flat"] = closed_loop_leg(dev, cpu=False, flat=True)
            extra["flat_battery_c1"] = flat_leg(dev, ref=ref)
            extra["battery_n50"] = flat_leg(dev, horizon=50, N=50, ref=ref)
            extra["flat_tol_c1"] = flat_tol_leg(dev, batch=65536)
            extra["flat_tol_n50"] = flat_tol_leg(dev, horizon=50, tol=1e-3, batch=16384)
        side_value = side["iters_all"] / side["dt"]
        out = {
            "metric": "GPAD iterations/s (instance-iterations, solve to eps=1e-4)",
            "value": value,
            "unit": "GPAD iterations/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": ("synthetic (seeded SURVEY.md §8d generator; shared ML/G, per-instance q/b; "
                     + ("the same q/b every step" if args.repeat_inputs else
                        "FRESH q/b draws every step, resident in HBM before timing") + ")"),
            "config": {"workload": f"C4 shard: {B} instances/GPU, N={args.horizon} (n={n}), m={m}, "
                                   f"shared ML/G, Algorithm 1 eps={args.tol}, K=10",
                       "batch_per_gpu": B, "global_batch": B * world, "n": n, "m": m,
                       "inputs": "repeated" if args.repeat_inputs else "fresh per step",
                       "parallelism": (f"instance-sharded x{world}, "
                                       + ("RCCL gather" if args.dist_backend == "nccl" else "gloo gather")
                                       if world > 1 else "single GPU (no gather)")},
            "qp_solves_per_s": solves,
            "mean_iters_to_eps": mean_iters,
            ("value_fresh_inputs" if args.repeat_inputs else "value_repeated_inputs"): side_value,
            "repeated_inputs_note": "the same q/b every step: the phase plan and the finisher's "
                                    "longest-first queue are built from the previous solve's exact "
                                    "per-instance counts, i.e. perfect foresight",
            "eps_parity": "iteration counts to eps are parity unpinned against the reference (its "
                          "termination test is commented out, acceldualgrad.m:66-79, absent from "
                          "main.cu); bit-exact with the oracle restatement, fp64 max(G z* - g) <= eps "
                          "certified (DESIGN.md section 3)",
            "batching": util,
            "converged": int(head["converged_all"]),
            "multi_gpu": multi,
            "kernel": st["kernel"],
            "single_instance": singles["c2"],
            "single_instance_c1": singles["c1"],
            "roofline": {"bound": "mfma", "achieved": achieved_tf, "peak": FP32_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": achieved_tf / FP32_PEAK_TFLOPS,
                         "traffic": traffic, "traffic_source": traffic_src,
                         "hbm_algorithmic_gbs": hbm_alg_gbs, "hbm_algorithmic_frac": hbm_alg_gbs / HBM_PEAK_GBS,
                         "hbm_note": "SURVEY.md §8d algorithmic bytes, 4 (2nm + B (4m + 3n)) per batch-iteration x "
                                     "mean iterations to eps, per GPU per step time, / 8 TB/s; the shared "
                                     "matrices are L2-resident, so HBM sees far less (traffic)",
                         "kernel_ms": avg_kernel_s * 1e3, "launches_per_solve": launches,
                         "kernel_frac": kernel_frac,
                         "kernel_frac_detail": {
                             "kernel": kname, "panel_instance_iterations": pan_iters,
                             "finisher_instance_iterations": fin_iters, "finisher_takeover": v_take,
                             "panel_ms_per_solve": pan_ms, "source": pan_src,
                             "note": "useful flops on the panel kernel (F per instance-iteration up to the "
                                     "finisher takeover of the last fresh-input solve) / the panel kernel's "
                                     "rocprof time per solve in the committed profile of this command, / "
                                     "the fp32 matrix peak; frac above is the whole step"},
                         "note": "fp32 matrix-core bound (shared matrices stay in L2, traffic = "
                                 "per-instance vectors); achieved = useful flops (F = 4nm+5m+4n "
                                 "per executed instance-iteration) of one solve / its device time "
                                 "(HIP events on the solve stream around the K back-to-back timed "
                                 "steps / K: the solve's chain of phase launches plus the z/y resets "
                                 "and the iteration-count reduction, ~10 us per step; the rocprof "
                                 "per-launch durations of the phase chain agree to that margin); "
                                 "traffic = PMC HBM bytes of the panel kernel per solve (profiled "
                                 "run's total / its solves)"},
            "cpu_baseline": cpu,
            "legs": extra,
        }
        print(json.dumps(out), flush=True)
    if hung:  # a multi-device call never returned: leave without joining it (guarded)
        sys.stderr.flush()
        os._exit(0)
    solver.close()
    if world > 1:
        try:
            dist.barrier(group=host_pg)
            dist.destroy_process_group()
        except Exception as e:  # rank 0 left early (guarded): the results are already printed
            print(f"bench.py rank {rank}: final barrier: {type(e).__name__}: {e}", file=sys.stderr)


if __name__ == "__main__":
    main()
