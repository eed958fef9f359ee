"""Randomised parity cases: the HIP path through the C-ABI against the oracle on random shapes,
batch sizes, kernels, modes, test periods, warm starts, schedule options, the multi-device group
API (shards over a repeated device) and repeated solves on one handle (the planner then follows the previous solve's counts).  Bar: z*, y* and per-instance
iteration counts bit-identical to oracle/gpad_oracle.c (which restates seq_functions.cpp:45-87
and acceldualgrad.m's Algorithm 1).

Used by tests/test_fuzz.py (a fixed seed, a few cases per run) and tools/fuzz_parity.py (many
seeds, on the GPU box).  Test infrastructure only: the oracle is the checker here."""
from __future__ import annotations

import numpy as np

SPECIAL = [1, 2, 15, 16, 17, 63, 64, 65, 127, 128, 129, 191, 192, 193, 199, 200, 201, 207, 208, 209, 240, 256]
BATCHES = [1, 2, 3, 15, 16, 17, 31, 33, 100, 257, 1000, 1025, 2049, 4097, 8191]


def draw_case(rng: np.random.Generator) -> dict:
    """One random configuration (plain dict, JSON-printable)."""
    def dim():
        return int(rng.choice(SPECIAL)) if rng.random() < 0.5 else int(rng.integers(1, 261))
    n, m = dim(), dim()
    big = max(n, m) <= 208
    batch = int(rng.choice([b for b in BATCHES if big or b <= 1025]))
    shared = bool(batch == 1 or rng.random() < 0.85 or batch > 64)
    kernels = ["auto", "auto", "panel", "stream"] + (["resident"] if max(n, m) <= 208 else [])
    kernel = str(rng.choice(kernels))
    if kernel == "panel" and not shared:
        kernel = "auto"
    tol_mode = bool(rng.random() < 0.6)
    cfg = dict(n=n, m=m, batch=batch, shared=shared, kernel=kernel, seed=int(rng.integers(1 << 30)),
               warm=bool(rng.random() < 0.3), device=bool(rng.random() < 0.5),
               solves=int(rng.integers(1, 4)), check_every=int(rng.choice([1, 2, 5, 10, 10, 10, 16])))
    if tol_mode:
        cfg.update(N=2000, tol=float(rng.choice([1e-2, 1e-3, 1e-4, 1e-4])))
    else:
        cfg.update(N=int(rng.integers(1, 151)), tol=0.0)
    opts = {}
    if rng.random() < 0.3:
        opts["phase_len"] = int(rng.choice([10, 20, 40, 100]))
    if rng.random() < 0.2:
        opts["finish_thresh"] = int(rng.choice([0, 64, 512, 100000]))
    if rng.random() < 0.15:
        opts["duo_max_grid"] = int(rng.choice([1, 3, 17]))
    if rng.random() < 0.1:
        opts["lpt"] = 0
    cfg["opts"] = opts
    # fp64 (the reference MATLAB precision): shared matrices, the stream kernel or the f64 panels
    cfg["f64"] = bool(shared and rng.random() < 0.2)
    # the multi-device group API over repeated device 0 (peer-copy shards): 2 or 3 shards
    cfg["group"] = int(rng.choice([0, 0, 0, 0, 0, 0, 2, 3])) if batch >= 2 else 0
    # the north-star one-shot gpad_solve (one cached handle per thread, reused across cases: the
    # cache compares contents, shapes and options); one solve, default options
    cfg["oneshot"] = bool(not cfg["group"] and rng.random() < 0.2)
    if cfg["oneshot"]:
        cfg["solves"], cfg["opts"] = 1, {}
    if cfg["f64"] and (kernel == "resident" or (kernel == "panel" and (not tol_mode or max(n, m) > 256))):
        cfg["kernel"] = "auto"
    return cfg


def _problem(cfg: dict):
    """The case's matrices and the q/b of every solve: shared matrices draw batch x solves
    instances at once (fresh q/b per solve on the same plant); per-instance matrices repeat."""
    from gpad_mpc import problems
    B, n, m, S = cfg["batch"], cfg["n"], cfg["m"], cfg["solves"]
    nb = B * S if cfg["shared"] else B
    qp = problems.synthetic_qp(n, m, batch=nb, seed=cfg["seed"], shared=cfg["shared"])
    dt = np.float64 if cfg.get("f64") else np.float32
    f = lambda a: np.ascontiguousarray(np.asarray(a, np.float64).astype(dt))  # noqa: E731
    return f(qp.ML), f(qp.G), f(qp.M).reshape(nb, n), f(qp.g).reshape(nb, m), dt(qp.L)


def run_case(cfg: dict, oracle, sample: int = 24, threads: int = 8) -> dict:
    """Solve cfg["solves"] fresh batches on one handle; check a sample of every batch's instances
    (first, last and random ones) bit for bit -- fp64 cases: counts equal to the fp64 oracle and
    z*, y* within 1e-11 norm-relative (acceldualgrad.m's elementwise order differs from the
    fp32 path's in the last bit).  Returns {"ok": bool, "checked": k, "why": ...}."""
    import torch

    import gpad_mpc
    from gpad_mpc import _lib
    B, n, m = cfg["batch"], cfg["n"], cfg["m"]
    kc = {"auto": _lib.KERNEL_AUTO, "stream": _lib.KERNEL_STREAM, "resident": _lib.KERNEL_RESIDENT,
          "panel": _lib.KERNEL_PANEL}[cfg["kernel"]]
    rng = np.random.default_rng(cfg["seed"])
    dev = torch.device("cuda:0")
    checked, kernels = 0, []
    ML, G, Mall, gall, Lk = _problem(cfg)
    grp = cfg.get("group", 0)
    if cfg.get("oneshot"):
        return _run_oneshot(cfg, oracle, ML, G, Mall, gall, Lk, kc, sample)
    with (gpad_mpc.GpadGroup([0] * grp) if grp else gpad_mpc.GpadSolver(0)) as s:
        put = (lambda a: torch.from_numpy(a).to(dev)) if cfg["device"] else (lambda a: a)  # noqa: E731
        s.setup(put(ML), put(G), float(Lk), n=n, m=m, batch=B, shared=cfg["shared"], kernel=kc,
                check_every=cfg["check_every"])
        if not grp:  # (a group takes its shards' defaults)
            s.set_options(**cfg["opts"])
        for k in range(cfg["solves"]):
            o = k * B if cfg["shared"] else 0
            M, g = np.ascontiguousarray(Mall[o:o + B]), np.ascontiguousarray(gall[o:o + B])
            if cfg["warm"]:
                z0 = rng.uniform(-0.5, 0.5, (B, n)).astype(ML.dtype)
                y0 = np.maximum(rng.normal(0.0, 0.3, (B, m)), 0.0).astype(ML.dtype)
            else:
                z0 = np.zeros((B, n), ML.dtype)
                y0 = np.zeros((B, m), ML.dtype)
            iters = np.zeros(B, np.int32)
            if cfg["device"]:
                zt, yt = torch.from_numpy(z0.copy()).to(dev), torch.from_numpy(y0.copy()).to(dev)
                st = s.run(zt, yt, put(M), put(g), cfg["N"], cfg["tol"], iters=iters)
                z, y = zt.cpu().numpy(), yt.cpu().numpy()
            else:
                z, y = z0.copy(), y0.copy()
                st = s.run(z, y, M, g, cfg["N"], cfg["tol"], iters=iters)
            kernels.append(st.get("kernel", "group") if not grp else f"group{grp}")
            # first, last, random, and the four longest (the finisher's tail) instances
            longest = [int(i) for i in np.argsort(iters)[-4:]] if cfg["tol"] > 0 else []
            pick = sorted(set([0, B - 1] + longest + [int(i) for i in rng.integers(0, B, min(sample, B))]))
            if cfg.get("f64"):
                Zo, Yo, Io = [], [], []
                for b in pick:
                    zo, yo, it, _ = oracle.solve_f64(z0[b], y0[b], ML, M[b], G, g[b], cfg["N"], float(Lk),
                                                     cfg["tol"], cfg["check_every"])
                    Zo.append(zo)
                    Yo.append(yo)
                    Io.append(it)
                Zo, Yo, Io = np.array(Zo), np.array(Yo), np.array(Io)
            elif cfg["shared"]:
                O = oracle
                MGneg, GL, _ = O.scale(ML, G, g[0], Lk)
                PD = O.scale_vec(g[pick], Lk)
                Zo, Yo, Io, _ = O.solve_batch_f32(z0[pick], y0[pick], MGneg, M[pick], GL, PD, cfg["N"], Lk,
                                                  cfg["tol"], cfg["check_every"], shared=True, threads=threads)
            else:
                Zo, Yo, Io = [], [], []
                for b in pick:
                    zo, yo, it, _ = oracle.solve_f32(z0[b], y0[b], ML[b], M[b], G[b], g[b], cfg["N"], Lk,
                                                     cfg["tol"], cfg["check_every"])
                    Zo.append(zo)
                    Yo.append(yo)
                    Io.append(it)
                Zo, Yo, Io = np.array(Zo), np.array(Yo), np.array(Io)
            for j, b in enumerate(pick):
                exp_it = int(Io[j]) if cfg["tol"] > 0 else cfg["N"]
                if cfg["tol"] > 0 and int(iters[b]) != exp_it:
                    return dict(ok=False, checked=checked, kernels=kernels,
                                why=f"solve {k} instance {b}: {int(iters[b])} iterations, oracle {exp_it}")
                for what, a, o in (("z", z[b], Zo[j]), ("y", y[b], Yo[j])):
                    if cfg.get("f64"):
                        e = np.linalg.norm(a - o) / max(np.linalg.norm(o), 1e-300)
                        if e > 1e-11:
                            return dict(ok=False, checked=checked, kernels=kernels,
                                        why=f"solve {k} instance {b} {what}: f64 norm-relative {e:.3g}")
                        continue
                    if not np.array_equal(a, o, equal_nan=True):  # (infeasible draws diverge to NaN in both)
                        d = np.abs(a.astype(np.float64) - o.astype(np.float64))
                        return dict(ok=False, checked=checked, kernels=kernels,
                                    why=f"solve {k} instance {b} {what}: {int((d > 0).sum())} of {a.size} differ, "
                                        f"max {d.max():.3g} (kernel {st['kernel']})")
                checked += 1
            if cfg["tol"] > 0 and st["total_iterations"] != int(iters.sum()):
                return dict(ok=False, checked=checked, kernels=kernels, why="total_iterations != sum of counts")
    return dict(ok=True, checked=checked, kernels=kernels)


def draw_flat_case(rng: np.random.Generator) -> dict:
    """A random flat battery case (gpad_setup_flat; seq_functions.cpp:5-43's data): n_u cells over
    a horizon N (n = n_u N, m = 4 n_u N + 2N), a scenario batch on one plant."""
    n_u = int(rng.choice([1, 2, 3, 4, 4, 5, 8, 16]))
    Nh = int(rng.integers(1, 61 if n_u <= 8 else 13))
    batch = int(rng.choice([1, 2, 5, 16, 17, 49, 100, 257, 1025, 4097]))
    cfg = dict(flat=True, n_u=n_u, Nh=Nh, batch=batch, seed=int(rng.integers(1 << 30)),
               kernel=str(rng.choice(["auto", "auto", "panel", "stream"])), warm=bool(rng.random() < 0.3),
               device=bool(rng.random() < 0.5), solves=int(rng.integers(1, 3)),
               check_every=int(rng.choice([1, 5, 10, 10])))
    if rng.random() < 0.6:
        cfg.update(N=3000, tol=float(rng.choice([1e-3, 1e-4])))
    else:
        cfg.update(N=int(rng.integers(1, 121)), tol=0.0)
    opts = {}
    if rng.random() < 0.3:
        opts["flat_panels"] = int(rng.choice([1, 2, 3, 4]))
    elif rng.random() < 0.15:
        opts["flat_waves"] = 8
    if rng.random() < 0.3:
        opts["phased"] = int(rng.choice([0, 2]))
    if rng.random() < 0.3:
        opts["phase_len"] = int(rng.choice([10, 20, 30]))
    cfg["opts"] = opts
    return cfg


def run_flat_case(cfg: dict, oracle, sample: int = 16) -> dict:
    """Flat battery solves on one handle (fresh initial states per solve) against the oracle's flat
    solve (orc_solve_flat_f32) on a sample of instances: z*, y*, counts bit for bit."""
    import torch

    import gpad_mpc
    from gpad_mpc import _lib, problems
    n_u, Nh, B, S = cfg["n_u"], cfg["Nh"], cfg["batch"], cfg["solves"]
    kc = {"auto": _lib.KERNEL_AUTO, "stream": _lib.KERNEL_STREAM, "panel": _lib.KERNEL_PANEL}[cfg["kernel"]]
    rng = np.random.default_rng(cfg["seed"])
    qp = problems.battery_scenarios(n_u, Nh, B * S, seed=cfg["seed"])
    MGf, GLf, L = problems.flatten_battery(qp, n_u, Nh)
    f32 = lambda a: np.ascontiguousarray(np.asarray(a, np.float64).astype(np.float32))  # noqa: E731
    L32 = np.float32(L)
    MGf32, GLf32 = f32(MGf), f32(GLf)
    GPall = f32(qp.M).reshape(B * S, -1)
    PDall = np.ascontiguousarray(oracle.scale_vec(f32(qp.g).reshape(B * S, -1), L32))
    n, m = GPall.shape[1], PDall.shape[1]
    dev = torch.device("cuda:0")
    put = (lambda a: torch.from_numpy(a).to(dev)) if cfg["device"] else (lambda a: a)  # noqa: E731
    checked, kernels = 0, []
    with gpad_mpc.GpadSolver(0) as s:
        s.setup_flat(put(MGf32), put(GLf32), float(L32), n_u=n_u, batch=B, kernel=kc,
                     check_every=cfg["check_every"])
        s.set_options(**cfg["opts"])
        for k in range(S):
            GP = np.ascontiguousarray(GPall[k * B:(k + 1) * B])
            PD = np.ascontiguousarray(PDall[k * B:(k + 1) * B])
            if cfg["warm"]:
                z0 = rng.uniform(-0.5, 0.5, (B, n)).astype(np.float32)
                y0 = np.maximum(rng.normal(0.0, 0.3, (B, m)), 0.0).astype(np.float32)
            else:
                z0 = np.zeros((B, n), np.float32)
                y0 = np.zeros((B, m), np.float32)
            iters = np.zeros(B, np.int32)
            if cfg["device"]:
                zt, yt = torch.from_numpy(z0.copy()).to(dev), torch.from_numpy(y0.copy()).to(dev)
                st = s.run(zt, yt, put(GP), put(PD), cfg["N"], cfg["tol"], scaled=True, iters=iters)
                z, y = zt.cpu().numpy(), yt.cpu().numpy()
            else:
                z, y = z0.copy(), y0.copy()
                st = s.run(z, y, GP, PD, cfg["N"], cfg["tol"], scaled=True, iters=iters)
            kernels.append(st["kernel"])
            pick = sorted(set([0, B - 1] + [int(i) for i in rng.integers(0, B, min(sample, B))]))
            for b in pick:
                zo, yo, it, _ = oracle.solve_flat_f32(z0[b], y0[b], MGf32, GP[b], GLf32, PD[b], n_u, cfg["N"], L32,
                                                      cfg["tol"], cfg["check_every"])
                exp_it = int(it) if cfg["tol"] > 0 else cfg["N"]
                if cfg["tol"] > 0 and int(iters[b]) != exp_it:
                    return dict(ok=False, checked=checked, kernels=kernels,
                                why=f"flat solve {k} instance {b}: {int(iters[b])} iterations, oracle {exp_it}")
                for what, a, o in (("z", z[b], zo), ("y", y[b], yo)):
                    # Infeasible draws (horizon 1) diverge: once an iterate overflows, the register-resident
                    # flat chains' structural-zero terms (0 * inf = NaN) may turn the
                    # reference's +-inf into NaN -- the non-finite positions must agree, finite values bit-exact.
                    fa, fo = np.isfinite(a), np.isfinite(o)
                    same = np.array_equal(fa, fo) and np.array_equal(a[fa], o[fo])
                    if not same:
                        d = np.abs(a.astype(np.float64) - o.astype(np.float64))
                        return dict(ok=False, checked=checked, kernels=kernels,
                                    why=f"flat solve {k} instance {b} {what}: {int((d > 0).sum())} of {a.size} "
                                        f"differ, max {d.max():.3g} (kernel {st['kernel']})")
                checked += 1
    return dict(ok=True, checked=checked, kernels=kernels)


def draw_value_case(rng: np.random.Generator) -> dict:
    """Algorithm 1 with the value-function branches (gpad_setup_hessian; acceldualgrad.m:73,76):
    the feasible point shifted away from 0 so both branches occur; f32 on the stream kernel, f64 on
    the stream kernel or the f64 panels."""
    f64 = bool(rng.random() < 0.5)
    n = int(rng.choice([1, 2, 8, 16, 17, 20, 40, 64, 65, 100, 129, 200, 208, 256]))
    m = int(rng.choice([1, 3, 16, 33, 40, 64, 100, 127, 200, 256]))
    batch = int(rng.choice([1, 2, 16, 17, 64, 257, 1025, 4097]))
    kernel = str(rng.choice(["auto", "stream"] + (["panel"] if f64 and max(n, m) <= 256 else [])))
    tol = float(rng.choice([1e-2, 1e-3, 1e-4]))
    return dict(value=True, f64=f64, n=n, m=m, batch=batch, kernel=kernel, seed=int(rng.integers(1 << 30)),
                shift=float(rng.choice([0.0, 1.0, 3.0])), tol=tol,
                tol_gap=float(tol * rng.choice([1.0, 10.0])), check_every=int(rng.choice([1, 5, 10])),
                N=int(rng.choice([3000, 20000 if f64 else 5000])), device=bool(rng.random() < 0.5))


def _value_problem(cfg: dict):
    """H = R'R + I, G ~ N(0, 1/n), b = G z_f + U(0.1, 1) with z_f ~ U(shift, shift + 1), q ~ N(0, 0.1),
    shared H, G; per-instance q, b (tests/test_value.py's generator, restated)."""
    n, m, B = cfg["n"], cfg["m"], cfg["batch"]
    rng = np.random.default_rng(cfg["seed"])
    R = rng.normal(0, 1 / np.sqrt(n), (n, n))
    H = R.T @ R + np.eye(n)
    G = rng.normal(0, 1 / np.sqrt(n), (m, n))
    Hi = np.linalg.inv(H)
    ML = Hi @ G.T
    L = float(np.linalg.norm(G @ ML, "fro"))
    zf = rng.uniform(cfg["shift"], cfg["shift"] + 1, (B, n))
    Q = rng.normal(0, 0.1, (B, n))
    g = zf @ G.T + rng.uniform(0.1, 1.0, (B, m))
    dt = np.float64 if cfg["f64"] else np.float32
    c = lambda a: np.ascontiguousarray(np.asarray(a, np.float64).astype(dt))  # noqa: E731
    return c(H), c(ML), c(Q @ Hi.T), c(G), c(g), (float(L) if cfg["f64"] else np.float32(L))


def run_value_case(cfg: dict, oracle, sample: int = 16) -> dict:
    """Counts and termination codes equal to the oracle's value-branch solve on a sample of
    instances; z*, y* bit-identical (f32) or within 1e-11 norm-relative (f64)."""
    import torch

    import gpad_mpc
    from gpad_mpc import _lib
    n, m, B = cfg["n"], cfg["m"], cfg["batch"]
    kc = {"auto": _lib.KERNEL_AUTO, "stream": _lib.KERNEL_STREAM, "panel": _lib.KERNEL_PANEL}[cfg["kernel"]]
    H, ML, M, G, g, L = _value_problem(cfg)
    dev = torch.device("cuda:0")
    put = (lambda a: torch.from_numpy(a).to(dev)) if cfg["device"] else (lambda a: a)  # noqa: E731
    z0 = np.zeros((B, n), ML.dtype)
    y0 = np.zeros((B, m), ML.dtype)
    iters = np.zeros(B, np.int32)
    codes = np.full(B, -1, np.int32)
    with gpad_mpc.GpadSolver(0) as s:
        s.setup(put(ML), put(G), float(L), n=n, m=m, batch=B, kernel=kc, check_every=cfg["check_every"],
                tol_gap=cfg["tol_gap"])
        s.setup_hessian(put(H))
        if cfg["device"]:
            zt, yt = put(z0.copy()), put(y0.copy())
            st = s.run(zt, yt, put(M), put(g), cfg["N"], cfg["tol"], iters=iters, codes=codes)
            z, y = zt.cpu().numpy(), yt.cpu().numpy()
        else:
            z, y = z0.copy(), y0.copy()
            st = s.run(z, y, M, g, cfg["N"], cfg["tol"], iters=iters, codes=codes)
    rng = np.random.default_rng(cfg["seed"] + 1)
    pick = sorted(set([0, B - 1] + [int(i) for i in rng.integers(0, B, min(sample, B))]))
    solve = oracle.solve_value_f64 if cfg["f64"] else oracle.solve_value_f32
    checked = 0
    for b in pick:
        zo, yo, ito, co = solve(z0[b], y0[b], ML, M[b], G, g[b], H, cfg["N"], L, cfg["tol"],
                                check_every=cfg["check_every"], tol_gap=cfg["tol_gap"])
        if (int(iters[b]), int(codes[b])) != (int(ito), int(co)):
            return dict(ok=False, checked=checked, kernels=[st["kernel"]],
                        why=f"instance {b}: (iterations, code) {(int(iters[b]), int(codes[b]))}, oracle {(ito, co)}")
        for what, a, o in (("z", z[b], zo), ("y", y[b], yo)):
            if cfg["f64"]:
                e = np.linalg.norm(a - o) / max(np.linalg.norm(o), 1e-300)
                bad = e > 1e-11
            else:
                bad = not np.array_equal(a, o, equal_nan=True)
            if bad:
                return dict(ok=False, checked=checked, kernels=[st["kernel"]],
                            why=f"instance {b} {what} differs (kernel {st['kernel']})")
        checked += 1
    return dict(ok=True, checked=checked, kernels=[st["kernel"]], codes=sorted(set(int(c) for c in codes)))


def draw_loop_case(rng: np.random.Generator) -> dict:
    """The closed-loop MPC runner (gpad_closed_loop, gpad.m:79-95): a battery plant of n_u cells over
    a horizon N, a batch of packs from random states, several receding-horizon steps."""
    n_u = int(rng.integers(1, 5))
    Nh = int(rng.integers(2, 13))
    tol_mode = bool(rng.random() < 0.5)
    kernels = ["auto", "auto", "panel", "stream"] + (["resident"] if 4 * n_u * Nh + 2 * Nh <= 208 else [])
    return dict(loop=True, n_u=n_u, Nh=Nh, batch=int(rng.choice([1, 3, 17, 64, 300, 1100, 4100])),
                steps=int(rng.integers(1, 11)), N=(2000 if tol_mode else int(rng.integers(1, 121))),
                tol=(float(rng.choice([1e-3, 1e-4])) if tol_mode else 0.0), warm=bool(rng.random() < 0.5),
                kernel=str(rng.choice(kernels)), device=bool(rng.random() < 0.5), seed=int(rng.integers(1 << 30)))


def run_loop_case(cfg: dict, oracle, sample: int = 6) -> dict:
    """Every trajectory value, final state, z*, y* and per-step count of a sample of packs bit for
    bit against the oracle's closed loop (orc_closed_loop_f32)."""
    import torch

    import gpad_mpc
    from gpad_mpc import _lib, problems
    n_u, B, S = cfg["n_u"], cfg["batch"], cfg["steps"]
    qp, pl = problems.battery_plant(n_u, cfg["Nh"])
    f32 = lambda a: np.ascontiguousarray(np.asarray(a, np.float64).astype(np.float32))  # noqa: E731
    kc = {"auto": _lib.KERNEL_AUTO, "stream": _lib.KERNEL_STREAM, "panel": _lib.KERNEL_PANEL,
          "resident": _lib.KERNEL_RESIDENT}[cfg["kernel"]]
    dev = torch.device("cuda:0")
    put = (lambda a: torch.from_numpy(f32(a)).to(dev)) if cfg["device"] else f32  # noqa: E731
    rng = np.random.default_rng(cfg["seed"])
    X0 = (rng.random((B, n_u)) - 0.5).astype(np.float32)
    L = np.float32(qp.L)
    with gpad_mpc.GpadSolver(0) as s:
        s.setup(put(qp.ML), put(qp.G), float(L), n=qp.n, m=qp.m, batch=B, shared=True, kernel=kc)
        s.setup_plant(put(pl.PM), put(pl.Pg), g0=put(pl.g0), A=put(pl.A), B=put(pl.B))
        IT = np.zeros(S * B, np.int32)
        if cfg["device"]:
            X, Z, Y = put(X0), torch.zeros(B, qp.n, device=dev), torch.zeros(B, qp.m, device=dev)
            XS, US = torch.zeros(S, B, n_u, device=dev), torch.zeros(S, B, n_u, device=dev)
            st = s.closed_loop(X, Z, Y, S, cfg["N"], cfg["tol"], warm=cfg["warm"], xs=XS, us=US, iters=IT)
            X, Z, Y, XS, US = (a.cpu().numpy() for a in (X, Z, Y, XS, US))
        else:
            X, Z, Y = X0.copy(), np.zeros((B, qp.n), np.float32), np.zeros((B, qp.m), np.float32)
            XS, US = np.zeros((S, B, n_u), np.float32), np.zeros((S, B, n_u), np.float32)
            st = s.closed_loop(X, Z, Y, S, cfg["N"], cfg["tol"], warm=cfg["warm"], xs=XS, us=US, iters=IT)
    IT = IT.reshape(S, B)
    MGneg, GL, _ = oracle.scale(f32(qp.ML), f32(qp.G), f32(qp.g), L)
    pick = sorted(set([0, B - 1] + [int(i) for i in rng.integers(0, B, min(sample, B))]))
    for b in pick:
        x, z, y, xs, us, its = oracle.closed_loop_f32(X0[b], MGneg, GL, L, pl.PM, pl.Pg, pl.A, pl.B, S, cfg["N"],
                                                      cfg["tol"], g0=pl.g0, warm=cfg["warm"])
        for what, a, o in (("xs", XS[:, b], xs), ("us", US[:, b], us), ("x", X[b], x), ("z", Z[b], z),
                           ("y", Y[b], y), ("iters", IT[:, b], its)):
            if not np.array_equal(a, o, equal_nan=True):
                return dict(ok=False, checked=0, kernels=[st["kernel"]], why=f"pack {b}: {what} differs")
    if st["total_iterations"] != int(IT.sum()):
        return dict(ok=False, checked=0, kernels=[st["kernel"]], why="total_iterations != sum of counts")
    return dict(ok=True, checked=len(pick), kernels=[st["kernel"]])


def _run_oneshot(cfg, oracle, ML, G, M, g, L, kc, sample):
    """gpad_solve(z0, y0, ML, M, G, g, N, L, tol, dims, stats) through ctypes (include/gpad.h), host
    pointers for numpy, device pointers for torch tensors."""
    import ctypes as C

    import torch

    from gpad_mpc import _lib
    lib = _lib.load()
    B, n, m = cfg["batch"], cfg["n"], cfg["m"]
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(cfg["seed"] + 5)
    if cfg["warm"]:
        z0 = rng.uniform(-0.5, 0.5, (B, n)).astype(ML.dtype)
        y0 = np.maximum(rng.normal(0.0, 0.3, (B, m)), 0.0).astype(ML.dtype)
    else:
        z0, y0 = np.zeros((B, n), ML.dtype), np.zeros((B, m), ML.dtype)
    mem = int(cfg["device"])
    # (copies: gpad_solve writes z*, y* over its z0, y0 and the oracle needs the starting point)
    t = (lambda a: torch.from_numpy(np.array(a, copy=True)).to(dev)) if mem else (lambda a: np.array(a, copy=True))  # noqa: E731
    args = [t(a) for a in (z0, y0, ML, M, G, g)]
    ptr = (lambda a: C.c_void_p(a.data_ptr())) if mem else (lambda a: C.c_void_p(a.ctypes.data))  # noqa: E731
    d = _lib.Dims(n=n, m=m, batch=B, shared=int(cfg["shared"]), dtype=int(ML.dtype == np.float64), memory=mem,
                  schedule=_lib.SCHEDULE_MATLAB, check_every=cfg["check_every"], kernel=kc)
    st = _lib.Stats()
    iters = np.zeros(B, np.int32)
    st.iters = iters.ctypes.data_as(C.POINTER(C.c_int))
    _lib.check(lib.gpad_solve(*[ptr(a) for a in args], int(cfg["N"]), float(L), float(cfg["tol"]), C.byref(d),
                              C.byref(st)), "gpad_solve")
    z, y = (a.cpu().numpy() if mem else a for a in args[:2])
    pick = sorted(set([0, B - 1] + [int(i) for i in rng.integers(0, B, min(sample, B))]))
    for b in pick:
        if cfg.get("f64"):
            zo, yo, it, _ = oracle.solve_f64(z0[b], y0[b], ML, M[b], G, g[b], cfg["N"], float(L), cfg["tol"],
                                             cfg["check_every"])
        else:
            ml, gg = (ML, G) if cfg["shared"] else (ML[b], G[b])
            zo, yo, it, _ = oracle.solve_f32(z0[b], y0[b], ml, M[b], gg, g[b], cfg["N"], L, cfg["tol"],
                                             cfg["check_every"])
        if cfg["tol"] > 0 and int(iters[b]) != int(it):
            return dict(ok=False, checked=0, kernels=["oneshot"], why=f"gpad_solve instance {b}: count {iters[b]} vs {it}")
        for what, a, o in (("z", z[b], zo), ("y", y[b], yo)):
            if cfg.get("f64"):
                bad = np.linalg.norm(a - o) / max(np.linalg.norm(o), 1e-300) > 1e-11
            else:
                bad = not np.array_equal(a, o, equal_nan=True)
            if bad:
                return dict(ok=False, checked=0, kernels=["oneshot"], why=f"gpad_solve instance {b} {what} differs")
    return dict(ok=True, checked=len(pick), kernels=["oneshot"])


def draw_heavy_case(rng: np.random.Generator) -> dict:
    """C3 / C4-shaped phased solves (shared 200 x 200-ish matrices, thousands of instances to eps, the
    planner over 2-3 fresh solves, the duo finisher's tail) with random schedule options."""
    n = int(rng.choice([200, 200, int(rng.integers(150, 209))]))
    m = int(rng.choice([200, 200, int(rng.integers(150, 209))]))
    opts = {}
    for name, choices, p in (("phase_len", [10, 20, 40, 60], 0.3), ("finish_thresh", [0, 256, 512, 2048], 0.3),
                             ("duo_max_grid", [1, 7, 64, 255], 0.2), ("panel_max_grid", [1, 3, 64, 200], 0.2),
                             ("lpt", [0], 0.15), ("plan", [0], 0.15), ("phased", [0], 0.1)):
        if rng.random() < p:
            opts[name] = int(rng.choice(choices))
    return dict(n=n, m=m, batch=int(rng.choice([4096, 4100, 8192, 8197, 12000, 16384])), shared=True,
                kernel=str(rng.choice(["auto", "auto", "panel"])), seed=int(rng.integers(1 << 30)),
                warm=bool(rng.random() < 0.2), device=bool(rng.random() < 0.7), solves=int(rng.integers(2, 4)),
                check_every=int(rng.choice([10, 10, 5, 20])), N=5000, tol=float(rng.choice([1e-4, 1e-4, 1e-3])),
                opts=opts, f64=False, group=0, oneshot=False, heavy=True)


def run_steps_case(seed: int, oracle) -> dict:
    """The per-step entry points (gpad_step1..4, the kernel_functions.h mirror) on random sizes and
    values against the oracle's steps 8a-8d (seq_functions.cpp:45-87), bit for bit."""
    import torch

    import gpad_mpc
    rng = np.random.default_rng(seed)
    n = int(rng.choice(SPECIAL + [300, 511, 512, 513, 1000, 1500]))
    m = int(rng.choice(SPECIAL + [300, 511, 512, 513, 1000, 1500]))
    dev = torch.device("cuda:0")
    f = lambda *s: rng.normal(0, 1, s).astype(np.float32)  # noqa: E731
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    MGneg, GL, gP, pD = f(n, m), f(m, n), f(n), f(m)
    y, ym1, zm1 = np.maximum(f(m), 0), np.maximum(f(m), 0), f(n)
    beta, theta = float(np.float32(rng.uniform(0, 1))), float(np.float32(rng.uniform(0, 1)))
    w, zh, z, yp = (torch.empty(m, device=dev), torch.empty(n, device=dev), torch.empty(n, device=dev),
                    torch.empty(m, device=dev))
    with gpad_mpc.GpadSolver(0) as s:
        s.step1(t(y), t(ym1), w, beta)
        s.step2(t(MGneg), w, t(gP), zh)
        s.step3(theta, t(zm1), zh, z)
        s.step4(t(GL), yp, w, t(pD), zh)
        s.sync()
    wo = oracle.step1(y, ym1, np.float32(beta))
    zho = oracle.step2(MGneg, wo, gP)
    zo = oracle.step3(np.float32(theta), zm1, zho)
    ypo = oracle.step4(GL, wo, pD, zho)
    for what, a, o in (("8a", w, wo), ("8b", zh, zho), ("8c", z, zo), ("8d", yp, ypo)):
        if not np.array_equal(a.cpu().numpy(), o):
            return dict(ok=False, checked=0, kernels=["steps"], why=f"step {what} differs at n={n} m={m}")
    return dict(ok=True, checked=1, kernels=["steps"])
