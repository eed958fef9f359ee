"""Problem construction for the GPAD path (row a8 of SURVEY.md §8a; off the per-iteration path).

Two families:

* ``battery_mpc`` -- the reference's battery-balancing MPC, a line-by-line
  restatement of ``Code/MATLAB/gpad.m:4-85`` (model, condensed Hessian, constraint
  stack) followed by the precompute of ``Code/MATLAB/acceldualgrad.m:11,20-23``.
* ``synthetic_qp`` -- the seeded generic generator of SURVEY.md §8d used for the
  C2..C5 shapes (strictly feasible by construction, L = ||G M^-1 G'||_F).

Everything returned is the north-star ``solve(z0, y0, ML, M, G, g, N, L, tol)`` input
set: ``ML = H^-1 G'`` (n x m), ``M = H^-1 q`` (n; the "M.g" product), ``G`` (m x n),
``g`` (m), ``L``.  Arrays are float64; callers cast to float32 for the fp32 path.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np


@dataclass
class QP:
    """Condensed MPC QP in GPAD form:  min 1/2 z'Hz + q'z  s.t.  G z <= g."""

    ML: np.ndarray  # n x m, H^-1 G'
    M: np.ndarray  # n or (batch, n), H^-1 q
    G: np.ndarray  # m x n
    g: np.ndarray  # m or (batch, m)
    L: float
    H: np.ndarray | None = None
    q: np.ndarray | None = None
    meta: dict = field(default_factory=dict)

    @property
    def n(self) -> int:
        return self.ML.shape[-2]

    @property
    def m(self) -> int:
        return self.ML.shape[-1]


def battery_matrices(n_u: int, N: int, capacity_ah: float = 0.027 * 4.1, qx: float = 100.0,
                     qu: float = 1.0):
    """gpad.m:18-77 -- A, B, M_ak, M_ab, K, H, F for ``n_u`` cells over horizon ``N``."""
    n, p = n_u, N
    cap = np.full(n, capacity_ah)
    A = np.eye(n)
    B = np.diag(-1.0 / (3600.0 * cap))                                   # gpad.m:38-41
    M_ak = np.zeros((n * p, n))
    for i in range(1, p + 1):                                            # gpad.m:42-44
        M_ak[(i - 1) * n:i * n, :] = np.linalg.matrix_power(A, i)
    M_ab = np.zeros((n * p, n * p))
    for i in range(1, p + 1):                                            # gpad.m:47-55
        for j in range(1, p + 1):
            if j <= i:
                M_ab[(i - 1) * n:i * n, (j - 1) * n:j * n] = np.linalg.matrix_power(A, i - j) @ B
    K = np.zeros((p, n * p))
    for i in range(1, p + 1):                                            # gpad.m:57-65
        for j in range(1, n * p + 1):
            if (j - 1) // n + 1 == i:
                K[i - 1, j - 1] = 1.0
    Mx = qx * np.eye(n * p)
    Mu = qu * np.eye(n * p)
    H = M_ab.T @ Mx @ M_ab + Mu                                          # gpad.m:68
    F = M_ak.T @ Mx @ M_ab                                               # gpad.m:69
    return dict(A=A, B=B, M_ak=M_ak, M_ab=M_ab, K=K, H=H, F=F)


def battery_constraints(mats: dict, x0: np.ndarray, n_u: int, N: int, xmax: float = 0.5,
                        xmin: float = -0.5, umax: float = 0.3, umin: float = -0.3):
    """gpad.m:73-85 -- f = x0'F, A_i, b_i for the state x0 (m = 4 n_u N + 2 N rows)."""
    n, p = n_u, N
    M_ab, M_ak, K = mats["M_ab"], mats["M_ak"], mats["K"]
    f = x0 @ mats["F"]
    A_i = np.vstack([M_ab, -M_ab, np.eye(n * p), -np.eye(n * p), K, -K])
    b_i = np.concatenate([
        np.full(n * p, xmax) - M_ak @ x0,
        -np.full(n * p, xmin) + M_ak @ x0,
        np.full(n * p, umax),
        -np.full(n * p, umin),
        np.zeros(p),
        np.zeros(p),
    ])
    return f, A_i, b_i


def gpad_precompute(H: np.ndarray, f: np.ndarray, A_i: np.ndarray, b_i: np.ndarray,
                    L: float | None = None) -> QP:
    """acceldualgrad.m:11,20-23: L = ||H||_F^2 (reference choice), M_G = inv(H) A',
    g_P = inv(H) f'.  Returns the unscaled solve() inputs (G = A_i, g = b_i)."""
    Hinv = np.linalg.inv(H)
    if L is None:
        L = float(np.linalg.norm(H, "fro") ** 2)                         # acceldualgrad.m:11
    return QP(ML=Hinv @ A_i.T, M=Hinv @ np.asarray(f).reshape(-1), G=A_i.copy(),
              g=np.asarray(b_i, dtype=np.float64).copy(), L=float(L), H=H,
              q=np.asarray(f).reshape(-1).copy())


def battery_x0(n_u: int, seed: int = 0) -> np.ndarray:
    """gpad.m:9-15: fixed states for 10 and 5 cells, otherwise U(-0.5, 0.5) (seeded here)."""
    if n_u == 10:
        return np.array([-0.1, 0.45, -0.09, 0.05, 0, -0.05, 0.3, 0.2, 0.25, -0.45], dtype=np.float64)
    if n_u == 5:
        return np.array([-0.1, 0.05, 0, -0.05, 0.1], dtype=np.float64)
    return np.random.default_rng(seed).random(n_u) - 0.5


def battery_mpc(n_u: int = 4, N: int = 10, x0: np.ndarray | None = None, seed: int = 0) -> QP:
    """Config C1 (n_u = 4, N = 10 -> n = 40, m = 180) and friends."""
    if x0 is None:
        x0 = battery_x0(n_u, seed)
    mats = battery_matrices(n_u, N)
    f, A_i, b_i = battery_constraints(mats, x0, n_u, N)
    qp = gpad_precompute(mats["H"], f, A_i, b_i)
    qp.meta = dict(kind="battery", n_u=n_u, N=N, x0=np.asarray(x0, dtype=np.float64), B=mats["B"])
    return qp


def battery_scenarios(n_u: int, N: int, batch: int, seed: int = 0) -> QP:
    """A battery-balancing scenario batch: one plant (shared ML, G, L) and ``batch`` initial
    states of charge x0 ~ U(-0.45, 0.45) -> per-instance M = H^-1 F'x0 and g = b_i(x0)."""
    mats = battery_matrices(n_u, N)
    rng = np.random.default_rng(seed)
    X0 = rng.uniform(-0.45, 0.45, size=(batch, n_u))
    f0, A_i, b0 = battery_constraints(mats, X0[0], n_u, N)
    qp = gpad_precompute(mats["H"], f0, A_i, b0)
    Hinv = np.linalg.inv(mats["H"])
    F = mats["F"]
    M = (X0 @ F) @ Hinv.T
    g = np.stack([battery_constraints(mats, x, n_u, N)[2] for x in X0])
    return QP(ML=qp.ML, M=M, G=qp.G, g=g, L=qp.L, H=mats["H"], q=X0 @ F,
              meta=dict(kind="battery_batch", n_u=n_u, N=N, X0=X0))


@dataclass
class Plant:
    """Affine state dependence of the MPC QP and the plant model (gpad_setup_plant):
    M(x) = M0 + PM x, g(x) = g0 + Pg x, x+ = A x + B u with u = z*[0:nu]."""

    PM: np.ndarray  # n x nx
    Pg: np.ndarray  # m x nx
    A: np.ndarray   # nx x nx
    B: np.ndarray   # nx x nu
    M0: np.ndarray | None = None  # n
    g0: np.ndarray | None = None  # m

    @property
    def nx(self) -> int:
        return self.PM.shape[1]

    @property
    def nu(self) -> int:
        return self.B.shape[1]


def battery_plant(n_u: int = 4, N: int = 10, xmax: float = 0.5, xmin: float = -0.5,
                  umax: float = 0.3, umin: float = -0.3):
    """The battery-balancing MPC of gpad.m as (QP, Plant): the constant ML, G, L of the QP
    and the affine maps of gpad.m:81-85 -- f = x0'F so M(x) = H^-1 F' x (M0 = 0);
    b_i(x) = [xmax - M_ak x; -xmin + M_ak x; umax; -umin; 0; 0] -- plus x+ = A x + B u
    (gpad.m:93).  Everything float64."""
    mats = battery_matrices(n_u, N)
    x0 = np.zeros(n_u)
    f0, A_i, b0 = battery_constraints(mats, x0, n_u, N, xmax, xmin, umax, umin)
    qp = gpad_precompute(mats["H"], f0, A_i, b0)
    Hinv = np.linalg.inv(mats["H"])
    PM = Hinv @ mats["F"].T
    M_ak = mats["M_ak"]
    z = np.zeros_like(M_ak)
    Pg = np.vstack([-M_ak, M_ak, z, z, np.zeros((N, n_u)), np.zeros((N, n_u))])
    plant = Plant(PM=PM, Pg=Pg, A=mats["A"], B=mats["B"], M0=None, g0=b0)
    qp.meta = dict(kind="battery_plant", n_u=n_u, N=N)
    return qp, plant


def flatten_battery(qp: QP, n_u: int, N: int, L: float | None = None):
    """The reference's "flat" battery data (ENABLE_FLATTEN_MATRICES; seq_functions.cpp:5-43) from
    the full problem, valid for equal cell capacities: with H = kron(Hs, I_{n_u}), column k of
    the first 4 n_u N constraints touches only cell k % n_u, and the 2N coupling rows touch all
    cells equally.  Returns float64 (MGf (N x m) = flat -ML, GLf (m x N) = flat G/L, L);
    M, g stay as in ``qp`` (g_P = M, p_D = -g/L)."""
    L = float(qp.L if L is None else L)
    n, m = qp.n, qp.m
    mc = 4 * n_u * N
    assert n == n_u * N and m >= mc
    ML, G = np.asarray(qp.ML, np.float64), np.asarray(qp.G, np.float64)
    MGf = np.empty((N, m))
    GLf = np.empty((m, N))
    for i in range(N):
        for k in range(m):
            MGf[i, k] = -ML[i * n_u + (k % n_u if k < mc else 0), k]
    for r in range(m):
        for t in range(N):
            GLf[r, t] = G[r, t * n_u + (r % n_u if r < mc else 0)] / L
    return MGf, GLf, L


def synthetic_qp(n: int, m: int, batch: int = 1, seed: int = 0, shared: bool = True) -> QP:
    """SURVEY.md §8d generic generator: M = R'R + I with R ~ N(0, 1/n); G ~ N(0, 1/n);
    b = G z_f + U(0.1, 1) with z_f ~ U(-0.5, 0.5) (strictly feasible); q ~ N(0, 1);
    L = ||G M^-1 G'||_F (a valid dual Lipschitz bound).  With ``shared`` the Hessian and G
    come from ``seed`` and only q, b vary per instance (seeds seed+1 ...); otherwise every
    instance draws its own matrices and ML/G are returned stacked (batch, n, m)/(batch, m, n)."""

    def one(rng):
        R = rng.normal(0.0, 1.0 / np.sqrt(n), size=(n, n))
        H = R.T @ R + np.eye(n)
        G = rng.normal(0.0, 1.0 / np.sqrt(n), size=(m, n))
        return H, G

    def rhs(rng, G):
        zf = rng.uniform(-0.5, 0.5, size=n)
        b = G @ zf + rng.uniform(0.1, 1.0, size=m)
        q = rng.normal(0.0, 1.0, size=n)
        return q, b

    if shared:
        H, G = one(np.random.default_rng(seed))
        Hinv = np.linalg.inv(H)
        ML = Hinv @ G.T
        L = float(np.linalg.norm(G @ ML, "fro"))
        qs, bs = [], []
        for b in range(batch):
            q, bb = rhs(np.random.default_rng(seed + 1 + b), G)
            qs.append(q)
            bs.append(bb)
        Q = np.stack(qs)
        Bm = np.stack(bs)
        M = Q @ Hinv.T
        if batch == 1:
            return QP(ML=ML, M=M[0], G=G, g=Bm[0], L=L, H=H, q=Q[0],
                      meta=dict(kind="synthetic", seed=seed))
        return QP(ML=ML, M=M, G=G, g=Bm, L=L, H=H, q=Q,
                  meta=dict(kind="synthetic_shared", seed=seed))
    MLs, Ms, Gs, gs, Ls = [], [], [], [], []
    for b in range(batch):
        rng = np.random.default_rng(seed + b)
        H, G = one(rng)
        q, bb = rhs(rng, G)
        Hinv = np.linalg.inv(H)
        ML = Hinv @ G.T
        MLs.append(ML)
        Ms.append(Hinv @ q)
        Gs.append(G)
        gs.append(bb)
        Ls.append(float(np.linalg.norm(G @ ML, "fro")))
    # one L for the whole batch (the C-ABI takes a scalar L): the max is valid for every member
    return QP(ML=np.stack(MLs), M=np.stack(Ms), G=np.stack(Gs), g=np.stack(gs), L=max(Ls),
              meta=dict(kind="synthetic_distinct", seed=seed))
