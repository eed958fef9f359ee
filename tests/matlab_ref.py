"""numpy restatement of Code/MATLAB/acceldualgrad.m (fp64).  TEST INFRASTRUCTURE ONLY.

MATLAB/Octave are not available, so the reference's semantic oracle is restated line by
line here (this container only, to generate and check golden vectors).  The restatement
is a transcription of the algorithm's *behaviour* -- the file itself is not copied.
"""
from __future__ import annotations

import numpy as np


def schedule(N: int, kind: str = "matlab"):
    """acceldualgrad.m:18,27,55-56 (kind='matlab', beta lagged one iteration) or eq. (8e)."""
    th, thm1, b = 1.0, 1.0, 0.0
    theta = np.empty(N)
    beta = np.empty(N)
    for v in range(N):
        thn = (np.sqrt(th ** 4 + 4 * th ** 2) - th ** 2) / 2
        theta[v] = th
        if kind == "paper":
            beta[v] = th * (1.0 / thm1 - 1.0)
        else:
            beta[v] = b
            b = th * (1.0 / thm1 - 1.0)
        thm1, th = th, thn
    return theta, beta


def acceldualgrad(H, f, A_i, b_i, n_u, num_iterations=100, kind="matlab", z_m1=None, y0=None,
                  L=None):
    """[u, z, y] after ``num_iterations`` GPAD iterations, acceldualgrad.m:1-85 order."""
    m = A_i.shape[0]
    n = H.shape[1]
    if L is None:
        L = np.linalg.norm(H, "fro") ** 2                     # :11
    y_v = np.zeros(m) if y0 is None else np.array(y0, float)  # :16
    y_vm1 = y_v.copy()
    z_vm1 = np.zeros(n) if z_m1 is None else np.array(z_m1, float)  # :17
    Hinv = np.linalg.inv(H)
    M_G = Hinv @ A_i.T                                        # :20
    g_P = Hinv @ np.asarray(f).reshape(-1)                    # :21
    G_L = (1.0 / L) * A_i                                     # :22
    p_D = (-1.0 / L) * b_i                                    # :23
    theta, beta = schedule(num_iterations, kind)
    z_v = z_vm1
    for v in range(num_iterations):                           # :39
        w_v = y_v + beta[v] * (y_v - y_vm1)                   # :43 (8a)
        zhat_v = -1 * M_G @ w_v - g_P                         # :46 (8b)
        z_v = (1 - theta[v]) * z_vm1 + theta[v] * zhat_v      # :49 (8c)
        y_vp1 = np.maximum(w_v + G_L @ zhat_v + p_D, 0)       # :52 (8d)
        y_vm1, y_v, z_vm1 = y_v, y_vp1, z_v                   # :60-64
    return z_v[:n_u], z_v, y_v


def acceldualgrad_alg1(H, f, A_i, b_i, L, e_g, e_V, N, check_every=1, kind="matlab"):
    """acceldualgrad.m with its commented termination test (:66-79) switched on, fp64, literally:
    valuefcn/lagrangian/dualtoprimal/dualfcn/g as :30-34, the test tree as :67-78, tested every
    ``check_every`` iterations.  Returns (z, y, iterations, code) with the code of the branch that
    stopped (1: max(g(z)) <= e_g; 2: :71; 3: :73; 4: :76; 0: ran to N) and the point the paper
    returns for it (z for 1, zhat otherwise; the commented MATLAB returns z_v in every branch)."""
    m, n = A_i.shape
    f = np.asarray(f, float).reshape(-1)
    Hinv = np.linalg.inv(H)
    M_G = Hinv @ A_i.T
    g_P = Hinv @ f
    G_L = (1.0 / L) * A_i
    p_D = (-1.0 / L) * b_i
    valuefcn = lambda z: (0.5 * z @ H + f) @ z                                    # noqa: E731  :30
    lagrangian = lambda z, y: (0.5 * z @ H + f + y @ A_i) @ z - y @ b_i           # noqa: E731  :31
    dualtoprimal = lambda y: -1 * Hinv @ (f + A_i.T @ y)                           # noqa: E731  :32
    dualfcn = lambda y: lagrangian(dualtoprimal(y), y)                             # noqa: E731  :33
    g = lambda z: A_i @ z - b_i                                                    # noqa: E731  :34
    theta, beta = schedule(N, kind)
    y_v = np.zeros(m)
    y_vm1 = y_v.copy()
    z_vm1 = np.zeros(n)
    for v in range(N):
        w_v = y_v + beta[v] * (y_v - y_vm1)
        zhat_v = -1 * M_G @ w_v - g_P
        z_v = (1 - theta[v]) * z_vm1 + theta[v] * zhat_v
        y_vp1 = np.maximum(w_v + G_L @ zhat_v + p_D, 0)
        y_vm1, y_v, z_vm1 = y_v, y_vp1, z_v
        if (v + 1) % check_every:
            continue
        if np.all(np.maximum(g(z_v), 0) <= e_g):                                  # :67
            return z_v, y_v, v + 1, 1
        if np.all(np.maximum(g(zhat_v), 0) <= e_g):                               # :69
            if np.all(w_v >= 0):                                                   # :70
                if -1 * w_v @ g(zhat_v) <= e_V:                                    # :71
                    return zhat_v, y_v, v + 1, 2
                if -1 * w_v @ g(zhat_v) <= valuefcn(zhat_v) * e_V / (1 + e_V):    # :73
                    return zhat_v, y_v, v + 1, 3
            elif valuefcn(zhat_v) - dualfcn(y_vp1) <= e_V * max(dualfcn(y_vp1), 1):  # :76
                return zhat_v, y_v, v + 1, 4
    return z_v, y_v, N, 0
