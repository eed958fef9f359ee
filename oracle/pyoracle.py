"""ctypes front-end for the CPU ORACLE (TEST INFRASTRUCTURE ONLY).

Loads ``oracle/liboracle.so`` (our C restatement, gpad_oracle.c) and, where it was built,
``oracle/_ref/libref_seq.so`` (the reference's own seq_functions.cpp compiled in place by
``make -C oracle ref``).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg import this module -- it is the checker, never the product path.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")
REF = os.path.join(HERE, "_ref", "libref_seq.so")
REF_O3 = os.path.join(HERE, "_ref", "libref_seq_o3.so")

_f = C.POINTER(C.c_float)
_d = C.POINTER(C.c_double)
_i = C.POINTER(C.c_int)

SCHEDULE_MATLAB = 0
SCHEDULE_PAPER = 1


def build(ref: bool | None = None) -> None:
    """Compile liboracle.so (and _ref/ when the reference tree is present)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    if ref is None:
        ref = os.path.isdir("/root/reference")
    if ref:
        subprocess.run(["make", "-s", "-C", HERE, "ref"], check=True)


def _fp(a):
    return a.ctypes.data_as(_f)


def _dp(a):
    return a.ctypes.data_as(_d)


class Oracle:
    def __init__(self, path: str = LIB):
        if not os.path.exists(path):
            build(ref=False)
        L = C.CDLL(path)
        L.orc_step1_f32.argtypes = [_f, _f, _f, C.c_float, C.c_int]
        L.orc_step2_f32.argtypes = [_f, _f, _f, _f, C.c_int, C.c_int]
        L.orc_step3_f32.argtypes = [C.c_float, C.c_int, _f, _f, _f]
        L.orc_step4_f32.argtypes = [_f, _f, _f, _f, _f, C.c_int, C.c_int]
        L.orc_scale_f32.argtypes = [_f, _f, _f, C.c_float, C.c_int, C.c_int, _f, _f, _f]
        L.orc_schedule.argtypes = [C.c_int, C.c_int, _d, _d]
        L.orc_solve_f32.argtypes = [_f, _f, _f, _f, _f, _f, C.c_int, C.c_int, C.c_int, C.c_float,
                                    C.c_double, C.c_double, C.c_int, _f, _f, _i]
        L.orc_solve_f32.restype = C.c_int
        L.orc_solve_f64.argtypes = [_d, _d, _d, _d, _d, _d, C.c_int, C.c_int, C.c_int, C.c_double,
                                    C.c_double, C.c_double, C.c_int, C.c_int, _i]
        L.orc_solve_f64.restype = C.c_int
        L.orc_solve_value_f32.argtypes = [_f, _f, _f, _f, _f, _f, _f, C.c_int, C.c_int, C.c_int, C.c_float,
                                          C.c_double, C.c_double, C.c_int, _f, _f, C.POINTER(C.c_int)]
        L.orc_solve_value_f32.restype = C.c_int
        L.orc_solve_value_f64.argtypes = [_d, _d, _d, _d, _d, _d, _d, C.c_int, C.c_int, C.c_int, C.c_double,
                                          C.c_double, C.c_double, C.c_int, C.c_int, C.POINTER(C.c_int)]
        L.orc_solve_value_f64.restype = C.c_int
        L.orc_solve_batch_f32.argtypes = [_f, _f, _f, _f, _f, _f, C.c_int, C.c_int, C.c_int, C.c_int,
                                          C.c_int, C.c_float, C.c_double, C.c_double, C.c_int, _f, _f, _i,
                                          C.c_int]
        L.orc_solve_batch_f32.restype = C.c_longlong
        L.orc_affine_f32.argtypes = [_f, _f, _f, _f, C.c_int, C.c_int]
        L.orc_plant_step_f32.argtypes = [_f, _f, _f, _f, _f, C.c_int, C.c_int]
        L.orc_closed_loop_f32.argtypes = [_f, _f, _f, _f, _f, C.c_float, C.c_int, C.c_int, _f, _f, _f,
                                          _f, _f, _f, C.c_int, C.c_int, C.c_int, C.c_int, C.c_double,
                                          C.c_double, C.c_int, _f, _f, C.c_int, _f, _f, _i]
        L.orc_closed_loop_f32.restype = C.c_longlong
        L.orc_step2_flat_f32.argtypes = [_f, _f, _f, _f, C.c_int, C.c_int, C.c_int]
        L.orc_step4_flat_f32.argtypes = [_f, _f, _f, _f, _f, C.c_int, C.c_int, C.c_int]
        L.orc_solve_flat_f32.argtypes = [_f, _f, _f, _f, _f, _f, C.c_int, C.c_int, C.c_int, C.c_int,
                                         C.c_float, C.c_double, C.c_double, C.c_int, _f, _f, _i]
        L.orc_solve_flat_f32.restype = C.c_int
        self.lib = L

    # -- steps ------------------------------------------------------------------
    def step1(self, y, ym1, beta):
        y = np.ascontiguousarray(y, np.float32); ym1 = np.ascontiguousarray(ym1, np.float32)
        w = np.empty_like(y)
        self.lib.orc_step1_f32(_fp(y), _fp(ym1), _fp(w), beta, y.size)
        return w

    def step2(self, MGneg, w, gP):
        MGneg = np.ascontiguousarray(MGneg, np.float32); n, m = MGneg.shape
        w = np.ascontiguousarray(w, np.float32); gP = np.ascontiguousarray(gP, np.float32)
        zh = np.empty(n, np.float32)
        self.lib.orc_step2_f32(_fp(MGneg), _fp(w), _fp(gP), _fp(zh), n, m)
        return zh

    def step3(self, theta, zm1, zhat):
        zm1 = np.ascontiguousarray(zm1, np.float32); zhat = np.ascontiguousarray(zhat, np.float32)
        z = np.empty_like(zm1)
        self.lib.orc_step3_f32(theta, zm1.size, _fp(zm1), _fp(zhat), _fp(z))
        return z

    def step4(self, GL, w, pD, zhat):
        GL = np.ascontiguousarray(GL, np.float32); m, n = GL.shape
        w = np.ascontiguousarray(w, np.float32); pD = np.ascontiguousarray(pD, np.float32)
        zhat = np.ascontiguousarray(zhat, np.float32)
        y = np.empty(m, np.float32)
        self.lib.orc_step4_f32(_fp(GL), _fp(y), _fp(w), _fp(pD), _fp(zhat), n, m)
        return y

    # -- inputs -----------------------------------------------------------------
    def scale(self, ML, G, g, L):
        ML = np.ascontiguousarray(ML, np.float32); n, m = ML.shape
        G = np.ascontiguousarray(G, np.float32); g = np.ascontiguousarray(g, np.float32)
        MGneg = np.empty((n, m), np.float32); GL = np.empty((m, n), np.float32)
        pD = np.empty(m, np.float32)
        self.lib.orc_scale_f32(_fp(ML), _fp(G), _fp(g), np.float32(L), n, m, _fp(MGneg), _fp(GL),
                               _fp(pD))
        return MGneg, GL, pD

    def scale_vec(self, g, L):
        """pD = fl32((-1/L)_64 * g) for a (batch, m) array."""
        g = np.asarray(g, np.float32)
        return ((-1.0 / np.float64(np.float32(L))) * g.astype(np.float64)).astype(np.float32)

    def schedule(self, N, kind=SCHEDULE_MATLAB):
        th = np.empty(N, np.float64); be = np.empty(N, np.float64)
        self.lib.orc_schedule(N, kind, _dp(th), _dp(be))
        return th, be

    def schedule_f32(self, N, kind=SCHEDULE_MATLAB):
        th, be = self.schedule(N, kind)
        return th.astype(np.float32), be.astype(np.float32)

    # -- solves -----------------------------------------------------------------
    def solve_f32(self, z0, y0, ML, M, G, g, N, L, tol=0.0, check_every=10,
                  schedule=SCHEDULE_MATLAB, tol_gap=0.0):
        """solve(z0, y0, ML, M, G, g, N, L, tol) restated on the CPU in fp32 (tol = e_g,
        tol_gap = e_V; <= 0: = tol)."""
        MGneg, GL, pD = self.scale(ML, G, g, L)
        return self.solve_scaled_f32(z0, y0, MGneg, M, GL, pD, N, L, tol, check_every, schedule,
                                     tol_gap=tol_gap)

    def solve_scaled_f32(self, z0, y0, MGneg, gP, GL, pD, N, L, tol=0.0, check_every=10,
                         schedule=SCHEDULE_MATLAB, theta=None, beta=None, tol_gap=0.0):
        n, m = MGneg.shape
        z = np.array(z0, np.float32, copy=True).reshape(n)
        y = np.array(y0, np.float32, copy=True).reshape(m)
        if theta is None:
            theta, beta = self.schedule_f32(max(N, 1), schedule)
        theta = np.ascontiguousarray(theta, np.float32); beta = np.ascontiguousarray(beta, np.float32)
        conv = C.c_int(0)
        it = self.lib.orc_solve_f32(_fp(z), _fp(y), _fp(np.ascontiguousarray(MGneg, np.float32)),
                                    _fp(np.ascontiguousarray(gP, np.float32)),
                                    _fp(np.ascontiguousarray(GL, np.float32)),
                                    _fp(np.ascontiguousarray(pD, np.float32)), n, m, N,
                                    np.float32(L), float(tol), float(tol_gap), check_every, _fp(theta),
                                    _fp(beta), C.byref(conv))
        return z, y, it, bool(conv.value)

    def solve_f64(self, z0, y0, ML, M, G, g, N, L, tol=0.0, check_every=10,
                  schedule=SCHEDULE_MATLAB, tol_gap=0.0):
        ML = np.ascontiguousarray(ML, np.float64); n, m = ML.shape
        z = np.array(z0, np.float64, copy=True).reshape(n)
        y = np.array(y0, np.float64, copy=True).reshape(m)
        conv = C.c_int(0)
        it = self.lib.orc_solve_f64(_dp(z), _dp(y), _dp(ML), _dp(np.ascontiguousarray(M, np.float64)),
                                    _dp(np.ascontiguousarray(G, np.float64)),
                                    _dp(np.ascontiguousarray(g, np.float64)), n, m, N, float(L),
                                    float(tol), float(tol_gap), check_every, schedule, C.byref(conv))
        return z, y, it, bool(conv.value)

    # -- Algorithm 1 with the value-function branches (acceldualgrad.m:73,76; f = H M) -------
    def solve_value_f32(self, z0, y0, ML, M, G, g, H, N, L, tol=0.0, check_every=10,
                        schedule=SCHEDULE_MATLAB, tol_gap=0.0):
        """solve_f32 with the QP Hessian H bound: returns (z, y, iterations, code), code 0..4."""
        MGneg, GL, pD = self.scale(ML, G, g, L)
        n, m = MGneg.shape
        z = np.array(z0, np.float32, copy=True).reshape(n)
        y = np.array(y0, np.float32, copy=True).reshape(m)
        theta, beta = self.schedule_f32(max(N, 1), schedule)
        conv = C.c_int(0)
        it = self.lib.orc_solve_value_f32(_fp(z), _fp(y), _fp(MGneg), _fp(np.ascontiguousarray(M, np.float32).reshape(n)),
                                          _fp(GL), _fp(pD), _fp(np.ascontiguousarray(H, np.float32)), n, m, N,
                                          np.float32(L), float(tol), float(tol_gap), check_every, _fp(theta),
                                          _fp(beta), C.byref(conv))
        return z, y, it, conv.value

    def solve_value_f64(self, z0, y0, ML, M, G, g, H, N, L, tol=0.0, check_every=10,
                        schedule=SCHEDULE_MATLAB, tol_gap=0.0):
        ML = np.ascontiguousarray(ML, np.float64); n, m = ML.shape
        z = np.array(z0, np.float64, copy=True).reshape(n)
        y = np.array(y0, np.float64, copy=True).reshape(m)
        conv = C.c_int(0)
        it = self.lib.orc_solve_value_f64(_dp(z), _dp(y), _dp(ML), _dp(np.ascontiguousarray(M, np.float64)),
                                          _dp(np.ascontiguousarray(G, np.float64)),
                                          _dp(np.ascontiguousarray(g, np.float64)),
                                          _dp(np.ascontiguousarray(H, np.float64)), n, m, N, float(L),
                                          float(tol), float(tol_gap), check_every, schedule, C.byref(conv))
        return z, y, it, conv.value

    def solve_batch_f32(self, Z0, Y0, MGneg, GP, GL, PD, N, L, tol=0.0, check_every=10,
                        shared=True, threads=1, schedule=SCHEDULE_MATLAB, tol_gap=0.0):
        """Batch of instances; per-instance vectors packed [batch][n] / [batch][m]."""
        Z = np.array(Z0, np.float32, copy=True); Y = np.array(Y0, np.float32, copy=True)
        batch, n = Z.shape
        m = Y.shape[1]
        theta, beta = self.schedule_f32(max(N, 1), schedule)
        iters = np.zeros(batch, np.int32)
        total = self.lib.orc_solve_batch_f32(
            _fp(Z), _fp(Y), _fp(np.ascontiguousarray(MGneg, np.float32)),
            _fp(np.ascontiguousarray(GP, np.float32)), _fp(np.ascontiguousarray(GL, np.float32)),
            _fp(np.ascontiguousarray(PD, np.float32)), n, m, batch, int(bool(shared)), N,
            np.float32(L), float(tol), float(tol_gap), check_every, _fp(theta), _fp(beta),
            iters.ctypes.data_as(_i), threads)
        return Z, Y, iters, int(total)


    # -- flat battery steps (seq_functions.cpp:5-43) ------------------------------
    def step2_flat(self, MGf, w, gP, n_u):
        MGf = np.ascontiguousarray(MGf, np.float32); Nh, m = MGf.shape
        zh = np.empty(Nh * n_u, np.float32)
        self.lib.orc_step2_flat_f32(_fp(MGf), _fp(np.ascontiguousarray(w, np.float32)),
                                    _fp(np.ascontiguousarray(gP, np.float32)), _fp(zh), Nh, n_u, m)
        return zh

    def step4_flat(self, GLf, w, pD, zhat, n_u):
        GLf = np.ascontiguousarray(GLf, np.float32); m, Nh = GLf.shape
        yp = np.empty(m, np.float32)
        self.lib.orc_step4_flat_f32(_fp(GLf), _fp(yp), _fp(np.ascontiguousarray(w, np.float32)),
                                    _fp(np.ascontiguousarray(pD, np.float32)),
                                    _fp(np.ascontiguousarray(zhat, np.float32)), Nh, n_u, m)
        return yp

    def solve_flat_f32(self, z0, y0, MGf, gP, GLf, pD, n_u, N, L, tol=0.0, check_every=10,
                       schedule=SCHEDULE_MATLAB, theta=None, beta=None, tol_gap=0.0):
        MGf = np.ascontiguousarray(MGf, np.float32); Nh, m = MGf.shape
        n = Nh * n_u
        z = np.array(z0, np.float32, copy=True).reshape(n)
        y = np.array(y0, np.float32, copy=True).reshape(m)
        if theta is None:
            theta, beta = self.schedule_f32(max(N, 1), schedule)
        conv = C.c_int(0)
        it = self.lib.orc_solve_flat_f32(_fp(z), _fp(y), _fp(MGf), _fp(np.ascontiguousarray(gP, np.float32)),
                                         _fp(np.ascontiguousarray(GLf, np.float32)),
                                         _fp(np.ascontiguousarray(pD, np.float32)), Nh, n_u, m, N,
                                         np.float32(L), float(tol), float(tol_gap), check_every,
                                         _fp(np.ascontiguousarray(theta, np.float32)),
                                         _fp(np.ascontiguousarray(beta, np.float32)), C.byref(conv))
        return z, y, it, conv.value

    # -- per-state data / closed loop (gpad.m:79-95) -----------------------------
    def affine(self, P, c0, x):
        P = np.ascontiguousarray(P, np.float32); rows, nx = P.shape
        out = np.empty(rows, np.float32)
        c = None if c0 is None else _fp(np.ascontiguousarray(c0, np.float32))
        self.lib.orc_affine_f32(_fp(P), c, _fp(np.ascontiguousarray(x, np.float32)), _fp(out), rows, nx)
        return out

    def closed_loop_f32(self, x0, MGneg, GL, L, PM, Pg, A, B, steps, N, tol=0.0, M0=None, g0=None,
                        check_every=10, warm=False, z0=None, y0=None, schedule=SCHEDULE_MATLAB, tol_gap=0.0):
        """One instance: returns (x_T, z, y, xs [steps][nx], us [steps][nu], iters [steps])."""
        MGneg = np.ascontiguousarray(MGneg, np.float32); n, m = MGneg.shape
        c = lambda a: np.ascontiguousarray(a, np.float32)  # noqa: E731
        PM, Pg, A, B = c(PM), c(Pg), c(A), c(B)
        nx, nu = PM.shape[1], B.shape[1]
        x = np.array(x0, np.float32, copy=True).reshape(nx)
        z = np.zeros(n, np.float32) if z0 is None else np.array(z0, np.float32, copy=True)
        y = np.zeros(m, np.float32) if y0 is None else np.array(y0, np.float32, copy=True)
        xs = np.zeros((steps, nx), np.float32); us = np.zeros((steps, nu), np.float32)
        iters = np.zeros(steps, np.int32)
        theta, beta = self.schedule_f32(max(N, 1), schedule)
        opt = lambda a: None if a is None else _fp(c(a))  # noqa: E731
        self.lib.orc_closed_loop_f32(
            _fp(x), _fp(z), _fp(y), _fp(MGneg), _fp(c(GL)), np.float32(L), n, m, _fp(PM), opt(M0),
            _fp(Pg), opt(g0), _fp(A), _fp(B), nx, nu, steps, N, float(tol), float(tol_gap), check_every,
            _fp(theta), _fp(beta), int(bool(warm)), _fp(xs), _fp(us), iters.ctypes.data_as(_i))
        return x, z, y, xs, us, iters


class RefSeq:
    """The reference's own seq_functions.cpp (extern "C", seq_functions.h:4-17), composed in
    main.cu:160-175 loop order by ``solve``.  Available only where ``make -C oracle ref`` ran."""

    def __init__(self, path: str = REF):
        L = C.CDLL(path)
        L.StepOneGPADSequential.argtypes = [_f, _f, _f, C.c_float, C.c_int]
        L.StepTwoGPADSequential.argtypes = [_f, _f, _f, _f, C.c_int, C.c_int, C.c_int]
        L.StepThreeGPADSequential.argtypes = [C.c_float, C.c_int, _f, _f, _f]
        L.StepFourGPADSequential.argtypes = [_f, _f, _f, _f, _f, C.c_int, C.c_int, C.c_int]
        L.ref_solve_f32.argtypes = [_f, _f, _f, _f, _f, _f, C.c_int, C.c_int, C.c_int, _f, _f]
        L.ref_solve_batch_f32.argtypes = [_f, _f, _f, _f, _f, _f, C.c_int, C.c_int, C.c_int,
                                          C.c_int, C.c_int, _f, _f, C.c_int]
        L.StepTwoGPADFlatSequential.argtypes = [_f, _f, _f, _f, C.c_int, C.c_int, C.c_int]
        L.StepFourGPADFlatSequential.argtypes = [_f, _f, _f, _f, _f, C.c_int, C.c_int, C.c_int]
        L.ref_solve_flat_f32.argtypes = [_f, _f, _f, _f, _f, _f, C.c_int, C.c_int, C.c_int, C.c_int,
                                         _f, _f]
        self.lib = L

    @staticmethod
    def available(path: str = REF) -> bool:
        return os.path.exists(path)

    def step1(self, y, ym1, beta):
        y = np.ascontiguousarray(y, np.float32); ym1 = np.ascontiguousarray(ym1, np.float32)
        w = np.empty_like(y)
        self.lib.StepOneGPADSequential(_fp(y), _fp(ym1), _fp(w), beta, y.size)
        return w

    def step2(self, MGneg, w, gP):
        MGneg = np.ascontiguousarray(MGneg, np.float32); n, m = MGneg.shape
        zh = np.empty(n, np.float32)
        self.lib.StepTwoGPADSequential(_fp(MGneg), _fp(np.ascontiguousarray(w, np.float32)),
                                       _fp(np.ascontiguousarray(gP, np.float32)), _fp(zh), n, 1, m)
        return zh

    def step3(self, theta, zm1, zhat):
        zm1 = np.ascontiguousarray(zm1, np.float32)
        z = np.empty_like(zm1)
        self.lib.StepThreeGPADSequential(theta, zm1.size, _fp(zm1),
                                         _fp(np.ascontiguousarray(zhat, np.float32)), _fp(z))
        return z

    def step4(self, GL, w, pD, zhat):
        GL = np.ascontiguousarray(GL, np.float32); m, n = GL.shape
        y = np.empty(m, np.float32)
        self.lib.StepFourGPADSequential(_fp(GL), _fp(y), _fp(np.ascontiguousarray(w, np.float32)),
                                        _fp(np.ascontiguousarray(pD, np.float32)),
                                        _fp(np.ascontiguousarray(zhat, np.float32)), n, 1, m)
        return y

    def step2_flat(self, MGf, w, gP, n_u):
        MGf = np.ascontiguousarray(MGf, np.float32); Nh, m = MGf.shape
        zh = np.empty(Nh * n_u, np.float32)
        self.lib.StepTwoGPADFlatSequential(_fp(MGf), _fp(np.ascontiguousarray(w, np.float32)),
                                           _fp(np.ascontiguousarray(gP, np.float32)), _fp(zh), Nh, n_u, m)
        return zh

    def step4_flat(self, GLf, w, pD, zhat, n_u):
        GLf = np.ascontiguousarray(GLf, np.float32); m, Nh = GLf.shape
        y = np.empty(m, np.float32)
        self.lib.StepFourGPADFlatSequential(_fp(GLf), _fp(y), _fp(np.ascontiguousarray(w, np.float32)),
                                            _fp(np.ascontiguousarray(pD, np.float32)),
                                            _fp(np.ascontiguousarray(zhat, np.float32)), Nh, n_u, m)
        return y

    def solve_flat_c(self, z0, y0, MGf, gP, GLf, pD, n_u, theta, beta, N):
        """The reference's flat steps in the main_prof.cu loop (oracle/ref_driver.c)."""
        MGf = np.ascontiguousarray(MGf, np.float32); Nh, m = MGf.shape
        z = np.array(z0, np.float32, copy=True); y = np.array(y0, np.float32, copy=True)
        self.lib.ref_solve_flat_f32(_fp(z), _fp(y), _fp(MGf), _fp(np.ascontiguousarray(gP, np.float32)),
                                    _fp(np.ascontiguousarray(GLf, np.float32)),
                                    _fp(np.ascontiguousarray(pD, np.float32)), Nh, n_u, m, N,
                                    _fp(np.ascontiguousarray(theta, np.float32)),
                                    _fp(np.ascontiguousarray(beta, np.float32)))
        return z, y

    def solve_c(self, z0, y0, MGneg, gP, GL, pD, theta, beta, N):
        """Same loop as ``solve`` but driven from C (oracle/ref_driver.c)."""
        MGneg = np.ascontiguousarray(MGneg, np.float32); n, m = MGneg.shape
        z = np.array(z0, np.float32, copy=True); y = np.array(y0, np.float32, copy=True)
        self.lib.ref_solve_f32(_fp(z), _fp(y), _fp(MGneg), _fp(np.ascontiguousarray(gP, np.float32)),
                               _fp(np.ascontiguousarray(GL, np.float32)),
                               _fp(np.ascontiguousarray(pD, np.float32)), n, m, N,
                               _fp(np.ascontiguousarray(theta, np.float32)),
                               _fp(np.ascontiguousarray(beta, np.float32)))
        return z, y

    def solve_batch_c(self, Z0, Y0, MGneg, GP, GL, PD, theta, beta, N, shared=True, threads=1):
        Z = np.array(Z0, np.float32, copy=True); Y = np.array(Y0, np.float32, copy=True)
        batch, n = Z.shape
        m = Y.shape[1]
        self.lib.ref_solve_batch_f32(_fp(Z), _fp(Y), _fp(np.ascontiguousarray(MGneg, np.float32)),
                                     _fp(np.ascontiguousarray(GP, np.float32)),
                                     _fp(np.ascontiguousarray(GL, np.float32)),
                                     _fp(np.ascontiguousarray(PD, np.float32)), n, m, batch,
                                     int(bool(shared)), N,
                                     _fp(np.ascontiguousarray(theta, np.float32)),
                                     _fp(np.ascontiguousarray(beta, np.float32)), threads)
        return Z, Y

    def solve(self, z0, y0, MGneg, gP, GL, pD, theta, beta, N):
        """main.cu:160-175: step1 -> step2 (+copy) -> step3 -> step4, N fixed iterations."""
        z = np.array(z0, np.float32, copy=True)
        ycur = np.array(y0, np.float32, copy=True)
        yprev = ycur.copy()
        for v in range(N):
            w = self.step1(ycur, yprev, np.float32(beta[v]))
            zh = self.step2(MGneg, w, gP)
            z = self.step3(np.float32(theta[v]), z, zh)
            ynew = self.step4(GL, w, pD, zh)
            yprev, ycur = ycur, ynew
        return z, ycur
