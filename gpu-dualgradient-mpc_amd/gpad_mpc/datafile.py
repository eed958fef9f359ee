"""The reference's text data-file boundary (Code/CUDA/FinalProject/main.cu:29-67 readData),
read and written by libgpad (gpad_datafile_read / gpad_datafile_write, include/gpad.h).

A data file holds the scaled GPAD inputs of one QP: ``M_G = -H^-1 G'`` (n x m), ``g_P``
(n), ``G_L = G/L`` (m x n), ``p_D = -g/L`` (m) and the theta/beta tables.  ``read`` returns
them as numpy float32 arrays in the mathematical orientation; ``layout`` says how the file
stores the matrices (``FILE_ROWMAJOR``: seq_functions.cpp; ``FILE_FLIPPED``:
kernel_functions.cu ENABLE_FLIPPING).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import FILE_FLAT, FILE_FLIPPED, FILE_ROWMAJOR, DataFile, check

__all__ = ["GpadData", "read", "write", "from_qp", "FILE_ROWMAJOR", "FILE_FLIPPED", "FILE_FLAT"]


@dataclass
class GpadData:
    n_u: int
    N: int
    m: int
    L: float
    M_G: np.ndarray   # (n, m) float32, sign-folded -H^-1 G'
    g_P: np.ndarray   # (n,)
    G_L: np.ndarray   # (m, n)
    p_D: np.ndarray   # (m,)
    theta: np.ndarray  # (num_iterations,)
    beta: np.ndarray   # (num_iterations,)

    @property
    def n(self) -> int:
        return self.n_u * self.N

    @property
    def num_iterations(self) -> int:
        return int(self.theta.shape[0])


def read(path: str, layout: int = FILE_ROWMAJOR) -> GpadData:
    lib = _lib.load()
    f = DataFile()
    check(lib.gpad_datafile_read(str(path).encode(), layout, C.byref(f)), "gpad_datafile_read")
    try:
        n, m, k = f.n_u * f.N, f.m, f.num_iterations
        rows = f.N if layout == FILE_FLAT else n  # flat files: M_G N x m, G_L m x N
        arr = lambda p, cnt: np.ctypeslib.as_array(p, shape=(max(cnt, 1),))[:cnt].copy()  # noqa: E731
        return GpadData(n_u=f.n_u, N=f.N, m=m, L=float(f.L),
                        M_G=arr(f.M_G, rows * m).reshape(rows, m), g_P=arr(f.g_P, n),
                        G_L=arr(f.G_L, rows * m).reshape(m, rows), p_D=arr(f.p_D, m),
                        theta=arr(f.theta, k), beta=arr(f.beta, k))
    finally:
        lib.gpad_datafile_free(C.byref(f))


def write(path: str, d: GpadData, layout: int = FILE_ROWMAJOR) -> None:
    lib = _lib.load()
    keep = [np.ascontiguousarray(a, np.float32) for a in (d.M_G, d.g_P, d.G_L, d.p_D, d.theta, d.beta)]
    fp = lambda a: a.ctypes.data_as(C.POINTER(C.c_float))  # noqa: E731
    f = DataFile(n_u=d.n_u, N=d.N, m=d.m, num_iterations=d.num_iterations, L=d.L,
                 M_G=fp(keep[0]), g_P=fp(keep[1]), G_L=fp(keep[2]), p_D=fp(keep[3]),
                 theta=fp(keep[4]), beta=fp(keep[5]))
    check(lib.gpad_datafile_write(str(path).encode(), layout, C.byref(f)), "gpad_datafile_write")


def from_qp(qp, n_u: int, N: int, num_iterations: int = 100, schedule: int = _lib.SCHEDULE_MATLAB) -> GpadData:
    """The data file the reference's off-line precompute would write for ``qp`` (float32
    rounding of the fp64 products, as main.cu reads them): M_G = -ML, G_L = G/L, p_D = -g/L,
    theta/beta from the MATLAB schedule (acceldualgrad.m:18,27,55-56)."""
    from .solver import schedule as sched
    L = float(qp.L)
    th, be = sched(num_iterations, schedule)
    return GpadData(n_u=n_u, N=N, m=qp.m, L=L,
                    M_G=(-np.asarray(qp.ML, np.float64)).astype(np.float32),
                    g_P=np.asarray(qp.M, np.float64).astype(np.float32),
                    G_L=(np.asarray(qp.G, np.float64) * (1.0 / L)).astype(np.float32),
                    p_D=(np.asarray(qp.g, np.float64) * (-1.0 / L)).astype(np.float32),
                    theta=th.astype(np.float32), beta=be.astype(np.float32))
