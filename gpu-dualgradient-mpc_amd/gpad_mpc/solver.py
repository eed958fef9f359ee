"""Host-side mirror of the reference's GPAD interfaces, on top of libgpad.so.

* ``solve(z0, y0, ML, M, G, g, N, L, tol)`` -- the north-star entry surface (BASELINE.json),
  numpy in / numpy out (host memory) or torch device tensors (device memory, in place).
* ``acceldualgrad(H, f, A_i, b_i, Qx, Qu, n_u)`` -- the reference MATLAB function
  (Code/MATLAB/acceldualgrad.m:1) with the same arguments and return ``u = z(1:n_u)``;
  precompute as acceldualgrad.m:11,20-23, the 100-iteration loop on the GPU.
* ``GpadSolver`` -- a handle: ``setup`` once per plant (constant ML/G), ``run`` per state.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import Dims, Stats, check


def _is_torch(x) -> bool:
    return type(x).__module__.startswith("torch")


def _count_array(arr, field: str, entries: int):
    """A caller's host iters / codes array for gpad_stats_t: int32, C-contiguous, >= entries."""
    if not isinstance(arr, np.ndarray) or arr.dtype != np.int32 or not arr.flags["C_CONTIGUOUS"] \
            or arr.size < entries:
        raise ValueError(f"{field} must be a C-contiguous host int32 array with >= {entries} entries")
    return arr.ctypes.data_as(C.POINTER(C.c_int))


def _dtype_code(x) -> int:
    if _is_torch(x):
        import torch
        if x.dtype == torch.float64:
            return _lib.DTYPE_F64
        if x.dtype == torch.float32:
            return _lib.DTYPE_F32
        raise TypeError(f"unsupported torch dtype {x.dtype}")
    if x.dtype == np.float64:
        return _lib.DTYPE_F64
    if x.dtype == np.float32:
        return _lib.DTYPE_F32
    raise TypeError(f"unsupported dtype {x.dtype}")


def _ptr(x):
    if _is_torch(x):
        if not x.is_contiguous():
            raise ValueError("device tensors must be contiguous")
        return C.c_void_p(x.data_ptr())
    if not x.flags["C_CONTIGUOUS"]:
        raise ValueError("host arrays must be C-contiguous")
    return C.c_void_p(x.ctypes.data)


class GpadSolver:
    """One libgpad handle (device + HIP stream + packed matrices + workspaces)."""

    def __init__(self, device: int = 0, stream=None):
        self.lib = _lib.load()
        self.h = C.c_void_p()
        if stream is None and self._torch_device_ready():
            # order the solve after torch's pending work on this device (0 = HIP null stream)
            import torch
            stream = torch.cuda.current_stream(device).cuda_stream
        check(self.lib.gpad_create(C.byref(self.h), device, C.c_void_p(stream or 0)), "gpad_create")
        self._device = device
        self.dims = None

    def last_phases(self) -> dict:
        """The phases the last phased panel solve launched (include/gpad.h gpad_last_phases): ends,
        finisher thresholds, survivors after each phase, whether the shape's plan prior was followed,
        and the finisher takeover (the first phase whose input the finisher took, its start
        iteration; None when the panels ran the whole solve)."""
        cap = 64
        ends, fins, counts = (C.c_int * cap)(), (C.c_int * cap)(), (C.c_int * cap)()
        prior = C.c_int(0)
        n = self.lib.gpad_last_phases(self.h, ends, fins, counts, cap, C.byref(prior))
        check(min(n, 0), "gpad_last_phases")
        e, f, c = list(ends[:n]), list(fins[:n]), list(counts[:n])
        take = None
        for ph in range(1, n):
            if f[ph] > 0 and c[ph - 1] <= f[ph]:
                take = dict(phase=ph, iteration=e[ph - 1], survivors=c[ph - 1])
                break
        return dict(ends=e, fins=f, counts=c, prior=bool(prior.value), takeover=take)

    @staticmethod
    def _torch_device_ready() -> bool:
        try:
            import torch
            return torch.cuda.is_available()
        except Exception:  # noqa: BLE001 - torch is optional for host-memory use
            return False

    def close(self):
        if self.h:
            self.lib.gpad_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def set_option(self, name, value: int = _lib.OPT_DEFAULT) -> None:
        """gpad_set_option: schedule / launch tuning (``name`` in _lib.OPTIONS or a GPAD_OPT_*
        code); never changes results.  ``value`` -1 restores the default."""
        code = _lib.OPTIONS[name] if isinstance(name, str) else int(name)
        check(self.lib.gpad_set_option(self.h, code, int(value)), f"gpad_set_option({name})")

    def set_options(self, **kw) -> None:
        for k, v in kw.items():
            self.set_option(k, v)

    def set_stream(self, stream) -> None:
        check(self.lib.gpad_set_stream(self.h, C.c_void_p(stream or 0)), "gpad_set_stream")

    def setup(self, ML, G, L: float, *, n: int, m: int, batch: int = 1, shared: bool = True,
              schedule: int = _lib.SCHEDULE_MATLAB, check_every: int = 10,
              kernel: int = _lib.KERNEL_AUTO, scaled: bool = False, tol_gap: float = 0.0) -> None:
        """Bind (ML, G, L) -- or (MGneg, GL, L) with ``scaled`` (reference data-file form).
        ``tol_gap``: e_V of test (B)'s gap term (acceldualgrad.m:13; 0 = the run's tol)."""
        mem = _lib.MEM_DEVICE if _is_torch(ML) else _lib.MEM_HOST
        if _is_torch(ML) and not ML.is_cuda:
            raise ValueError("torch inputs must live on the GPU (use numpy for host memory)")
        self.dims = Dims(n=n, m=m, batch=batch, shared=int(bool(shared)), dtype=_dtype_code(ML),
                         memory=mem, schedule=schedule, check_every=check_every, kernel=kernel,
                         tol_gap=float(tol_gap))
        fn = self.lib.gpad_setup_scaled if scaled else self.lib.gpad_setup
        check(fn(self.h, C.byref(self.dims), _ptr(ML), _ptr(G), float(L)), "gpad_setup")

    def setup_flat(self, MGf, GLf, L: float, *, n_u: int, batch: int = 1,
                   schedule: int = _lib.SCHEDULE_MATLAB, check_every: int = 10,
                   kernel: int = _lib.KERNEL_AUTO, tol_gap: float = 0.0) -> None:
        """Bind the reference's flat battery data (seq_functions.cpp:5-43): MGf (N x m) flat
        sign-folded M_G, GLf (m x N) flat G_L; then ``run(..., scaled=True)`` with g_P, p_D.
        kernel=KERNEL_STREAM forces the LDS flat kernel (else the register-resident one when
        6N, n <= 208)."""
        Nh, m = MGf.shape
        mem = _lib.MEM_DEVICE if _is_torch(MGf) else _lib.MEM_HOST
        self.dims = Dims(n=n_u * Nh, m=m, batch=batch, shared=1, dtype=_lib.DTYPE_F32, memory=mem,
                         schedule=schedule, check_every=check_every, kernel=kernel, tol_gap=float(tol_gap))
        check(self.lib.gpad_setup_flat(self.h, C.byref(self.dims), int(n_u), _ptr(MGf), _ptr(GLf),
                                       float(L)), "gpad_setup_flat")

    def setup_hessian(self, H) -> None:
        """gpad_setup_hessian: bind the QP Hessian (same dtype / memory kind as ``setup``) so
        tol > 0 runs also evaluate the value-function branches (acceldualgrad.m:73,76); None
        unbinds."""
        check(self.lib.gpad_setup_hessian(self.h, _ptr(H) if H is not None else None), "gpad_setup_hessian")

    def run(self, z, y, M, g, N: int, tol: float = 0.0, *, stats: bool = True, iters=None,
            scaled: bool = False, theta=None, beta=None, codes=None):
        """Run GPAD in place on z [batch][n] / y [batch][m].  Returns a dict of stats, or None
        when ``stats`` is False and the inputs are device tensors (asynchronous launch)."""
        st = Stats()
        nb = max(1, self.dims.batch if self.dims else 1)
        if iters is not None:
            st.iters = _count_array(iters, "iters", nb)
        if codes is not None:  # per-instance termination codes 0..4 (host int32 [batch])
            st.codes = _count_array(codes, "codes", nb)
        want = stats or not _is_torch(z)
        for tab in (theta, beta):  # host tables whatever the memory kind (include/gpad.h)
            if tab is not None and (_is_torch(tab) or not isinstance(tab, np.ndarray)):
                raise TypeError("theta/beta must be host numpy arrays (include/gpad.h gpad_run_scaled)")
        if scaled:
            rc = self.lib.gpad_run_scaled(self.h, _ptr(z), _ptr(y), _ptr(M), _ptr(g), int(N),
                                          float(tol), _ptr(theta) if theta is not None else None,
                                          _ptr(beta) if beta is not None else None,
                                          C.byref(st) if want else None)
        else:
            rc = self.lib.gpad_run(self.h, _ptr(z), _ptr(y), _ptr(M), _ptr(g), int(N), float(tol),
                                   C.byref(st) if want else None)
        check(rc, "gpad_run")
        if not want:
            return None
        return self._stats_dict(st)

    def last_stats(self, iters=None) -> dict:
        st = Stats()
        if iters is not None:
            st.iters = _count_array(iters, "iters", max(1, self.dims.batch if self.dims else 1))
        check(self.lib.gpad_last_stats(self.h, C.byref(st)), "gpad_last_stats")
        return self._stats_dict(st)

    def phase_plan(self) -> dict:
        """The phase plan the next phased panel solve follows (include/gpad.h gpad_phase_plan):
        phase ends, finisher thresholds, modelled time; empty lists = the default schedule."""
        cap = 64
        ends = (C.c_int * cap)()
        fins = (C.c_int * cap)()
        cost = C.c_double(0.0)
        n = self.lib.gpad_phase_plan(self.h, ends, fins, cap, C.byref(cost))
        check(min(n, 0), "gpad_phase_plan")
        return dict(ends=list(ends[:n]), fins=list(fins[:n]), cost_us=cost.value)

    def phase_counts(self) -> list:
        """Survivors after each phase of the last phased panel solve (gpad_phase_counts); trailing
        zeros trimmed."""
        cap = 64
        buf = (C.c_int * cap)()
        n = self.lib.gpad_phase_counts(self.h, buf, cap)
        check(min(n, 0), "gpad_phase_counts")
        out = list(buf[:n])
        while out and out[-1] == 0:
            out.pop()
        return out

    @staticmethod
    def plan_phases(iters, n: int, m: int, N: int, check_every: int = 10, num_cus: int = 256) -> dict:
        """gpad_plan_phases: the phase plan the panel solver would make from these per-instance
        iteration counts (host-only; runs without a GPU)."""
        L = _lib.load()
        it = np.ascontiguousarray(iters, np.int32)
        cap = 64
        ends = (C.c_int * cap)()
        fins = (C.c_int * cap)()
        cost = C.c_double(0.0)
        k = L.gpad_plan_phases(it.ctypes.data, it.size, n, m, N, check_every, num_cus, ends, fins, cap,
                               C.byref(cost))
        check(min(k, 0), "gpad_plan_phases")
        return dict(ends=list(ends[:k]), fins=list(fins[:k]), cost_us=cost.value)

    @staticmethod
    def _stats_dict(st: Stats) -> dict:
        return dict(iterations=st.iterations, converged=st.converged,
                    total_iterations=st.total_iterations, kernel=_lib.KERNEL_NAMES.get(st.kernel),
                    kernel_ms=st.kernel_ms, tol_floor=st.tol_floor,
                    below_tol_floor=bool(st.flags & _lib.FLAG_TOL_FLOOR),
                    nonfinite_g=bool(st.flags & _lib.FLAG_NONFINITE_G))

    def sync(self) -> None:
        check(self.lib.gpad_sync(self.h), "gpad_sync")

    # ---- per-state QP data / closed loop (gpad.m:79-95; include/gpad.h gpad_setup_plant) ---
    def accumulate_iterations(self, acc) -> None:
        """Enqueue acc += sum of the last run's per-instance iteration counts (acc: a 1-element
        int64 device tensor on this handle's device); no host synchronisation."""
        import torch
        if not (_is_torch(acc) and acc.is_cuda and acc.dtype == torch.int64 and acc.numel() >= 1):
            raise TypeError("acc must be an int64 CUDA tensor with at least one element")
        if self._device is not None and acc.device.index != self._device:
            raise ValueError(f"acc lives on cuda:{acc.device.index}, the handle on cuda:{self._device}")
        check(self.lib.gpad_accumulate_iterations(self.h, _ptr(acc)), "gpad_accumulate_iterations")

    def precompute(self, H, A, f=None, *, shared: bool = True):
        """acceldualgrad.m:11,20-21 on the device in fp64 (gpad_precompute): returns
        (ML = inv(H) A', gP = inv(H) f' or None, L = ||H||_F^2).  shared: one H (n x n), A (m x n)
        and f [batch][n]; else H [batch][n][n], A [batch][m][n], f [batch][n].  numpy in ->
        numpy out; torch (device, float64) in -> torch out."""
        dev = _is_torch(H)
        n = H.shape[-1]
        m = A.shape[-2]
        batch = (f.shape[0] if f is not None and f.ndim == 2 else 1) if shared else H.shape[0]
        nmat = 1 if shared else batch
        if dev:
            import torch
            H = H.to(torch.float64).contiguous()
            A = A.to(torch.float64).contiguous()
            f = None if f is None else f.to(torch.float64).contiguous()
            ML = torch.empty((nmat, n, m) if not shared else (n, m), dtype=torch.float64, device=H.device)
            gP = None if f is None else torch.empty_like(f)
            L = torch.empty(nmat, dtype=torch.float64, device=H.device)
            mem = _lib.MEM_DEVICE
        else:
            H = np.ascontiguousarray(H, np.float64)
            A = np.ascontiguousarray(A, np.float64)
            f = None if f is None else np.ascontiguousarray(f, np.float64)
            ML = np.empty((nmat, n, m) if not shared else (n, m))
            gP = None if f is None else np.empty_like(f)
            L = np.empty(nmat)
            mem = _lib.MEM_HOST
        opt = lambda a: _ptr(a) if a is not None else None  # noqa: E731
        check(self.lib.gpad_precompute(self.h, n, m, batch, 1 if shared else 0, mem, _ptr(H), _ptr(A), opt(f),
                                       _ptr(ML), opt(gP), _ptr(L)), "gpad_precompute")
        return ML, gP, (float(L[0]) if shared else L)

    def setup_plant(self, PM, Pg, *, M0=None, g0=None, A=None, B=None) -> None:
        """Bind M(x) = M0 + PM x, g(x) = g0 + Pg x and (optionally) x+ = A x + B u.
        Same dtype / memory kind as the preceding ``setup``."""
        nx = PM.shape[-1]
        nu = 0 if B is None else B.shape[-1]
        opt = lambda a: _ptr(a) if a is not None else None  # noqa: E731
        check(self.lib.gpad_setup_plant(self.h, nx, nu, _ptr(PM), opt(M0), _ptr(Pg), opt(g0),
                                        opt(A), opt(B)), "gpad_setup_plant")

    def run_state(self, x, z, y, N: int, tol: float = 0.0, *, stats: bool = True):
        """GPAD for every instance's state x [batch][nx] (M(x), g(x) formed on the device)."""
        st = Stats()
        want = stats or not _is_torch(z)
        check(self.lib.gpad_run_state(self.h, _ptr(x), _ptr(z), _ptr(y), int(N), float(tol),
                                      C.byref(st) if want else None), "gpad_run_state")
        return self._stats_dict(st) if want else None

    def closed_loop(self, x, z, y, steps: int, N: int, tol: float = 0.0, *, warm: bool = False,
                    xs=None, us=None, iters=None, codes=None, stats: bool = True):
        """gpad.m:79-95 on the device: ``steps`` receding-horizon MPC steps for every instance.
        x [batch][nx] is advanced in place; xs [steps][batch][nx] / us [steps][batch][nu]
        receive the trajectories when given; ``iters`` / ``codes`` (host int32 [steps*batch]) the
        counts and termination codes."""
        st = Stats()
        for arr, field in ((iters, "iters"), (codes, "codes")):
            if arr is not None:
                setattr(st, field, _count_array(arr, field, steps * max(1, self.dims.batch if self.dims else 1)))
        want = stats or iters is not None or codes is not None or not _is_torch(z)
        opt = lambda a: _ptr(a) if a is not None else None  # noqa: E731
        check(self.lib.gpad_closed_loop(self.h, _ptr(x), _ptr(z), _ptr(y), int(steps), int(N),
                                        float(tol), int(bool(warm)), opt(xs), opt(us),
                                        C.byref(st) if want else None), "gpad_closed_loop")
        return self._stats_dict(st) if want else None

    # ---- per-step entry points (device tensors; kernel_functions.h one-for-one) ----------
    def step1(self, y, ym1, w, beta: float):
        check(self.lib.gpad_step1_extrapolate(self.h, _ptr(y), _ptr(ym1), _ptr(w), float(beta),
                                              y.numel()), "gpad_step1")

    def step2(self, MGneg, w, gP, zhat):
        n, m = MGneg.shape
        check(self.lib.gpad_step2_primal(self.h, _ptr(MGneg), _ptr(w), _ptr(gP), _ptr(zhat), n, m),
              "gpad_step2")

    def step2_flat(self, MGf, w, gP, zhat, n_u: int):
        """StepTwoGPADFlatSequential (seq_functions.cpp:5-20) on device tensors."""
        Nh, m = MGf.shape
        check(self.lib.gpad_step2_primal_flat(self.h, _ptr(MGf), _ptr(w), _ptr(gP), _ptr(zhat), Nh,
                                              n_u, m), "gpad_step2_flat")

    def step4_flat(self, GLf, yp1, w, pD, zhat, n_u: int):
        """StepFourGPADFlatSequential / StepFourGPADFlatParRows on device tensors."""
        m, Nh = GLf.shape
        check(self.lib.gpad_step4_project_flat(self.h, _ptr(GLf), _ptr(yp1), _ptr(w), _ptr(pD),
                                               _ptr(zhat), Nh, n_u, m), "gpad_step4_flat")

    def step3(self, theta: float, zm1, zhat, z):
        check(self.lib.gpad_step3_average(self.h, float(theta), _ptr(zm1), _ptr(zhat), _ptr(z),
                                          z.numel()), "gpad_step3")

    def step4(self, GL, yp1, w, pD, zhat):
        m, n = GL.shape
        check(self.lib.gpad_step4_project(self.h, _ptr(GL), _ptr(yp1), _ptr(w), _ptr(pD),
                                          _ptr(zhat), n, m), "gpad_step4")


class GpadGroup:
    """Several devices from one process (include/gpad.h gpad_group_*): contiguous instance shards,
    RCCL scatter/gather to devices[0] for device memory (peer copies when a device repeats)."""

    def __init__(self, devices):
        self.lib = _lib.load()
        self.devices = list(devices)
        arr = (C.c_int * len(self.devices))(*self.devices)
        self.g = C.c_void_p()
        check(self.lib.gpad_group_create(C.byref(self.g), len(self.devices), arr), "gpad_group_create")
        self.dims = None

    @property
    def transport(self) -> str:
        t = self.lib.gpad_group_transport(self.g)
        check(min(t, 0), "gpad_group_transport")
        return "rccl" if t == _lib.GROUP_RCCL else "peer"

    def close(self):
        if self.g:
            self.lib.gpad_group_destroy(self.g)
            self.g = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def setup(self, ML, G, L: float, *, n: int, m: int, batch: int, shared: bool = True,
              schedule: int = _lib.SCHEDULE_MATLAB, check_every: int = 10, kernel: int = _lib.KERNEL_AUTO,
              tol_gap: float = 0.0) -> None:
        mem = _lib.MEM_DEVICE if _is_torch(ML) else _lib.MEM_HOST
        self.dims = Dims(n=n, m=m, batch=batch, shared=int(bool(shared)), dtype=_dtype_code(ML), memory=mem,
                         schedule=schedule, check_every=check_every, kernel=kernel, tol_gap=float(tol_gap))
        check(self.lib.gpad_group_setup(self.g, C.byref(self.dims), _ptr(ML), _ptr(G), float(L)),
              "gpad_group_setup")

    def run(self, z, y, M, g, N: int, tol: float = 0.0, *, iters=None, codes=None) -> dict:
        st = Stats()
        nb = max(1, self.dims.batch if self.dims else 1)
        if iters is not None:
            st.iters = _count_array(iters, "iters", nb)
        if codes is not None:  # per-instance termination codes, [batch] in global order
            st.codes = _count_array(codes, "codes", nb)
        check(self.lib.gpad_group_run(self.g, _ptr(z), _ptr(y), _ptr(M), _ptr(g), int(N), float(tol),
                                      C.byref(st)), "gpad_group_run")
        return GpadSolver._stats_dict(st)


def schedule(N: int, kind: int = _lib.SCHEDULE_MATLAB):
    """theta[v], beta[v] (acceldualgrad.m:18,27,55-56) from the library's host routine."""
    lib = _lib.load()
    th = np.empty(max(N, 1), np.float64)
    be = np.empty(max(N, 1), np.float64)
    check(lib.gpad_schedule(N, kind, th.ctypes.data_as(C.POINTER(C.c_double)),
                            be.ctypes.data_as(C.POINTER(C.c_double))), "gpad_schedule")
    return th[:N], be[:N]


def solve(z0, y0, ML, M, G, g, N: int, L: float, tol: float = 0.0, *, shared: bool = True,
          schedule: int = _lib.SCHEDULE_MATLAB, check_every: int = 10,
          kernel: int = _lib.KERNEL_AUTO, device: int = 0, tol_gap: float = 0.0):
    """solve(z0, y0, ML, M, G, g, N, L, tol) -> (z*, y*, stats).

    Shapes: z0 (n,) or (batch, n); y0 (m,) or (batch, m); ML (n, m) or (batch, n, m); M like z0;
    G (m, n) or (batch, m, n); g like y0.  numpy inputs are copied (host memory); torch device
    tensors are updated in place."""
    torch_in = _is_torch(z0)
    if torch_in:
        z, y = z0, y0
    else:
        dt = np.float64 if np.asarray(ML).dtype == np.float64 else np.float32
        z = np.array(z0, dtype=dt, copy=True, order="C")
        y = np.array(y0, dtype=dt, copy=True, order="C")
        ML = np.ascontiguousarray(ML, dt)
        G = np.ascontiguousarray(G, dt)
        M = np.ascontiguousarray(M, dt)
        g = np.ascontiguousarray(g, dt)
    n, m = ML.shape[-2], ML.shape[-1]
    batch = z.shape[0] if z.ndim == 2 else 1
    shared = shared and ML.ndim == 2
    with GpadSolver(device) as s:
        s.setup(ML, G, L, n=n, m=m, batch=batch, shared=shared, schedule=schedule,
                check_every=check_every, kernel=kernel, tol_gap=tol_gap)
        st = s.run(z, y, M, g, N, tol)
    return z, y, st


def acceldualgrad(H, f, A_i, b_i, Qx=None, Qu=None, n_u: int = 1, num_iterations: int = 100,
                  dtype=np.float64, tol: float = 0.0):
    """Code/MATLAB/acceldualgrad.m:1 -- [u, z, y] with u = z(1:n_u) (:83).  Qx/Qu are accepted
    and unused, as in the reference.  Precompute (:11,20-23) on the host in fp64; the GPAD
    iterations run in libgpad on the GPU."""
    H = np.asarray(H, np.float64)
    A_i = np.asarray(A_i, np.float64)
    Hinv = np.linalg.inv(H)
    L = float(np.linalg.norm(H, "fro") ** 2)                    # acceldualgrad.m:11
    ML = Hinv @ A_i.T                                           # :20
    M = Hinv @ np.asarray(f, np.float64).reshape(-1)            # :21
    n, m = ML.shape
    z, y, _ = solve(np.zeros(n), np.zeros(m), ML.astype(dtype), M.astype(dtype), A_i.astype(dtype),
                    np.asarray(b_i, np.float64).astype(dtype), num_iterations, L, tol)
    return z[:n_u], z, y
