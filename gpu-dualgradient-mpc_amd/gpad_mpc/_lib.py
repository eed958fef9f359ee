"""ctypes binding of libgpad.so (include/gpad.h).

The shared library is built in-tree (``make -C gpu-dualgradient-mpc_amd``) next to this file
so it travels with the repository.  There is no fallback: if the library is missing or does
not load, every entry point raises -- the product path never silently drops to Python.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libgpad.so")

VERSION_MAJOR, VERSION_MINOR = 0, 5  # include/gpad.h GPAD_VERSION_*: the layouts this binding declares
GPAD_OK = 0
ERR_INVALID, ERR_HIP, ERR_NOMEM, ERR_UNSUPPORTED, ERR_NOT_SETUP, ERR_NO_DEVICE = -1, -2, -3, -4, -5, -6
ERR_DEVICE = -7  # a kernel reported a device-side failure (include/gpad.h)
FLAG_TOL_FLOOR = 1  # gpad_stats_t.flags: tol below the certification floor
FLAG_NONFINITE_G = 2  # ... g holds a NaN / infinity (tol_floor not finite)
SCHEDULE_MATLAB, SCHEDULE_PAPER = 0, 1
MEM_HOST, MEM_DEVICE = 0, 1
DTYPE_F32, DTYPE_F64 = 0, 1
KERNEL_AUTO, KERNEL_STREAM, KERNEL_RESIDENT, KERNEL_PANEL, KERNEL_FLAT = 0, 1, 2, 3, 4
KERNEL_NAMES = {KERNEL_AUTO: "auto", KERNEL_STREAM: "stream", KERNEL_RESIDENT: "resident",
                KERNEL_PANEL: "panel", KERNEL_FLAT: "flat"}

# every symbol include/gpad.h declares (checked by tests/test_abi.py)
EXPORTS = [
    "gpad_version", "gpad_strerror", "gpad_last_error", "gpad_create", "gpad_destroy",
    "gpad_set_stream", "gpad_setup", "gpad_setup_scaled", "gpad_run", "gpad_run_scaled",
    "gpad_last_stats", "gpad_phase_plan", "gpad_plan_phases", "gpad_solve", "gpad_step1_extrapolate",
    "gpad_step2_primal",
    "gpad_step3_average", "gpad_step4_project", "gpad_schedule", "gpad_sync",
    "gpad_setup_plant", "gpad_run_state", "gpad_closed_loop",
    "gpad_datafile_read", "gpad_datafile_write", "gpad_datafile_free",
    "gpad_setup_flat", "gpad_step2_primal_flat", "gpad_step4_project_flat", "gpad_precompute",
    "gpad_accumulate_iterations", "gpad_set_option",
    "gpad_group_create", "gpad_group_destroy", "gpad_group_transport", "gpad_group_setup", "gpad_group_run",
    "gpad_solve_sharded", "gpad_device_count", "gpad_group_set_stream",
    "gpad_setup_hessian", "gpad_release_cached", "gpad_phase_counts", "gpad_last_phases",
    "gpad_group_rccl_library",
]
GROUP_RCCL, GROUP_PEER = 1, 2

# gpad_set_option (include/gpad.h GPAD_OPT_*): schedule / launch tuning, never results
OPT_DEFAULT = -1
OPT_PHASE_LEN, OPT_FINISH_THRESH, OPT_PLAN, OPT_PHASED, OPT_LPT = 1, 2, 3, 4, 6
OPT_PANEL_MAX_GRID, OPT_DUO_MAX_GRID, OPT_FLAT_PANEL_MIN, OPT_FLAT_PANELS = 7, 8, 9, 10
OPT_FLAT_WAVES, OPT_FLAT_A_LDS = 11, 12
OPT_DEBUG_DROP_HANDOFF = 16  # test-only fault injection
OPT_P64_RELAY = 18  # f64 panels: 16-wave relay layout at T = 9, 13 (default 1)
OPT_P64_REFILL = 19  # f64 panels: refill finished columns from the batch (default 1)
OPT_RETIRED = (5, 13, 14, 15, 17, 20, 21)  # finisher kind, solo finisher workgroups, plan finisher cost
# (0.3); condensed panels (0.4, with the condensed operator); 17: the opt-in pair layouts measured in
# round 4 and left out of the product (W32, TailPair); 20, 21: the panel dataflow boundaries and the
# finisher mailbox measured in round 5 and removed in 0.5
OPTIONS = {"phase_len": OPT_PHASE_LEN, "finish_thresh": OPT_FINISH_THRESH, "plan": OPT_PLAN,
           "phased": OPT_PHASED, "lpt": OPT_LPT,
           "panel_max_grid": OPT_PANEL_MAX_GRID, "duo_max_grid": OPT_DUO_MAX_GRID,
           "flat_panel_min": OPT_FLAT_PANEL_MIN, "flat_panels": OPT_FLAT_PANELS,
           "flat_waves": OPT_FLAT_WAVES, "flat_a_lds": OPT_FLAT_A_LDS,
           "debug_drop_handoff": OPT_DEBUG_DROP_HANDOFF, "p64_relay": OPT_P64_RELAY,
           "p64_refill": OPT_P64_REFILL}

FILE_ROWMAJOR, FILE_FLIPPED, FILE_FLAT = 0, 1, 2


class Dims(C.Structure):
    _fields_ = [("n", C.c_int), ("m", C.c_int), ("batch", C.c_int), ("shared", C.c_int),
                ("dtype", C.c_int), ("memory", C.c_int), ("schedule", C.c_int),
                ("check_every", C.c_int), ("kernel", C.c_int), ("reserved", C.c_int),
                ("tol_gap", C.c_double)]


class Stats(C.Structure):
    _fields_ = [("iterations", C.c_int), ("converged", C.c_int),
                ("total_iterations", C.c_longlong), ("kernel", C.c_int),
                ("kernel_ms", C.c_double), ("iters", C.POINTER(C.c_int)),
                ("tol_floor", C.c_double), ("flags", C.c_int), ("codes", C.POINTER(C.c_int))]


class DataFile(C.Structure):
    """gpad_datafile_t (include/gpad.h): the reference's text data file (main.cu:29-67)."""
    _fields_ = [("n_u", C.c_int), ("N", C.c_int), ("m", C.c_int), ("num_iterations", C.c_int),
                ("L", C.c_float), ("M_G", C.POINTER(C.c_float)), ("g_P", C.POINTER(C.c_float)),
                ("G_L", C.POINTER(C.c_float)), ("p_D", C.POINTER(C.c_float)),
                ("theta", C.POINTER(C.c_float)), ("beta", C.POINTER(C.c_float))]


class GpadError(RuntimeError):
    def __init__(self, code: int, where: str, detail: str = ""):
        self.code = code
        super().__init__(f"{where}: status {code}" + (f" ({detail})" if detail else ""))


_LIB = None


def _check_version(L) -> None:
    """The library's gpad_version() ("gpad-mi355x MAJOR.MINOR ...") must be the version this binding
    declares its structs for (Dims / Stats layouts change between minors)."""
    txt = (L.gpad_version() or b"").decode(errors="replace")
    parts = txt.split()
    try:
        major, minor = (int(x) for x in parts[1].split(".")[:2])
    except (IndexError, ValueError):
        raise ImportError(f"libgpad: unrecognised gpad_version() {txt!r}") from None
    if (major, minor) != (VERSION_MAJOR, VERSION_MINOR):
        raise ImportError(f"libgpad version {major}.{minor} does not match the binding's "
                          f"{VERSION_MAJOR}.{VERSION_MINOR} (rebuild: make -C gpu-dualgradient-mpc_amd)")


def load(path: str | None = None) -> C.CDLL:
    """Load libgpad.so once.  Raises (loudly) when the HIP library is absent or its version is not
    the one this binding declares.  ``GPAD_LIB`` may point at another build of the same library;
    ``GPAD_LIB_TOLERANT=1`` (A/B benchmarking of older builds only) binds what such a build
    exports -- missing entry points become stubs returning ERR_UNSUPPORTED -- and skips the
    version check."""
    global _LIB
    if _LIB is not None:
        return _LIB
    path = path or os.environ.get("GPAD_LIB") or LIB_PATH
    if not os.path.exists(path):
        raise ImportError(f"libgpad.so not built at {path}: run `make -C gpu-dualgradient-mpc_amd` "
                          "(or __graft_entry__.build()); there is no CPU fallback")
    # One HIP runtime per process.  PyTorch-ROCm ships its own libamdhip64 / libhsa-runtime64: with
    # torch loaded first, libgpad's libamdhip64.so.7 dependency binds to torch's copy; with libgpad
    # loaded first (it links /opt/rocm's), a later `import torch` maps a second HIP + HSA runtime pair
    # and torch then sees no GPU ("No HIP GPUs are available", found by tools/fuzz_parity.py).
    try:
        import torch  # noqa: F401
    except ImportError:  # plain-C / numpy callers: /opt/rocm's runtime
        pass
    L = C.CDLL(path)
    tolerant = os.environ.get("GPAD_LIB_TOLERANT") == "1"
    if tolerant:  # A/B runs may load an older build: bind what it exports
        class _Tolerant:
            def __init__(self, lib):
                self.__dict__["_lib"] = lib

            def __getattr__(self, name):
                try:
                    return getattr(self._lib, name)
                except AttributeError:
                    return C.CFUNCTYPE(C.c_int)(lambda *a: ERR_UNSUPPORTED)

            def __setattr__(self, name, value):
                setattr(self._lib, name, value)
        L = _Tolerant(L)
    vp, cvp, i, d = C.c_void_p, C.c_void_p, C.c_int, C.c_double
    L.gpad_version.restype = C.c_char_p
    if not tolerant:
        _check_version(L)
    L.gpad_strerror.restype = C.c_char_p
    L.gpad_strerror.argtypes = [i]
    L.gpad_last_error.restype = C.c_char_p
    L.gpad_create.argtypes = [C.POINTER(vp), i, vp]
    L.gpad_destroy.argtypes = [vp]
    L.gpad_set_stream.argtypes = [vp, vp]
    L.gpad_sync.argtypes = [vp]
    L.gpad_setup.argtypes = [vp, C.POINTER(Dims), cvp, cvp, d]
    L.gpad_setup_scaled.argtypes = [vp, C.POINTER(Dims), cvp, cvp, d]
    L.gpad_setup_hessian.argtypes = [vp, cvp]
    L.gpad_run.argtypes = [vp, vp, vp, cvp, cvp, i, d, C.POINTER(Stats)]
    L.gpad_run_scaled.argtypes = [vp, vp, vp, cvp, cvp, i, d, cvp, cvp, C.POINTER(Stats)]
    L.gpad_last_stats.argtypes = [vp, C.POINTER(Stats)]
    L.gpad_phase_plan.argtypes = [vp, C.POINTER(i), C.POINTER(i), i, C.POINTER(d)]
    L.gpad_plan_phases.argtypes = [vp, i, i, i, i, i, i, C.POINTER(i), C.POINTER(i), i, C.POINTER(d)]
    L.gpad_solve.argtypes = [vp, vp, cvp, cvp, cvp, cvp, i, d, d, C.POINTER(Dims), C.POINTER(Stats)]
    f = C.POINTER(C.c_float)
    L.gpad_step1_extrapolate.argtypes = [vp, vp, vp, vp, C.c_float, i]
    L.gpad_step2_primal.argtypes = [vp, vp, vp, vp, vp, i, i]
    L.gpad_step3_average.argtypes = [vp, C.c_float, vp, vp, vp, i]
    L.gpad_step4_project.argtypes = [vp, vp, vp, vp, vp, vp, i, i]
    L.gpad_schedule.argtypes = [i, i, C.POINTER(C.c_double), C.POINTER(C.c_double)]
    del f
    L.gpad_setup_plant.argtypes = [vp, i, i, cvp, cvp, cvp, cvp, cvp, cvp]
    L.gpad_run_state.argtypes = [vp, cvp, vp, vp, i, d, C.POINTER(Stats)]
    L.gpad_closed_loop.argtypes = [vp, vp, vp, vp, i, i, d, i, vp, vp, C.POINTER(Stats)]
    L.gpad_datafile_read.argtypes = [C.c_char_p, i, C.POINTER(DataFile)]
    L.gpad_datafile_write.argtypes = [C.c_char_p, i, C.POINTER(DataFile)]
    L.gpad_datafile_free.argtypes = [C.POINTER(DataFile)]
    L.gpad_datafile_free.restype = None
    L.gpad_setup_flat.argtypes = [vp, C.POINTER(Dims), i, cvp, cvp, d]
    L.gpad_precompute.argtypes = [vp, i, i, i, i, i, cvp, cvp, cvp, vp, vp, vp]
    L.gpad_accumulate_iterations.argtypes = [vp, vp]
    L.gpad_set_option.argtypes = [vp, i, i]
    ip = C.POINTER(C.c_int)
    L.gpad_group_create.argtypes = [C.POINTER(vp), i, ip]
    L.gpad_group_destroy.argtypes = [vp]
    L.gpad_group_transport.argtypes = [vp]
    L.gpad_group_set_stream.argtypes = [vp, vp]
    L.gpad_group_setup.argtypes = [vp, C.POINTER(Dims), cvp, cvp, d]
    L.gpad_group_run.argtypes = [vp, vp, vp, cvp, cvp, i, d, C.POINTER(Stats)]
    L.gpad_solve_sharded.argtypes = [i, ip, vp, vp, cvp, cvp, cvp, cvp, i, d, d, C.POINTER(Dims), C.POINTER(Stats)]
    L.gpad_step2_primal_flat.argtypes = [vp, vp, vp, vp, vp, i, i, i]
    L.gpad_step4_project_flat.argtypes = [vp, vp, vp, vp, vp, vp, i, i, i]
    for name in ["gpad_create", "gpad_destroy", "gpad_set_stream", "gpad_sync", "gpad_setup", "gpad_setup_hessian",
                 "gpad_setup_scaled", "gpad_run", "gpad_run_scaled", "gpad_last_stats",
                 "gpad_phase_plan", "gpad_plan_phases", "gpad_solve", "gpad_step1_extrapolate", "gpad_step2_primal",
                 "gpad_step3_average", "gpad_step4_project", "gpad_schedule", "gpad_setup_plant",
                 "gpad_run_state", "gpad_closed_loop", "gpad_datafile_read",
                 "gpad_datafile_write", "gpad_setup_flat", "gpad_step2_primal_flat",
                 "gpad_step4_project_flat", "gpad_precompute", "gpad_accumulate_iterations",
                 "gpad_set_option", "gpad_group_create", "gpad_group_destroy", "gpad_group_transport",
                 "gpad_group_set_stream", "gpad_group_setup", "gpad_group_run", "gpad_solve_sharded"]:
        getattr(L, name).restype = i
    L.gpad_phase_counts.argtypes = [vp, ip, i]
    L.gpad_phase_counts.restype = i
    if hasattr(L, "gpad_group_rccl_library"):  # (0.5)
        L.gpad_group_rccl_library.argtypes = [C.c_char_p, i]
        L.gpad_group_rccl_library.restype = i
    if hasattr(L, "gpad_last_phases"):  # (0.5)
        L.gpad_last_phases.argtypes = [vp, ip, ip, ip, i, ip]
        L.gpad_last_phases.restype = i
    if hasattr(L, "gpad_release_cached"):
        L.gpad_release_cached.argtypes = []
        L.gpad_release_cached.restype = None
    _LIB = L
    return L


def check(code: int, where: str) -> None:
    if code != GPAD_OK:
        L = load()
        detail = (L.gpad_last_error() or b"").decode(errors="replace")
        raise GpadError(code, where, detail or L.gpad_strerror(code).decode())
