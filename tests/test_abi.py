"""CPU tests of the drop-in boundary: libgpad.so builds for gfx950, loads, and exports every
symbol include/gpad.h declares.  No compute call needs a GPU here."""
from __future__ import annotations

import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import PKG, ROOT

HEADER = os.path.join(ROOT, "include", "gpad.h")


def declared_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(gpad_\w+)\s*\(", txt, re.M)))


def test_header_declares_the_north_star_surface():
    syms = declared_symbols()
    assert "gpad_solve" in syms and "gpad_setup" in syms and "gpad_run" in syms
    # solve(z0, y0, ML, M, G, g, N, L, tol) argument order is kept
    txt = open(HEADER).read()
    sig = re.search(r"int gpad_solve\(([^;]*)\);", txt, re.S).group(1)
    names = [re.findall(r"(\w+)\s*$", a.strip())[0] for a in sig.split(",")]
    assert names[:9] == ["z0", "y0", "ML", "M", "G", "g", "N", "L", "tol"]


def test_library_is_built_for_gfx950():
    lib = os.path.join(PKG, "gpad_mpc", "libgpad.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-s", "-C", PKG], check=True)
    blob = open(lib, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob  # the embedded code object's target id


def test_library_exports_every_declared_symbol():
    import gpad_mpc
    from gpad_mpc import _lib
    L = gpad_mpc.load()
    syms = declared_symbols()
    assert syms, "no symbols parsed from include/gpad.h"
    for s in syms:
        assert hasattr(L, s), f"libgpad.so does not export {s}"
    assert sorted(_lib.EXPORTS) == syms


def test_library_loads_rccl_lazily():
    """single-GPU users must not need librccl -- it is dlopen'ed by the first group over
    distinct devices (gpad_group.cpp rccl()), never a NEEDED entry of libgpad.so."""
    import shutil
    lib = os.path.join(PKG, "gpad_mpc", "libgpad.so")
    if not shutil.which("readelf"):
        pytest.skip("readelf not available")
    dyn = subprocess.run(["readelf", "-d", lib], capture_output=True, text=True, check=True).stdout
    needed = re.findall(r"\(NEEDED\).*\[(.*)\]", dyn)
    assert needed and not any("rccl" in n for n in needed), needed


def test_release_cached_without_handles_is_a_noop():
    from gpad_mpc import _lib
    L = _lib.load()
    L.gpad_release_cached()  # nothing cached on this thread: returns, touches no device
    L.gpad_release_cached()


def test_host_only_entry_points():
    from gpad_mpc import _lib, solver
    L = _lib.load()
    assert b"gfx950" in L.gpad_version()
    assert L.gpad_strerror(-4) == b"unsupported shape/kernel combination"
    th, be = solver.schedule(100)
    import pyoracle
    O = pyoracle.Oracle()
    tho, beo = O.schedule(100)
    np.testing.assert_array_equal(th, tho)
    np.testing.assert_array_equal(be, beo)
    thp, bep = solver.schedule(100, _lib.SCHEDULE_PAPER)
    np.testing.assert_array_equal(be[1:], bep[:-1])


def test_invalid_arguments_fail_cleanly():
    from gpad_mpc import _lib
    L = _lib.load()
    # null handle pointer / null handle: reported, not crashed
    assert L.gpad_create(None, 0, None) == _lib.ERR_INVALID
    assert L.gpad_run(None, None, None, None, None, 10, 0.0, None) == _lib.ERR_INVALID
    assert L.gpad_setup(None, None, None, None, 1.0) == _lib.ERR_INVALID
    assert L.gpad_schedule(-1, 0, None, None) == _lib.ERR_INVALID
    assert L.gpad_destroy(None) == _lib.GPAD_OK


def test_create_without_gpu_reports_no_device():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    from gpad_mpc import _lib
    L = _lib.load()
    h = C.c_void_p()
    rc = L.gpad_create(C.byref(h), 0, None)
    assert rc in (_lib.ERR_NO_DEVICE, _lib.ERR_HIP)
    assert not h.value
    # the failure names the HIP status it came from (name and number), or says
    # the runtime reported zero devices -- never a bare "no device"
    msg = L.gpad_last_error().decode()
    assert msg.startswith("gpad_create: hipGetDeviceCount"), msg
    assert ("hipError" in msg and "(code " in msg) or "reported 0 devices" in msg, msg
    n = L.gpad_device_count()
    if n < 0:
        assert "hipError" in L.gpad_last_error().decode()


def test_binding_checks_library_version():
    """the ctypes binding refuses a library whose gpad_version() is not the version
    its Dims / Stats layouts are declared for (GPAD_VERSION_MINOR of include/gpad.h)."""
    import re as _re

    from gpad_mpc import _lib
    hdr = open(HEADER).read()
    minor = int(_re.search(r"#define GPAD_VERSION_MINOR (\d+)", hdr).group(1))
    assert (_lib.VERSION_MAJOR, _lib.VERSION_MINOR) == (0, minor)
    assert f"0.{minor}".encode() in _lib.load().gpad_version()

    class Fake:
        def __init__(self, v):
            self.v = v

        def gpad_version(self):
            return self.v
    _lib._check_version(Fake(f"gpad-mi355x 0.{minor} (gfx950)".encode()))
    for bad in (b"gpad-mi355x 0.4 (gfx950)", b"garbage"):
        with pytest.raises(ImportError):
            _lib._check_version(Fake(bad))


def test_product_path_has_no_oracle_dependency():
    """The shipped library and package never reference the oracle."""
    lib = open(os.path.join(PKG, "gpad_mpc", "libgpad.so"), "rb").read()
    assert b"orc_" not in lib and b"liboracle" not in lib
    for f in os.listdir(os.path.join(PKG, "gpad_mpc")):
        if f.endswith(".py"):
            src = open(os.path.join(PKG, "gpad_mpc", f)).read()
            assert "pyoracle" not in src and "liboracle" not in src, f


def test_phase_planner_host_only():
    """gpad_plan_phases (the panel solver's phase planner, csrc/gpad_panel.hip panel_plan) on
    synthetic survival curves: ends strictly increasing and closing at N, takeover threshold
    covering the previous solve's survivors, and the degenerate inputs."""
    from gpad_mpc.solver import GpadSolver
    rng = np.random.default_rng(0)
    # a C4-like spread: convergence between 170 and 380 iterations
    it = np.clip(rng.normal(265, 30, 8192), 170, 380).astype(np.int32)
    p = GpadSolver.plan_phases(it, 200, 200, 5000)
    e = p["ends"]
    assert e and e[-1] == 5000 and all(a < b for a, b in zip(e, e[1:])), p
    assert all(x % 10 == 0 for x in e[:-1])                       # phases end right after a test
    assert e[0] <= int(it.min()) + 100                            # one long first phase, no earlier
    v_take = e[-2] if len(e) > 1 else 0                           # the last phase starts here ...
    assert p["fins"][-1] >= int((it > v_take).sum())              # ... and the finisher covers it
    assert p["cost_us"] > 0
    # nobody converges: one phase to N per plan slot at most, still closing at N
    p2 = GpadSolver.plan_phases(np.full(1000, 300, np.int32), 200, 200, 300)
    assert p2["ends"][-1] == 300 and len(p2["ends"]) <= 46
    # everyone at iteration 10 (first test): plan is a single phase
    p3 = GpadSolver.plan_phases(np.full(4096, 10, np.int32), 40, 180, 5000)
    assert p3["ends"] == [5000] or p3["ends"][0] == 10
    # shapes the panel kernels do not take: no plan
    assert GpadSolver.plan_phases(it, 300, 300, 5000)["ends"] == []
    from gpad_mpc import _lib
    with pytest.raises(_lib.GpadError):
        GpadSolver.plan_phases(it[:0], 200, 200, 5000)


@pytest.mark.parametrize("arr", [np.zeros(8, np.int64), np.zeros(7, np.int32), np.zeros(16, np.int32)[::2],
                                 [0] * 8])
def test_count_arrays_are_checked(arr):
    """iters / codes handed to the C stats collection must be host int32, contiguous and
    large enough -- an int64 or short array would be written out of bounds."""
    from gpad_mpc.solver import _count_array
    with pytest.raises(ValueError):
        _count_array(arr, "iters", 8)
    assert _count_array(np.zeros(8, np.int32), "iters", 8) is not None


def test_python_option_names_match_the_header():
    """Every gpad_set_option name of the Python mirror (gpad_mpc._lib.OPTIONS) is the number the
    header defines for it, and every live option of the header has a Python name."""
    from gpad_mpc import _lib
    hdr = {k.lower(): int(v) for k, v in re.findall(r"#define GPAD_OPT_(\w+)\s+(\d+)", open(HEADER).read())}
    hdr.pop("default", None)
    for name, num in _lib.OPTIONS.items():
        assert hdr.get(name) == num, name
    live = {k: v for k, v in hdr.items() if v not in _lib.OPT_RETIRED}
    assert set(live) <= set(_lib.OPTIONS), set(live) - set(_lib.OPTIONS)


def test_rccl_library_override_cpu():
    """gpad_group_rccl_library (the test / integration hook of the group transport) on the CPU: an
    unloadable library is reported as GPAD_ERR_UNSUPPORTED with a message that groups fall back to
    peer copies; the tests' stub (tests/rccl_stub, every RCCL entry point libgpad binds) loads; the
    default is restored.  No device is touched."""
    from gpad_mpc import _lib
    lib = _lib.load()
    stub = os.path.join(ROOT, "tests", "rccl_stub", "librccl_stub.so")
    if not os.path.exists(stub):
        subprocess.run(["make", "-s", "-C", os.path.dirname(stub)], check=True, timeout=120)
    try:
        assert lib.gpad_group_rccl_library(b"/nonexistent/librccl_missing.so", 1) == _lib.ERR_UNSUPPORTED
        assert b"peer copies" in lib.gpad_last_error()
        assert lib.gpad_group_rccl_library(stub.encode(), 1) == _lib.GPAD_OK
    finally:
        lib.gpad_group_rccl_library(None, 0)


def test_one_hip_runtime_whatever_the_import_order():
    """Loading libgpad before `import torch` must not map a second HIP / HSA runtime pair (torch then
    finds no GPU): _lib.load() brings torch's runtime in first, so libgpad binds to it."""
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from gpad_mpc import _lib\n_lib.load()\nimport torch\n"
            "maps = open('/proc/self/maps').read().splitlines()\n"
            "libs = sorted(set(l.split()[-1] for l in maps if 'libamdhip64' in l or 'libhsa-runtime64' in l))\n"
            "print(len([x for x in libs if 'amdhip64' in x]), len([x for x in libs if 'hsa-runtime64' in x]))\n"
            % PKG)
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    assert out.stdout.split() == ["1", "1"], out.stdout


def test_phase_planner_random_inputs():
    """gpad_plan_phases on random survival data (any batch, counts incl. 0 and > N, any N, test
    period, CU count, panel-taken shape): never an error or a crash, and every plan it returns is
    well formed -- strictly increasing ends closing at N, after a test each, within the slots."""
    from gpad_mpc.solver import GpadSolver
    rng = np.random.default_rng(3)
    for _ in range(400):
        B = int(rng.choice([1, 2, 15, 16, 17, 255, 1000, 4096, 8193, 70000]))
        N = int(rng.choice([1, 9, 10, 11, 100, 300, 5000, 20000]))
        K = int(rng.choice([1, 2, 5, 10, 16, 100]))
        kind = rng.integers(0, 4)
        if kind == 0:
            it = rng.integers(0, N + 50, B)
        elif kind == 1:
            it = np.clip(rng.normal(rng.uniform(0, N + 1), rng.uniform(1, 200), B), 0, N)
        elif kind == 2:
            it = np.full(B, int(rng.integers(0, N + 1)))
        else:
            it = rng.geometric(rng.uniform(0.001, 0.5), B)
        n, m = int(rng.choice([8, 40, 129, 200, 208, 256])), int(rng.choice([8, 64, 180, 200, 256]))
        p = GpadSolver.plan_phases(it.astype(np.int32), n, m, N, K, int(rng.choice([1, 8, 256, 304])))
        e = p["ends"]
        if not e:
            continue
        assert e[-1] == N and all(a < b for a, b in zip(e, e[1:])), (B, N, K, e)
        assert all(x % K == 0 for x in e[:-1]), (K, e)
        assert len(e) <= 64 and len(p["fins"]) == len(e)
