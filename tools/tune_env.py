"""Tools only: map the legacy GPAD_* tuning environment variables of the A/B scripts onto the
handle options of include/gpad.h (gpad_set_option).  Importing this module wraps
GpadSolver.setup / setup_flat so every handle a tool creates gets the options the environment
names.  The library itself reads no environment."""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gpu-dualgradient-mpc_amd"))

import gpad_mpc  # noqa: E402

_MAP = {  # env name -> (option, value transform)
    "GPAD_PANEL_PHASE": ("phase_len", int),
    "GPAD_FINISH_THRESH": ("finish_thresh", int),
    "GPAD_PANEL_NOPLAN": ("plan", lambda v: 0),
    "GPAD_PANEL_NOPHASE": ("phased", lambda v: 0),
    "GPAD_NO_LPT": ("lpt", lambda v: 0),
    "GPAD_PANEL_MAX_GRID": ("panel_max_grid", int),
    "GPAD_DUO_MAX_GRID": ("duo_max_grid", int),
    "GPAD_FLAT_PANEL_MIN": ("flat_panel_min", int),
    "GPAD_FLAT_PANELS": ("flat_panels", int),
    "GPAD_FLAT_WAVES": ("flat_waves", int),
    "GPAD_FLAT_NO_ALDS": ("flat_a_lds", lambda v: 0),
}


def options_from_env(env=os.environ) -> dict:
    return {opt: fn(env[k]) for k, (opt, fn) in _MAP.items() if k in env}


def apply(solver, env=os.environ) -> None:
    solver.set_options(**options_from_env(env))


def _wrap(name):
    orig = getattr(gpad_mpc.GpadSolver, name)

    def wrapped(self, *a, **kw):
        r = orig(self, *a, **kw)
        apply(self)
        return r
    setattr(gpad_mpc.GpadSolver, name, wrapped)


for _n in ("setup", "setup_flat"):
    _wrap(_n)
