"""Shared pytest setup.

Markers: ``gpu`` -- needs a real MI355X (run with ``-m gpu``); everything else runs on CPU.
The oracle (oracle/) is test infrastructure: tests load it as the checker only.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "gpu-dualgradient-mpc_amd")
for p in (PKG, os.path.join(ROOT, "oracle"), os.path.dirname(os.path.abspath(__file__))):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")
GOLDEN_SETS = ["battery_c1", "battery_10x4", "synth_small"]


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X GPU (run with -m gpu)")


def load_golden(name: str) -> dict:
    with np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def f32_inputs(gd: dict):
    """The fp32 solve() inputs a caller would pass: fl32 of the fp64 problem."""
    c = lambda k: np.ascontiguousarray(gd[k].astype(np.float32))  # noqa: E731
    return c("ML"), c("M"), c("G"), c("g"), np.float32(gd["L"])


@pytest.fixture(scope="session")
def oracle():
    import pyoracle
    if not os.path.exists(pyoracle.LIB):
        pyoracle.build(ref=False)
    return pyoracle.Oracle()


@pytest.fixture(scope="session")
def gpu():
    """Skip when no GPU is visible; FAIL (not skip) when the HIP library is missing."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    import gpad_mpc
    gpad_mpc.load()  # raises ImportError loudly if libgpad.so was not built
    return torch.device("cuda:0")
