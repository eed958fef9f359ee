"""gpad_mpc -- MI355X-native GPAD solver for embedded linear MPC (host side).

The compute path is libgpad.so (HIP kernels for gfx950 + C++ runtime, C-ABI in
include/gpad.h); this package binds it with ctypes and adds problem construction and
multi-GPU sharding.  Importing it does not touch the GPU.
"""
from . import datafile, problems
from ._lib import (DTYPE_F32, DTYPE_F64, KERNEL_AUTO, KERNEL_PANEL, KERNEL_RESIDENT,
                   KERNEL_STREAM, MEM_DEVICE, MEM_HOST, SCHEDULE_MATLAB, SCHEDULE_PAPER, GpadError,
                   load)
from .solver import GpadGroup, GpadSolver, acceldualgrad, schedule, solve

__all__ = [
    "problems", "datafile", "load", "GpadSolver", "GpadGroup", "GpadError", "solve", "acceldualgrad", "schedule",
    "DTYPE_F32", "DTYPE_F64", "KERNEL_AUTO", "KERNEL_STREAM", "KERNEL_RESIDENT", "KERNEL_PANEL",
    "MEM_HOST", "MEM_DEVICE", "SCHEDULE_MATLAB", "SCHEDULE_PAPER",
]
