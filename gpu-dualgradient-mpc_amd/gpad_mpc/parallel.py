"""Instance-sharded multi-GPU GPAD.

MPC instances are independent, so the batch is split into contiguous shards, one per rank
(one process per GPU, torch.distributed over RCCL on ROCm); each rank solves its shard with no
communication at all, and one gather brings (z*, y*, iterations) to rank 0.  The shared
matrices (ML, G) are replicated -- every rank packs its own device copy at setup.

The compute step is a callable so the same plumbing runs on GPUs (``gpu_solve``, libgpad) and,
in the CPU tests, on the gloo backend with a host solver.
"""
from __future__ import annotations

from typing import Callable

import numpy as np


def shard_range(total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous [start, start + count) shard of ``total`` instances for ``rank`` (sizes differ by
    at most one, the larger shards first)."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError("bad rank/world")
    base, extra = divmod(total, world)
    count = base + (1 if rank < extra else 0)
    start = rank * base + min(rank, extra)
    return start, count


def gather_rows(local, world: int, rank: int, counts, dst: int = 0):
    """Gather variable-length row blocks (torch tensors, same trailing shape) to ``dst``.
    Pads every block to the largest count (gather needs equal shapes), then trims."""
    import torch
    import torch.distributed as dist
    if world == 1:
        return local
    mx = max(counts)
    buf = torch.zeros((mx,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    buf[: local.shape[0]] = local
    gl = [torch.empty_like(buf) for _ in range(world)] if rank == dst else None
    dist.gather(buf, gl, dst=dst)
    if rank != dst:
        return None
    return torch.cat([g[:c] for g, c in zip(gl, counts)], dim=0)


def solve_sharded(total: int, make_shard: Callable[[int, int], dict],
                  solve_fn: Callable[[dict], tuple], world: int, rank: int, comm_device=None):
    """Solve ``total`` instances across ``world`` ranks.

    make_shard(start, count) -> dict of this rank's inputs (host or device arrays)
    solve_fn(shard) -> (z [count, n], y [count, m], iters [count]) as torch tensors
    comm_device: where the gather runs (None: where solve_fn left the tensors -- the GPU for
    RCCL; torch.device("cpu") for gloo)
    Returns (Z, Y, iters) for all instances on rank 0, None elsewhere."""
    import torch
    counts = [shard_range(total, r, world)[1] for r in range(world)]
    start, count = shard_range(total, rank, world)
    shard = make_shard(start, count)
    z, y, iters = solve_fn(shard)
    if comm_device is not None:
        z, y, iters = z.to(comm_device), y.to(comm_device), iters.to(comm_device)
    n = z.shape[1]
    # two messages in the solution's own types: (z*, y*) rows in their float type (fp32: 1.6 KB
    # per C4 instance) and the int32 iteration counts -- no widening, no float round trip
    zy = gather_rows(torch.cat([z, y.to(z.dtype)], dim=1).contiguous(), world, rank, counts)
    it = gather_rows(iters.to(torch.int32).reshape(-1, 1).contiguous(), world, rank, counts)
    if zy is None:
        return None
    return zy[:, :n], zy[:, n:].to(y.dtype), it[:, 0].to(torch.int64)


def gpu_solve_fn(ML, G, L, N, tol, device, check_every: int = 10):
    """A ``solve_fn`` running libgpad on ``device`` for shards sharing (ML, G, L)."""
    import torch

    from .solver import GpadSolver

    def run(shard):
        M = shard["M"]
        g = shard["g"]
        count, n = M.shape
        m = g.shape[1]
        z = torch.zeros(count, n, dtype=torch.float32, device=device)
        y = torch.zeros(count, m, dtype=torch.float32, device=device)
        iters = np.zeros(count, np.int32)
        with GpadSolver(device.index if device.index is not None else 0,
                        stream=torch.cuda.current_stream(device).cuda_stream) as s:
            s.setup(ML, G, float(L), n=n, m=m, batch=count, shared=True, check_every=check_every)
            s.run(z, y, M, g, N, tol, iters=iters)
        return z, y, torch.from_numpy(iters).to(device)

    return run
