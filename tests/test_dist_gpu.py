"""Multi-rank runs of the real sharded path on the GPU (north_star: instance
shards, one gather of the solutions to rank 0).  Two ranks share cuda:0 over gloo -- the
driver's 8-GPU SCALE run uses one GPU per rank over RCCL with the same code.

* parallel.solve_sharded + parallel.gpu_solve_fn (libgpad on each rank, C4-generator shards
  of 1100 instances each, phased panel solves to eps = 1e-4) gathered to rank 0: every
  instance bit-exact vs the oracle, iteration counts included.
* bench.py under torch.distributed.run with 2 ranks, and plain ``python bench.py --gpus 2`` (the
  bench starts its own ranks): the JSON line's n_gpus, global batch and converged count are
  consistent; with one device the rank-0 gpad_group leg over devices 0..N-1 reports skipped.
"""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

N_, M_ = 200, 200


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gpu_worker(rank, world, port, total, out_path):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, ROOT)
    import bench
    from gpad_mpc import parallel
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    ML, G, L, _, _ = bench.make_shard(N_, M_, 1, 0)
    f32 = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(dev)  # noqa: E731
    solve_fn = parallel.gpu_solve_fn(f32(ML), f32(G), float(np.float32(L)), 5000, 1e-4, dev)

    def make_shard(start, count):
        _, _, _, M, g = bench.make_shard(N_, M_, count, start)
        return {"M": f32(M), "g": f32(g)}

    res = parallel.solve_sharded(total, make_shard, solve_fn, world, rank, comm_device=torch.device("cpu"))
    if rank == 0:
        Z, Y, it = res
        np.savez(out_path, Z=Z.numpy(), Y=Y.numpy(), it=it.numpy())
    else:
        assert res is None
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_libgpad_two_ranks_bitexact(gpu, oracle, tmp_path):
    import torch.multiprocessing as mp
    sys.path.insert(0, ROOT)
    import bench
    world, total = 2, 2200
    out = str(tmp_path / "res.npz")
    mp.start_processes(_gpu_worker, args=(world, free_port(), total, out), nprocs=world, join=True,
                       start_method="spawn")
    res = np.load(out)
    assert res["Z"].shape == (total, N_) and res["Z"].dtype == np.float32
    assert res["Y"].shape == (total, M_) and res["it"].shape == (total,)
    ML, G, L, M, g = bench.make_shard(N_, M_, total, 0)
    ML32, G32, L32 = ML.astype(np.float32), G.astype(np.float32), np.float32(L)
    MGneg, GL, _ = oracle.scale(ML32, G32, g[0].astype(np.float32), L32)
    PD = oracle.scale_vec(g.astype(np.float32), L32)
    Z, Y, iters, _ = oracle.solve_batch_f32(np.zeros((total, N_)), np.zeros((total, M_)), MGneg,
                                            M.astype(np.float32), GL, PD, 5000, L32, 1e-4,
                                            threads=min(16, os.cpu_count() or 1))
    np.testing.assert_array_equal(res["it"], iters)
    np.testing.assert_array_equal(res["Z"], Z)
    np.testing.assert_array_equal(res["Y"], Y)


@pytest.mark.parametrize("launcher", ["torchrun", "self"])
def test_bench_two_ranks_rehearsal(gpu, launcher):
    """bench.py for N = 2 (gloo, both ranks on cuda:0): as the driver launches it under
    torch.distributed.run, and as plain ``python bench.py --gpus 2`` (bench.py starts the ranks)."""
    args = [os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo", "--no-extra", "--no-cpu",
            "--steps", "3", "--warmup", "2", "--batch", "2048"]
    pre = (["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
            "--master-port", str(free_port())] if launcher == "torchrun" else [])
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, *pre, *args], capture_output=True, text=True, timeout=300, cwd=ROOT,
                       env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    d = json.loads(line)
    assert d["n_gpus"] == 2
    assert d["config"]["global_batch"] == 4096 and d["config"]["batch_per_gpu"] == 2048
    assert d["converged"] == 4096
    assert d["value"] > 0 and d["steps"] == 3
    mg = d["multi_gpu"]  # attribution of a scaling loss: per-rank solve, drain and gather times
    assert len(mg["per_rank_step_ms"]) == 2 and len(mg["per_rank_kernel_ms"]) == 2
    assert 0 < mg["solve_ms_min"] <= mg["solve_ms_max"]
    assert mg["gather_ms"] > 0 and mg["drain_ms_max"] >= 0
    assert mg["gather_bytes_per_rank"] == 2048 * 400 * 4
    assert d["config"]["parallelism"] == "instance-sharded x2, gloo gather"
    import torch
    if torch.cuda.device_count() < 2:
        assert "skipped" in mg["sharded_c4_global"]


def test_bench_sharded_leg_runs_bitexact(gpu):
    """bench.sharded_leg -- the rank-0 gpad_group leg of an N > 1 run -- over devices [0, 0] (the
    peer-copy transport of one GPU; distinct devices use the RCCL clique): it runs, converges, and
    the group's counts, z*, y* equal one handle's on the same fresh batches."""
    sys.path.insert(0, ROOT)
    import bench
    r = bench.sharded_leg(gpu, 2, batch=4096, steps=2, warmup=1, devices=[0, 0])
    assert r["transport"] == "peer" and r["n_devices"] == 2
    assert r["bitexact_vs_one_handle"] is True
    assert r["converged_last"] == 4096 and r["kernel"] == "panel"
    assert r["ms_per_solve"] > 0 and r["one_gpu_ms_per_solve"] > 0
