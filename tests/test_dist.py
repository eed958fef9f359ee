"""world_size-2 gloo tests of the instance-sharded path (CPU).  The compute step is the
host oracle here (the plumbing under test is sharding + the rank-0 gather); on GPUs the same
plumbing runs libgpad (bench.py, parallel.gpu_solve_fn)."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gpad_mpc import parallel, problems


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("total,world", [(10, 2), (7, 3), (2, 2), (5, 1)])
def test_shard_range_partitions(total, world):
    seen = []
    sizes = []
    for r in range(world):
        st, c = parallel.shard_range(total, r, world)
        seen += list(range(st, st + c))
        sizes.append(c)
    assert seen == list(range(total))
    assert max(sizes) - min(sizes) <= 1


def _problem(total):
    return problems.synthetic_qp(24, 40, batch=total, seed=13)


def _worker(rank, world, port, total, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import pyoracle
    O = pyoracle.Oracle()
    qp = _problem(total)
    ML, G, L = qp.ML.astype(np.float32), qp.G.astype(np.float32), np.float32(qp.L)

    def make_shard(start, count):
        return {"M": qp.M[start:start + count].astype(np.float32),
                "g": qp.g[start:start + count].astype(np.float32)}

    def solve_fn(shard):
        MGneg, GL, _ = O.scale(ML, G, shard["g"][0], L)
        PD = O.scale_vec(shard["g"], L)
        count = shard["M"].shape[0]
        Z, Y, iters, _ = O.solve_batch_f32(np.zeros((count, 24)), np.zeros((count, 40)), MGneg,
                                           shard["M"], GL, PD, 3000, L, 1e-4, threads=1)
        return torch.from_numpy(Z), torch.from_numpy(Y), torch.from_numpy(iters.astype(np.int64))

    res = parallel.solve_sharded(total, make_shard, solve_fn, world, rank)
    if rank == 0:
        Z, Y, it = res
        np.savez(out_path, Z=Z.numpy(), Y=Y.numpy(), it=it.numpy())
    else:
        assert res is None
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,total", [(2, 11), (2, 2)])
def test_sharded_solve_gloo_matches_single_process(tmp_path, oracle, world, total):
    out = str(tmp_path / "res.npz")
    mp.start_processes(_worker, args=(world, free_port(), total, out), nprocs=world, join=True,
                       start_method="spawn")
    res = np.load(out)
    qp = _problem(total)
    ML, G, L = qp.ML.astype(np.float32), qp.G.astype(np.float32), np.float32(qp.L)
    for b in range(total):
        z, y, it, _ = oracle.solve_f32(np.zeros(24), np.zeros(40), ML, qp.M[b].astype(np.float32), G,
                                       qp.g[b].astype(np.float32), 3000, L, 1e-4)
        assert np.array_equal(res["Z"][b], z) and np.array_equal(res["Y"][b], y)
        assert res["it"][b] == it


@pytest.mark.parametrize("gpus,world", [(2, "3"), (1, "2"), (8, "1")])
def test_bench_rejects_gpus_world_size_mismatch(gpus, world):
    """bench.py --gpus N under a launcher that started a different number of ranks exits non-zero
    before touching torch or the GPU (the driver's scaling run must not silently measure fewer)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE=world, RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", str(gpus), "--no-cpu"],
                       capture_output=True, text=True, timeout=60, env=env, cwd=root)
    assert r.returncode == 2
    assert f"--gpus {gpus} but WORLD_SIZE={world}" in r.stderr
    assert not r.stdout.strip()


def test_bench_guarded_leg_times_out_and_reports_errors():
    """bench.guarded: a multi-device leg that never returns (or raises) becomes a "skipped" record,
    so rank 0 still prints the JSON line."""
    import threading

    import bench
    done = threading.Event()
    r, hung = bench.guarded(lambda: done.wait(30) and {"ok": 1}, 0.2, "leg")
    assert hung and "did not finish" in r["skipped"]
    done.set()
    r, hung = bench.guarded(lambda: 1 / 0, 5, "leg")
    assert not hung and "ZeroDivisionError" in r["skipped"]
    r, hung = bench.guarded(lambda: {"ms": 1.0}, 5, "leg")
    assert not hung and r == {"ms": 1.0}
