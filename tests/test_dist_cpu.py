"""Data-parallel semantics on CPU (gloo, world_size 2, 127.0.0.1).

The product's multi-GPU path (learner.hip) shards envs per rank and all-reduces (sums) the per-rank
gradients over RCCL, then clip_by_norm + Adam use sum / world.  With equal per-rank batches that is the
gradient of the Huber *mean over the union batch*, i.e. exactly the single-process train step on the
concatenated batch.  These tests check that identity with the fp32 oracle in two gloo processes, and
exercise bench.py's control plane (barrier, max-reduce, unique-id broadcast).
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _batch(rank, B):
    rng = np.random.default_rng(100 + rank)
    x = np.zeros((B, 84, 84, 4), np.uint8)
    for b in range(B):
        for _ in range(5):
            i, j = rng.integers(0, 80, 2)
            x[b, i:i + 4, j:j + 4, rng.integers(0, 4)] = rng.choice([96, 236, 255])
    a = rng.integers(0, 3, B).astype(np.uint8)
    y = rng.normal(0, 2, B).astype(np.float32)
    return x, a, y


def _worker(rank, world, port, B, out_path):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle as O
    sys.path.insert(0, ROOT)
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    ctl = bench.Control()                     # bench.py's control plane: gloo process group from the env
    assert ctl.world == world and ctl.rank == rank and dist.is_initialized()
    net = O.QNet(seed=21)
    x, a, y = _batch(rank, B)
    _, grads, _ = net.train(x, a, y)          # local gradients (train also applies Adam locally; unused)
    flat = torch.from_numpy(np.concatenate([g.ravel() for g in grads]).astype(np.float64))
    dist.all_reduce(flat)                     # RCCL sum in the product
    mean = (flat / world).numpy()
    # control plane used by bench.py: max over ranks of the timed interval, unique-id broadcast, barrier
    tmax = ctl.max(float(rank + 1))
    uid = ctl.bcast_bytes(bytes(range(128)) if rank == 0 else bytes(128))
    ctl.barrier()
    if rank == 0:
        np.savez(out_path, mean=mean, tmax=tmax, uid=np.frombuffer(uid, np.uint8))
    dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_dp_allreduce_mean_equals_union_batch_gradient(tmp_path):
    import oracle as O
    world, B = 2, 4
    out = str(tmp_path / "dp.npz")
    mp.spawn(_worker, args=(world, _free_port(), B, out), nprocs=world, join=True)
    r = np.load(out)
    assert r["tmax"] == world
    assert np.array_equal(r["uid"], np.arange(128, dtype=np.uint8))
    # single process on the union batch
    xs, as_, ys = zip(*[_batch(k, B) for k in range(world)])
    net = O.QNet(seed=21)
    _, grads, _ = net.train(np.concatenate(xs), np.concatenate(as_), np.concatenate(ys))
    ref = np.concatenate([g.ravel() for g in grads]).astype(np.float64)
    assert np.abs(r["mean"] - ref).max() <= 1e-5 * np.abs(ref).max()


def test_bench_control_single_process():
    sys.path.insert(0, ROOT)
    import bench
    os.environ.pop("WORLD_SIZE", None)
    c = bench.Control()
    assert c.world == 1 and c.max(3.5) == 3.5 and c.bcast_bytes(b"x") == b"x"
    c.barrier()


@pytest.mark.timeout(300)
def test_bench_spawns_ranks_and_runs_control_plane():
    """`bench.py --gpus 2` without a torch.distributed.run environment starts two rank processes itself (before any GPU
    call) and their gloo control plane agrees: world 2, max / sum over ranks, rank 0's unique id on both ranks."""
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--control-only"],
                         capture_output=True, text=True, env=env, timeout=240, check=True)
    line = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(line) == 1, out.stdout
    r = json.loads(line[0])
    assert r == {"world": 2, "max_rank": 1.0, "min_rank": 0.0, "sum_ones": 2.0, "uid_ok": True}
