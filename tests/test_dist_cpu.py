"""Data-parallel semantics on CPU (gloo, world_size 2, 127.0.0.1).

The product's multi-GPU path (learner.hip) shards envs per rank and all-reduces (sums) the per-rank
gradients over RCCL, then clip_by_norm + Adam use sum / world.  With equal per-rank batches that is the
gradient of the Huber *mean over the union batch*, i.e. exactly the single-process train step on the
concatenated batch.  These tests check that identity with the oracle in two gloo processes, restate the
fp32 two-bucket update of learner.hip on the fp32 chain oracle (the definition the GPU is bit-exact to at world 1), and
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


KVAR_OFFSET_DENSE = 77984   # q-learning_amd/csrc/qnet.h kVarOffsetDense: W3 onward is the dense bucket


def _batch_env(rank, B):
    """rank's batch of env-rendered Breakout frames (the restated env, random play), actions and targets"""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle as O
    _, _, _, _, x = O.envs_run(0xD15 + rank, B, 30 + 7 * rank, 11 + rank, want_tensors=True)
    rng = np.random.default_rng(200 + rank)
    return x, rng.integers(0, 3, B).astype(np.uint8), rng.normal(0, 2, B).astype(np.float32)


def _worker_f32(rank, world, port, B, steps, out_dir):
    """One rank of the product's data-parallel update on the fp32 chain definition (learner.hip learner_update): local
    fp32 gradients of the rank's batch, the dense bucket (W3, b3, W4, b4) all-reduced first, then the conv bucket (fp32
    sums), then clip_by_norm + Adam on sum * (1 / world)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle as O
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    net = O.QNet(seed=21, f32=True)
    x, a, y = _batch_env(rank, B)
    sums = []
    for t in range(steps):
        scratch = O.QNet(seed=21, f32=True)
        scratch.load_state_from(net)
        _, grads, _ = scratch.train(x, a, y)             # this rank's raw gradients at the current weights
        flat = torch.from_numpy(np.concatenate([g.ravel() for g in grads]).astype(np.float32))
        dense, conv = flat[KVAR_OFFSET_DENSE:].clone(), flat[:KVAR_OFFSET_DENSE].clone()
        dist.all_reduce(dense)                            # communicator stream, beside the conv backward
        dist.all_reduce(conv)                             # learner stream, after the dense bucket
        total = torch.cat([conv, dense]).numpy()
        sums.append(total)
        O.qnet32_apply(net, total, np.float32(1.0 / world))
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), sums=np.stack(sums),
             **{f"w{v}_{k}": net.get(v, k) for v in range(10) for k in range(3)})
    dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_dp_fp32_chain_two_buckets_world2(tmp_path):
    """The fp32 data-parallel update at world 2, restated on the fp32 chain oracle with the product's bucket order
    (learner.hip:397-423): (1) both ranks end every update with identical weights and Adam slots, bit for bit; (2) the
    all-reduced gradient is the fp32 sum of the per-rank chain gradients (a two-term sum: exact IEEE, order-free), so the
    world-2 update is a fixed function of the per-rank batches; (3) against the single-GPU update on the union batch
    (one chain over all 2 B samples) it differs only by fp32 reassociation - the stated multi-rank tolerance (DESIGN.md
    §6): gradients <= 1e-5 of the variable's max |g|, weights after 3 updates within 2e-6 max |w| + 1e-4 x (3 alpha)
    (Adam's first steps move every weight by ~alpha = 7.9e-5 whatever |g| is: the biases start at 0, so their max |w|
    is itself a few alpha)."""
    import oracle as O
    world, B, steps = 2, 16, 3
    mp.spawn(_worker_f32, args=(world, _free_port(), B, steps, str(tmp_path)), nprocs=world, join=True)
    r = [np.load(str(tmp_path / f"rank{k}.npz")) for k in range(world)]
    for key in r[0].files:
        assert np.array_equal(r[0][key], r[1][key]), f"ranks differ: {key}"
    # (2) step 0: the sum is the fp32 sum of the two ranks' chain gradients
    per_rank = []
    for k in range(world):
        x, a, y = _batch_env(k, B)
        _, g, _ = O.QNet(seed=21, f32=True).train(x, a, y)
        per_rank.append(np.concatenate([v.ravel() for v in g]).astype(np.float32))
    assert np.array_equal(r[0]["sums"][0], per_rank[0] + per_rank[1])
    # (3) single GPU, union batch, same number of updates
    xs, as_, ys = zip(*[_batch_env(k, B) for k in range(world)])
    X, A, Y = np.concatenate(xs), np.concatenate(as_), np.concatenate(ys)
    one = O.QNet(seed=21, f32=True)
    for t in range(steps):
        scratch = O.QNet(seed=21, f32=True)
        scratch.load_state_from(one)
        _, g, _ = scratch.train(X, A, Y)
        flat = np.concatenate([v.ravel() for v in g]).astype(np.float64)
        if t == 0:
            off = 0
            for v in range(10):
                n = O.VAR_SIZES[v]
                mean = r[0]["sums"][0][off:off + n].astype(np.float64) / world
                assert np.abs(mean - flat[off:off + n]).max() <= 1e-5 * np.abs(flat[off:off + n]).max(), v
                off += n
        one.train(X, A, Y)
    alpha = 2.5e-4 * np.sqrt(1 - 0.999) / (1 - 0.9)
    for v in range(10):
        w1 = one.get(v, 0)
        d = np.abs(r[0][f"w{v}_0"] - w1).max()
        assert d <= 2e-6 * np.abs(w1).max() + 1e-4 * alpha * steps, v


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
