#!/usr/bin/env python3
"""Benchmark of the MI355X-native DQN hot path: env-step -> replay-sample -> Q-net update (Breakout 84x84x4).

One "step" = one vector step of the learner on every GPU: n_envs env-steps (epsilon-greedy acting forward,
batched Breakout physics + frame render, replay push, episode bookkeeping) plus the Q-net updates those
env-steps trigger (update every `update_after_actions` env-steps with batch B, replay ratio B/update_after
= 8 samples per env-step as in the reference: B 32 every 4 steps).  Each update = sample + gather, target
forward, online forward, Huber, backward, [RCCL all-reduce], clip_by_norm + Adam.

    python bench.py --gpus N --steps K --warmup W
Multi-GPU: launched by torch.distributed.run, one process per GPU; envs are sharded (weak scaling) and
gradients are all-reduced over RCCL inside libqlx.  torch.distributed (gloo) is only the control plane.
Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "q-learning_amd"))

METRIC = "env-steps/sec + grad-updates/sec, Breakout 84×84×4, 1/2/4/8 MI355X"
PEAK_BF16_TFLOPS = 2500.0     # MI355X dense bf16 MFMA (MI355X_MICROARCH.md, chip-level parameters)
PEAK_HBM_GBS = 8000.0         # HBM3E spec
GEMM_SCOPES = ("trunk_fwd", "trunk_fwd_nostore", "trunk_bwd_data", "fc1_fwd", "fc1_bwd", "conv23_wgrad", "conv1_wgrad")
# profiler scope -> the rocprofv3 kernel symbol it launches (for the committed PMC traffic lookup)
SCOPE_KERNEL = {"trunk_fwd": "k_trunk_fwdILb1E", "trunk_fwd_nostore": "k_trunk_fwdILb0E", "trunk_bwd_data": "k_trunk_bwd_data",
                "conv1_wgrad": "k_conv1_wgrad", "conv23_wgrad": "k_conv23_wgrad", "fc1_bwd": "k_fc1_bwd"}
HBM_SCOPES = ("adam", "env_step", "replay_push")
# per-sample algorithmic work of the scopes the roofline can name: (FLOP, HBM bytes).  trunk_fwd (the online forward
# that keeps its activations for the backward): 2 (400*32*256 + 81*64*512 + 49*64*576) FLOP; 4 x 7,056 B frames
# in + a1 25,600 + a2 10,368 + a3 6,272 B out.  219.6 FLOP/B is below the bf16 ridge (2,500 / 8 = 312.5): HBM class.
SCOPE_ALGO = {"trunk_fwd": (15_474_688.0, 70_464.0), "trunk_fwd_nostore": (15_474_688.0, 28_224.0 + 6_272.0)}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=55, help="vector steps before timing (covers the 50k pure-random phase)")
    ap.add_argument("--envs", type=int, default=1024, help="envs per GPU (config C2: 1024)")
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--replay-ratio", type=int, default=8, help="samples per env-step (reference: 32 per 4 steps)")
    ap.add_argument("--replay", type=int, default=100_000, help="replay capacity per GPU (config C2: 100k)")
    ap.add_argument("--cpu-sample", type=int, default=2000, help="env-steps of the CPU baseline sample, ~15 s (0 = skip)")
    ap.add_argument("--profile-steps", type=int, default=3)
    ap.add_argument("--double-dqn", action="store_true", help="extension (config C5): double-DQN targets")
    ap.add_argument("--per", action="store_true", help="extension (config C5): proportional prioritized replay")
    return ap.parse_args()


class Control:
    """Barrier / max-reduce / broadcast over torch.distributed gloo (control plane only)."""

    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.dist = None
        if self.world > 1:
            import torch.distributed as dist
            dist.init_process_group("gloo")
            self.dist = dist

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def max(self, x):
        if not self.dist:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def bcast_bytes(self, b):
        if not self.dist:
            return b
        obj = [b]
        self.dist.broadcast_object_list(obj, src=0)
        return obj[0]


def cpu_baseline(sample_steps):
    exe = os.path.join(ROOT, "oracle", "cpu_baseline")
    if sample_steps <= 0 or not os.path.exists(exe):
        return None
    threads = min(16, os.cpu_count() or 1)
    env = dict(os.environ, OMP_NUM_THREADS=str(threads))
    out = subprocess.run([exe, str(sample_steps)], capture_output=True, text=True, env=env, timeout=600, check=True)
    r = json.loads(out.stdout.strip().splitlines()[-1])
    return {"value": round(r["env_steps_per_sec"], 3), "unit": "env-steps/s", "cores": r["threads"], "kind": "port",
            "sample": f"{r['env_steps']} env-steps of the C++ restatement of the reference loop (oracle/): 1 env, "
                      f"Parameter::default(), B=32, {r['updates']} fp32 Q-net train_model updates, "
                      f"{r['seconds']:.1f} s; env+replay single-threaded, Q-net OpenMP",
            "grad_updates_per_sec": round(r["updates_per_sec"], 3)}


def roofline(scope, work, launches, avg_us, tflops, traffic, traffic_src):
    """Roofline entry for the dominant kernel: the bound follows its arithmetic intensity (algorithmic FLOP per
    algorithmic HBM byte against the ridge PEAK_BF16 / PEAK_HBM); achieved = algorithmic work per launch / the
    live average launch duration.  Both rates are kept for the record."""
    flops_launch = work / max(launches, 1)
    fl, by = SCOPE_ALGO.get(scope, (None, None))
    r = {"kernel": scope, "avg_us": round(avg_us, 2), "launches": launches, "flops_per_launch": round(flops_launch),
         "traffic": traffic, "traffic_unit": "bytes/launch", "traffic_source": traffic_src,
         "mfma_tflops": round(tflops, 2), "mfma_frac": round(tflops / PEAK_BF16_TFLOPS, 4)}
    if fl is None:
        r.update({"bound": "mfma", "achieved": round(tflops, 2), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                  "frac": round(tflops / PEAK_BF16_TFLOPS, 4)})
        return r
    bytes_launch = flops_launch / fl * by
    gbs = bytes_launch / (avg_us * 1e-6) / 1e9 if avg_us > 0 else 0.0
    intensity = fl / by
    r["algorithmic_bytes_per_launch"] = round(bytes_launch)
    r["flop_per_byte"] = round(intensity, 1)
    if intensity < PEAK_BF16_TFLOPS * 1e12 / (PEAK_HBM_GBS * 1e9):
        r.update({"bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                  "frac": round(gbs / PEAK_HBM_GBS, 4)})
    else:
        r.update({"bound": "mfma", "achieved": round(tflops, 2), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                  "frac": round(tflops / PEAK_BF16_TFLOPS, 4)})
    return r


def pmc_traffic(scope):
    """HBM bytes per launch of the scope's kernel from the newest committed PMC pass (profiles/*/pmc_traffic.json,
    written by scripts/pmc.sh + scripts/pmc_traffic.py on the same build), or None."""
    import glob
    key = SCOPE_KERNEL.get(scope)
    import re
    # natural order of the round / version directories (r01_v10 after r01_v9)
    nat = lambda f: [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", f)]
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "pmc_traffic.json")), key=nat)
    if not key or not files:
        return None, None
    data = json.load(open(files[-1]))["kernels"]
    hits = [v for k, v in data.items() if key in k]
    if len(hits) != 1:
        return None, None
    return hits[0]["hbm_bytes"], os.path.relpath(files[-1], ROOT)


def main():
    args = parse()
    ctl = Control()
    import qlx
    N, B = args.envs, args.batch
    assert B % args.replay_ratio == 0
    ua = B // args.replay_ratio
    flags = (qlx.DOUBLE_DQN if args.double_dqn else 0) | (qlx.PER if args.per else 0)
    p = qlx.Parameter(n_envs=N, batch_size=B, update_after_actions=ua, history_buffer_len=args.replay, rank=ctl.rank,
                      flags=flags)
    L = qlx.SelfDrivingQLearner(p, device=ctl.local)
    if ctl.world > 1:
        uid = ctl.bcast_bytes(qlx.dist_unique_id() if ctl.rank == 0 else bytes(128))
        L.dist_init(ctl.world, ctl.rank, uid)

    L.run(args.warmup)
    L.sync()
    # short profiled pass: per-kernel device time, pick the dominant GEMM kernel
    L.profile(True)
    L.run(args.profile_steps)
    L.sync()
    comps = {}
    for name in L.profile_names():
        us, work, n = L.profile_get(name)
        if n:
            comps[name] = {"avg_us": us / n, "launches_per_step": n / args.profile_steps, "total_us_per_step":
                           us / args.profile_steps}
            if name in GEMM_SCOPES and us > 0:
                comps[name]["tflops"] = work / us / 1e6
            if name in HBM_SCOPES and us > 0:
                comps[name]["gbs"] = work / us / 1e3
    dominant = max((n for n in comps if n in GEMM_SCOPES), key=lambda n: comps[n]["total_us_per_step"])
    L.profile(False)

    # timed region: events only around the dominant kernel's launches
    L.profile(True)
    # every 7th launch (coprime with the 8 updates of a vector step, so the samples rotate through the update
    # positions) keeps the event cost off the clock
    L.profile_filter(dominant, stride=7)
    s0 = L.stats()
    ctl.barrier()
    L.sync()
    t0 = time.perf_counter()
    L.run(args.steps)
    L.sync()
    ctl.barrier()
    dt = time.perf_counter() - t0
    dt = ctl.max(dt)
    s1 = L.stats()
    us, work, launches = L.profile_get(dominant)
    L.profile(False)

    env_steps = N * args.steps * ctl.world
    updates = s1["update_count"] - s0["update_count"]      # global updates (all-reduced: same on every rank)
    if ctl.rank != 0:
        return
    avg_us = us / max(launches, 1)
    achieved = work / us / 1e6 if us > 0 else 0.0
    traffic, traffic_src = pmc_traffic(dominant)
    line = {
        "metric": METRIC,
        "value": round(env_steps / dt, 1),
        "unit": "env-steps/s",
        "n_gpus": ctl.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic: frames rendered by the batched Breakout env kernel from live play; "
                "random-init (GlorotUniform) Nature-DQN",
        "config": {"workload": f"{'C5' if flags else 'C2'}: {N} Breakout envs per GPU, replay {args.replay} in HBM, Nature-DQN "
                               f"(3 conv + 2 dense), B={B}, update every {ua} env-steps (replay ratio "
                               f"{args.replay_ratio} samples/env-step), epsilon-greedy acting"
                               + (" + double-DQN" if args.double_dqn else "") + (" + prioritized replay" if args.per else ""),
                   "envs_per_gpu": N, "batch": B, "replay_capacity": args.replay, "update_after_actions": ua,
                   "parallelism": f"dp{ctl.world}" if ctl.world > 1 else "single", "env_dtype": "fp32",
                   "qnet_dtype": "bf16 MFMA, fp32 accumulate + master weights"},
        "grad_updates_per_sec": round(updates / dt, 2),
        "samples_per_sec": round(updates * B * ctl.world / dt, 1),
        "roofline": roofline(dominant, work, launches, avg_us, achieved, traffic, traffic_src),
        "components": {k: {kk: (round(vv, 3) if isinstance(vv, float) else vv) for kk, vv in v.items()}
                       for k, v in sorted(comps.items(), key=lambda kv: -kv[1]["total_us_per_step"])},
        "episodes": s1["episode_count"],
        "last_loss": s1["last_loss"],
    }
    if ctl.world == 1:
        line["cpu_baseline"] = cpu_baseline(args.cpu_sample)
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
