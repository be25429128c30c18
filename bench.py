#!/usr/bin/env python3
"""Benchmark of the MI355X-native DQN hot path: env-step -> replay-sample -> Q-net update (Breakout 84x84x4).

One "step" = one vector step of the learner on every GPU: n_envs env-steps (epsilon-greedy acting forward,
batched Breakout physics + frame render, replay push, episode bookkeeping) plus the Q-net updates those
env-steps trigger (update every `update_after_actions` env-steps with batch B, replay ratio B/update_after
= 8 samples per env-step as in the reference: B 32 every 4 steps).  Each update = sample + gather, target
forward, online forward, Huber, backward, [RCCL all-reduce], clip_by_norm + Adam.

    python bench.py --gpus N --steps K --warmup W

Default workload (N = 1): config C3 of SURVEY.md §8(d) - 8,192 envs per GPU, replay 1,000,000 in HBM, B = 1024,
fp32 Q-net (the reference's arithmetic).  Steady state regardless of --warmup: before anything is timed the replay
is prefilled to capacity, which also runs the loop past the 50k-step pure-random phase, so the timed vector steps
include the greedy acting forward, brick contacts and episode ends; then it keeps stepping (no updates) until episode
ends are spread over the steps as in a long run (all envs launch together and the untrained policy's episodes have
nearly one length, so their ends come in waves): after the first wave the envs' next episodes are started at staggered
steps (Run._steady), then one mean episode length of vector steps must each hold within +-50 % of the expected
n_envs / mean-length episode ends.  Then W untimed training vector steps, then K timed ones (asserted to contain
episode ends).  Beside the headline, measured in the same run: the same loop with the frozen target net evaluated per
sampled batch as the reference does (value_no_target_memo), fp32 with the exact zero skips off (value_dense_frames:
every conv1 step and conv2 / conv3 row computed), the per-step fractions those skips leave out (skipped_fractions), and
the bf16 fast path (labelled, not the headline).

Multi-GPU: with --gpus N > 1 and no WORLD_SIZE in the environment, this process starts
`torch.distributed.run --nproc-per-node N` on itself before touching the GPU and exits with its code; each rank owns
one GPU, envs and replay are sharded (weak scaling), gradients are all-reduced over RCCL inside libqlx, rank 0's
initial weights are broadcast over RCCL.  torch.distributed (gloo) is only the control plane.
Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "q-learning_amd"))

METRIC = "env-steps/sec + grad-updates/sec, Breakout 84×84×4, 1/2/4/8 MI355X"
PEAK_TFLOPS = {"fp32": 157.3, "bf16": 2500.0}   # MI355X dense MFMA peaks (MI355X_MICROARCH.md: f32-input MFMA, bf16)
# steady state before timing (Run._steady): a window of one mean episode length T whose episode ends per vector step average
# within +-STEADY_MEAN_TOL of n_envs / T with a coefficient of variation <= STEADY_MAX_CV (waves: CV >> 1; a steady
# stream of independent ends: ~1 / sqrt(n_envs / T))
STEADY_MEAN_TOL, STEADY_MAX_CV, MAX_STEADY = 0.1, 0.5, 4000
PEAK_HBM_GBS = 8000.0                            # HBM3E
# per-sample algorithmic FLOPs of the Q-net: forward 18,689,024; per trained sample 68,202,496
FWD_FLOP, TRAIN_FLOP = 18_689_024, 68_202_496
TRANSITION_BYTES = 56_454          # logical (a, s, s', r, done) of one sampled transition
# with the Bellman-target memo (learner.hip ycache_fill: the frozen target net's y computed once per transition at
# insertion) a sampled transition delivers (a, s, y); s' is read once, by the memo pass over the new transitions
MEMO_SAMPLED_BYTES = 1 + 4 * 7056 + 4
ADAM_BYTES = 53_941_344            # clip_by_norm + Adam per update: g read twice, w / m / v read and written
# profiler scopes of each precision: the GEMM-shaped kernels (FLOP work) and their per-layer grouping
GEMM_SCOPES = {
    "fp32": ("f32_conv1_fwd", "f32_conv2_fwd", "f32_conv3_fwd", "f32_fc1_fwd", "f32_conv1_fwd_big", "f32_conv2_fwd_big",
             "f32_conv3_fwd_big", "f32_fc1_fwd_big", "f32_fc1_bwd", "f32_conv3_bwd", "f32_conv2_bwd", "f32_conv1_wgrad"),
    "bf16": ("trunk_fwd", "trunk_fwd_nostore", "trunk_bwd_data", "fc1_fwd", "fc1_bwd", "conv23_wgrad", "conv1_wgrad"),
}
ADAM_SCOPES = {"fp32": ("f32_norms", "f32_adam"), "bf16": ("sumsq", "adam")}
# the kernels that deliver sampled transitions into the net: index draw, gather, and the conv1 frame fetch of the
# online pass (s) and of the batched target pass (s'; conv1_fwd_big, which also runs the one acting chunk: its share is
# taken by sample count)
SAMPLE_SCOPES = {"fp32": ("sample", "gather", "f32_conv1_fwd", "f32_conv1_fwd_big"), "bf16": ("sample", "gather")}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10, help="timed vector steps")
    ap.add_argument("--warmup", type=int, default=2, help="untimed training vector steps after the steady-state prefill")
    ap.add_argument("--envs", type=int, default=8192, help="envs per GPU (C3: 8192; C2: 1024; C4: 4096 x 8)")
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--replay-ratio", type=int, default=8, help="samples per env-step (reference: 32 per 4 steps)")
    ap.add_argument("--replay", type=int, default=1_000_000, help="replay capacity per GPU (C3: 1M; C2: 100k)")
    ap.add_argument("--precision", choices=("fp32", "bf16"), default="fp32", help="headline Q-net arithmetic")
    ap.add_argument("--beside-steps", type=int, default=5, help="timed vector steps of the other precision (0 = skip)")
    ap.add_argument("--nomemo-steps", type=int, default=5,
                    help="timed vector steps of the headline precision with the target net evaluated per sampled batch "
                         "(QLX_TARGET_CACHE=0, the reference's work; 0 = skip)")
    ap.add_argument("--dense-steps", type=int, default=5,
                    help="fp32: timed vector steps of a learner built with the exact zero skips off (QLX_F32_BG=0 "
                         "QLX_F32_C1_SKIP=0: every conv1 step and conv2 / conv3 row computed; 0 = skip)")
    ap.add_argument("--refwork-steps", type=int, default=5,
                    help="fp32: timed vector steps doing the reference's work - the target net per sampled batch AND the "
                         "exact zero skips off (QLX_TARGET_CACHE=0 QLX_F32_BG=0 QLX_F32_C1_SKIP=0; 0 = skip)")
    ap.add_argument("--dp1-steps", type=int, default=5,
                    help="one GPU: timed vector steps of the data-parallel update path on a single-rank RCCL communicator "
                         "(bucketed all-reduce + the DP update tail; the cost C4 pays per rank besides the link; 0 = skip)")
    ap.add_argument("--c5-steps", type=int, default=5,
                    help="one GPU: timed vector steps of C5's per-GPU shard (double DQN + prioritized replay, fp32, the "
                         "same envs / replay / batch) beside the headline; 0 = skip")
    ap.add_argument("--sparsity-steps", type=int, default=8,
                    help="fp32: untimed vector steps after the timed window, each reporting the fractions of conv work "
                         "the skips left out (qlx_learner_frame_sparsity)")
    ap.add_argument("--cpu-sample", type=int, default=4_000,
                    help="env-steps of the CPU baseline: the first N of C1's 10,000 (~26 s on the box's host; 0 = skip)")
    ap.add_argument("--profile-steps", type=int, default=1)
    ap.add_argument("--double-dqn", action="store_true", help="extension (config C5): double-DQN targets")
    ap.add_argument("--per", action="store_true", help="extension (config C5): proportional prioritized replay")
    ap.add_argument("--no-target-memo", action="store_true",
                    help="evaluate the frozen target net per sampled batch (QLX_TARGET_CACHE=0) instead of once per "
                         "transition at insertion (same values; the reference's per-batch work)")
    ap.add_argument("--control-only", action="store_true",
                    help="exercise the rank spawn + gloo control plane only (no GPU; CPU test of the N > 1 path)")
    return ap.parse_args()


def spawn_ranks(args):
    """--gpus N > 1 without a torch.distributed.run environment: start N rank processes on this bench (before
    any GPU call in this process) and return their exit code."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


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

    def min(self, x):
        if not self.dist:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MIN)
        return float(t.item())

    def sum(self, x):
        if not self.dist:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return float(t.item())

    def bcast_bytes(self, b):
        if not self.dist:
            return b
        obj = [b]
        self.dist.broadcast_object_list(obj, src=0)
        return obj[0]


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(sample_steps):
    """C1 on the host: the oracle's restatement of the reference loop (1 env, Parameter::default(), B = 32).  The loop
    runs on one pinned core (the OpenMP master thread, OMP_PROC_BIND=close on an explicit place list); the Q-net's
    OpenMP regions use up to 16 of the cores this process may run on."""
    exe = os.path.join(ROOT, "oracle", "cpu_baseline")
    if sample_steps <= 0 or not os.path.exists(exe):
        return None
    cpus = sorted(os.sched_getaffinity(0))[:16]
    env = dict(os.environ, OMP_NUM_THREADS=str(len(cpus)), OMP_PROC_BIND="close",
               OMP_PLACES=",".join("{%d}" % c for c in cpus))
    out = subprocess.run([exe, str(sample_steps)], capture_output=True, text=True, env=env, timeout=900, check=True)
    r = json.loads(out.stdout.strip().splitlines()[-1])
    return {"value": round(r["env_steps_per_sec"], 3), "unit": "env-steps/s", "cores": r["threads"], "kind": "port",
            "sample": f"C1 (its first {r['env_steps']} of 10,000 env-steps, a bounded sample): the C++ restatement of the "
                      f"reference loop (oracle/): 1 env, "
                      f"Parameter::default(), B=32, {r['updates']} fp32 Q-net updates, {r['seconds']:.1f} s; env loop "
                      f"single-threaded on one pinned core, Q-net OpenMP on {r['threads']} cores ({cpu_model()})",
            "grad_updates_per_sec": round(r["updates_per_sec"], 3)}


def config_label(N, replay, flags, world):
    if flags == 0 and world == 1 and N == 1024 and replay == 100_000:
        return "C2"
    if flags == 0 and world == 1 and N == 8192 and replay == 1_000_000:
        return "C3"
    if flags == 0 and world == 8 and N == 4096:
        return "C4"
    if flags == 3 and world == 8 and N == 8192:
        return "C5"
    if flags == 3 and world == 1 and N == 8192:
        return "C5 (one GPU's shard)"
    if flags == 0 and world > 1 and N == 8192 and replay == 1_000_000:
        return f"C3 per GPU x {world} (weak scaling)"
    return f"custom ({world} GPU)"


class stdout_to_stderr:
    """fd 1 -> fd 2 while RCCL initialises a communicator (its version banner goes to stdout; the bench's stdout is the
    one JSON line)"""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        os.dup2(self.saved, 1)
        os.close(self.saved)


def log(msg):
    """progress on stderr (one line per phase, so a long run shows it is alive)"""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def rate(work, us, div):
    return work / us / div if us > 0 else 0.0


class Run:
    """One learner measured on the steady-state workload."""

    def __init__(self, args, ctl, precision, steps, warmup, flags, sparsity_steps=0, dp1=False):
        import qlx
        self.args, self.ctl, self.precision = args, ctl, precision
        N, B = args.envs, args.batch
        self.ua = B // args.replay_ratio
        prec = qlx.PREC_F32 if precision == "fp32" else qlx.PREC_BF16
        p = qlx.Parameter(n_envs=N, batch_size=B, update_after_actions=self.ua, history_buffer_len=args.replay,
                          rank=ctl.rank, flags=flags, qnet_precision=prec)
        L = qlx.SelfDrivingQLearner(p, device=ctl.local)
        self.L = L
        self.rccl_world = 1
        try:
            if ctl.world > 1:
                uid = ctl.bcast_bytes(qlx.dist_unique_id() if ctl.rank == 0 else bytes(128))
                with stdout_to_stderr():
                    L.dist_init(ctl.world, ctl.rank, uid)
            elif dp1:   # a single-rank communicator: the data-parallel update path on one GPU
                with stdout_to_stderr():
                    L.dist_init(1, 0, qlx.dist_unique_id())
            self.rccl_world = L.comm_size()   # read back from the communicator (ncclCommCount)
            # steady state: replay at capacity and past the pure-random phase, whatever --warmup is
            prefill = max(-(-args.replay // N), -(-p.epsilon_pure_random_steps // N))
            log(f"{precision}: prefill {prefill} vector steps")
            L.prefill(prefill)
            # ... and episode ends spread over the steps as in a long run (all envs launch together, so their first
            # episodes end together)
            prefill += self._steady(L)
            L.run(max(warmup, 1))
            L.sync()
            s = L.stats()
            assert s["replay_len"] == args.replay and s["episode_count"] > 0, s
            assert s["step_count"] >= p.epsilon_pure_random_steps, s
            self.prefill = prefill
            log(f"{precision}: profile pass")
            self.comps = self._profile()
            log(f"{precision}: timed {steps} vector steps")
            self._timed(steps)
            log(f"{precision}: {self.value():.1f} env-steps/s")
            self.sparsity = self._sparsity(sparsity_steps) if sparsity_steps > 0 else None
        finally:
            L.close()

    def _steady(self, L):
        """Vector steps without updates until episode ends are spread over the steps as in a long run.  All envs launch
        together and the untrained policy's episodes have nearly one length, so left alone their ends come in waves that
        persist for thousands of vector steps (measured: 0..275 ends per step after 4,000).  So: (1) step until the first
        wave has passed (one finished episode per env on average) and take the mean episode length T from it; (2) a
        staggered start - over T steps, step k ends the current episode of the envs e = k (mod T) (the
        max_steps_per_episode path, qlx_learner_end_episodes); (3) step until one window of T vector steps has its
        episode ends per step averaging within STEADY_MEAN_TOL of n_envs / T with a coefficient of variation of at most
        STEADY_MAX_CV, for at most 3 T vector steps - when no window qualifies the bench still measures, but the JSON line
        carries steady_state.steady = false and the log warns.  Decisions are global (every rank runs the same number
        of vector steps: each one carries collectives)."""
        import numpy as np
        N, ctl = self.args.envs, self.ctl
        n = 0
        while n < MAX_STEADY:
            s = L.stats()
            if ctl.sum(float(s["episode_count"])) >= N * ctl.world:
                break
            L.prefill(1)
            n += 1
        s = L.stats()
        mean_len = ctl.sum(float(s["step_count"])) / max(ctl.sum(float(s["episode_count"])), 1.0)
        T = max(1, int(round(mean_len)))
        eids = np.arange(N)
        for k in range(T):
            L.end_episodes((eids % T) == k)
            L.prefill(1)
            n += 1
        expect = N / mean_len
        last, ends, ok = L.stats()["episode_count"], [], False
        def window_stats(w):
            w = np.asarray(w, np.float64)
            return w.mean(), w.std() / max(w.mean(), 1e-9)
        for _ in range(3 * T):
            L.prefill(1)
            n += 1
            e = L.stats()["episode_count"]
            ends.append(e - last)
            last = e
            mine = False
            if len(ends) >= T:
                mean, cv = window_stats(ends[-T:])
                mine = abs(mean - expect) <= STEADY_MEAN_TOL * expect and cv <= STEADY_MAX_CV
            if ctl.min(1.0 if mine else 0.0) > 0:
                ok = True
                break
        mean, cv = window_stats(ends[-T:])
        self.mean_len, self.expect_ends, self.steady_ok = mean_len, expect, ok
        self.steady_window = {"steps": T, "mean_ends": round(mean, 2), "cv": round(cv, 3), "min": int(min(ends[-T:])),
                              "max": int(max(ends[-T:]))}
        if not ok:
            log(f"WARNING {self.precision}: no steady window within {3 * T} vector steps; the line says steady: false")
        log(f"{self.precision}: {n} more vector steps to steady episode ends (mean episode {mean_len:.1f} env-steps, "
            f"staggered over {T}; {expect:.1f} ends expected per vector step; last window {self.steady_window}, steady {ok})")
        return n

    def _profile(self):
        """Event-timed per-scope device time over profile_steps vector steps (every launch bracketed by events, so
        the sum exceeds the un-instrumented step; for attribution only)."""
        L, n = self.L, self.args.profile_steps
        L.profile(True)
        L.run(n)
        L.sync()
        comps = {}
        for name in L.profile_names():
            us, work, k = L.profile_get(name)
            if k:
                comps[name] = {"avg_us": us / k, "launches_per_step": k / n, "total_us_per_step": us / n, "work": work / n}
        L.profile(False)
        return comps

    def _timed(self, steps):
        L, ctl, gemm = self.L, self.ctl, GEMM_SCOPES[self.precision]
        self.dominant = max((c for c in self.comps if c in gemm), key=lambda c: self.comps[c]["total_us_per_step"])
        # events only around the dominant kernel, on every 7th launch (keeps the event cost off the clock)
        L.profile(True)
        L.profile_filter(self.dominant, stride=7)
        s0 = L.stats()
        ctl.barrier()
        L.sync()
        t0 = time.perf_counter()
        L.run(steps)
        L.sync()
        ctl.barrier()
        dt = ctl.max(time.perf_counter() - t0)
        s1 = L.stats()
        self.dom_us, self.dom_work, self.dom_launches = L.profile_get(self.dominant)
        L.profile(False)
        self.steps, self.dt = steps, dt
        self.env_steps = self.args.envs * steps * ctl.world
        self.updates = s1["update_count"] - s0["update_count"]
        self.episodes = int(ctl.sum(s1["episode_count"] - s0["episode_count"]))
        self.ends_per_step = self.episodes / max(steps, 1)
        self.episodes_total = int(ctl.sum(s1["episode_count"]))
        self.last_loss = s1["last_loss"]
        self.running_reward = s1["running_reward"]
        self.epsilon = s1["epsilon"]

    def _sparsity(self, n):
        """Per vector step (untimed, after the timed window): the fractions of the fp32 conv work the exact zero skips
        left out - conv1 forward / weight-gradient all-zero steps, conv2 / conv3 background rows - over the step's sampled
        training states and over its acting frames (qlx_learner_frame_sparsity, the kernels' own predicates)."""
        import numpy as np
        L = self.L
        tr, ac = [], []
        for _ in range(n):
            L.run(1)
            f = L.frame_sparsity()
            if not np.isnan(f["train"][0]):
                tr.append(f["train"])
            ac.append(f["act"])
        names = ("conv1_fwd_zero_steps", "conv1_wgrad_zero_steps", "conv2_background_rows", "conv3_background_rows")
        def summ(rows):
            if not rows:
                return None
            a = np.asarray(rows)
            return {k: {"mean": round(float(a[:, i].mean()), 4), "min": round(float(a[:, i].min()), 4),
                        "max": round(float(a[:, i].max()), 4)} for i, k in enumerate(names)}
        return {"vector_steps": n, "train_batches": summ(tr), "acting": summ(ac),
                "note": "fractions of the dense conv work not issued (exact skips, DESIGN.md 4.1), per vector step after "
                        "the timed window; train = the step's U x B sampled states, acting = the n_envs frames"}

    def roofline(self):
        """The dominant kernel against the MFMA peak of this precision (the Q-net is MFMA class):
        achieved = algorithmic FLOP per launch / live average launch duration (HIP events bound to the kernel's own
        dispatch on the learner stream, every 7th launch of the timed region)."""
        peak = PEAK_TFLOPS[self.precision]
        avg_us = self.dom_us / max(self.dom_launches, 1)
        tflops = rate(self.dom_work, self.dom_us, 1e6)
        traffic, src = pmc_traffic(self.precision, self.dominant)
        out = {"kernel": self.dominant, "bound": "mfma", "achieved": round(tflops, 2), "peak": peak, "unit": "TFLOP/s",
               "frac": round(tflops / peak, 4), "traffic": traffic, "traffic_unit": "HBM bytes/launch",
               "traffic_source": src, "avg_us": round(avg_us, 2), "launches_timed": self.dom_launches,
               "flops_per_launch": round(self.dom_work / max(self.dom_launches, 1))}
        if self.dominant in ZERO_STEP_SCOPES:
            # a launch that does not issue part of its dense work: achieved = the issued FLOP (dense x (1 - share x the
            # measured skipped fraction)) per launch / time; the dense-equivalent rate beside it
            _, (half, key), share = zero_step_scope(self.dominant)
            skip = self.skipped(half, key)
            if skip is not None:
                f = 1.0 - share * skip
                out.update({"achieved": round(tflops * f, 2), "frac": round(tflops * f / peak, 4),
                            "flops_per_launch": round(self.dom_work * f / max(self.dom_launches, 1)),
                            "achieved_dense_equivalent": round(tflops, 2), "skipped_fraction": round(skip, 4),
                            "skipped_share_of_launch": share,
                            "flops_per_launch_dense": round(self.dom_work / max(self.dom_launches, 1))})
        return out

    def report(self):
        """north_star's extra rates from the event-timed profile pass: per-layer MFMA utilisation, replay-sampling
        and clip+Adam HBM fractions."""
        c, peak = self.comps, PEAK_TFLOPS[self.precision]
        layers = {}
        for k in GEMM_SCOPES[self.precision]:
            if k in c and c[k]["total_us_per_step"] > 0:
                t = rate(c[k]["work"], c[k]["total_us_per_step"], 1e6)
                if k in ZERO_STEP_SCOPES:
                    # part of the dense work is not issued: the MFMA utilisation is the issued work, dense FLOP x (1 - the
                    # scope's measured skipped fraction x the share of the launch's work it applies to), over the time;
                    # the dense-equivalent rate stays beside it
                    note, (half, key), share = zero_step_scope(k)
                    skip = self.skipped(half, key)
                    issued = None if skip is None else t * (1.0 - share * skip)
                    layers[k] = {"tflops_issued": None if issued is None else round(issued, 2),
                                 "mfma_frac": None if issued is None else round(issued / peak, 4),
                                 "skipped_fraction": None if skip is None else round(skip, 4),
                                 "skipped_fraction_source": f"skipped_fractions.{half}.{key}.mean",
                                 "skipped_share_of_launch": share,
                                 "tflops_dense_equivalent": round(t, 2), "avg_us": round(c[k]["avg_us"], 2), "note": note}
                else:
                    layers[k] = {"tflops": round(t, 2), "mfma_frac": round(t / peak, 4), "avg_us": round(c[k]["avg_us"], 2)}
        upd = self.updates / max(self.steps, 1) / max(self.ctl.world, 1)   # updates per vector step on one GPU
        B = self.args.batch
        t_samp = sum(c[k]["total_us_per_step"] for k in SAMPLE_SCOPES[self.precision][:3] if k in c)
        memo = "target_memo" in c
        if memo:
            tb, note = MEMO_SAMPLED_BYTES, ("logical bytes of a sampled transition (a, s, y: the target memo holds y) "
                                            "delivered into the net / time of index draw + gather + the online pass's "
                                            "conv1 frame fetch")
        else:
            tb, note = TRANSITION_BYTES, ("logical transition bytes (a, s, s', r, done) delivered into the net / time "
                                          "of index draw + gather + conv1 frame-fetch launches")
            if "f32_conv1_fwd_big" in c:   # the target chunks' share (U*B of the U*B + n_envs samples per vector step)
                t_samp += c["f32_conv1_fwd_big"]["total_us_per_step"] * upd * B / (upd * B + self.args.envs)
        samp_gbs = rate(upd * B * tb, t_samp, 1e3)
        t_adam = sum(c[k]["total_us_per_step"] for k in ADAM_SCOPES[self.precision] if k in c)
        adam_gbs = rate(upd * ADAM_BYTES, t_adam, 1e3)
        return {
            "mfma_per_layer": layers,
            "replay_sampling": {"gbs": round(samp_gbs, 1), "frac": round(samp_gbs / PEAK_HBM_GBS, 4),
                                "bytes_per_transition": tb,
                                "scopes": list(SAMPLE_SCOPES[self.precision][:3 if memo else 4]), "note": note},
            "clip_adam": {"gbs": round(adam_gbs, 1), "frac": round(adam_gbs / PEAK_HBM_GBS, 4),
                          "bytes_per_update": ADAM_BYTES, "scopes": list(ADAM_SCOPES[self.precision])},
        }

    def value(self):
        return self.env_steps / self.dt

    def skipped(self, half, key):
        """mean skipped fraction of one skip predicate over the sparsity pass (None without one)"""
        s = self.sparsity
        if not s or not s.get(half):
            return None
        return s[half][key]["mean"]


# launches that do not issue part of their layer's dense work (exact), each with the skipped fraction that
# applies to it: the training-batch launches take the sampled states' fraction, the chunk launches (the acting forward and
# the target memo over the new transitions' s' - the same frames one vector step apart) the acting frames'
_C1_NOTE = ("MFMA steps whose frame operands are all 0 are not issued (exact, DESIGN.md 4.1): mfma_frac = dense FLOP x (1 - "
            "skipped_fraction) / time / peak; tflops_dense_equivalent = dense FLOP / time")
_BG_NOTE = ("the background rows (receptive field all-zero frame pixels) are one constant row, computed once and written, "
            "the GEMM runs the other rows (exact, DESIGN.md 4.1): mfma_frac = dense FLOP x (1 - skipped_fraction) / time / "
            "peak; tflops_dense_equivalent = dense FLOP / time")
_WG_NOTE = ("backward pair (weight gradient + backward data, equal dense FLOP): the weight-gradient tiles reduce over the "
            "non-background rows only - a background row's im2col row is the layer's constant input row, its share a rank-1 "
            "term added in the reduction (DESIGN.md §6): mfma_frac = dense FLOP x (1 - skipped_fraction / 2) / time / peak; "
            "tflops_dense_equivalent = dense FLOP / time")
ZERO_STEP_SCOPES = {
    "f32_conv2_bwd": (_WG_NOTE, ("train_batches", "conv2_background_rows"), 0.5),
    "f32_conv3_bwd": (_WG_NOTE, ("train_batches", "conv3_background_rows"), 0.5),
    "f32_conv1_fwd": (_C1_NOTE, ("train_batches", "conv1_fwd_zero_steps")),
    "f32_conv1_fwd_big": (_C1_NOTE, ("acting", "conv1_fwd_zero_steps")),
    "f32_conv1_wgrad": (_C1_NOTE, ("train_batches", "conv1_wgrad_zero_steps")),
    "f32_conv2_fwd": (_BG_NOTE, ("train_batches", "conv2_background_rows")),
    "f32_conv2_fwd_big": (_BG_NOTE, ("acting", "conv2_background_rows")),
    "f32_conv3_fwd": (_BG_NOTE, ("train_batches", "conv3_background_rows")),
    "f32_conv3_fwd_big": (_BG_NOTE, ("acting", "conv3_background_rows")),
}


def zero_step_scope(k):
    """(note, (half, key), share of the launch's dense work the skipped fraction applies to)"""
    v = ZERO_STEP_SCOPES[k]
    return (v[0], v[1], v[2] if len(v) > 2 else 1.0)


def pmc_traffic(precision, scope):
    """HBM bytes per launch of the scope's kernel from the newest committed PMC pass of this precision
    (profiles/*/pmc_traffic_<precision>.json, written by scripts/pmc.sh + scripts/pmc_traffic.py), or None."""
    import glob
    import re
    nat = lambda f: [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", f)]
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*", f"pmc_traffic_{precision}.json")), key=nat)
    if not files:
        return None, None
    d = json.load(open(files[-1]))
    hit = d.get("scopes", {}).get(scope)
    if hit is None:
        return None, None
    return hit["hbm_bytes"], os.path.relpath(files[-1], ROOT)


def control_check(ctl):
    """The control plane bench.py relies on, without the GPU: barrier, max / sum over ranks, rank 0's unique id on
    every rank.  Rank 0 prints one JSON line."""
    uid = ctl.bcast_bytes(bytes(range(128)) if ctl.rank == 0 else bytes(128))
    ctl.barrier()
    out = {"world": ctl.world, "max_rank": ctl.max(float(ctl.rank)), "min_rank": ctl.min(float(ctl.rank)),
           "sum_ones": ctl.sum(1.0), "uid_ok": ctl.sum(1.0 if uid == bytes(range(128)) else 0.0) == ctl.world}
    ctl.barrier()
    if ctl.rank == 0:
        print(json.dumps(out), flush=True)


def run_with_env(env, *a, **kw):
    """A Run with some QLX_* switches set while its learner is built (the switches are read per model / learner)."""
    prev = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return Run(*a, **kw)
    finally:
        for k, v in prev.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


def main():
    args = parse()
    if args.no_target_memo:
        os.environ["QLX_TARGET_CACHE"] = "0"
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))
    ctl = Control()
    assert ctl.world == args.gpus, f"--gpus {args.gpus} but WORLD_SIZE {ctl.world}"
    if args.control_only:
        control_check(ctl)
        return
    assert args.batch % args.replay_ratio == 0
    import qlx
    flags = (qlx.DOUBLE_DQN if args.double_dqn else 0) | (qlx.PER if args.per else 0)
    f32 = args.precision == "fp32"
    head = Run(args, ctl, args.precision, args.steps, args.warmup, flags, args.sparsity_steps if f32 else 0)
    nomemo = None
    if args.nomemo_steps > 0 and "target_memo" in head.comps:
        # the reference's per-batch target work (same values, tests/test_gpu_learner.py), measured in this run
        nomemo = run_with_env({"QLX_TARGET_CACHE": "0"}, args, ctl, args.precision, args.nomemo_steps, 1, flags)
        assert "target_memo" not in nomemo.comps
    dense = None
    if f32 and args.dense_steps > 0:
        # the same loop on a learner built with the exact zero skips off (every conv1 step, every conv2 / conv3 row)
        dense = run_with_env({"QLX_F32_BG": "0", "QLX_F32_C1_SKIP": "0"}, args, ctl, "fp32", args.dense_steps, 1, flags)
    refwork = None
    if f32 and args.refwork_steps > 0 and not args.no_target_memo:
        # the reference's whole work: the target forward per sampled batch and every dense conv step / row
        refwork = run_with_env({"QLX_TARGET_CACHE": "0", "QLX_F32_BG": "0", "QLX_F32_C1_SKIP": "0"}, args, ctl, "fp32",
                               args.refwork_steps, 1, flags)
        assert "target_memo" not in refwork.comps
    dp1 = None
    if ctl.world == 1 and args.dp1_steps > 0:
        dp1 = Run(args, ctl, args.precision, args.dp1_steps, 1, flags, dp1=True)
    c5 = None
    if ctl.world == 1 and args.c5_steps > 0 and flags == 0:
        # C5's per-GPU shard: the same workload with double-DQN targets and proportional prioritized replay (fp32)
        c5 = Run(args, ctl, "fp32", args.c5_steps, 1, qlx.DOUBLE_DQN | qlx.PER)
    other = "bf16" if args.precision == "fp32" else "fp32"
    beside = Run(args, ctl, other, args.beside_steps, 1, flags, args.sparsity_steps if other == "fp32" else 0) \
        if args.beside_steps > 0 else None
    # the measured window is the steady-state loop: greedy acting and episode ends inside it
    assert "act_forward" in head.comps, "acting forward missing from the measured loop"
    assert head.episodes > 0, "no episode ended inside the timed window"
    if ctl.rank != 0:
        return
    N, B = args.envs, args.batch
    label = config_label(N, args.replay, flags, ctl.world)
    comps = {k: {kk: round(vv, 3) for kk, vv in v.items() if kk != "work"}
             for k, v in sorted(head.comps.items(), key=lambda kv: -kv[1]["total_us_per_step"])}
    line = {
        "metric": METRIC,
        "value": round(head.value(), 1),
        "unit": "env-steps/s",
        "n_gpus": ctl.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(head.dt / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.precision,
        "data": "synthetic: frames rendered by the batched Breakout env kernel from live play; random-init "
                "(GlorotUniform) Nature-DQN; replay prefilled to capacity before timing",
        "config": {"workload": f"{label}: {N} Breakout envs per GPU, replay {args.replay} per GPU in HBM (prefilled), "
                               f"Nature-DQN (3 conv + 2 dense) in {args.precision}, B={B}, update every {head.ua} "
                               f"env-steps per GPU (replay ratio {args.replay_ratio} samples/env-step), epsilon-greedy "
                               f"acting" + (" + double-DQN" if args.double_dqn else "")
                               + (" + prioritized replay" if args.per else ""),
                   "envs_per_gpu": N, "batch": B, "replay_capacity": args.replay, "update_after_actions": head.ua,
                   "parallelism": f"dp{ctl.world}" if ctl.world > 1 else "single", "rccl_world": head.rccl_world,
                   "global_batch_per_update": B * head.rccl_world,
                   "target_memo": "target_memo" in head.comps,
                   "env_dtype": "fp32 physics, u8 frames",
                   "qnet_dtype": "fp32 (exact-fp32 MFMA v_mfma_f32_16x16x4_f32)" if args.precision == "fp32"
                   else "bf16 MFMA operands, fp32 accumulate + master weights"},
        "grad_updates_per_sec": round(head.updates / head.dt, 2),
        "samples_per_sec": round(head.updates * B * ctl.world / head.dt, 1),
        "replay_ratio": args.replay_ratio,
        "roofline": head.roofline(),
        **head.report(),
        "steady_state": {"prefill_vector_steps": head.prefill, "episodes_in_window": head.episodes,
                         "episode_ends_per_step": round(head.ends_per_step, 2),
                         "expected_ends_per_step": round(head.expect_ends * ctl.world, 2),
                         "mean_episode_env_steps": round(head.mean_len, 1), "steady": head.steady_ok,
                         "steady_window": head.steady_window,
                         "episodes_total": head.episodes_total, "epsilon": round(head.epsilon, 4),
                         "running_reward": head.running_reward, "last_loss": head.last_loss},
        "components_event_timed": comps,
    }
    if nomemo is not None:
        line["value_no_target_memo"] = round(nomemo.value(), 1)
        line["no_target_memo"] = {
            "value": round(nomemo.value(), 1), "unit": "env-steps/s", "steps": nomemo.steps,
            "ms_per_step": round(nomemo.dt / nomemo.steps * 1e3, 3), "episodes_in_window": nomemo.episodes,
            "grad_updates_per_sec": round(nomemo.updates / nomemo.dt, 2),
            "note": "same loop and precision with the frozen target net evaluated per sampled batch (U*B target forwards "
                    "per vector step, the reference's work: self_driving_tf_q_learner.rs:189-199) instead of once per "
                    "transition at insertion; identical targets (tests/test_gpu_learner.py)"}
    if dense is not None:
        line["value_dense_frames"] = round(dense.value(), 1)
        line["dense_frames"] = {
            "value": round(dense.value(), 1), "unit": "env-steps/s", "steps": dense.steps,
            "ms_per_step": round(dense.dt / dense.steps * 1e3, 3), "grad_updates_per_sec": round(dense.updates / dense.dt, 2),
            "note": "fp32 with the exact zero skips off (QLX_F32_BG=0 QLX_F32_C1_SKIP=0, a learner built so in this run): "
                    "every conv1 MFMA step and every conv2 / conv3 row computed - the rate on frames without black "
                    "background; bit-identical results (tests/test_gpu_qnet32_paths.py)"}
    if refwork is not None:
        line["value_reference_work"] = round(refwork.value(), 1)
        line["reference_work"] = {
            "value": round(refwork.value(), 1), "unit": "env-steps/s", "steps": refwork.steps,
            "ms_per_step": round(refwork.dt / refwork.steps * 1e3, 3),
            "grad_updates_per_sec": round(refwork.updates / refwork.dt, 2),
            "note": "fp32 doing the reference's whole work: the frozen target net evaluated per sampled batch (no memo) AND the "
                    "exact zero skips off (QLX_TARGET_CACHE=0 QLX_F32_BG=0 QLX_F32_C1_SKIP=0, a learner built so in this "
                    "run); identical results"}
    if dp1 is not None:
        def per_update(run, names):
            return {n: round(run.comps[n]["avg_us"], 2) for n in names if n in run.comps}
        tail_plain = ("f32_wgrad_reduce", "f32_adam") if f32 else ("wgrad_reduce", "adam")
        tail_dp = ("allreduce_dense", "f32_norms", "allreduce_conv", "f32_wgrad_reduce", "f32_adam") if f32 else \
            ("allreduce_dense", "allreduce_conv", "wgrad_reduce", "norms", "adam")
        line["value_dp_single_rank"] = round(dp1.value(), 1)
        line["dp_single_rank"] = {
            "value": round(dp1.value(), 1), "unit": "env-steps/s", "steps": dp1.steps,
            "ms_per_step": round(dp1.dt / dp1.steps * 1e3, 3), "vs_plain": round(dp1.value() / head.value(), 4),
            "rccl_world": dp1.rccl_world,
            "per_update_us_event_timed": {"dp": per_update(dp1, tail_dp), "plain": per_update(head, tail_plain)},
            "note": "the same workload with the learner on a single-rank RCCL communicator (qlx_learner_dist_init(1, 0)): "
                    "the data-parallel update path - dense bucket all-reduced on the communicator stream beside the conv "
                    "backward, its clip-norm partials after it there, conv bucket all-reduced on the learner stream, the "
                    "k_update32 tail - whose per-rank cost C4 pays besides the xGMI transfer; bit-identical to the plain "
                    "path at world 1 (tests/test_gpu_learner.py)"}
    if c5 is not None:
        upd = c5.updates / max(c5.steps, 1)
        per_scopes = ("sample", "per_tree_build", "per_draw", "gather", "priorities", "per_push")
        line["value_c5_shard"] = round(c5.value(), 1)
        line["c5_shard"] = {
            "value": round(c5.value(), 1), "unit": "env-steps/s", "steps": c5.steps,
            "ms_per_step": round(c5.dt / c5.steps * 1e3, 3), "grad_updates_per_sec": round(c5.updates / c5.dt, 2),
            "episodes_in_window": c5.episodes, "config": config_label(N, args.replay, 3, 1),
            "per_update_us_event_timed": {
                n: round(c5.comps[n]["total_us_per_step"] / max(upd, 1e-9), 2) for n in per_scopes if n in c5.comps},
            "note": "C5's one-GPU shard (SURVEY 8(d)): the headline's envs, replay and batch with double-DQN targets (online "
                    "argmax over s', target-net value; the target net evaluated per sampled batch, so no memo) and "
                    "proportional prioritized replay (HBM f32 sum tree: per_tree_build = bottom-up rebuild, per_draw = "
                    "stratified draws + IS weights, priorities = |td| write-back, per_push = new leaves at max priority), "
                    "fp32, bit-exact vs the oracle (tests/test_gpu_per.py::test_f32_c5_shard); per-update figures = the "
                    "profile pass's per-step device time / updates per step"}
    if head.sparsity is not None:
        line["skipped_fractions"] = head.sparsity
    if beside is not None:
        line[f"{other}_beside"] = {
            "value": round(beside.value(), 1), "unit": "env-steps/s", "steps": beside.steps,
            "ms_per_step": round(beside.dt / beside.steps * 1e3, 3),
            "grad_updates_per_sec": round(beside.updates / beside.dt, 2), "roofline": beside.roofline(),
            "mfma_per_layer": beside.report()["mfma_per_layer"],
            "components_event_timed": {k: {"avg_us": round(v["avg_us"], 2), "launches_per_step": round(v["launches_per_step"], 2)}
                                       for k, v in sorted(beside.comps.items(), key=lambda kv: -kv[1]["total_us_per_step"])},
            "note": "bf16 MFMA operands, fp32 accumulation and master weights: the labelled fast path, not the reference's "
                    "arithmetic; its tolerance contract vs the fp32 oracle (DESIGN.md §6, tests/test_gpu_qnet_bf16.py): Q "
                    "<= 1.5e-2 and activations <= 3e-2 max|ref|, loss <= 3e-2 relative, per-variable gradients relative "
                    "L2 <= 0.13 with cosine >= 0.992" if other == "bf16"
            else "fp32: the reference's arithmetic"}
    if ctl.world == 1:
        log(f"cpu baseline: {args.cpu_sample} env-steps")
        line["cpu_baseline"] = cpu_baseline(args.cpu_sample)
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
