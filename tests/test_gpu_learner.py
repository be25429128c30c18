"""GPU SelfDrivingQLearner (vector steps) vs the oracle's sequential restatement.

fp32 (qnet_precision = QLX_PREC_F32, the reference's arithmetic; the default): EVERYTHING is bit-exact - actions
(random and greedy), env rewards / dones / mechanics, replay contents, sampled indices, Bellman targets, losses, the
online weights and Adam slots after any number of updates (the Q-net is one fmaf chain per output in the order
DESIGN.md §6 defines, tests/test_gpu_qnet32.py).
bf16 (QLX_PREC_BF16, the labelled fast path): env / replay / indices exact; targets and losses within the stated
bf16 tolerances (3e-2 of max|y|; lockstep losses 10 %).
"""
import hashlib
import os

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu


def _qlx():
    import qlx
    return qlx


def make(N, B, prec=0, **kw):
    qlx = _qlx()
    p = dict(n_envs=N, batch_size=B, history_buffer_len=3000, update_after_actions=4,
             epsilon_pure_random_steps=50_000, max_steps_per_episode=10_000, qnet_precision=prec)
    p.update(kw)
    return qlx.SelfDrivingQLearner(qlx.Parameter(**p)), O.Learner(O.default_params(**p))


def same(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return a.shape == b.shape and a.tobytes() == b.tobytes()


def assert_step_equal(g, r, v):
    for k in ("actions", "rewards", "dones", "indices", "targets", "losses"):
        assert same(g[k], r[k]), f"{k} differ @ vector step {v}"


def assert_models_equal(gpu_model, ref_qnet):
    for var in range(10):
        for which in range(3):
            assert same(gpu_model.get(var, which), ref_qnet.get(var, which)), (var, which)


def test_f32_pure_random_phase_bit_exact():
    N, B = 16, 32
    gpu, ref = make(N, B, max_steps_per_episode=45)
    n_updates = 0
    for v in range(30):
        gpu.vector_step()
        ref.vector_step()
        g, r = gpu.last(), ref.last()
        assert_step_equal(g, r, v)
        n_updates += len(r["losses"])
    assert n_updates > 50
    assert_models_equal(gpu.model, ref.qnet(0))
    sg, sr = gpu.stats(), ref.counters()
    for k in ("step_count", "update_count", "episode_count", "replay_len"):
        assert sg[k] == sr[k], k
    assert sg["running_reward"] == sr["running_reward"] and sg["epsilon"] == sr["epsilon"]


def test_f32_greedy_phase_bit_exact():
    """Greedy acting from the online net while it learns: the acting forward, argmax, every update and the
    resulting trajectories stay identical (epsilon 0.3 -> 0.05 over the run, one update per 16 env-steps)."""
    N, B = 64, 32
    gpu, ref = make(N, B, epsilon_pure_random_steps=200, epsilon_max=0.3, epsilon_min=0.05, epsilon_greedy_steps=2000.0,
                    update_after_actions=16, max_steps_per_episode=200)
    greedy = 0
    for v in range(24):
        gpu.vector_step()
        ref.vector_step()
        g, r = gpu.last(), ref.last()
        assert_step_equal(g, r, v)
        greedy += int(len(r["q"]) > 0)
    assert greedy >= 20
    assert_models_equal(gpu.model, ref.qnet(0))
    mech = gpu.environment.mechanics()
    for e in range(N):
        ro = ref.env_state(e)
        for k in O.STATE_DTYPE.names:
            assert mech[k][e] == ro[k], (e, k)


def test_f32_c2_config_bit_exact():
    """Config C2: 1,024 envs, replay 100,000 filled to capacity (98 prefill vector steps, the FIFO
    wraps), B = 1,024, replay ratio 8 (update every 128 env-steps); then 2 full vector steps (16 updates, greedy
    acting at epsilon ~0.1) compared bit for bit."""
    N, B = 1024, 1024
    kw = dict(history_buffer_len=100_000, update_after_actions=128, epsilon_pure_random_steps=98 * 1024,
              epsilon_greedy_steps=100_000.0, stats_after_steps=0)
    gpu, ref = make(N, B, **kw)
    gpu.prefill(98)
    ref.prefill(98)
    assert gpu.stats()["replay_len"] == ref.counters()["replay_len"] == 100_000
    for v in range(2):
        gpu.vector_step()
        ref.vector_step()
        g, r = gpu.last(), ref.last()
        assert len(r["losses"]) == 8
        assert_step_equal(g, r, v)
    assert_models_equal(gpu.model, ref.qnet(0))


def test_f32_c3_config():
    """Config C3: 8,192 envs, replay 1,000,000 filled to capacity, B = 1,024 (64 updates per vector step).  The
    oracle cannot hold 1M state pairs, so: sampled indices of all 64 updates = the sequential sampler at len 1M
    (bit-exact); the Bellman targets of the first two updates and the first update's loss, gradients and weights =
    the fp32 oracle fed the product's own gathered transitions and pre-step weights (bit-exact)."""
    qlx = _qlx()
    N, B = 8192, 1024
    p = qlx.Parameter(n_envs=N, batch_size=B, history_buffer_len=1_000_000, update_after_actions=128,
                      epsilon_pure_random_steps=123 * N, epsilon_greedy_steps=1_000_000.0, stats_after_steps=0)
    L = qlx.SelfDrivingQLearner(p)
    L.prefill(123)
    st = L.stats()
    assert st["replay_len"] == 1_000_000 and st["update_count"] == 0
    w0 = [[L.model.get(v, which) for which in range(3)] for v in range(10)]
    tw = [L.stabilized_model.get(v) for v in range(10)]
    L.vector_step()
    g = L.last()
    assert g["losses"].shape[0] == 64
    for u in range(64):
        ref_idx = O.sample_distinct(p.learner_seed, u, 0, 1_000_000, B)
        assert same(g["indices"][u], ref_idx), f"update {u} indices"
    tnet = O.QNet(seed=1, f32=True)
    for v in range(10):
        tnet.set(v, tw[v])
    for u in range(2):
        batch = L.replay_buffer.get_many(g["indices"][u])
        q = tnet.forward(batch["state_next"])
        y = np.where(batch["done"], batch["reward"],
                     (batch["reward"] + (q.max(axis=1) * np.float32(p.gamma)).astype(np.float32)).astype(np.float32))
        assert same(g["targets"][u], y.astype(np.float32)), f"targets of update {u}"
    online = O.QNet(seed=1, f32=True)
    for v in range(10):
        for which in range(3):
            online.set(v, w0[v][which], which)
    batch = L.replay_buffer.get_many(g["indices"][0])
    loss, _, _ = online.train(batch["state"], batch["action"], g["targets"][0])
    assert same(np.float32(loss), g["losses"][0])


# (n_envs, B, update_after_actions, replay, vector steps, step of the target-weight write): a tiny shape, and a C2-like one
# where the memo's chunks (n_envs = 1024 samples) and the per-batch pass (U * B = 8 * 1024) fall on different batch sizes
MEMO_SHAPES = {"tiny": (64, 32, 8, 1000, 30, 18), "c2like": (1024, 1024, 128, 20_000, 8, 5)}


@pytest.mark.parametrize("shape", sorted(MEMO_SHAPES))
@pytest.mark.parametrize("prec", [0, 1])
def test_target_memo_matches_per_batch_target_pass(monkeypatch, prec, shape):
    """The per-slot Bellman-target memo (default while the target net is frozen, learner.hip ycache_fill) gives the
    same targets, losses and weights as the per-batch target pass (QLX_TARGET_CACHE=0) - bit for bit, also across
    the replay FIFO wrap and after the target weights are overwritten mid-run (the memo is rebuilt for every slot)."""
    qlx = _qlx()
    N, B, ua, cap, steps, write_at = MEMO_SHAPES[shape]

    def run(cache):
        monkeypatch.setenv("QLX_TARGET_CACHE", "1" if cache else "0")
        p = qlx.Parameter(n_envs=N, batch_size=B, history_buffer_len=cap, update_after_actions=ua,
                          epsilon_pure_random_steps=400, epsilon_greedy_steps=2000.0, max_steps_per_episode=200,
                          stats_after_steps=0, qnet_precision=prec)
        L = qlx.SelfDrivingQLearner(p)
        out = []
        for v in range(steps):
            if v == write_at:
                w = L.stabilized_model.get(9)
                L.stabilized_model.set(9, (w + np.float32(0.01)).astype(np.float32))
            L.vector_step()
            g = L.last()
            out.append((g["targets"].copy(), g["losses"].copy()))
        return out, [L.model.get(v) for v in range(10)]

    memo, w_memo = run(True)
    plain, w_plain = run(False)
    for v, ((ym, lm), (yp, lp)) in enumerate(zip(memo, plain)):
        assert same(ym, yp), f"targets differ @ vector step {v}"
        assert same(lm, lp), f"losses differ @ vector step {v}"
    for a, b in zip(w_memo, w_plain):
        assert same(a, b)


C1_GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "c1_learner_f32.npz")


def test_f32_c1_reference_loop_golden():
    """Config C1: the reference loop itself - 1 env, Parameter::default(), B = 32, 10,000 env-steps
    (all random: 50k pure-random steps), 2,492 updates - on the GPU learner, against the fp32 oracle's run of the
    same loop committed as tests/golden/c1_learner_f32.npz (tests/golden/make_c1_golden.py): actions, rewards,
    dones and all 2,492 losses bit-exact; targets, indices and the final weights / Adam slots by SHA-256."""
    qlx = _qlx()
    gold = np.load(C1_GOLDEN, allow_pickle=False)
    L = qlx.SelfDrivingQLearner(qlx.Parameter(n_envs=1, batch_size=32))
    acts, rews, dones, losses = [], [], [], []
    h_idx, h_tg = hashlib.sha256(), hashlib.sha256()
    for _ in range(10_000):
        L.vector_step()
        g = L.last()
        acts.append(g["actions"][0]); rews.append(g["rewards"][0]); dones.append(g["dones"][0])
        if len(g["losses"]):
            losses.extend(g["losses"].tolist())
            h_idx.update(g["indices"].astype(np.uint64).tobytes())
            h_tg.update(g["targets"].astype(np.float32).tobytes())
    assert same(np.array(acts, np.uint8), gold["actions"])
    assert same(np.array(rews, np.float32), gold["rewards"])
    assert same(np.array(dones, np.uint8), gold["dones"])
    assert len(losses) == 2492
    assert same(np.array(losses, np.float32), gold["losses"])
    assert h_idx.hexdigest() == str(gold["indices_sha256"]) and h_tg.hexdigest() == str(gold["targets_sha256"])
    hw = hashlib.sha256()
    for v in range(10):
        for which in range(3):
            hw.update(L.model.get(v, which).astype(np.float32).tobytes())
    assert hw.hexdigest() == str(gold["model_sha256"])


def test_stats_events_and_checkpoint(tmp_path):
    """stats_after_steps (self_driving_tf_q_learner.rs:204-212): the learner writes its checkpoint and the
    learning_update_log once per vector step that crosses a multiple - same event count as the oracle; the file
    holds the online weights of that moment and the log text is the learning_update_log of that moment (before the
    first finished episode, where the reference's log would assert, the counters only)."""
    qlx = _qlx()
    path = str(tmp_path / "ql.ckpt")
    gpu, ref = make(32, 32, stats_after_steps=320, checkpoint_file=path, max_steps_per_episode=60, update_after_actions=8)
    seen, with_episodes = 0, 0
    for v in range(80):
        gpu.vector_step()
        ref.vector_step()
        assert gpu.stats_events() == ref.stats_events(), v
        if gpu.stats_events() > seen:
            seen = gpu.stats_events()
            log = gpu.last_log()
            if gpu.stats()["episode_count"] > 0:
                assert log == gpu.learning_update_log() and "reward_distribution" in log
                with_episodes += 1
            else:
                assert "no finished episode yet" in log
            m2 = qlx.DeepQLearningModel(seed=99)
            m2.read_checkpoint(path)
            for var in range(10):
                assert same(m2.get(var), gpu.model.get(var))
            m2.close()
    assert seen >= 8 and with_episodes >= 2


def test_solved_events_without_periodic_stats(tmp_path):
    """stats_after_steps = 0 turns off only the periodic event: solved() is still checked after every vector step in which
    an episode ended (self_driving_tf_q_learner.rs:226-230) and then writes the checkpoint and the log.  The goal is mocked
    (episode_reward_goal, a test double of Environment::episode_reward_goal_mean) so the random-init net reaches it:
    same event count as the oracle at every step, and the checkpoint holds the online weights of that moment."""
    qlx = _qlx()
    path = str(tmp_path / "solved.ckpt")
    gpu, ref = make(32, 32, stats_after_steps=0, checkpoint_file=path, max_steps_per_episode=15, update_after_actions=8,
                    episode_reward_goal=-1.0)
    fired = 0
    for v in range(40):
        gpu.vector_step()
        ref.vector_step()
        assert gpu.stats_events() == ref.stats_events(), v
        if gpu.stats_events() > fired:
            fired = gpu.stats_events()
            assert gpu.stats()["solved"] == 1 and "reward_distribution" in gpu.last_log()
            m2 = qlx.DeepQLearningModel(seed=99)
            m2.read_checkpoint(path)
            for var in range(10):
                assert same(m2.get(var), gpu.model.get(var))
            m2.close()
    assert fired >= 2


def test_end_episodes_is_the_truncation_path():
    """qlx_learner_end_episodes (the bench's staggered start): the masked envs' episodes end as at
    max_steps_per_episode - episode_count advances by the mask's count, their running episode rewards enter the
    history in env order, the envs reset (reset_count + 1, fresh state) - and the others are untouched; no transition."""
    N = 64
    gpu, _ = make(N, 32, max_steps_per_episode=10_000)
    for _ in range(12):
        gpu.vector_step()
    s0 = gpu.stats()
    mech0 = gpu.environment.mechanics()
    rewards0 = gpu.episode_rewards()
    mask = (np.arange(N) % 3 == 1).astype(np.uint8)
    gpu.end_episodes(mask)
    s1 = gpu.stats()
    mech1 = gpu.environment.mechanics()
    assert s1["episode_count"] == s0["episode_count"] + int(mask.sum())
    assert s1["replay_len"] == s0["replay_len"] and s1["step_count"] == s0["step_count"]
    for e in range(N):
        if mask[e]:
            assert mech1["reset_count"][e] == mech0["reset_count"][e] + 1, e
        else:
            assert all(mech1[k][e] == mech0[k][e] for k in O.STATE_DTYPE.names), e
    assert len(gpu.episode_rewards()) == min(100, len(rewards0) + int(mask.sum()))
    gpu.vector_step()   # the loop continues from there
    assert gpu.stats()["step_count"] == s0["step_count"] + N


def test_bf16_pure_random_phase_parity():
    """bf16 learner against the oracle in lockstep: before every vector step the oracle's online net takes the product's
    weights + Adam slots, so the first update of each step starts from identical state and its loss is held to a
    per-update bound (the later updates of a step start from weights that bf16 gradient noise has already moved: Adam's
    sign-like first steps turn it into full lr-sized steps); env, replay, sampling exact throughout."""
    N, B = 16, 32
    gpu, ref = make(N, B, prec=1, max_steps_per_episode=45)
    ref_online = ref.qnet(0)
    n_updates = 0
    rel_errs = []
    for v in range(30):
        ref_online.load_state_from(gpu.model)
        gpu.vector_step()
        ref.vector_step()
        g, r = gpu.last(), ref.last()
        assert np.array_equal(g["actions"], r["actions"]), f"actions @ {v}"
        assert np.array_equal(g["rewards"], r["rewards"]) and np.array_equal(g["dones"], r["dones"])
        assert np.array_equal(g["indices"], r["indices"]), f"indices @ {v}"
        if len(r["losses"]):
            n_updates += len(r["losses"])
            tg, tr = g["targets"], r["targets"]
            # the target net is never synced (reference behaviour): identical weights on both sides
            assert np.abs(tg - tr).max() <= 3e-2 * max(1.0, np.abs(tr).max()), f"targets @ {v}"
            assert np.isfinite(g["losses"]).all()
            # lockstep: the step's first update; |dloss| <= 0.1 max(|loss|, 0.1) (the bf16 forward's Q error, <= 3e-2
            # max|Q|, times the Huber gradient |e| <= 1 of the residual; the measured max is printed)
            rel = abs(g["losses"][0] - r["losses"][0]) / max(abs(r["losses"][0]), 0.1)
            rel_errs.append(rel)
            assert rel <= 0.1, (v, g["losses"][0], r["losses"][0])
    assert n_updates > 50
    print("bf16 lockstep loss error, max / mean of max(|loss|, 0.1):", max(rel_errs), np.mean(rel_errs))
    sg, sr = gpu.stats(), ref.counters()
    for k in ("step_count", "update_count", "episode_count", "replay_len"):
        assert sg[k] == sr[k], k
    assert sg["running_reward"] == sr["running_reward"]
    assert abs(sg["epsilon"] - sr["epsilon"]) == 0.0
    mech = gpu.environment.mechanics()
    for e in range(N):
        ro = ref.env_state(e)
        for k in O.STATE_DTYPE.names:
            assert mech[k][e] == ro[k], (e, k)
    obs = gpu.environment.state()
    for e in range(N):
        assert np.array_equal(obs[e], ref.env_tensor(e))
    idx = np.array([0, 1, 17, 100, 255, 400, sr["replay_len"] - 1], np.uint64)
    got = gpu.replay_buffer.get_many(idx)
    s, sn, a, rw, d = ref.replay_get(idx)
    assert np.array_equal(got["state"], s) and np.array_equal(got["state_next"], sn)
    assert np.array_equal(got["action"], a) and np.array_equal(got["reward"], rw)
    assert np.array_equal(got["done"].astype(np.uint8), d)


def test_bf16_lockstep_update_losses():
    """One update per vector step; before each step the oracle's online net is re-synced to the product's
    weights + Adam slots, so every loss is compared from identical state (Q-forward tolerance)."""
    N, B = 32, 32
    gpu, ref = make(N, B, prec=1, update_after_actions=N)
    ref_online = ref.qnet(0)
    n = 0
    for v in range(12):
        ref_online.load_state_from(gpu.model)
        gpu.vector_step()
        ref.vector_step()
        g, r = gpu.last(), ref.last()
        assert np.array_equal(g["indices"], r["indices"])
        if len(r["losses"]):
            n += 1
            # dloss ~ mean|e| * dq with dq <= 3e-2 max|Q|: bounded by 10% of the loss (or 0.01) here
            assert abs(g["losses"][0] - r["losses"][0]) <= 0.1 * max(abs(r["losses"][0]), 0.1), (v, g["losses"], r["losses"])
    assert n >= 10


def test_epsilon_random_branch_is_exact():
    # epsilon_max = epsilon_min = 1, no pure-random phase: every action comes from the epsilon branch
    gpu, ref = make(64, 32, epsilon_pure_random_steps=0, epsilon_max=1.0, epsilon_min=1.0)
    for _ in range(3):
        gpu.vector_step()
        ref.vector_step()
        assert np.array_equal(gpu.last()["actions"], ref.last()["actions"])


def test_bf16_greedy_actions_match_where_margin_is_clear():
    gpu, ref = make(128, 32, prec=1, epsilon_pure_random_steps=0, epsilon_max=0.0, epsilon_min=0.0)
    checked = 0
    for _ in range(4):       # early steps: weights identical or one update apart
        obs = gpu.environment.state()
        q_gpu, _ = gpu.model.q_values(obs)          # the product's own Q with the acting weights
        gpu.vector_step()
        ref.vector_step()
        ga, r = gpu.last()["actions"], ref.last()
        # (1) greedy selection = tf.argmax (first maximal index) of the product's Q, exactly
        assert np.array_equal(ga, np.argmax(q_gpu, axis=1).astype(np.uint8))
        if gpu.stats()["update_count"] > 0:
            break
        # (2) product Q vs oracle Q within the forward tolerance; actions equal where the oracle's
        # top-2 margin exceeds twice the observed Q error
        q = r["q"]
        assert np.abs(q_gpu - q).max() <= 3e-2 * np.abs(q).max()
        err_e = np.abs(q_gpu - q).max(axis=1)
        srt = np.sort(q, axis=1)
        sure = (srt[:, -1] - srt[:, -2]) > 2 * err_e
        checked += int(sure.sum())
        assert np.array_equal(ga[sure], r["actions"][sure])
        if not np.array_equal(ga, r["actions"]):
            break   # a near-tie flipped: the envs diverge from here on by construction


def test_learner_runs_many_steps_without_faults():
    qlx = _qlx()
    p = qlx.Parameter(n_envs=256, batch_size=64, history_buffer_len=20_000, update_after_actions=64,
                      epsilon_pure_random_steps=1000, epsilon_greedy_steps=5000.0, target_sync_steps=2000)
    L = qlx.SelfDrivingQLearner(p)
    L.run(60)
    st = L.stats()
    assert st["step_count"] == 60 * 256 and st["update_count"] > 100
    assert np.isfinite(st["last_loss"])
    assert (L.environment.mechanics()["fault"] == 0).all()
    w = L.model.get(6)
    assert np.isfinite(w).all()


@pytest.mark.parametrize("prec,fold", [(0, "1"), (0, "0"), (1, "1")], ids=["fp32", "fp32_norms_launch", "bf16"])
@pytest.mark.parametrize("overlap", ["1", "0"], ids=["two_buckets", "one_allreduce"])
def test_data_parallel_path_single_rank_bit_identical(monkeypatch, overlap, prec, fold):
    """The data-parallel update path on a single-rank RCCL communicator equals the plain single-GPU path bit for bit, in
    both precisions and both DP schedules: QLX_DP_OVERLAP=1 (the default: dense gradient bucket all-reduced on the
    communicator's stream while the conv backward runs; fp32: its clip-norm partials in the conv backward's reduction launch
    once it has landed, or with QLX_DP_FOLD=0 in a launch of their own on the communicator stream; then the conv bucket,
    the update tail after both) and QLX_DP_OVERLAP=0 (one whole-gradient all-reduce after the backward, then the tail): the stream
    hand-offs order every read and write.  (At world 1 the tail's scale is exactly 1; scale != 1 is
    test_update_tail_scaled_gradient.)"""
    qlx = _qlx()
    monkeypatch.setenv("QLX_DP_OVERLAP", overlap)   # read by dist_init
    monkeypatch.setenv("QLX_DP_FOLD", fold)         # fp32: dense norm partials in the reduction launch (1) or their own (0)
    p = dict(n_envs=64, batch_size=64, history_buffer_len=4000, update_after_actions=16, epsilon_pure_random_steps=1000,
             max_steps_per_episode=300, qnet_precision=prec)
    plain = qlx.SelfDrivingQLearner(qlx.Parameter(**p))
    dp = qlx.SelfDrivingQLearner(qlx.Parameter(**p))
    dp.dist_init(1, 0, qlx.dist_unique_id())
    for v in range(25):
        plain.vector_step()
        dp.vector_step()
        a, b = plain.last(), dp.last()
        assert np.array_equal(a["actions"], b["actions"]) and np.array_equal(a["indices"], b["indices"]), v
        assert np.array_equal(a["losses"], b["losses"]), v
    for var in range(10):
        for which in range(3):
            assert np.array_equal(plain.model.get(var, which), dp.model.get(var, which)), (var, which)
    assert plain.stats()["update_count"] == dp.stats()["update_count"] > 50


@pytest.mark.parametrize("scale", [0.5, 0.25, 1.0 / 3.0, 1.0 / 8.0, 1.0])
def test_update_tail_scaled_gradient(scale):
    """The update tail a data-parallel rank runs after the all-reduce (learner.hip learner_update: model_norms +
    model_adam at scale = 1 / world) on a known gradient, bit for bit against the oracle's clip_by_norm(g * scale) + legacy
    Adam (oracle/qnet32_ref.cpp, orc_qnet32_apply - the definition tests/test_dist_cpu.py's world-2 restatement uses):
    three consecutive updates with different gradients, clip norms and w / m / v after each.  The gradients are the
    oracle's own chain gradients of a batch, so some variables clip (norm > 1) and some do not."""
    qlx = _qlx()
    ref = O.QNet(seed=31, f32=True)
    gpu = qlx.DeepQLearningModel(seed=31)
    for v in range(10):
        gpu.set(v, ref.get(v, 0))
    rng = np.random.default_rng(77)
    x = rng.integers(0, 256, (64, 84, 84, 4), dtype=np.uint8)
    x[:, 20:60] = 0
    a = rng.integers(0, 3, 64).astype(np.uint8)
    for t in range(3):
        scratch = O.QNet(seed=31, f32=True)
        scratch.load_state_from(ref)
        y = rng.normal(0, 4.0 * (t + 1), 64).astype(np.float32)
        _, grads, _ = scratch.train(x, a, y)
        flat = np.concatenate([g.ravel() for g in grads]).astype(np.float32) * np.float32(3.0 - t)
        want = O.qnet32_apply(ref, flat, np.float32(scale))
        got = gpu.apply_gradient(flat, scale)
        assert same(got, want), (t, got, want)
        assert (want > 1.0).any() and (want < 1.0).any(), want   # both sides of clip_by_norm exercised
        for var in range(10):
            for which in range(3):
                assert same(gpu.get(var, which), ref.get(var, which)), (scale, t, var, which)
    assert gpu.iterations() == ref.iterations() == 3


def test_invalid_parameters_fail_loudly():
    """Bad parameters are rejected with the library's message (QlError), like the reference's Result errors; the
    create path releases whatever it built before failing (repeated failures do not accumulate device memory)."""
    qlx = _qlx()
    bad = [dict(n_envs=0), dict(batch_size=0), dict(update_after_actions=0), dict(history_buffer_len=8, batch_size=32),
           dict(episode_reward_history_buffer_len=0), dict(flags=8), dict(flags=qlx.PER, per_eps=0.0)]
    for kw in bad:
        p = dict(n_envs=16, batch_size=32, history_buffer_len=1000)
        p.update(kw)
        for cls in (qlx.SelfDrivingQLearner, qlx.BallGameLearner):
            with pytest.raises(qlx.QlError):
                cls(qlx.Parameter(**p))
    import torch
    free0 = torch.cuda.mem_get_info()[0]
    for _ in range(20):   # fails after env, replay and both models were built
        with pytest.raises(qlx.QlError):
            qlx.SelfDrivingQLearner(qlx.Parameter(n_envs=16, batch_size=32, history_buffer_len=1000, flags=qlx.PER,
                                                  per_eps=-1.0))
    assert torch.cuda.mem_get_info()[0] >= free0 - (64 << 20)
