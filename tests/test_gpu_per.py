"""GPU double DQN + prioritized replay (per.hip, learner.hip flags) vs the oracle (oracle/learner_ref.h).

fp32 Q-net (qnet_precision 0, the default): EVERYTHING is bit-exact at every vector step, with no re-sync of the oracle -
actions, rewards, sampled indices (uniform under double DQN, proportional under PER), IS weights, double-DQN targets,
losses, every sum-tree leaf and per_max after the priority write, and the online / target weights and Adam slots at the
end.  Both sides evaluate the prioritized replay's x^y by the build's own definition (det_powf / per_powf),
so nothing depends on a library powf.
bf16 Q-net (qnet_precision 1, the labelled fast path): env and sampling exact; double-DQN targets within 3e-2 of max|y|
for >= 98 % of samples with the oracle re-synced before each step (an online-net argmax near-tie may pick the other
action); the first prioritized batch's priorities within 5e-2 relative.
Config C5's one-GPU shard (8,192 envs, 1M replay, DDQN + PER, target sync on): `test_f32_c5_shard`.
"""
import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu


def _qlx():
    import qlx
    return qlx


def same(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return a.shape == b.shape and a.tobytes() == b.tobytes()


@pytest.mark.parametrize("cap,length", [(1, 1), (3, 2), (1000, 1000), (5000, 3777), (70_000, 65_537)])
def test_sumtree_sample_matches_oracle(cap, length):
    qlx = _qlx()
    rng = np.random.default_rng(cap)
    leaves = np.zeros(cap, np.float32)
    leaves[:length] = (rng.gamma(0.4, 1.0, length) + 1e-6).astype(np.float32) ** 0.6
    if length > 10:
        leaves[rng.integers(0, length, length // 10)] = 0.0
    t = qlx.SumTree(cap)
    t.set_leaves(leaves)
    got_leaves, total, pmax = t.get()
    assert np.array_equal(got_leaves, leaves) and pmax == 1.0
    for B, U in ((1, 1), (64, 3), (300, 2)):
        s_ref, w_ref, t_ref = O.per_sample(leaves, 0xABC, 17, U, 2, length, 0.4, B)
        assert total == t_ref
        slots, w = t.sample(0xABC, 17, U, 2, length, 0.4, B)
        assert same(slots, s_ref), (B, U)
        assert same(w, w_ref), (B, U)
    with pytest.raises(qlx.QlError):
        t.sample(1, 0, 1, 0, cap + 1, 0.4, 8)


def test_sumtree_update_last_writer_wins():
    qlx = _qlx()
    cap = 1000
    t = qlx.SumTree(cap)
    t.set_leaves(np.ones(cap, np.float32))
    rng = np.random.default_rng(5)
    slots = rng.integers(0, 50, 400).astype(np.uint64)   # many repeats
    td = rng.random(400).astype(np.float32) * 3
    t.update(slots, td, 0.6, 1e-6)
    leaves, total, pmax = t.get()
    ref = np.ones(cap, np.float32)
    pr = O.det_powf(td + np.float32(1e-6), 0.6)
    for k in range(400):
        ref[slots[k]] = pr[k]
    assert same(leaves, ref)
    assert pmax == max(np.float32(1.0), pr.max())
    _, _, t_ref = O.per_sample(leaves, 0, 0, 1, 0, cap, 0.4, 1)
    assert total == t_ref


def make(flags, N=16, B=32, prec=0, **kw):
    qlx = _qlx()
    p = dict(n_envs=N, batch_size=B, history_buffer_len=3000, update_after_actions=4, epsilon_pure_random_steps=50_000,
             max_steps_per_episode=45, target_sync_steps=0, flags=flags, qnet_precision=prec)
    p.update(kw)
    return qlx.SelfDrivingQLearner(qlx.Parameter(**p)), O.Learner(O.default_params(**p))


def assert_models_equal(gpu_model, ref_qnet):
    for var in range(10):
        for which in range(3):
            assert same(gpu_model.get(var, which), ref_qnet.get(var, which)), (var, which)


def run_lockstep(gpu, ref, steps, per):
    """Both learners in lockstep, no re-sync: every per-step output and the replay priorities equal bit for bit."""
    n_updates = 0
    for v in range(steps):
        gpu.vector_step()
        ref.vector_step()
        g, r = gpu.last(), ref.last()
        for k in ("actions", "rewards", "dones", "indices", "targets", "losses"):
            assert same(g[k], r[k]), f"{k} differ @ vector step {v}"
        n_updates += len(r["losses"])
        if per:
            wg, lg, pg = gpu.priorities()
            wr, lr, pr = ref.priorities()
            assert same(wg, wr), f"IS weights @ {v}"
            assert same(lg, lr), f"sum-tree leaves @ {v}"
            assert pg == pr, f"per_max @ {v}"
    sg, sr = gpu.stats(), ref.counters()
    for k in ("step_count", "update_count", "episode_count", "replay_len"):
        assert sg[k] == sr[k], k
    return n_updates


def test_f32_double_dqn_learner_bit_exact():
    """Double DQN on the fp32 path: y = r + gamma Q_target(s', argmax Q_online(s')) with the online net as it stands
    before the vector step's updates; 4 updates per vector step, 32 steps, no re-sync."""
    qlx = _qlx()
    gpu, ref = make(qlx.DOUBLE_DQN)
    n = run_lockstep(gpu, ref, 32, per=False)
    assert n >= 100
    assert_models_equal(gpu.model, ref.qnet(0))
    assert_models_equal(gpu.stabilized_model, ref.qnet(1))


def test_f32_double_dqn_with_target_sync_bit_exact():
    """Double DQN with the target net synced every 64 env-steps (between vector steps, as the oracle does)."""
    qlx = _qlx()
    gpu, ref = make(qlx.DOUBLE_DQN, target_sync_steps=64)
    n = run_lockstep(gpu, ref, 24, per=False)
    assert n >= 60
    assert_models_equal(gpu.model, ref.qnet(0))
    assert_models_equal(gpu.stabilized_model, ref.qnet(1))


@pytest.mark.parametrize("ua", [16, 4])
def test_f32_prioritized_learner_bit_exact(ua):
    """PER + double DQN on the fp32 path: proportional draws, IS weights, the weighted Huber loss and its gradients,
    the |td| priorities written back (a slot drawn twice keeps its last draw's value: with 4 updates of 32 draws per
    vector step from a few hundred transitions, repeats are frequent), per_max, all bit for bit at every step."""
    qlx = _qlx()
    gpu, ref = make(qlx.PER | qlx.DOUBLE_DQN, update_after_actions=ua)
    n = run_lockstep(gpu, ref, 40, per=True)
    assert n >= (30 if ua == 16 else 150)
    _, leaves, _ = gpu.priorities()
    assert (leaves[leaves > 0] != 1.0).any()   # priorities were written (not only the initial 1)
    assert_models_equal(gpu.model, ref.qnet(0))


def test_bf16_double_dqn_learner_parity():
    """bf16 Q-net: before each vector step the oracle's online net is re-synced to the product's weights, so the
    double-DQN argmax on both sides comes from the same weights (the nets otherwise drift apart after the first update:
    Adam's sign-like first steps turn bf16 gradient noise into lr-sized steps)."""
    qlx = _qlx()
    gpu, ref = make(qlx.DOUBLE_DQN, prec=1)
    ref_online = ref.qnet(0)
    n, close = 0, 0
    for v in range(24):
        ref_online.load_state_from(gpu.model)
        gpu.vector_step()
        ref.vector_step()
        g, r = gpu.last(), ref.last()
        assert np.array_equal(g["actions"], r["actions"]) and np.array_equal(g["rewards"], r["rewards"])
        assert np.array_equal(g["indices"], r["indices"]), v
        if len(r["losses"]):
            tg, tr = g["targets"], r["targets"]
            n += tg.size
            close += int((np.abs(tg - tr) <= 3e-2 * max(1.0, np.abs(tr).max())).sum())
            assert np.isfinite(g["losses"]).all()
    assert n > 1000 and close >= 0.98 * n, (close, n)


def test_bf16_prioritized_learner_parity():
    qlx = _qlx()
    gpu, ref = make(qlx.PER | qlx.DOUBLE_DQN, prec=1, update_after_actions=16)
    first = None
    for v in range(40):
        gpu.vector_step()
        ref.vector_step()
        g, r = gpu.last(), ref.last()
        if not len(r["losses"]):
            continue
        wg, lg, pg = gpu.priorities()
        wr, lr, pr = ref.priorities()
        if first is None:   # all stored transitions entered at priority 1: same uniform draws, unit weights
            first = v
            assert np.array_equal(g["indices"], r["indices"])
            assert (wg == 1.0).all() and (wr == 1.0).all()
            # one update per vector step: its priorities from the TD errors of the same batch on identical weights,
            # through the bf16 network
            live = lr > 0
            assert np.array_equal(lg > 0, live)
            assert np.allclose(lg[live], lr[live], rtol=5e-2, atol=1e-2)
        for w, leaves, pmax in ((wg, lg, pg), (wr, lr, pr)):
            assert ((w > 0) & (w <= 1)).all() and (w.max(axis=1) == 1.0).all()
            assert pmax >= leaves.max() * (1 - 1e-6)
        assert (g["indices"] < gpu.stats()["replay_len"]).all()
    assert first is not None
    sg, sr = gpu.stats(), ref.counters()
    for k in ("step_count", "update_count", "replay_len"):
        assert sg[k] == sr[k], k


def test_f32_c5_shard():
    """Config C5's one-GPU shard (65,536 envs over 8 GPUs = 8,192 per rank): 8,192 envs, replay 1,000,000
    filled to capacity, B = 1,024, replay ratio 8 (64 updates per vector step), double DQN + prioritized replay, target
    sync every 32,768 env-steps.  The oracle cannot hold 1M state pairs, so, bit for bit: the prefill leaves every leaf at
    priority 1; all 64 updates' proportional draws and IS weights = the oracle sampler over the product's leaves; the first
    update's double-DQN targets and loss = the fp32 oracle nets (online and target weights as they stood before the step)
    fed the product's own gathered transitions; the priorities of the slots whose last draw was in update 0 =
    det_powf(|Q_online(s)[a] - y| + eps, alpha) of those values."""
    qlx = _qlx()
    N, B, cap = 8192, 1024, 1_000_000
    p = qlx.Parameter(n_envs=N, batch_size=B, history_buffer_len=cap, update_after_actions=128,
                      epsilon_pure_random_steps=123 * N, epsilon_greedy_steps=1_000_000.0, stats_after_steps=0,
                      target_sync_steps=4 * N, flags=qlx.PER | qlx.DOUBLE_DQN)
    L = qlx.SelfDrivingQLearner(p)
    L.prefill(123)
    st = L.stats()
    assert st["replay_len"] == cap and st["update_count"] == 0
    _, leaves0, pmax0 = L.priorities()
    assert (leaves0 == 1.0).all() and pmax0 == 1.0
    w0 = [[L.model.get(v, which) for which in range(3)] for v in range(10)]
    tw = [L.stabilized_model.get(v) for v in range(10)]
    L.vector_step()
    g = L.last()
    assert g["losses"].shape[0] == 64
    isw, leaves1, pmax1 = L.priorities()
    total_pushed = 124 * N
    start = (total_pushed - cap) % cap
    # the step's pushes enter at per_max = 1 before the draws: the sampled tree is all ones
    ref_slots, ref_w, total = O.per_sample(np.ones(cap, np.float32), p.learner_seed, 0, 64, 0, cap, p.per_beta, B)
    assert total == np.float32(cap)
    ref_idx = (ref_slots + np.uint64(cap - start)) % np.uint64(cap)
    assert same(g["indices"], ref_idx)
    assert same(isw, ref_w) and (isw == 1.0).all()
    online = O.QNet(seed=1, f32=True)
    target = O.QNet(seed=1, f32=True)
    for v in range(10):
        target.set(v, tw[v])
        for which in range(3):
            online.set(v, w0[v][which], which)
    batch = L.replay_buffer.get_many(g["indices"][0])
    qt = target.forward(batch["state_next"])
    qo = online.forward(batch["state_next"])
    a_star = np.argmax(qo, axis=1)
    v_sel = qt[np.arange(B), a_star]
    y = np.where(batch["done"], batch["reward"],
                 (batch["reward"] + (v_sel * np.float32(p.gamma)).astype(np.float32)).astype(np.float32)).astype(np.float32)
    assert same(g["targets"][0], y), "double-DQN targets of update 0"
    q_s = online.forward(batch["state"])
    loss, _, _ = online.train(batch["state"], batch["action"], y)
    assert same(np.float32(loss), g["losses"][0])
    td = np.abs((q_s[np.arange(B), batch["action"].astype(np.int64)] - y).astype(np.float32))
    pr = O.det_powf(td + np.float32(p.per_eps), p.per_alpha)
    flat = g["indices"].reshape(-1)
    last_draw = {}
    for k, i in enumerate(flat.tolist()):
        last_draw[i] = k
    slots0 = [(i, k) for i, k in last_draw.items() if k < B]
    assert len(slots0) > 100
    for i, k in slots0:
        assert leaves1[(start + i) % cap] == pr[k], (i, k)
    assert pmax1 >= pr.max()
