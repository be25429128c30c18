"""GPU double DQN + prioritized replay (per.hip, learner.hip flags) vs the oracle (oracle/learner_ref.h).

Bit-exact: the HBM sum tree's total and the proportional stratified draws (physical slots) for the same leaves
and stream; last-writer-wins priority updates; the first prioritized batches of a learner (all leaves at the
initial max priority) and its uniform-sampling indices under double DQN.
Within tolerance: IS weights 1e-6 relative (device powf vs glibc powf); priorities (|td| + eps)^alpha from the
bf16 network's TD errors, 5e-2 relative; double-DQN targets within 3e-2 of max|y| for at least 98% of samples
(an online-net argmax near-tie may pick the other action on the two sides).
"""
import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu


def _qlx():
    import qlx
    return qlx


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
        assert np.array_equal(slots, s_ref), (B, U)
        assert np.allclose(w, w_ref, rtol=1e-6, atol=0), (B, U)
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
    pr = np.power(td + np.float32(1e-6), np.float32(0.6), dtype=np.float32)
    for k in range(400):
        ref[slots[k]] = pr[k]
    assert np.allclose(leaves, ref, rtol=1e-6, atol=0)
    assert np.isclose(pmax, max(1.0, pr.max()), rtol=1e-6)
    _, _, t_ref = O.per_sample(leaves, 0, 0, 1, 0, cap, 0.4, 1)
    assert total == t_ref


def make(flags, N=16, B=32, **kw):
    qlx = _qlx()
    p = dict(n_envs=N, batch_size=B, history_buffer_len=3000, update_after_actions=4, epsilon_pure_random_steps=50_000,
             max_steps_per_episode=45, target_sync_steps=0, flags=flags)
    p.update(kw)
    return qlx.SelfDrivingQLearner(qlx.Parameter(**p)), O.Learner(O.default_params(**p))


def test_double_dqn_learner_matches_oracle():
    """Lockstep: before each vector step the oracle's online net is re-synced to the product's weights, so the
    double-DQN argmax on both sides comes from the same weights (the nets otherwise drift apart after the first
    update: Adam's sign-like first steps turn bf16 gradient noise into lr-sized steps)."""
    qlx = _qlx()
    gpu, ref = make(qlx.DOUBLE_DQN)
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


def test_prioritized_learner_matches_oracle():
    qlx = _qlx()
    gpu, ref = make(qlx.PER | qlx.DOUBLE_DQN, update_after_actions=16)
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
            # one update per vector step (16 envs, update_after_actions 16): its priorities from the TD errors
            # of the same batch on identical weights
            live = lr > 0
            assert np.array_equal(lg > 0, live)
            assert np.allclose(lg[live], lr[live], rtol=5e-2, atol=1e-2)
        # invariants on both sides
        for w, leaves, pmax in ((wg, lg, pg), (wr, lr, pr)):
            assert ((w > 0) & (w <= 1)).all() and (w.max(axis=1) == 1.0).all()
            assert pmax >= leaves.max() * (1 - 1e-6)
        assert (g["indices"] < gpu.stats()["replay_len"]).all()
    assert first is not None
    sg, sr = gpu.stats(), ref.counters()
    for k in ("step_count", "update_count", "replay_len"):
        assert sg[k] == sr[k], k


def test_prioritized_replay_bench_scale_runs():
    """Bench-shaped learner with both extensions: many updates per vector step, 1M-slot tree (two build levels)."""
    qlx = _qlx()
    p = qlx.Parameter(n_envs=512, batch_size=64, history_buffer_len=1_100_000, update_after_actions=64,
                      epsilon_pure_random_steps=0, max_steps_per_episode=2000, target_sync_steps=4096,
                      flags=qlx.PER | qlx.DOUBLE_DQN)
    L = qlx.SelfDrivingQLearner(p)
    L.run(20)
    st = L.stats()
    assert st["update_count"] == 20 * 8 and st["replay_len"] == 20 * 512
    w, leaves, pmax = L.priorities()
    assert w.shape == (8, 64) and ((w > 0) & (w <= 1)).all()
    assert (leaves[:st["replay_len"]] > 0).all() and (leaves[st["replay_len"]:] == 0).all()
    assert np.isfinite(st["last_loss"])
