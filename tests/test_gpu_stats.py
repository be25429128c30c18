"""GPU learning statistics (stats.hip) vs the oracle: the action histogram over the replay (exact counts) and the
learning_update_log text (self_driving_tf_q_learner.rs:235-273) for both learners (exact string)."""
import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu


def _qlx():
    import qlx
    return qlx


def test_breakout_action_counts_and_log_match_oracle():
    qlx = _qlx()
    p = dict(n_envs=16, batch_size=32, history_buffer_len=3000, update_after_actions=16, epsilon_pure_random_steps=50_000,
             max_steps_per_episode=30, episode_reward_history_buffer_len=20)
    gpu, ref = qlx.SelfDrivingQLearner(qlx.Parameter(**p)), O.Learner(O.default_params(**p))
    for _ in range(70):
        gpu.vector_step()
        ref.vector_step()
    st, rc = gpu.stats(), ref.counters()
    assert st["episode_count"] == rc["episode_count"] > 0
    n = rc["replay_len"]
    _, _, acts, _, _ = ref.replay_get(np.arange(n, dtype=np.uint64))
    want = np.bincount(acts, minlength=3).astype(np.uint64)
    assert np.array_equal(gpu.action_counts(), want)
    rewards = gpu.episode_rewards()
    assert rewards.shape[0] == min(rc["episode_count"], 20)
    txt = gpu.learning_update_log()
    assert txt == O.update_log(st["episode_count"], st["step_count"], p.get("gamma", 0.99), st["epsilon"], 59.0, 0.9, rewards,
                               want)
    assert "action_distribution (of last " in txt and "None " in txt


def test_ballgame_log_matches_oracle_format():
    qlx = _qlx()
    p = qlx.Parameter(n_envs=64, batch_size=64, history_buffer_len=5000, update_after_actions=8, epsilon_pure_random_steps=500,
                      episode_reward_history_buffer_len=100, gamma=0.95)
    L = qlx.BallGameLearner(p)
    L.run(40)
    st = L.stats()
    counts = L.action_counts()
    assert counts.sum() == st["replay_len"] and (counts > 0).all()
    rewards = L.episode_rewards()
    assert rewards.shape[0] == min(st["episode_count"], 100) > 0
    txt = L.learning_update_log()
    assert txt == O.update_log(st["episode_count"], st["step_count"], np.float32(0.95), st["epsilon"], 9.5, 0.9, rewards,
                               counts, ballgame=True)
    print(txt)


def test_action_histogram_large_replay():
    qlx = _qlx()
    p = qlx.Parameter(n_envs=2048, batch_size=64, history_buffer_len=100_003, update_after_actions=100_000,
                      epsilon_pure_random_steps=10**9, max_steps_per_episode=500)
    L = qlx.SelfDrivingQLearner(p)
    L.run(60)   # 122,880 pushes: the ring has wrapped
    c = L.action_counts()
    assert c.sum() == 100_003
    # pure-random actions: each of the 3 within 1% of a third
    assert np.abs(c / c.sum() - 1 / 3).max() < 0.01
