"""GPU BallGame (env kernel, fp32 Q-model kernels, vector-step learner) vs the CPU oracle (oracle/ballgame_ref.cpp).

Bit-exact: initial states, the reference's scripted episode (ballgame_test_environment.rs:333-410), batched
random play with resets, epsilon-greedy random actions, replay sampling indices, rewards / dones / episode
counters of the learner.
Within tolerance (fp32 SIMT kernels vs the fp32 oracle with float64 dot products): Q values and loss 1e-4
relative, raw gradients 1e-3 relative L2 per variable, post-Adam weights 2e-7 absolute (Adam's first steps
are +-lr-sized, so a flipped sign of a tiny gradient would show as a 2*lr jump; none are expected at fp32).
A learning check trains the GPU learner until the running reward over the last 200 episodes exceeds 9.0
(optimal play scores 9.96, random play about -10).
"""
import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

WEST, NORTH, EAST, SOUTH, NOTHING = 0, 1, 2, 3, 4


def _qlx():
    import qlx
    return qlx


def test_initial_states_match_oracle():
    qlx = _qlx()
    env = qlx.BallGameEnvironment(n_envs=300, seed=0xBA11)
    st = env.states()
    for e in range(300):
        ref = O.bg_initial_state(0xBA11, e, 0)
        assert st[e].tobytes() == ref[0].tobytes(), e
    obs = env.state()
    for e in range(0, 300, 37):
        assert np.array_equal(obs[e], O.bg_obs(O.bg_initial_state(0xBA11, e, 0)))


def test_reference_kat_episode_on_gpu():
    qlx = _qlx()
    env = qlx.BallGameEnvironment(n_envs=1)
    f = np.zeros((3, 3), np.uint8)
    f[0, 0], f[0, 1], f[1, 1], f[2, 2] = 1, 3, 3, 2
    st = O.bg_state_from_field(f, (2, 2))
    env.set_states(st.astype(qlx.BG_STATE_DTYPE))
    seq = [EAST, SOUTH, NORTH, WEST, EAST, NORTH, NORTH, WEST, NORTH, WEST]
    for k, a in enumerate(seq):
        r_ref, d_ref = O.bg_step(st, a)
        r, d = env.step(np.array([a], np.uint8))
        assert r[0] == np.float32(r_ref) and bool(d[0]) == d_ref, k
        assert env.states()[0].tobytes() == st[0].tobytes(), k
    assert d[0] and r[0] == 10.0 and tuple(env.states()[0]["field"].reshape(3, 3)[0, :2]) == (2, 3)


def test_batched_random_play_with_resets_bit_exact():
    qlx = _qlx()
    N, T = 512, 60
    env = qlx.BallGameEnvironment(n_envs=N, seed=77)
    ref = [O.bg_initial_state(77, e, 0) for e in range(N)]
    rng = np.random.default_rng(3)
    for t in range(T):
        a = rng.integers(0, 5, N).astype(np.uint8)
        r, d = env.step(a)
        for e in range(N):
            rr, dd = O.bg_step(ref[e], a[e])
            assert r[e] == np.float32(rr) and bool(d[e]) == dd, (t, e)
        if d.any():
            env.reset(d.astype(np.uint8))
            for e in np.flatnonzero(d):
                ref[e] = O.bg_initial_state(77, int(e), int(ref[e]["reset_count"][0]) + 1)
        if t % 10 == 9:
            st = env.states()
            for e in range(N):
                assert st[e].tobytes() == ref[e][0].tobytes(), (t, e)
    with pytest.raises(qlx.QlError):
        env.step(np.full(N, 5, np.uint8))


def rand_obs(B, seed):
    out = np.zeros((B, 3, 3, 4), np.uint8)
    rng = np.random.default_rng(seed)
    for b in range(B):
        st = O.bg_initial_state(seed, b, 0)
        for _ in range(int(rng.integers(0, 6))):
            O.bg_step(st, int(rng.integers(0, 5)))
        out[b] = O.bg_obs(st)
    return out


def test_model_forward_and_train_match_oracle():
    qlx = _qlx()
    m = qlx.BallGameModel(seed=5)
    ref = O.BgNet(seed=5)
    for v in range(8):
        assert np.array_equal(m.get(v), ref.get(v)), v   # identical GlorotUniform draws
    for v in (1, 3, 5, 7):
        b = np.linspace(-0.05, 0.05, int(np.prod(qlx.BG_VAR_SHAPES[v])), dtype=np.float32)
        m.set(v, b)
        ref.set(v, b)
    B = 512
    x = rand_obs(B, 9)
    q, a = m.q_values(x)
    qr = ref.forward(x)
    assert np.allclose(q, qr, rtol=1e-4, atol=1e-5 * max(1.0, np.abs(qr).max()))
    assert (a == qr.argmax(axis=1)).mean() > 0.99
    mx = m.batch_predict_max_future_reward(x)
    assert np.allclose(mx, qr.max(axis=1), rtol=1e-4, atol=1e-5)
    acts = (np.arange(B) % 5).astype(np.uint8)
    y = (qr[np.arange(B), acts] + np.sin(np.arange(B)).astype(np.float32)).astype(np.float32)
    for it in range(3):
        loss, g, nrm = m.train(x, acts, y, want_grads=True)
        lr_, gr, nr = ref.train(x, acts, y)
        assert abs(loss - lr_) <= 1e-4 * max(1.0, abs(lr_)), it
        off = 0
        for v, n in enumerate(O.BG_VAR_SIZES):
            gv, rv = g[off:off + n], gr[off:off + n]
            assert np.linalg.norm(gv - rv) <= 1e-3 * max(np.linalg.norm(rv), 1e-12), (it, v)
            assert abs(nrm[v] - nr[v]) <= 1e-3 * max(nr[v], 1e-12), (it, v)
            off += n
        for v in range(8):
            assert np.abs(m.get(v) - ref.get(v)).max() <= 2e-7 * (it + 1), (it, v)
    assert m.iterations() == 3


def make_learners(**kw):
    qlx = _qlx()
    p = dict(n_envs=32, batch_size=64, history_buffer_len=2000, update_after_actions=4, gamma=0.95,
             epsilon_pure_random_steps=600, epsilon_greedy_steps=5000.0, max_steps_per_episode=10_000,
             target_sync_steps=256, episode_reward_history_buffer_len=50, env_seed=0xBA11, learner_seed=7, init_seed=3)
    p.update(kw)
    return qlx.BallGameLearner(qlx.Parameter(**p)), O.BgLearner(O.default_params(**p))


def test_learner_matches_oracle():
    gpu, ref = make_learners()
    n_upd = 0
    for v in range(30):   # 19 pure-random vector steps, then epsilon-greedy with live Q values
        gpu.vector_step()
        ref.vector_step()
        g, r = gpu.last(), ref.last()
        if v < 19:
            assert np.array_equal(g["actions"], r["actions"]), v
        else:   # greedy choices follow fp32 Q values: allow the rare near-tie flip
            assert (g["actions"] == r["actions"]).mean() >= 0.9, v
        if v < 19:
            assert np.array_equal(g["rewards"], r["rewards"]) and np.array_equal(g["dones"], r["dones"]), v
        assert np.array_equal(g["indices"], r["indices"]), v
        if len(r["losses"]):
            n_upd += len(r["losses"])
            assert np.allclose(g["targets"], r["targets"], rtol=1e-3, atol=1e-3), v
            assert np.allclose(g["losses"], r["losses"], rtol=2e-2, atol=1e-3), v
    assert n_upd >= 150
    sg, sr = gpu.stats(), ref.counters()
    for k in ("step_count", "update_count", "replay_len"):
        assert sg[k] == sr[k], k


def test_learner_learns_ballgame():
    """End-to-end learning check: DQN with a periodically synced target net masters the 3x3 ball game."""
    gpu, _ = make_learners(n_envs=64, batch_size=256, history_buffer_len=100_000, epsilon_pure_random_steps=5_000,
                           epsilon_greedy_steps=60_000.0, epsilon_min=0.01, target_sync_steps=2_000,
                           episode_reward_history_buffer_len=200, update_after_actions=8)
    best = -100.0
    for chunk in range(40):
        gpu.run(100)
        st = gpu.stats()
        best = max(best, st["running_reward"])
        if st["running_reward"] >= 9.0:
            break
    print(f"\nballgame learning: running_reward {st['running_reward']:.3f} after {st['step_count']} env-steps, "
          f"{st['update_count']} updates, {st['episode_count']} episodes, epsilon {st['epsilon']:.3f}")
    assert best >= 9.0, (best, st)


def test_reference_saved_weights_load_and_forward():
    """The reference's own exported BallGame variables (tests/golden) loaded through the TF-bundle reader
    into the GPU model: identical weights, Adam slots and iterations; Q values equal the oracle's on them."""
    import os
    qlx = _qlx()
    prefix = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ballgame_saved_variables", "variables")
    m = qlx.BallGameModel(seed=99)
    m.load_tf(prefix)
    bundle = qlx.TfBundle(prefix)
    ref = O.BgNet(seed=99)
    for v in range(8):
        name = f"layer_with_weights-{v // 2}/{('kernel', 'bias')[v % 2]}/.ATTRIBUTES/VARIABLE_VALUE"
        w = bundle.read(name)
        assert np.array_equal(m.get(v), w), v
        assert not m.get(v, which=1).any() and not m.get(v, which=2).any()
        ref.set(v, w)
    assert m.iterations() == 0
    x = rand_obs(256, 4)
    q, _ = m.q_values(x)
    assert np.allclose(q, ref.forward(x), rtol=1e-4, atol=1e-5)


def test_double_dqn_prioritized_learner_matches_oracle():
    """BallGame learner with double DQN + prioritized replay vs the oracle: identical first prioritized batches
    (every leaf at the initial max priority), priorities (|td| + eps)^alpha from the same TD errors, and the
    counters; later draws follow each side's own priorities."""
    qlx = _qlx()
    gpu, ref = make_learners(update_after_actions=32, flags=qlx.DOUBLE_DQN | qlx.PER, epsilon_pure_random_steps=10**6)
    first = None
    for v in range(12):
        gpu.vector_step()
        ref.vector_step()
        g, r = gpu.last(), ref.last()
        assert np.array_equal(g["actions"], r["actions"]) and np.array_equal(g["rewards"], r["rewards"]), v
        if not len(r["losses"]):
            continue
        wg, lg, pg = gpu.priorities()
        lr, pr = ref.priorities()
        assert ((wg > 0) & (wg <= 1)).all() and (wg.max(axis=1) == 1.0).all()
        assert pg >= lg.max() * (1 - 1e-6)
        if first is None:
            first = v
            assert np.array_equal(g["indices"], r["indices"])
            assert (wg == 1.0).all()
            assert np.allclose(g["targets"], r["targets"], rtol=1e-3, atol=1e-3)
            assert np.allclose(lg, lr, rtol=1e-4, atol=1e-6)   # fp32 nets: TD errors agree closely
    assert first is not None
    sg, sr = gpu.stats(), ref.counters()
    for k in ("step_count", "update_count", "replay_len"):
        assert sg[k] == sr[k], k


def test_double_dqn_prioritized_learner_learns_ballgame():
    """End-to-end learning check of the extensions: double DQN + prioritized replay also masters the game."""
    qlx = _qlx()
    gpu, _ = make_learners(n_envs=64, batch_size=256, history_buffer_len=100_000, epsilon_pure_random_steps=5_000,
                           epsilon_greedy_steps=60_000.0, epsilon_min=0.01, target_sync_steps=2_000,
                           episode_reward_history_buffer_len=200, update_after_actions=8,
                           flags=qlx.DOUBLE_DQN | qlx.PER)
    best = -100.0
    for chunk in range(40):
        gpu.run(100)
        st = gpu.stats()
        best = max(best, st["running_reward"])
        if st["running_reward"] >= 9.0:
            break
    print(f"\nballgame ddqn+per learning: running_reward {st['running_reward']:.3f} after {st['step_count']} env-steps, "
          f"{st['update_count']} updates, {st['episode_count']} episodes")
    assert best >= 9.0, (best, st)


def test_reference_learner_single_episode():
    """The reference's own learner test (self_driving_tf_q_learner.rs:325-344 test_learner_single_episode): one
    BallGame env, Parameter::default(), both nets loaded from the reference's exported model
    (QL_MODEL_BALLGAME_3x3x4_5_512_PATH; tests/golden/ballgame_saved_variables); not solved, then learn_episode (vector
    steps of one env until its first episode ends), then still not solved, step_count > 1, episode_count == 1."""
    import os
    qlx = _qlx()
    prefix = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ballgame_saved_variables", "variables")
    L = qlx.BallGameLearner(qlx.Parameter(n_envs=1))   # Parameter::default() (B = 32, 50k pure-random steps, ...)
    L.model.load_tf(prefix)
    L.stabilized_model.load_tf(prefix)   # SelfDrivingQLearner::new loads the stabilized model the same way (:94-116)
    assert not L.solved()
    steps = 0
    while L.stats()["episode_count"] == 0:   # learn_episode: until the episode ends (done or max_steps_per_episode)
        L.vector_step()
        steps += 1
        assert steps <= 10_000
    st = L.stats()
    assert not L.solved()
    assert st["step_count"] > 1
    assert st["episode_count"] == 1
    L.close()
