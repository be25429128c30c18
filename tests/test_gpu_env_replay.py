"""GPU parity of the batched Breakout env kernel and the HBM replay ring against the CPU oracle.

Bit-exact bar: mechanics state, frames (through a per-step checksum of every env and step, plus the
final 84x84x4 observations), rewards/dones, sampled indices and gathered transitions.
"""
import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

ENV_SEED = 0x51A5EED
ACT_SEED = 9


def _qlx():
    import qlx
    return qlx


def _state_eq(a, b):
    for k in O.STATE_DTYPE.names:
        assert np.array_equal(a[k], b[k]), f"field {k} differs: {a[k][:4]} vs {b[k][:4]}"


def _run_gpu(n_envs, n_steps, max_steps=10_000):
    qlx = _qlx()
    env = qlx.BreakoutEnvironment(n_envs=n_envs, seed=ENV_SEED)
    ep = np.zeros(n_envs, np.int64)
    tot = np.zeros(n_envs, np.float32)
    episodes = np.zeros(n_envs, np.uint32)
    for t in range(n_steps):
        a = O.synth_actions(ACT_SEED, n_envs, t)
        _, r, d = env.step(a)
        tot += r
        ep += 1
        mask = d | (ep >= max_steps)
        if mask.any():
            env.reset(mask.astype(np.uint8))
            episodes += mask
            ep[mask] = 0
    return env, tot, episodes


def test_env_initial_state_matches_oracle():
    qlx = _qlx()
    env = qlx.BreakoutEnvironment(n_envs=64, seed=ENV_SEED)
    st = env.mechanics()
    for e in range(64):
        ref = O.Env(ENV_SEED, e).state()
        for k in O.STATE_DTYPE.names:
            assert st[k][e] == ref[k], (e, k)
    assert not env.state().any()


@pytest.mark.parametrize("n_envs,n_steps,max_steps", [(1024, 600, 10_000), (256, 400, 50)])
def test_env_bit_exact_vs_oracle(n_envs, n_steps, max_steps):
    env, tot, episodes = _run_gpu(n_envs, n_steps, max_steps)
    st_ref, h_ref, tr_ref, ep_ref, tens_ref = O.envs_run(ENV_SEED, n_envs, n_steps, ACT_SEED, max_steps, want_tensors=True)
    _state_eq(env.mechanics(), st_ref)
    assert np.array_equal(env.hashes(), h_ref), "per-step checksum of state+frame differs"
    assert np.array_equal(tot, tr_ref)
    assert np.array_equal(episodes, ep_ref)
    assert np.array_equal(env.state(), tens_ref)
    assert (st_ref["fault"] == 0).all()


def test_env_invalid_action_is_an_error():
    qlx = _qlx()
    env = qlx.BreakoutEnvironment(n_envs=4)
    with pytest.raises(qlx.QlError):
        env.step(np.array([0, 1, 2, 3], np.uint8))   # Action::try_from_numeric(3) -> Err


def test_replay_get_many_reconstructs_states():
    """ReplayBuffer::add/get_many semantics: s' of step t == s of step t+1, FIFO eviction, reset zeros."""
    qlx = _qlx()
    n, T, cap = 16, 120, 700
    env = qlx.BreakoutEnvironment(n_envs=n, seed=ENV_SEED)
    rb = qlx.ReplayBuffer(cap, n)
    log = []   # (s, a, r, s_next, done) per pushed transition, in push order
    ep = np.zeros(n, np.int64)
    for t in range(T):
        s = env.state()
        a = O.synth_actions(ACT_SEED, n, t)
        s_next, r, d = env.step(a)
        rb.add(env, a, r, d)
        for e in range(n):
            log.append((s[e], a[e], r[e], s_next[e], d[e]))
        ep += 1
        mask = d | (ep >= 37)       # short episodes: exercise reset/zero-frame reconstruction
        if mask.any():
            env.reset(mask.astype(np.uint8))
            ep[mask] = 0
    assert len(rb) == cap
    kept = log[-cap:]
    idx = np.array([0, 1, 2, 5, 63, 64, 100, 333, cap - 2, cap - 1] + list(range(200, 240)), np.uint64)
    got = rb.get_many(idx)
    for j, i in enumerate(idx.tolist()):
        s, a, r, sn, d = kept[i]
        assert np.array_equal(got["state"][j], s), f"state of logical index {i}"
        assert np.array_equal(got["state_next"][j], sn), f"state_next of logical index {i}"
        assert got["action"][j] == a and got["reward"][j] == r and got["done"][j] == d


@pytest.mark.parametrize("length,B", [(100, 50), (100_000, 32), (1_000_000, 1024), (40, 40)])
def test_sample_distinct_matches_oracle(length, B):
    qlx = _qlx()
    n = 8 if length < 10_000 else 2048
    env = qlx.BreakoutEnvironment(n_envs=n)
    rb = qlx.ReplayBuffer(length, n)
    zeros = np.zeros(n, np.uint8)
    steps = (length + n - 1) // n
    for _ in range(steps):
        _, r, d = env.step(zeros)
        rb.add(env, zeros, r, d)
    assert len(rb) == length
    for u in range(5):
        got = rb.sample_distinct(seed=77, update_idx=u, batch=B)
        ref = O.sample_distinct(77, u, 0, length, B)
        assert np.array_equal(got, ref)
        assert len(set(got.tolist())) == B
