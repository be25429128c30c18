"""BallGame oracle (oracle/ballgame_ref.cpp) pinned by the reference's own KAT and by independent restatements.

- The scripted episode of ballgame_test_environment.rs:333-410 (test_ballgame_environment) - exact.
- random_initial_state (:100-123): every generated state is one of all_possible_initial_states (:125-151)
  with the second obstacle off (1, 1), and all 54 such states occur.
- rand 0.8.5 `gen_range(0..3)` on usize (UniformInt::sample_single_inclusive, "(range << lz) - 1" zone)
  against a numpy restatement over the raw stream words.
- The fp32 Q-model (create_ql_model_ballgame_3x3x4_5_512.py:24-31, MSE train :71-85) against float64 torch
  autograd with Keras 'same' padding of a 2x2 kernel (one zero row / column after the data), and the
  legacy Adam + clip_by_norm step against numpy.
Parity of the raw bit stream is unpinned (the reference draws from the unseedable thread_rng).
"""
import numpy as np
import torch

import oracle as O

EMPTY, GOAL, BALL, OBST = 0, 1, 2, 3
WEST, NORTH, EAST, SOUTH, NOTHING = 0, 1, 2, 3, 4


def field_of(st):
    return st["field"][0].reshape(3, 3)   # [x][y]


def test_reference_kat_episode():
    # BallGameState::test_state_00_01_11_22 (:193-207): goal (0,0), obstacles (0,1), (1,1), ball (2,2)
    f = np.zeros((3, 3), np.uint8)
    f[0, 0], f[0, 1], f[1, 1], f[2, 2] = GOAL, OBST, OBST, BALL
    st = O.bg_state_from_field(f, (2, 2))
    init = field_of(st).copy()
    for a in (EAST, SOUTH):                      # blocked by the border: state unchanged, reward < 0
        r, d = O.bg_step(st, a)
        assert np.array_equal(field_of(st), init) and (st["ball_x"][0], st["ball_y"][0]) == (2, 2)
        assert r < 0 and not d
    r, d = O.bg_step(st, NORTH)
    assert (st["ball_x"][0], st["ball_y"][0]) == (2, 1)
    fx = field_of(st)
    assert fx[2, 1] == BALL and fx[2, 2] == EMPTY and fx[1, 2] == EMPTY and fx[0, 2] == EMPTY
    assert fx[1, 1] == OBST and fx[0, 1] == OBST and fx[2, 0] == EMPTY and fx[1, 0] == EMPTY and fx[0, 0] == GOAL
    assert r <= 0 and not d
    last = field_of(st).copy()
    O.bg_step(st, WEST)                          # into the (1,1) obstacle
    assert np.array_equal(field_of(st), last) and (st["ball_x"][0], st["ball_y"][0]) == (2, 1)
    r, d = O.bg_step(st, EAST)
    assert np.array_equal(field_of(st), last) and r <= 0 and not d
    r, d = O.bg_step(st, NORTH)
    assert (st["ball_x"][0], st["ball_y"][0]) == (2, 0) and field_of(st)[2, 1] == EMPTY and field_of(st)[2, 0] == BALL
    assert r <= 0 and not d
    last = field_of(st).copy()
    r, d = O.bg_step(st, NORTH)
    assert np.array_equal(field_of(st), last) and r <= 0 and not d
    r, d = O.bg_step(st, WEST)
    assert r <= 0 and not d and (st["ball_x"][0], st["ball_y"][0]) == (1, 0)
    assert field_of(st)[2, 0] == EMPTY and field_of(st)[1, 0] == BALL
    last = field_of(st).copy()
    r, d = O.bg_step(st, NORTH)
    assert np.array_equal(field_of(st), last) and r <= 0 and not d
    r, d = O.bg_step(st, WEST)
    assert (st["ball_x"][0], st["ball_y"][0]) == (0, 0)
    fx = field_of(st)
    assert fx[1, 0] == EMPTY and fx[0, 0] == BALL and fx[0, 1] == OBST and fx[1, 1] == OBST
    assert r > 9.5 and d                         # reward > episode_reward_goal_mean(), done


def test_exact_rewards_and_step_limit():
    # Environment::step (:69-86): +10 goal, -0.02 legal, -1 illegal, -10 / done once steps >= MAX_STEPS (16)
    f = np.zeros((3, 3), np.uint8)
    f[0, 0], f[0, 1], f[1, 1], f[2, 2] = GOAL, OBST, OBST, BALL
    st = O.bg_state_from_field(f, (2, 2))
    assert O.bg_step(st, NOTHING) == (np.float32(-0.02), False)   # Nothing is a legal stay
    assert O.bg_step(st, EAST) == (-1.0, False)
    for k in range(13):
        r, d = O.bg_step(st, NOTHING)
        assert not d and abs(r - (-0.02)) < 1e-7
    assert int(st["steps"][0]) == 15
    assert O.bg_step(st, NOTHING) == (-10.0, True)


def all_possible_initial_states():
    """BallGameState::all_possible_initial_states (:125-151) as (goal_x, ball_x, o2) tuples."""
    out = set()
    for gx in range(3):
        for bx in range(3):
            for ox in range(3):
                for oy in range(3):
                    if (ox, oy) != (gx, 0) and (ox, oy) != (bx, 2):
                        out.add((gx, bx, (ox, oy)))
    return out


def test_random_initial_states_are_valid_and_cover():
    allowed = {s for s in all_possible_initial_states() if s[2] != (1, 1)}
    assert len(allowed) == 54
    seen = set()
    for env_id in range(400):
        for rc in range(8):
            st = O.bg_initial_state(0xBA11, env_id, rc)
            f = field_of(st)
            assert int(st["steps"][0]) == 0 and int(st["ball_y"][0]) == 2
            gx = int(np.flatnonzero(f[:, 0] == GOAL)[0])
            bx = int(st["ball_x"][0])
            assert f[bx, 2] == BALL and f[1, 1] == OBST
            obst = [(x, y) for x in range(3) for y in range(3) if f[x, y] == OBST and (x, y) != (1, 1)]
            assert len(obst) == 1 and (f == EMPTY).sum() == 5
            key = (gx, bx, obst[0])
            assert key in allowed
            seen.add(key)
    assert seen == allowed


def test_gen_range_usize_single_matches_restatement():
    words = O.stream_u32(7, 3, 5, O.P_BALLGAME, 0, 64)
    zone = (3 << 62) - 1
    pos, expect = 0, []
    while len(expect) < 10:   # each draw consumes one u64 = (lo, hi) u32 words
        v = int(words[pos]) | (int(words[pos + 1]) << 32)
        pos += 2
        m = v * 3
        if (m & ((1 << 64) - 1)) <= zone:
            expect.append(m >> 64)
        else:
            expect.append(None)
    got, start = [], 0
    for e in expect:
        if e is None:
            start += 2
            continue
        got.append(O.gen_range_usize_single(7, 3, 5, O.P_BALLGAME, start, 3))
        start += 2
    assert got == [e for e in expect if e is not None]


def torch_bg_forward(ws, x_u8):
    t = lambda a: torch.as_tensor(np.asarray(a, dtype=np.float64))
    x = t(x_u8).permute(0, 3, 1, 2)                      # NHWC [x][y][c] -> NCHW (H = x, W = y)
    k0, b0, k1, b1, k2, b2, k3, b3 = [t(w).requires_grad_(True) for w in ws]
    h = torch.nn.functional.pad(x, (0, 1, 0, 1))           # TF 'same' 2x2 / stride 1: pad after
    h = torch.relu(torch.nn.functional.conv2d(h, k0.permute(3, 2, 0, 1), b0))
    h = torch.relu(torch.nn.functional.conv2d(h, k1.permute(3, 2, 0, 1), b1))
    h = h.permute(0, 2, 3, 1).reshape(x.shape[0], -1)     # Flatten (h, w, c)
    h = torch.relu(h @ k2 + b2)
    return h @ k3 + b3, [k0, b0, k1, b1, k2, b2, k3, b3]


def rand_obs(B, seed):
    out = np.zeros((B, 3, 3, 4), np.uint8)
    for b in range(B):
        st = O.bg_initial_state(seed, b, 0)
        for k in range(b % 5):
            O.bg_step(st, (b + k) % 5)
        out[b] = O.bg_obs(st)
    return out


def test_bg_obs_one_hot():
    st = O.bg_initial_state(1, 2, 3)
    x = O.bg_obs(st)
    assert x.sum() == 9 and np.array_equal(x.argmax(axis=2), field_of(st))


def test_bg_net_forward_and_train_match_torch():
    net = O.BgNet(seed=11)
    ws = [w.copy() for w in net.weights()]
    for v in (1, 3, 5, 7):   # non-zero biases so the bias paths are exercised
        ws[v] = np.linspace(-0.05, 0.05, ws[v].size, dtype=np.float32).reshape(ws[v].shape)
        net.set(v, ws[v])
    B = 16
    x = rand_obs(B, 5)
    q = net.forward(x)
    qt, params = torch_bg_forward(ws, x)
    assert np.allclose(q, qt.detach().numpy(), rtol=1e-5, atol=1e-6)
    a = (np.arange(B) % 5).astype(np.uint8)
    y = (q[np.arange(B), a] + np.linspace(-1.0, 1.0, B)).astype(np.float32)
    loss, grads, norms = net.train(x, a, y)
    qa = qt[torch.arange(B), torch.as_tensor(a.astype(np.int64))]
    lt = ((qa - torch.as_tensor(y.astype(np.float64))) ** 2).mean()
    lt.backward()
    assert abs(loss - lt.item()) <= 1e-5 * max(1.0, abs(lt.item()))
    off = 0
    for v, p in enumerate(params):
        g = grads[off:off + O.BG_VAR_SIZES[v]]
        gt = p.grad.numpy().reshape(-1)
        assert np.allclose(g, gt, rtol=1e-4, atol=1e-6 * max(1.0, np.abs(gt).max())), v
        assert abs(norms[v] - np.linalg.norm(gt)) <= 1e-4 * max(1e-6, np.linalg.norm(gt))
        off += O.BG_VAR_SIZES[v]
    # legacy Adam step t = 1 (clip_by_norm per variable, ResourceApplyAdam)
    alpha = np.float32(0.00025) * np.sqrt(np.float32(1) - np.float32(0.999)) / (np.float32(1) - np.float32(0.9))
    off = 0
    for v in range(8):
        g = grads[off:off + O.BG_VAR_SIZES[v]].astype(np.float32)
        gc = g * np.float32(1.0) / np.float32(max(norms[v], 1.0))
        m = gc * np.float32(0.1)
        vv = gc * gc * np.float32(0.001)
        w = ws[v].reshape(-1) - (m * alpha) / (np.sqrt(vv) + np.float32(1e-7))
        assert np.allclose(net.get(v).reshape(-1), w, rtol=1e-5, atol=1e-7), v
        off += O.BG_VAR_SIZES[v]


def test_bg_learner_runs_and_counts():
    p = O.default_params(n_envs=8, batch_size=32, history_buffer_len=300, update_after_actions=4,
                         epsilon_pure_random_steps=40, gamma=0.95, target_sync_steps=64)
    L = O.BgLearner(p)
    upd = 0
    for _ in range(20):
        L.vector_step()
        upd += len(L.last()["losses"])
    c = L.counters()
    assert c["step_count"] == 160 and c["update_count"] == upd > 0 and c["replay_len"] == 160
    assert c["episode_count"] > 0
