"""ctypes view of the CPU oracle (oracle/liboracle.so) — TEST INFRASTRUCTURE ONLY.

The oracle is the checker: only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load it.
Struct layouts mirror oracle/oracle_api.cpp and oracle/learner_ref.h.
"""
import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(ROOT, "oracle", "liboracle.so")

STATE_DTYPE = np.dtype([
    ("ball_x", "<f4"), ("ball_y", "<f4"), ("dir_x", "<f4"), ("dir_y", "<f4"),
    ("panel_min_x", "<f4"), ("panel_min_y", "<f4"), ("panel_max_x", "<f4"), ("panel_max_y", "<f4"),
    ("panel_speed", "<f4"),
    ("score", "<u4"), ("finished", "<u4"), ("next_slot", "<u4"), ("fault", "<u4"), ("reset_count", "<u4"),
    ("bricks", "<u8"),
])
assert STATE_DTYPE.itemsize == 64


class LearnerParams(C.Structure):
    _fields_ = [
        ("gamma", C.c_float),
        ("lowest_episode_reward_goal_threshold_pct", C.c_float),
        ("epsilon_max", C.c_double),
        ("epsilon_min", C.c_double),
        ("epsilon_greedy_steps", C.c_double),
        ("max_steps_per_episode", C.c_uint64),
        ("epsilon_pure_random_steps", C.c_uint64),
        ("history_buffer_len", C.c_uint64),
        ("update_after_actions", C.c_uint64),
        ("target_sync_steps", C.c_uint64),
        ("episode_reward_history_buffer_len", C.c_uint64),
        ("n_envs", C.c_uint32),
        ("batch_size", C.c_uint32),
        ("env_seed", C.c_uint64),
        ("learner_seed", C.c_uint64),
        ("init_seed", C.c_uint64),
        ("rank", C.c_uint32),
        ("flags", C.c_uint32),
        ("per_alpha", C.c_float),
        ("per_beta", C.c_float),
        ("per_eps", C.c_float),
        ("qnet_precision", C.c_uint32),
        ("stats_after_steps", C.c_uint64),
        ("checkpoint_file", C.c_char * 256),
        ("episode_reward_goal", C.c_float),
    ]


DOUBLE_DQN, PER = 1, 2   # LearnerParams.flags (include/qlx.h QLX_LEARNER_*)


def default_params(**kw):
    """Parameter::default() (self_driving_tf_q_learner.rs:50-67) + build fields."""
    p = LearnerParams(gamma=0.99, lowest_episode_reward_goal_threshold_pct=0.9, epsilon_max=1.0,
                      epsilon_min=0.1, epsilon_greedy_steps=1_000_000.0, max_steps_per_episode=10_000,
                      epsilon_pure_random_steps=50_000, history_buffer_len=1_000_000, update_after_actions=4,
                      target_sync_steps=0, episode_reward_history_buffer_len=100, n_envs=1, batch_size=32,
                      env_seed=0x51A5EED, learner_seed=1, init_seed=2, rank=0, flags=0, per_alpha=0.6,
                      per_beta=0.4, per_eps=1e-6, qnet_precision=0, stats_after_steps=25_000, checkpoint_file=b"",
                      episode_reward_goal=float("nan"))
    for k, v in kw.items():
        if k == "checkpoint_file" and isinstance(v, str):
            v = v.encode()
        setattr(p, k, v)
    return p


# BallGame state (oracle/ballgame_ref.h BgState = qlx_ballgame_state): field[x*3+y] in
# {0 empty, 1 goal, 2 ball, 3 obstacle}
BG_STATE_DTYPE = np.dtype([("field", "u1", (9,)), ("ball_x", "u1"), ("ball_y", "u1"), ("pad", "u1"), ("steps", "<u4"),
                           ("reset_count", "<u4")])
assert BG_STATE_DTYPE.itemsize == 20
BG_VAR_SHAPES = [(2, 2, 4, 32), (32,), (1, 1, 32, 32), (32,), (288, 512), (512,), (512, 5), (5,)]
BG_VAR_SIZES = [int(np.prod(s)) for s in BG_VAR_SHAPES]
P_BALLGAME = 6

VAR_SHAPES = [(8, 8, 4, 32), (32,), (4, 4, 32, 64), (64,), (3, 3, 64, 64), (64,), (3136, 512), (512,), (512, 3), (3,)]
VAR_SIZES = [int(np.prod(s)) for s in VAR_SHAPES]
STATE_BYTES = 84 * 84 * 4


def _p(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
        L = C.CDLL(LIB_PATH)
        vp, u64, u32, f32, i32 = C.c_void_p, C.c_uint64, C.c_uint32, C.c_float, C.c_int
        L.orc_philox.argtypes = [vp, vp, vp]
        L.orc_stream_u32.argtypes = [u64, u32, u32, u32, u64, i32, vp]
        L.orc_gen_range_f32.argtypes = [u64, u32, u32, u32, f32, f32]
        L.orc_gen_range_f32.restype = f32
        L.orc_gen_f64_01.argtypes = [u64, u32, u32, u32]
        L.orc_gen_f64_01.restype = C.c_double
        L.orc_gen_u8.argtypes = [u64, u32, u32, u32, u64, i32]
        L.orc_sample_distinct.argtypes = [u64, u32, u32, u64, i32, vp]
        L.orc_synth_actions.argtypes = [u64, u32, u32, vp]
        for n in ("orc_wall_left", "orc_wall_right"):
            getattr(L, n).argtypes = [f32] * 5 + [vp]
        L.orc_rect_check.argtypes = [f32] * 9 + [vp]
        L.orc_acos_threshold.restype = f32
        L.orc_env_new.argtypes = [u64, u32]
        L.orc_env_new.restype = vp
        L.orc_env_free.argtypes = [vp]
        L.orc_env_reset.argtypes = [vp]
        L.orc_env_step.argtypes = [vp, i32, vp, vp]
        L.orc_env_state.argtypes = [vp, vp]
        L.orc_env_tensor.argtypes = [vp, vp]
        L.orc_env_frame.argtypes = [vp, i32, vp]
        L.orc_envs_run.argtypes = [u64, u32, u32, u64, u64, vp, vp, vp, vp, vp]
        L.orc_qnet_new.argtypes = [u64]
        L.orc_qnet_new.restype = vp
        L.orc_qnet_free.argtypes = [vp]
        L.orc_qnet_get.argtypes = [vp, i32, i32, vp]
        L.orc_qnet_set.argtypes = [vp, i32, i32, vp]
        L.orc_qnet_iterations.argtypes = [vp]
        L.orc_qnet_iterations.restype = C.c_int64
        L.orc_qnet_set_iterations.argtypes = [vp, C.c_int64]
        L.orc_qnet_forward.argtypes = [vp, vp, i32, vp, vp, vp, vp, vp]
        L.orc_qnet_train.argtypes = [vp, vp, vp, vp, i32, vp, vp]
        L.orc_qnet_train.restype = f32
        L.orc_qnet32_forward.argtypes = [vp, vp, i32, vp, vp, vp, vp, vp]
        L.orc_qnet32_set_dense.argtypes = [i32]
        L.orc_qnet32_train.argtypes = [vp, vp, vp, vp, i32, vp, vp]
        L.orc_qnet32_train.restype = f32
        L.orc_qnet32_apply.argtypes = [vp, vp, f32, vp]
        L.orc_learner_prefill.argtypes = [vp, u64]
        L.orc_learner_stats_events.argtypes = [vp]
        L.orc_learner_stats_events.restype = u64
        L.orc_learner_new.argtypes = [C.POINTER(LearnerParams)]
        L.orc_learner_new.restype = vp
        L.orc_learner_free.argtypes = [vp]
        L.orc_learner_vector_step.argtypes = [vp]
        L.orc_learner_qnet.argtypes = [vp, i32]
        L.orc_learner_qnet.restype = vp
        L.orc_learner_counters.argtypes = [vp, vp, C.POINTER(C.c_double), C.POINTER(C.c_float)]
        L.orc_learner_last.argtypes = [vp] * 8
        L.orc_learner_last.restype = i32
        L.orc_learner_env_state.argtypes = [vp, u32, vp]
        L.orc_learner_env_tensor.argtypes = [vp, u32, vp]
        L.orc_learner_replay_get.argtypes = [vp, vp, i32, vp, vp, vp, vp, vp]
        L.orc_learner_params_size.restype = C.c_size_t
        L.orc_learner_per.argtypes = [vp, vp, vp, vp]
        L.orc_per_sample.argtypes = [vp, u64, u64, u32, u32, u32, u64, f32, i32, vp, vp, vp]
        L.orc_bg_learner_per.argtypes = [vp, vp, vp]
        L.orc_det_powf.argtypes = [vp, vp, u64, vp]
        L.orc_qnet_hparams.argtypes = [vp, vp]
        L.orc_bg_net_hparams.argtypes = [vp, vp]
        L.orc_dbscan_f32.argtypes = [vp, u64, f32, u64, vp]
        L.orc_dbscan_f32.restype = u64
        L.orc_dbscan_f32_format.argtypes = [vp, u64, f32, u64, C.c_char_p, C.c_size_t]
        L.orc_dbscan_f32_format.restype = C.c_size_t
        L.orc_update_log.argtypes = [u64, u64, f32, C.c_double, f32, f32, vp, u64, vp, i32, i32, C.c_char_p, C.c_size_t]
        L.orc_update_log.restype = C.c_size_t
        L.orc_state_size.restype = C.c_size_t
        # BallGame (oracle/ballgame_ref.h)
        L.orc_bg_state_size.restype = C.c_size_t
        L.orc_bg_initial_state.argtypes = [u64, u32, u32, vp]
        L.orc_bg_step.argtypes = [vp, i32, vp, vp]
        L.orc_bg_obs.argtypes = [vp, vp]
        L.orc_gen_range_usize_single.argtypes = [u64, u32, u32, u32, u64, u64]
        L.orc_gen_range_usize_single.restype = u64
        L.orc_bg_net_new.argtypes = [u64]
        L.orc_bg_net_new.restype = vp
        L.orc_bg_net_free.argtypes = [vp]
        L.orc_bg_net_get.argtypes = [vp, i32, i32, vp]
        L.orc_bg_net_set.argtypes = [vp, i32, i32, vp]
        L.orc_bg_net_forward.argtypes = [vp, vp, i32, vp, vp, vp, vp]
        L.orc_bg_net_train.argtypes = [vp, vp, vp, vp, i32, vp, vp]
        L.orc_bg_net_train.restype = f32
        L.orc_bg_learner_new.argtypes = [C.POINTER(LearnerParams)]
        L.orc_bg_learner_new.restype = vp
        L.orc_bg_learner_free.argtypes = [vp]
        L.orc_bg_learner_vector_step.argtypes = [vp]
        L.orc_bg_learner_net.argtypes = [vp, i32]
        L.orc_bg_learner_net.restype = vp
        L.orc_bg_learner_counters.argtypes = [vp, vp, C.POINTER(C.c_double), C.POINTER(C.c_float)]
        L.orc_bg_learner_last.argtypes = [vp] * 7
        L.orc_bg_learner_last.restype = i32
        L.orc_bg_learner_env_state.argtypes = [vp, u32, vp]
        assert L.orc_bg_state_size() == BG_STATE_DTYPE.itemsize
        assert L.orc_learner_params_size() == C.sizeof(LearnerParams)
        assert L.orc_state_size() == STATE_DTYPE.itemsize
        _lib = L
    return _lib


def philox(ctr, key):
    c = np.asarray(ctr, dtype=np.uint32)
    k = np.asarray(key, dtype=np.uint32)
    out = np.zeros(4, dtype=np.uint32)
    lib().orc_philox(_p(c), _p(k), _p(out))
    return out


def stream_u32(seed, c1, c2, purpose, start, n):
    out = np.zeros(n, dtype=np.uint32)
    lib().orc_stream_u32(seed, c1, c2, purpose, start, n, _p(out))
    return out


def sample_distinct(seed, update_idx, rank, length, B):
    out = np.zeros(B, dtype=np.uint64)
    lib().orc_sample_distinct(seed, update_idx, rank, length, B, _p(out))
    return out


def synth_actions(action_seed, n_envs, step):
    out = np.zeros(n_envs, dtype=np.uint8)
    lib().orc_synth_actions(action_seed, n_envs, step, _p(out))
    return out


def _surface(fn, *args):
    out = np.zeros(4, dtype=np.float32)
    hit = fn(*[float(a) for a in args], _p(out))
    return (float(out[0]), float(out[1]), float(out[2]), float(out[3])) if hit else None


def wall_left(center, radius, mv):
    return _surface(lib().orc_wall_left, center[0], center[1], radius, mv[0], mv[1])


def wall_right(center, radius, mv):
    return _surface(lib().orc_wall_right, center[0], center[1], radius, mv[0], mv[1])


def rect_check(center, radius, mv, lo, hi):
    return _surface(lib().orc_rect_check, center[0], center[1], radius, mv[0], mv[1], lo[0], lo[1], hi[0], hi[1])


class Env:
    """Single Breakout env (BreakoutEnvironment restatement)."""

    def __init__(self, seed, env_id=0):
        self.h = lib().orc_env_new(seed, env_id)

    def __del__(self):
        if getattr(self, "h", None):
            if _lib is not None:
                _lib.orc_env_free(self.h)
            self.h = None

    def reset(self):
        lib().orc_env_reset(self.h)

    def step(self, action):
        r = C.c_float()
        d = C.c_int()
        lib().orc_env_step(self.h, int(action), C.byref(r), C.byref(d))
        return r.value, bool(d.value)

    def state(self):
        s = np.zeros(1, dtype=STATE_DTYPE)
        lib().orc_env_state(self.h, _p(s))
        return s[0]

    def tensor(self):
        t = np.zeros((84, 84, 4), dtype=np.uint8)
        lib().orc_env_tensor(self.h, _p(t))
        return t

    def frame(self, slot):
        f = np.zeros((84, 84), dtype=np.uint8)
        lib().orc_env_frame(self.h, slot, _p(f))
        return f


def envs_run(env_seed, n_envs, n_steps, action_seed, max_steps=10_000, want_tensors=False):
    st = np.zeros(n_envs, dtype=STATE_DTYPE)
    h = np.zeros(n_envs, dtype=np.uint64)
    tr = np.zeros(n_envs, dtype=np.float32)
    ep = np.zeros(n_envs, dtype=np.uint32)
    tens = np.zeros((n_envs, 84, 84, 4), dtype=np.uint8) if want_tensors else None
    lib().orc_envs_run(env_seed, n_envs, n_steps, action_seed, max_steps, _p(st), _p(h), _p(tr), _p(ep), _p(tens))
    return st, h, tr, ep, tens


class QNet:
    """Q-net restatement.  f32=True: the fp32 arithmetic of QLX_ARCH_NATURE_DQN (oracle/qnet32_ref.cpp, every
    reduction one fmaf chain in the build's order: the product matches it bit for bit); f32=False: the
    double-accumulating restatement (oracle/qnet_ref.cpp) the bf16 product is held to within stated tolerances."""

    def __init__(self, seed=2, handle=None, owned=True, f32=False):
        self.f32 = f32
        self.owned = handle is None and owned
        self.h = handle if handle is not None else lib().orc_qnet_new(seed)

    def __del__(self):
        if getattr(self, "owned", False) and self.h:
            if _lib is not None:
                _lib.orc_qnet_free(self.h)
            self.h = None

    def get(self, var, which=0):
        out = np.zeros(VAR_SIZES[var], dtype=np.float32)
        lib().orc_qnet_get(self.h, var, which, _p(out))
        return out.reshape(VAR_SHAPES[var])

    def set(self, var, arr, which=0):
        a = np.ascontiguousarray(arr, dtype=np.float32).reshape(-1)
        assert a.size == VAR_SIZES[var]
        lib().orc_qnet_set(self.h, var, which, _p(a))

    def weights(self):
        return [self.get(v) for v in range(10)]

    def hparams(self):
        """(learning_rate, beta_1, beta_2, epsilon, clipnorm) as float32"""
        out = np.zeros(5, np.float32)
        lib().orc_qnet_hparams(self.h, _p(out))
        return out

    def iterations(self):
        return lib().orc_qnet_iterations(self.h)

    def set_iterations(self, it):
        lib().orc_qnet_set_iterations(self.h, int(it))

    def load_state_from(self, model):
        """Copy weights, Adam slots and iteration count from a product model (lockstep tests)."""
        for v in range(10):
            for which in range(3):
                self.set(v, model.get(v, which), which)
        self.set_iterations(model.iterations())

    def forward(self, x, acts=False):
        x = np.ascontiguousarray(x, dtype=np.uint8)
        B = x.shape[0]
        q = np.zeros((B, 3), dtype=np.float32)
        a = [np.zeros((B, 20, 20, 32), np.float32), np.zeros((B, 9, 9, 64), np.float32),
             np.zeros((B, 7, 7, 64), np.float32), np.zeros((B, 512), np.float32)] if acts else [None] * 4
        fn = lib().orc_qnet32_forward if self.f32 else lib().orc_qnet_forward
        fn(self.h, _p(x), B, _p(q), *[_p(t) for t in a])
        return (q, a) if acts else q

    def train(self, x, actions, y):
        x = np.ascontiguousarray(x, dtype=np.uint8)
        a = np.ascontiguousarray(actions, dtype=np.uint8)
        y = np.ascontiguousarray(y, dtype=np.float32)
        grads = np.zeros(sum(VAR_SIZES), dtype=np.float32)
        norms = np.zeros(10, dtype=np.float32)
        fn = lib().orc_qnet32_train if self.f32 else lib().orc_qnet_train
        loss = fn(self.h, _p(x), _p(a), _p(y), x.shape[0], _p(grads), _p(norms))
        out, off = [], 0
        for v in range(10):
            out.append(grads[off:off + VAR_SIZES[v]].reshape(VAR_SHAPES[v]))
            off += VAR_SIZES[v]
        return loss, out, norms


def qnet32_apply(net, flat_grads, scale):
    """clip_by_norm + Adam (fp32 chain definition) of net with flat_grads * scale; returns the clip norms"""
    g = np.ascontiguousarray(flat_grads, dtype=np.float32)
    assert g.size == sum(VAR_SIZES)
    norms = np.zeros(10, np.float32)
    lib().orc_qnet32_apply(net.h, _p(g), scale, _p(norms))
    return norms


def cluster_analysis(elements, eps, min_neighbors):
    """oracle/stats_ref.cpp generic DBSCAN: (clusters as index lists, noise indices)"""
    x = np.ascontiguousarray(elements, dtype=np.float32)
    labels = np.zeros(x.shape[0], np.int32)
    nc = lib().orc_dbscan_f32(_p(x), x.shape[0], eps, min_neighbors, _p(labels))
    return [np.flatnonzero(labels == c).tolist() for c in range(nc)], np.flatnonzero(labels < 0).tolist()


def cluster_analysis_text(elements, eps, min_neighbors):
    x = np.ascontiguousarray(elements, dtype=np.float32)
    n = lib().orc_dbscan_f32_format(_p(x), x.shape[0], eps, min_neighbors, None, 0)
    buf = C.create_string_buffer(n + 1)
    lib().orc_dbscan_f32_format(_p(x), x.shape[0], eps, min_neighbors, buf, n + 1)
    return buf.raw[:n].decode("utf-8")


def update_log(episode_count, step_count, gamma, epsilon, goal_mean, pct, rewards, counts, ballgame=False):
    """oracle/stats_ref.cpp learning_update_log text"""
    r = np.ascontiguousarray(rewards, dtype=np.float32)
    c = np.ascontiguousarray(counts, dtype=np.uint64)
    args = (episode_count, step_count, gamma, epsilon, goal_mean, pct, _p(r), r.shape[0], _p(c), c.shape[0], int(ballgame))
    n = lib().orc_update_log(*args, None, 0)
    buf = C.create_string_buffer(n + 1)
    lib().orc_update_log(*args, buf, n + 1)
    return buf.raw[:n].decode("utf-8")


def per_sample(leaves, seed, first_update, n_updates, rank, length, beta, batch):
    """oracle/learner_ref.h SumTree + per_sample over the given leaves: (slots [U][B], IS weights [U][B], total)"""
    x = np.ascontiguousarray(leaves, dtype=np.float32)
    slots = np.zeros(n_updates * batch, np.uint64)
    w = np.zeros(n_updates * batch, np.float32)
    total = C.c_float()
    lib().orc_per_sample(_p(x), x.shape[0], seed, first_update, n_updates, rank, length, beta, batch, _p(slots), _p(w),
                         C.byref(total))
    return slots.reshape(n_updates, batch), w.reshape(n_updates, batch), total.value


def det_powf(x, y):
    """oracle/learner_ref.cpp det_powf: the prioritized replay's x^y (binary64 from basic operations, one rounding)"""
    x = np.ascontiguousarray(x, dtype=np.float32)
    y = np.ascontiguousarray(np.broadcast_to(np.asarray(y, np.float32), x.shape), dtype=np.float32)
    out = np.zeros(x.shape, np.float32)
    lib().orc_det_powf(_p(x), _p(y), x.size, _p(out))
    return out


class Learner:
    def __init__(self, params):
        self.params = params
        self.N = params.n_envs
        self.B = params.batch_size
        self.h = lib().orc_learner_new(C.byref(params))

    def __del__(self):
        if getattr(self, "h", None):
            if _lib is not None:
                _lib.orc_learner_free(self.h)
            self.h = None

    def vector_step(self):
        lib().orc_learner_vector_step(self.h)

    def prefill(self, n_vector_steps):
        """vector steps without updates (act, env step, replay push, episode books)"""
        lib().orc_learner_prefill(self.h, n_vector_steps)

    def stats_events(self):
        return int(lib().orc_learner_stats_events(self.h))

    def counters(self):
        out = np.zeros(6, dtype=np.uint64)
        eps = C.c_double()
        rr = C.c_float()
        lib().orc_learner_counters(self.h, _p(out), C.byref(eps), C.byref(rr))
        keys = ["step_count", "vec_steps", "update_count", "episode_count", "replay_len", "solved"]
        d = {k: int(v) for k, v in zip(keys, out)}
        d["epsilon"] = eps.value
        d["running_reward"] = rr.value
        return d

    def last(self, max_updates=4096):
        N, B = self.N, self.B
        a = np.zeros(N, np.uint8)
        r = np.zeros(N, np.float32)
        d = np.zeros(N, np.uint8)
        losses = np.zeros(max_updates, np.float32)
        idx = np.zeros(max_updates * B, np.uint64)
        tg = np.zeros(max_updates * B, np.float32)
        q = np.zeros((N, 3), np.float32)
        n = lib().orc_learner_last(self.h, _p(a), _p(r), _p(d), _p(losses), _p(idx), _p(tg), _p(q))
        return dict(actions=a, rewards=r, dones=d, losses=losses[:n], indices=idx[:n * B].reshape(n, B),
                    targets=tg[:n * B].reshape(n, B), q=q)

    def priorities(self):
        """(IS weights [n_updates][B] of the last vector step, sum-tree leaves [cap], per_max)"""
        n = self.last()["losses"].shape[0]
        w = np.zeros(max(n, 1) * self.B, np.float32)
        leaves = np.zeros(self.params.history_buffer_len, np.float32)
        pmax = C.c_float()
        lib().orc_learner_per(self.h, _p(w), _p(leaves), C.byref(pmax))
        return w[:n * self.B].reshape(n, self.B), leaves, pmax.value

    def qnet(self, which=0):
        return QNet(handle=lib().orc_learner_qnet(self.h, which), owned=False, f32=self.params.qnet_precision == 0)

    def env_state(self, e):
        s = np.zeros(1, dtype=STATE_DTYPE)
        lib().orc_learner_env_state(self.h, e, _p(s))
        return s[0]

    def env_tensor(self, e):
        t = np.zeros((84, 84, 4), np.uint8)
        lib().orc_learner_env_tensor(self.h, e, _p(t))
        return t

    def replay_get(self, idx):
        idx = np.ascontiguousarray(idx, dtype=np.uint64)
        B = idx.size
        s = np.zeros((B, 84, 84, 4), np.uint8)
        sn = np.zeros((B, 84, 84, 4), np.uint8)
        a = np.zeros(B, np.uint8)
        r = np.zeros(B, np.float32)
        d = np.zeros(B, np.uint8)
        lib().orc_learner_replay_get(self.h, _p(idx), B, _p(s), _p(sn), _p(a), _p(r), _p(d))
        return s, sn, a, r, d


# ---------------- BallGame ----------------
def bg_initial_state(seed, env_id, reset_count=0):
    st = np.zeros(1, dtype=BG_STATE_DTYPE)
    lib().orc_bg_initial_state(seed, env_id, reset_count, _p(st))
    return st


def bg_step(st, action):
    """Environment::step on a 1-element BG_STATE_DTYPE array (in place): (reward, done)."""
    r = np.zeros(1, np.float32)
    d = np.zeros(1, np.uint8)
    lib().orc_bg_step(_p(st), int(action), _p(r), _p(d))
    return float(r[0]), bool(d[0])


def bg_obs(st):
    out = np.zeros((3, 3, 4), np.uint8)
    lib().orc_bg_obs(_p(st), _p(out))
    return out


def bg_state_from_field(field, ball, steps=0):
    st = np.zeros(1, dtype=BG_STATE_DTYPE)
    st["field"][0] = np.asarray(field, np.uint8).reshape(9)
    st["ball_x"], st["ball_y"], st["steps"] = ball[0], ball[1], steps
    return st


def gen_range_usize_single(seed, c1, c2, purpose, start, n):
    return int(lib().orc_gen_range_usize_single(seed, c1, c2, purpose, start, n))


class BgNet:
    def __init__(self, seed=2, handle=None, owned=True):
        self.h = handle if handle is not None else lib().orc_bg_net_new(seed)
        self.owned = owned and handle is None

    def __del__(self):
        if getattr(self, "owned", False) and getattr(self, "h", None):
            if _lib is not None:
                _lib.orc_bg_net_free(self.h)
            self.h = None

    def get(self, var, which=0):
        out = np.zeros(BG_VAR_SIZES[var], np.float32)
        lib().orc_bg_net_get(self.h, var, which, _p(out))
        return out.reshape(BG_VAR_SHAPES[var])

    def set(self, var, arr, which=0):
        a = np.ascontiguousarray(arr, dtype=np.float32).reshape(-1)
        assert a.size == BG_VAR_SIZES[var]
        lib().orc_bg_net_set(self.h, var, which, _p(a))

    def weights(self):
        return [self.get(v) for v in range(8)]

    def hparams(self):
        out = np.zeros(5, np.float32)
        lib().orc_bg_net_hparams(self.h, _p(out))
        return out

    def forward(self, x, acts=False):
        x = np.ascontiguousarray(x, dtype=np.uint8)
        B = x.shape[0]
        q = np.zeros((B, 5), np.float32)
        a1, a2, a3 = (np.zeros((B, 288), np.float32), np.zeros((B, 288), np.float32), np.zeros((B, 512), np.float32))
        lib().orc_bg_net_forward(self.h, _p(x), B, _p(q), _p(a1), _p(a2), _p(a3))
        return (q, a1, a2, a3) if acts else q

    def train(self, x, actions, y):
        x = np.ascontiguousarray(x, dtype=np.uint8)
        a = np.ascontiguousarray(actions, dtype=np.uint8)
        y = np.ascontiguousarray(y, dtype=np.float32)
        g = np.zeros(sum(BG_VAR_SIZES), np.float32)
        nrm = np.zeros(8, np.float32)
        loss = lib().orc_bg_net_train(self.h, _p(x), _p(a), _p(y), x.shape[0], _p(g), _p(nrm))
        return loss, g, nrm


class BgLearner:
    def __init__(self, params):
        self.params = params
        self.N = params.n_envs
        self.B = params.batch_size
        self.h = lib().orc_bg_learner_new(C.byref(params))

    def __del__(self):
        if getattr(self, "h", None):
            if _lib is not None:
                _lib.orc_bg_learner_free(self.h)
            self.h = None

    def vector_step(self):
        lib().orc_bg_learner_vector_step(self.h)

    def counters(self):
        out = np.zeros(6, dtype=np.uint64)
        eps = C.c_double()
        rr = C.c_float()
        lib().orc_bg_learner_counters(self.h, _p(out), C.byref(eps), C.byref(rr))
        keys = ["step_count", "vec_steps", "update_count", "episode_count", "replay_len", "solved"]
        d = {k: int(v) for k, v in zip(keys, out)}
        d["epsilon"] = eps.value
        d["running_reward"] = rr.value
        return d

    def last(self, max_updates=4096):
        N, B = self.N, self.B
        a, r, d = np.zeros(N, np.uint8), np.zeros(N, np.float32), np.zeros(N, np.uint8)
        losses = np.zeros(max_updates, np.float32)
        idx = np.zeros(max_updates * B, np.uint64)
        tg = np.zeros(max_updates * B, np.float32)
        n = lib().orc_bg_learner_last(self.h, _p(a), _p(r), _p(d), _p(losses), _p(idx), _p(tg))
        return dict(actions=a, rewards=r, dones=d, losses=losses[:n], indices=idx[:n * B].reshape(n, B),
                    targets=tg[:n * B].reshape(n, B))

    def priorities(self):
        """(sum-tree leaves [cap], per_max) of prioritized replay"""
        leaves = np.zeros(self.params.history_buffer_len, np.float32)
        pmax = C.c_float()
        lib().orc_bg_learner_per(self.h, _p(leaves), C.byref(pmax))
        return leaves, pmax.value

    def net(self, which=0):
        return BgNet(handle=lib().orc_bg_learner_net(self.h, which), owned=False)

    def env_state(self, e):
        s = np.zeros(1, dtype=BG_STATE_DTYPE)
        lib().orc_bg_learner_env_state(self.h, e, _p(s))
        return s[0]
