"""Host-side mirror of the reference's `ql` trait surface over libqlx's C ABI (include/qlx.h).

Names follow the reference so tests read like its own:
  Environment / Action           src/ql/src/prelude.rs:12-63
  BreakoutEnvironment            src/_breakout-ml/src/breakout_environment.rs:131-207   (batched: n envs)
  ReplayBuffer                   src/ql-with-tensorflow/src/learn/replay_buffer.rs:52-138
  DeepQLearningModel             src/ql-with-tensorflow/src/ml_model/model.rs:29-77
  Parameter / SelfDrivingQLearner  src/ql-with-tensorflow/src/learn/self_driving_tf_q_learner.rs:20-139

Everything here is plumbing: the compute runs in libqlx.so (HIP, gfx950).  There is no CPU fallback —
if the library or a GPU is missing, construction raises QlError.
"""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("QLX_LIB_PATH") or os.path.join(_HERE, "lib", "libqlx.so")   # override: A/B builds

ACTION_SPACE = 3           # BreakoutAction::ACTION_SPACE
FRAME = 84
SLOTS = 4
STATE_BYTES = FRAME * FRAME * SLOTS
NUM_VARS = 10
VAR_SHAPES = [(8, 8, 4, 32), (32,), (4, 4, 32, 64), (64,), (3, 3, 64, 64), (64,), (3136, 512), (512,), (512, 3), (3,)]
VAR_NAMES = ["convolution_layer1/kernel", "convolution_layer1/bias", "convolution_layer2/kernel",
             "convolution_layer2/bias", "convolution_layer3/kernel", "convolution_layer3/bias",
             "full_layer/kernel", "full_layer/bias", "action_layer/kernel", "action_layer/bias"]


class QlError(RuntimeError):
    """prelude.rs:70-86 QlError; raised for every non-zero status of the C ABI."""


STATE_DTYPE = np.dtype([
    ("ball_x", "<f4"), ("ball_y", "<f4"), ("dir_x", "<f4"), ("dir_y", "<f4"),
    ("panel_min_x", "<f4"), ("panel_min_y", "<f4"), ("panel_max_x", "<f4"), ("panel_max_y", "<f4"),
    ("panel_speed", "<f4"),
    ("score", "<u4"), ("finished", "<u4"), ("next_slot", "<u4"), ("fault", "<u4"), ("reset_count", "<u4"),
    ("bricks", "<u8"),
])


class Params(C.Structure):
    """qlx_params = Parameter (self_driving_tf_q_learner.rs:20-67) + build fields."""
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

DOUBLE_DQN = 1
PER = 2
PREC_F32 = 0    # QLX_PREC_F32: the reference's fp32 arithmetic (bit-exact against the oracle)
PREC_BF16 = 1   # QLX_PREC_BF16: bf16 MFMA operands, fp32 accumulation (the labelled fast path)
ARCH_F32 = 1    # QLX_ARCH_NATURE_DQN
ARCH_BF16 = 2   # QLX_ARCH_NATURE_DQN_BF16


class LearnerStats(C.Structure):
    _fields_ = [(k, C.c_uint64) for k in ("step_count", "vec_steps", "update_count", "episode_count",
                                          "replay_len", "solved")] + [
        ("epsilon", C.c_double), ("running_reward", C.c_float), ("last_loss", C.c_float)]


def Parameter(**kw):
    """Parameter::default() with overrides (self_driving_tf_q_learner.rs:50-67)."""
    p = Params(gamma=0.99, lowest_episode_reward_goal_threshold_pct=0.9, epsilon_max=1.0, epsilon_min=0.1,
               epsilon_greedy_steps=1_000_000.0, max_steps_per_episode=10_000, epsilon_pure_random_steps=50_000,
               history_buffer_len=1_000_000, update_after_actions=4, target_sync_steps=0,
               episode_reward_history_buffer_len=100, n_envs=1, batch_size=32, env_seed=0x51A5EED, learner_seed=1,
               init_seed=2, rank=0, flags=0, per_alpha=0.6, per_beta=0.4, per_eps=1e-6, qnet_precision=PREC_F32,
               stats_after_steps=25_000, checkpoint_file=b"", episode_reward_goal=float("nan"))
    for k, v in kw.items():
        if k == "checkpoint_file" and isinstance(v, str):
            v = v.encode()
        setattr(p, k, v)
    return p


_lib = None


def lib():
    """Load libqlx.so (fails loudly: the product has no CPU path)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise QlError(f"{LIB_PATH} not built — run `make lib` (or __graft_entry__.build())")
    L = C.CDLL(LIB_PATH)
    vp, u8p = C.c_void_p, C.c_void_p
    i32, u32, u64, f32 = C.c_int32, C.c_uint32, C.c_uint64, C.c_float
    sig = {
        "qlx_last_error": ([], C.c_char_p), "qlx_version": ([], i32),
        "qlx_env_action_space": ([i32], i32), "qlx_env_reward_goal_mean": ([i32], f32),
        "qlx_env_create": ([i32, u32, u64, i32, C.POINTER(vp)], i32), "qlx_env_destroy": ([vp], i32),
        "qlx_env_count": ([vp], u32), "qlx_env_reset": ([vp, u8p], i32), "qlx_env_step": ([vp, u8p, vp, u8p], i32),
        "qlx_env_step_dev": ([vp, vp, vp, vp], i32), "qlx_env_obs": ([vp, u8p], i32),
        "qlx_env_states": ([vp, vp], i32), "qlx_env_hashes": ([vp, vp], i32), "qlx_env_sync": ([vp], i32),
        "qlx_replay_create": ([u64, u32, i32, C.POINTER(vp)], i32), "qlx_replay_destroy": ([vp], i32),
        "qlx_replay_len": ([vp], u64), "qlx_replay_push_dev": ([vp, vp, vp, vp, vp], i32),
        "qlx_replay_push": ([vp, vp, vp, vp, vp], i32),
        "qlx_replay_sample_distinct": ([vp, u64, u32, u32, u32, vp], i32),
        "qlx_replay_get_many": ([vp, vp, u32, vp, vp, vp, vp, vp], i32),
        "qlx_model_create": ([i32, u64, i32, C.POINTER(vp)], i32), "qlx_model_destroy": ([vp], i32),
        "qlx_model_num_vars": ([], i32), "qlx_model_var_size": ([i32], C.c_int64), "qlx_model_hparams": ([vp], i32),
        "qlx_bg_model_hparams": ([vp], i32),
        "qlx_model_get_var": ([vp, i32, i32, vp], i32), "qlx_model_set_var": ([vp, i32, i32, vp], i32),
        "qlx_model_iterations": ([vp], C.c_int64), "qlx_model_copy_weights": ([vp, vp], i32),
        "qlx_model_predict": ([vp, vp, u32, vp, vp], i32), "qlx_model_batch_max_q": ([vp, vp, u32, vp], i32),
        "qlx_model_train": ([vp, vp, vp, vp, u32, vp, vp, vp], i32),
        "qlx_model_apply_gradient": ([vp, vp, C.c_float, vp], i32),
        "qlx_model_last_activation": ([vp, i32, vp], i32),
        "qlx_model_write_checkpoint": ([vp, C.c_char_p], i32), "qlx_model_read_checkpoint": ([vp, C.c_char_p], i32),
        "qlx_model_sync": ([vp], i32),
        "qlx_params_default": ([vp], None),
        "qlx_learner_create": ([C.POINTER(Params), i32, C.POINTER(vp)], i32), "qlx_learner_destroy": ([vp], i32),
        "qlx_learner_vector_step": ([vp], i32), "qlx_learner_run": ([vp, u64], i32), "qlx_learner_sync": ([vp], i32),
        "qlx_learner_prefill": ([vp, u64], i32), "qlx_learner_end_episodes": ([vp, vp], i32), "qlx_learner_stats_events": ([vp], u64),
        "qlx_learner_learn_till_mastered": ([vp, u64, C.POINTER(u64)], i32),
        "qlx_learner_last_log": ([vp, C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t)], i32),
        "qlx_learner_stats_get": ([vp, C.POINTER(LearnerStats)], i32),
        "qlx_learner_last": ([vp, vp, vp, vp, vp, vp, vp, C.POINTER(u32)], i32),
        "qlx_learner_env": ([vp], vp), "qlx_learner_replay": ([vp], vp), "qlx_learner_model": ([vp, i32], vp),
        "qlx_learner_priorities": ([vp, vp, vp, vp], i32),
        "qlx_learner_frame_sparsity": ([vp, vp], i32),
        "qlx_learner_action_counts": ([vp, vp], i32), "qlx_bg_learner_action_counts": ([vp, vp], i32),
        "qlx_learner_episode_rewards": ([vp, vp, u64, C.POINTER(u64)], i32),
        "qlx_bg_learner_episode_rewards": ([vp, vp, u64, C.POINTER(u64)], i32),
        "qlx_learner_update_log": ([vp, C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t)], i32),
        "qlx_bg_learner_update_log": ([vp, C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t)], i32),
        "qlx_dbscan_f32": ([vp, u64, C.c_float, u64, vp, C.POINTER(u64)], i32),
        "qlx_dbscan_f32_format": ([vp, u64, C.c_float, u64, C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t)], i32),
        "qlx_sumtree_create": ([u64, i32, C.POINTER(vp)], i32), "qlx_sumtree_destroy": ([vp], i32),
        "qlx_sumtree_set_leaves": ([vp, vp], i32), "qlx_sumtree_get": ([vp, vp, vp, vp], i32),
        "qlx_sumtree_sample": ([vp, u64, u32, u32, u32, u64, C.c_float, u32, vp, vp], i32),
        "qlx_sumtree_update": ([vp, vp, vp, u32, C.c_float, C.c_float], i32),
        "qlx_dist_unique_id": ([vp], i32), "qlx_learner_dist_init": ([vp, i32, i32, vp], i32),
        "qlx_learner_comm_size": ([vp, vp], i32),
        "qlx_learner_profile": ([vp, i32], i32),
        "qlx_learner_profile_get": ([vp, C.c_char_p, C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(u64)], i32),
        "qlx_learner_profile_filter": ([vp, C.c_char_p], i32),
        "qlx_learner_profile_sample": ([vp, C.c_char_p, u32], i32),
        "qlx_learner_profile_names": ([vp, C.c_char_p, C.c_size_t], i32),
        # BallGame
        "qlx_bg_env_create": ([u32, u64, i32, C.POINTER(vp)], i32), "qlx_bg_env_destroy": ([vp], i32),
        "qlx_bg_env_reset": ([vp, u8p], i32), "qlx_bg_env_step": ([vp, u8p, vp, u8p], i32),
        "qlx_bg_env_obs": ([vp, u8p], i32), "qlx_bg_env_states": ([vp, vp], i32), "qlx_bg_env_set_states": ([vp, vp], i32),
        "qlx_bg_model_create": ([u64, i32, C.POINTER(vp)], i32), "qlx_bg_model_destroy": ([vp], i32),
        "qlx_bg_model_var_size": ([i32], C.c_int64), "qlx_bg_model_get_var": ([vp, i32, i32, vp], i32),
        "qlx_bg_model_set_var": ([vp, i32, i32, vp], i32), "qlx_bg_model_iterations": ([vp], C.c_int64),
        "qlx_bg_model_predict": ([vp, vp, u32, vp, vp], i32), "qlx_bg_model_batch_max_q": ([vp, vp, u32, vp], i32),
        "qlx_bg_model_train": ([vp, vp, vp, vp, u32, vp, vp, vp], i32),
        "qlx_bg_learner_create": ([C.POINTER(Params), i32, C.POINTER(vp)], i32), "qlx_bg_learner_destroy": ([vp], i32),
        "qlx_bg_learner_run": ([vp, u64], i32), "qlx_bg_learner_sync": ([vp], i32),
        "qlx_bg_learner_stats_get": ([vp, C.POINTER(LearnerStats)], i32),
        "qlx_bg_learner_last": ([vp, vp, vp, vp, vp, vp, vp, C.POINTER(u32)], i32),
        "qlx_bg_learner_env": ([vp], vp), "qlx_bg_learner_model": ([vp, i32], vp),
        "qlx_bg_learner_priorities": ([vp, vp, vp, vp], i32),
        "qlx_bg_model_load_tf": ([vp, C.c_char_p], i32), "qlx_model_load_tf": ([vp, C.c_char_p], i32),
        "qlx_tf_bundle_open": ([C.c_char_p, C.POINTER(vp)], i32), "qlx_tf_bundle_close": ([vp], i32),
        "qlx_tf_bundle_count": ([vp], i32),
        "qlx_tf_bundle_entry": ([vp, i32, C.c_char_p, C.c_size_t, C.POINTER(i32), vp, C.POINTER(i32), C.POINTER(C.c_int64)], i32),
        "qlx_tf_bundle_read": ([vp, C.c_char_p, vp, C.c_size_t], i32),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name, None)
        if fn is None:
            continue
        fn.argtypes = args
        fn.restype = res
    _lib = L
    return L


def _text(fn, *args):
    n = C.c_size_t()
    _check(fn(*args, None, 0, C.byref(n)))
    buf = C.create_string_buffer(n.value + 1)
    _check(fn(*args, buf, n.value + 1, C.byref(n)))
    return buf.raw[:n.value].decode("utf-8")


def cluster_analysis(elements, max_neighbor_distance, core_point_min_neighbors):
    """dbscan::cluster_analysis (dbscan.rs:209-262) over f32 values: (clusters as index lists ordered by their lowest
    member, noise indices)"""
    x = np.ascontiguousarray(elements, dtype=np.float32)
    labels = np.zeros(x.shape[0], np.int32)
    nc = C.c_uint64()
    _check(lib().qlx_dbscan_f32(_p(x), x.shape[0], max_neighbor_distance, core_point_min_neighbors, _p(labels), C.byref(nc)))
    clusters = [np.flatnonzero(labels == c).tolist() for c in range(nc.value)]
    return clusters, np.flatnonzero(labels < 0).tolist()


def cluster_analysis_text(elements, max_neighbor_distance, core_point_min_neighbors):
    """Display of the ClusterAnalysisResult<f32> (dbscan.rs:91-133)"""
    x = np.ascontiguousarray(elements, dtype=np.float32)
    return _text(lib().qlx_dbscan_f32_format, _p(x), x.shape[0], max_neighbor_distance, core_point_min_neighbors)


class _LearningStats:
    """learning_update_log (self_driving_tf_q_learner.rs:235-273) for a learner handle"""
    _prefix = "qlx_learner"

    def action_counts(self):
        out = np.zeros(self._n_actions, np.uint64)
        _check(getattr(lib(), self._prefix + "_action_counts")(self.h, _p(out)))
        return out

    def episode_rewards(self):
        n = C.c_uint64()
        fn = getattr(lib(), self._prefix + "_episode_rewards")
        _check(fn(self.h, None, 0, C.byref(n)))
        out = np.zeros(n.value, np.float32)
        _check(fn(self.h, _p(out), n.value, C.byref(n)))
        return out

    def learning_update_log(self):
        return _text(getattr(lib(), self._prefix + "_update_log"), self.h)


def model_hparams(ballgame=False):
    """(learning_rate, beta_1, beta_2, epsilon, clipnorm) every model is created with (float32, no device needed)"""
    out = np.zeros(5, np.float32)
    _check((lib().qlx_bg_model_hparams if ballgame else lib().qlx_model_hparams)(_p(out)))
    return out


def exported_symbols():
    return [n for n in dir(lib()) if n.startswith("qlx_")]


def _check(status):
    if status != 0:
        msg = lib().qlx_last_error()
        raise QlError(f"qlx status {status}: {msg.decode() if msg else ''}")


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


class BreakoutEnvironment:
    """Batched `impl Environment for BreakoutEnvironment` on one MI355X (n independent envs)."""

    ACTION_SPACE = ACTION_SPACE

    def __init__(self, n_envs=1, seed=0x51A5EED, device=0, handle=None):
        self._owned = handle is None
        if handle is None:
            h = C.c_void_p()
            _check(lib().qlx_env_create(1, n_envs, seed, device, C.byref(h)))
            handle = h.value
        self.h = handle
        self.n = lib().qlx_env_count(self.h)

    def close(self):
        if getattr(self, "_owned", False) and getattr(self, "h", None):
            lib().qlx_env_destroy(self.h)
        self.h = None

    __del__ = close

    def reset(self, mask=None):
        m = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8)
        _check(lib().qlx_env_reset(self.h, _p(m)))

    def step(self, actions):
        a = np.ascontiguousarray(np.broadcast_to(actions, (self.n,)), dtype=np.uint8)
        r = np.zeros(self.n, np.float32)
        d = np.zeros(self.n, np.uint8)
        _check(lib().qlx_env_step(self.h, _p(a), _p(r), _p(d)))
        return self.state(), r, d.astype(bool)

    def state(self):
        """Reference tensor view [n][x][y][slot] u8 (ToMultiDimArray)."""
        out = np.zeros((self.n, FRAME, FRAME, SLOTS), np.uint8)
        _check(lib().qlx_env_obs(self.h, _p(out)))
        return out

    def mechanics(self):
        out = np.zeros(self.n, STATE_DTYPE)
        _check(lib().qlx_env_states(self.h, _p(out)))
        return out

    def hashes(self):
        out = np.zeros(self.n, np.uint64)
        _check(lib().qlx_env_hashes(self.h, _p(out)))
        return out

    @staticmethod
    def episode_reward_goal_mean():
        return lib().qlx_env_reward_goal_mean(1)


class ReplayBuffer:
    def __init__(self, capacity, n_envs, device=0, handle=None):
        self._owned = handle is None
        if handle is None:
            h = C.c_void_p()
            _check(lib().qlx_replay_create(capacity, n_envs, device, C.byref(h)))
            handle = h.value
        self.h = handle

    def close(self):
        if getattr(self, "_owned", False) and getattr(self, "h", None):
            lib().qlx_replay_destroy(self.h)
        self.h = None

    __del__ = close

    def __len__(self):
        return int(lib().qlx_replay_len(self.h))

    def add(self, env, actions, rewards, dones):
        """ReplayBuffer::add for the transition every env of `env` just made (replay_buffer.rs:85-98)."""
        a = np.ascontiguousarray(actions, dtype=np.uint8)
        r = np.ascontiguousarray(rewards, dtype=np.float32)
        d = np.ascontiguousarray(dones, dtype=np.uint8)
        _check(lib().qlx_replay_push(self.h, env.h, _p(a), _p(r), _p(d)))

    def sample_distinct(self, seed, update_idx, batch, rank=0):
        out = np.zeros(batch, np.uint64)
        _check(lib().qlx_replay_sample_distinct(self.h, seed, update_idx, rank, batch, _p(out)))
        return out

    def get_many(self, indices):
        idx = np.ascontiguousarray(indices, dtype=np.uint64)
        B = idx.size
        s = np.zeros((B, FRAME, FRAME, SLOTS), np.uint8)
        sn = np.zeros_like(s)
        a = np.zeros(B, np.uint8)
        r = np.zeros(B, np.float32)
        d = np.zeros(B, np.uint8)
        _check(lib().qlx_replay_get_many(self.h, _p(idx), B, _p(s), _p(sn), _p(a), _p(r), _p(d)))
        return dict(state=s, state_next=sn, action=a, reward=r, done=d.astype(bool))


class DeepQLearningModel:
    """Nature-DQN on MI355X: fp32 (the reference's arithmetic, fp32 MFMA, bit-exact against the oracle) or, with
    precision=PREC_BF16, bf16 MFMA operands with fp32 accumulation and fp32 master weights."""

    def __init__(self, seed=2, device=0, handle=None, precision=PREC_F32):
        self._owned = handle is None
        if handle is None:
            h = C.c_void_p()
            _check(lib().qlx_model_create(ARCH_BF16 if precision == PREC_BF16 else ARCH_F32, seed, device, C.byref(h)))
            handle = h.value
        self.h = handle

    def close(self):
        if getattr(self, "_owned", False) and getattr(self, "h", None):
            lib().qlx_model_destroy(self.h)
        self.h = None

    __del__ = close

    def get(self, var, which=0):
        out = np.zeros(int(np.prod(VAR_SHAPES[var])), np.float32)
        _check(lib().qlx_model_get_var(self.h, var, which, _p(out)))
        return out.reshape(VAR_SHAPES[var])

    def set(self, var, arr, which=0):
        a = np.ascontiguousarray(arr, dtype=np.float32).reshape(-1)
        _check(lib().qlx_model_set_var(self.h, var, which, _p(a)))

    def weights(self):
        return [self.get(v) for v in range(NUM_VARS)]

    def set_weights(self, ws):
        for v, w in enumerate(ws):
            self.set(v, w)

    def iterations(self):
        return int(lib().qlx_model_iterations(self.h))

    def copy_from(self, other):
        _check(lib().qlx_model_copy_weights(self.h, other.h))

    def load_tf(self, bundle_prefix):
        """Weights, Adam slots and iterations from a TF SavedModel / checkpoint bundle of the reference model."""
        _check(lib().qlx_model_load_tf(self.h, str(bundle_prefix).encode()))

    def q_values(self, states):
        x = np.ascontiguousarray(states, dtype=np.uint8)
        n = x.shape[0]
        q = np.zeros((n, ACTION_SPACE), np.float32)
        a = np.zeros(n, np.uint8)
        _check(lib().qlx_model_predict(self.h, _p(x), n, _p(q), _p(a)))
        return q, a

    def predict_action(self, state):
        """model.rs:39-42 for one state [84][84][4] (or a batch)."""
        x = np.asarray(state, dtype=np.uint8)
        single = x.ndim == 3
        _, a = self.q_values(x[None] if single else x)
        return int(a[0]) if single else a

    def batch_predict_max_future_reward(self, states):
        x = np.ascontiguousarray(states, dtype=np.uint8)
        out = np.zeros(x.shape[0], np.float32)
        _check(lib().qlx_model_batch_max_q(self.h, _p(x), x.shape[0], _p(out)))
        return out

    def train(self, states, actions, updated_q_values, want_grads=False):
        x = np.ascontiguousarray(states, dtype=np.uint8)
        a = np.ascontiguousarray(actions, dtype=np.uint8)
        y = np.ascontiguousarray(updated_q_values, dtype=np.float32)
        B = x.shape[0]
        loss = C.c_float()
        grads = np.zeros(sum(int(np.prod(s)) for s in VAR_SHAPES), np.float32) if want_grads else None
        norms = np.zeros(NUM_VARS, np.float32)
        _check(lib().qlx_model_train(self.h, _p(x), _p(a), _p(y), B, C.byref(loss), _p(grads), _p(norms)))
        if not want_grads:
            return loss.value
        out, off = [], 0
        for s in VAR_SHAPES:
            n = int(np.prod(s))
            out.append(grads[off:off + n].reshape(s))
            off += n
        return loss.value, out, norms

    def apply_gradient(self, flat_grads, scale=1.0):
        """the update tail alone (qlx_model_apply_gradient): clip_by_norm(flat_grads * scale) + Adam; the clip norms"""
        g = np.ascontiguousarray(flat_grads, dtype=np.float32)
        assert g.size == sum(int(np.prod(s)) for s in VAR_SHAPES)
        norms = np.zeros(NUM_VARS, np.float32)
        _check(lib().qlx_model_apply_gradient(self.h, _p(g), C.c_float(scale), _p(norms)))
        return norms

    def write_checkpoint(self, path):
        _check(lib().qlx_model_write_checkpoint(self.h, path.encode()))
        return path

    def read_checkpoint(self, path):
        _check(lib().qlx_model_read_checkpoint(self.h, path.encode()))


class SelfDrivingQLearner(_LearningStats):
    """SelfDrivingQLearner with n parallel envs on one GPU (vector-step generalisation)."""
    _n_actions = 3

    def __init__(self, param, device=0):
        self.param = param
        h = C.c_void_p()
        _check(lib().qlx_learner_create(C.byref(param), device, C.byref(h)))
        self.h = h.value
        self.environment = BreakoutEnvironment(handle=lib().qlx_learner_env(self.h))
        self.replay_buffer = ReplayBuffer(0, 0, handle=lib().qlx_learner_replay(self.h))
        self.model = DeepQLearningModel(handle=lib().qlx_learner_model(self.h, 0))
        self.stabilized_model = DeepQLearningModel(handle=lib().qlx_learner_model(self.h, 1))

    def close(self):
        if getattr(self, "h", None):
            lib().qlx_learner_destroy(self.h)
        self.h = None

    __del__ = close

    def vector_step(self):
        _check(lib().qlx_learner_vector_step(self.h))

    def run(self, n):
        _check(lib().qlx_learner_run(self.h, n))

    def prefill(self, n):
        """n vector steps without updates (replay fill before a measurement / parity check)"""
        _check(lib().qlx_learner_prefill(self.h, n))

    def end_episodes(self, mask):
        """end the current episode of every env with mask[e] (the max_steps_per_episode path; no transition added)"""
        m = np.ascontiguousarray(mask, dtype=np.uint8)
        assert m.shape == (self.param.n_envs,)
        _check(lib().qlx_learner_end_episodes(self.h, _p(m)))

    def learn_till_mastered(self, max_vector_steps):
        n = C.c_uint64()
        _check(lib().qlx_learner_learn_till_mastered(self.h, max_vector_steps, C.byref(n)))
        return n.value

    def stats_events(self):
        return int(lib().qlx_learner_stats_events(self.h))

    def last_log(self):
        return _text(lib().qlx_learner_last_log, self.h)

    def sync(self):
        _check(lib().qlx_learner_sync(self.h))

    def stats(self):
        s = LearnerStats()
        _check(lib().qlx_learner_stats_get(self.h, C.byref(s)))
        return {k: getattr(s, k) for k, _ in LearnerStats._fields_}

    def solved(self):
        return bool(self.stats()["solved"])

    def last(self, max_updates=4096):
        N, B = self.param.n_envs, self.param.batch_size
        a = np.zeros(N, np.uint8)
        r = np.zeros(N, np.float32)
        d = np.zeros(N, np.uint8)
        losses = np.zeros(max_updates, np.float32)
        idx = np.zeros(max_updates * B, np.uint64)
        tg = np.zeros(max_updates * B, np.float32)
        nu = C.c_uint32()
        _check(lib().qlx_learner_last(self.h, _p(a), _p(r), _p(d), _p(losses), _p(idx), _p(tg), C.byref(nu)))
        n = nu.value
        return dict(actions=a, rewards=r, dones=d, losses=losses[:n], indices=idx[:n * B].reshape(n, B),
                    targets=tg[:n * B].reshape(n, B))

    def priorities(self, max_updates=4096):
        """Prioritized replay (flags & PER): IS weights [n_updates][B] of the last vector step, sum-tree leaves
        [history_buffer_len], the priority new transitions enter with."""
        B = self.param.batch_size
        w = np.zeros(max_updates * B, np.float32)
        leaves = np.zeros(self.param.history_buffer_len, np.float32)
        pmax = C.c_float()
        n = self.last()["losses"].shape[0]
        _check(lib().qlx_learner_priorities(self.h, _p(w), _p(leaves), C.byref(pmax)))
        return w[:n * B].reshape(n, B), leaves, pmax.value

    def frame_sparsity(self):
        """Fractions of the fp32 conv work the exact zero skips leave out in the last vector step (diagnostic):
        {"train": [...], "act": [...]}, each [conv1 fwd zero steps, conv1 wgrad zero steps, conv2 bg rows, conv3 bg rows]
        (train: the step's sampled states, NaN without an update; act: the current acting frames - the observations the
        next vector step acts on, after this step's env step and resets)."""
        out = np.zeros(8, np.float64)
        _check(lib().qlx_learner_frame_sparsity(self.h, _p(out)))
        return {"train": out[:4].tolist(), "act": out[4:].tolist()}

    def dist_init(self, world, rank, uid):
        buf = (C.c_uint8 * 128).from_buffer_copy(bytes(uid))
        _check(lib().qlx_learner_dist_init(self.h, world, rank, buf))

    def comm_size(self):
        """ranks of the RCCL communicator (ncclCommCount), 1 without dist_init"""
        n = C.c_int32()
        _check(lib().qlx_learner_comm_size(self.h, C.byref(n)))
        return n.value

    def profile(self, enable=True):
        _check(lib().qlx_learner_profile(self.h, 1 if enable else 0))

    def profile_filter(self, name=None, stride=1):
        """Record only scope `name` (None = all), every `stride`-th launch of it."""
        _check(lib().qlx_learner_profile_sample(self.h, None if name is None else name.encode(), stride))

    def profile_get(self, name):
        """(total_us, total_work, launches) of a profiler scope since profile() was enabled."""
        us = C.c_double()
        work = C.c_double()
        n = C.c_uint64()
        _check(lib().qlx_learner_profile_get(self.h, name.encode(), C.byref(us), C.byref(work), C.byref(n)))
        return us.value, work.value, n.value

    def profile_names(self):
        buf = C.create_string_buffer(8192)
        _check(lib().qlx_learner_profile_names(self.h, buf, 8192))
        return [n for n in buf.value.decode().split(",") if n]


def dist_unique_id():
    buf = (C.c_uint8 * 128)()
    _check(lib().qlx_dist_unique_id(buf))
    return bytes(buf)


# ---------------- BallGame (the reference's second environment / model pair) ----------------
BG_ACTION_SPACE = 5
BG_VAR_SHAPES = [(2, 2, 4, 32), (32,), (1, 1, 32, 32), (32,), (288, 512), (512,), (512, 5), (5,)]
BG_STATE_DTYPE = np.dtype([("field", "u1", (9,)), ("ball_x", "u1"), ("ball_y", "u1"), ("pad", "u1"), ("steps", "<u4"),
                           ("reset_count", "<u4")])


class BallGameEnvironment:
    """Batched `impl Environment for BallGameTestEnvironment` (ballgame_test_environment.rs:59-89)."""

    ACTION_SPACE = BG_ACTION_SPACE

    def __init__(self, n_envs=1, seed=0xBA11, device=0, handle=None):
        self._owned = handle is None
        if handle is None:
            h = C.c_void_p()
            _check(lib().qlx_bg_env_create(n_envs, seed, device, C.byref(h)))
            handle = h.value
        self.h = handle
        self.n = n_envs

    def close(self):
        if getattr(self, "_owned", False) and getattr(self, "h", None):
            lib().qlx_bg_env_destroy(self.h)
        self.h = None

    __del__ = close

    def reset(self, mask=None):
        m = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8)
        _check(lib().qlx_bg_env_reset(self.h, _p(m)))

    def step(self, actions):
        a = np.ascontiguousarray(actions, dtype=np.uint8)
        r = np.zeros(self.n, np.float32)
        d = np.zeros(self.n, np.uint8)
        _check(lib().qlx_bg_env_step(self.h, _p(a), _p(r), _p(d)))
        return r, d.astype(bool)

    def state(self):
        out = np.zeros((self.n, 3, 3, 4), np.uint8)
        _check(lib().qlx_bg_env_obs(self.h, _p(out)))
        return out

    def states(self):
        out = np.zeros(self.n, dtype=BG_STATE_DTYPE)
        _check(lib().qlx_bg_env_states(self.h, _p(out)))
        return out

    def set_states(self, st):
        a = np.ascontiguousarray(st, dtype=BG_STATE_DTYPE)
        assert a.shape == (self.n,)
        _check(lib().qlx_bg_env_set_states(self.h, _p(a)))

    @staticmethod
    def episode_reward_goal_mean():
        return float(lib().qlx_env_reward_goal_mean(2))


class BallGameModel:
    """The 3x3x4 -> 5 Q-model (create_ql_model_ballgame_3x3x4_5_512.py) in fp32 HIP kernels."""

    def __init__(self, seed=2, device=0, handle=None):
        self._owned = handle is None
        if handle is None:
            h = C.c_void_p()
            _check(lib().qlx_bg_model_create(seed, device, C.byref(h)))
            handle = h.value
        self.h = handle

    def close(self):
        if getattr(self, "_owned", False) and getattr(self, "h", None):
            lib().qlx_bg_model_destroy(self.h)
        self.h = None

    __del__ = close

    def get(self, var, which=0):
        out = np.zeros(int(np.prod(BG_VAR_SHAPES[var])), np.float32)
        _check(lib().qlx_bg_model_get_var(self.h, var, which, _p(out)))
        return out.reshape(BG_VAR_SHAPES[var])

    def set(self, var, arr, which=0):
        a = np.ascontiguousarray(arr, dtype=np.float32).reshape(-1)
        _check(lib().qlx_bg_model_set_var(self.h, var, which, _p(a)))

    def weights(self):
        return [self.get(v) for v in range(8)]

    def iterations(self):
        return int(lib().qlx_bg_model_iterations(self.h))

    def load_tf(self, bundle_prefix):
        """Weights, Adam slots and iterations from the reference's SavedModel variables bundle."""
        _check(lib().qlx_bg_model_load_tf(self.h, str(bundle_prefix).encode()))

    def q_values(self, states):
        x = np.ascontiguousarray(states, dtype=np.uint8)
        n = x.shape[0]
        q = np.zeros((n, BG_ACTION_SPACE), np.float32)
        a = np.zeros(n, np.uint8)
        _check(lib().qlx_bg_model_predict(self.h, _p(x), n, _p(q), _p(a)))
        return q, a

    def batch_predict_max_future_reward(self, states):
        x = np.ascontiguousarray(states, dtype=np.uint8)
        out = np.zeros(x.shape[0], np.float32)
        _check(lib().qlx_bg_model_batch_max_q(self.h, _p(x), x.shape[0], _p(out)))
        return out

    def train(self, states, actions, updated_q_values, want_grads=False):
        x = np.ascontiguousarray(states, dtype=np.uint8)
        a = np.ascontiguousarray(actions, dtype=np.uint8)
        y = np.ascontiguousarray(updated_q_values, dtype=np.float32)
        loss = np.zeros(1, np.float32)
        nrm = np.zeros(8, np.float32)
        g = np.zeros(sum(int(np.prod(s)) for s in BG_VAR_SHAPES), np.float32) if want_grads else None
        _check(lib().qlx_bg_model_train(self.h, _p(x), _p(a), _p(y), x.shape[0], _p(loss), _p(g), _p(nrm)))
        return (float(loss[0]), g, nrm) if want_grads else float(loss[0])


class BallGameLearner(_LearningStats):
    """SelfDrivingQLearner over n BallGame envs on one GPU (same vector-step semantics as SelfDrivingQLearner)."""
    _prefix = "qlx_bg_learner"
    _n_actions = 5

    def __init__(self, param, device=0):
        self.param = param
        h = C.c_void_p()
        _check(lib().qlx_bg_learner_create(C.byref(param), device, C.byref(h)))
        self.h = h.value
        self.environment = BallGameEnvironment(handle=lib().qlx_bg_learner_env(self.h), n_envs=param.n_envs)
        self.model = BallGameModel(handle=lib().qlx_bg_learner_model(self.h, 0))
        self.stabilized_model = BallGameModel(handle=lib().qlx_bg_learner_model(self.h, 1))

    def close(self):
        if getattr(self, "h", None):
            lib().qlx_bg_learner_destroy(self.h)
        self.h = None

    __del__ = close

    def vector_step(self):
        _check(lib().qlx_bg_learner_run(self.h, 1))

    def run(self, n):
        _check(lib().qlx_bg_learner_run(self.h, n))

    def sync(self):
        _check(lib().qlx_bg_learner_sync(self.h))

    def stats(self):
        s = LearnerStats()
        _check(lib().qlx_bg_learner_stats_get(self.h, C.byref(s)))
        return {k: getattr(s, k) for k, _ in LearnerStats._fields_}

    def solved(self):
        return bool(self.stats()["solved"])

    def priorities(self, max_updates=4096):
        """Prioritized replay (flags & PER): IS weights [n_updates][B] of the last vector step, sum-tree leaves, per_max."""
        B = self.param.batch_size
        w = np.zeros(max_updates * B, np.float32)
        leaves = np.zeros(self.param.history_buffer_len, np.float32)
        pmax = C.c_float()
        n = self.last()["losses"].shape[0]
        _check(lib().qlx_bg_learner_priorities(self.h, _p(w), _p(leaves), C.byref(pmax)))
        return w[:n * B].reshape(n, B), leaves, pmax.value

    def last(self, max_updates=4096):
        N, B = self.param.n_envs, self.param.batch_size
        a, r, d = np.zeros(N, np.uint8), np.zeros(N, np.float32), np.zeros(N, np.uint8)
        losses = np.zeros(max_updates, np.float32)
        idx = np.zeros(max_updates * B, np.uint64)
        tg = np.zeros(max_updates * B, np.float32)
        nu = C.c_uint32()
        _check(lib().qlx_bg_learner_last(self.h, _p(a), _p(r), _p(d), _p(losses), _p(idx), _p(tg), C.byref(nu)))
        n = nu.value
        return dict(actions=a, rewards=r, dones=d, losses=losses[:n], indices=idx[:n * B].reshape(n, B),
                    targets=tg[:n * B].reshape(n, B))


TF_DTYPES = {1: np.float32, 2: np.float64, 3: np.int32, 9: np.int64}


class SumTree:
    """Proportional prioritized-replay sum tree in HBM (per.hip; beyond the reference)."""

    def __init__(self, capacity, device=0):
        self.capacity = int(capacity)
        h = C.c_void_p()
        _check(lib().qlx_sumtree_create(self.capacity, device, C.byref(h)))
        self.h = h.value

    def close(self):
        if getattr(self, "h", None):
            lib().qlx_sumtree_destroy(self.h)
        self.h = None

    __del__ = close

    def set_leaves(self, leaves):
        x = np.ascontiguousarray(leaves, dtype=np.float32)
        if x.shape != (self.capacity,):
            raise ValueError("leaves must have shape (capacity,)")
        _check(lib().qlx_sumtree_set_leaves(self.h, _p(x)))

    def get(self):
        leaves = np.zeros(self.capacity, np.float32)
        total, pmax = C.c_float(), C.c_float()
        _check(lib().qlx_sumtree_get(self.h, _p(leaves), C.byref(total), C.byref(pmax)))
        return leaves, total.value, pmax.value

    def sample(self, seed, first_update, n_updates, rank, length, beta, batch):
        slots = np.zeros(n_updates * batch, np.uint64)
        w = np.zeros(n_updates * batch, np.float32)
        _check(lib().qlx_sumtree_sample(self.h, seed, first_update, n_updates, rank, length, beta, batch, _p(slots), _p(w)))
        return slots.reshape(n_updates, batch), w.reshape(n_updates, batch)

    def update(self, slots, td_abs, alpha, eps):
        s_ = np.ascontiguousarray(slots, dtype=np.uint64).ravel()
        t_ = np.ascontiguousarray(td_abs, dtype=np.float32).ravel()
        if s_.shape != t_.shape:
            raise ValueError("slots and td_abs must have the same length")
        _check(lib().qlx_sumtree_update(self.h, _p(s_), _p(t_), s_.shape[0], alpha, eps))


class TfBundle:
    """TF tensor bundle (variables.index + variables.data-*) read by libqlx's host-side SSTable reader."""

    def __init__(self, prefix):
        h = C.c_void_p()
        _check(lib().qlx_tf_bundle_open(str(prefix).encode(), C.byref(h)))
        self.h = h.value

    def close(self):
        if getattr(self, "h", None):
            lib().qlx_tf_bundle_close(self.h)
        self.h = None

    __del__ = close

    def entries(self):
        """{name: (dtype enum, shape tuple, byte size)}"""
        out = {}
        for i in range(lib().qlx_tf_bundle_count(self.h)):
            name = C.create_string_buffer(512)
            dt, nd, nb = C.c_int32(), C.c_int32(), C.c_int64()
            dims = np.zeros(8, np.int64)
            _check(lib().qlx_tf_bundle_entry(self.h, i, name, 512, C.byref(dt), _p(dims), C.byref(nd), C.byref(nb)))
            out[name.value.decode()] = (dt.value, tuple(int(d) for d in dims[:nd.value]), nb.value)
        return out

    def read(self, name):
        dt, shape, nbytes = self.entries()[name]
        buf = np.zeros(nbytes, np.uint8)
        _check(lib().qlx_tf_bundle_read(self.h, name.encode(), _p(buf), nbytes))
        return buf.view(TF_DTYPES[dt]).reshape(shape)
