/* qlx.h — C ABI of the MI355X-native DQN hot path (env-step -> replay-sample -> Q-net update).
 *
 * This is the drop-in boundary for bitmagier/q-learning's Breakout DQN path.  Every entry point
 * names the reference interface it replaces (paths relative to the reference repo root):
 *
 *   ql::Environment / ql::Action         src/ql/src/prelude.rs:12-63
 *   BreakoutEnvironment (+ mechanics)   src/_breakout-ml/src/breakout_environment.rs:131-207,
 *                                        src/breakout-game/src/mechanics.rs:56-135
 *   ReplayBuffer / get_many             src/ql-with-tensorflow/src/learn/replay_buffer.rs:52-138
 *   generate_distinct_random_ids        src/ql-with-tensorflow/src/learn/self_driving_tf_q_learner.rs:276-296
 *   DeepQLearningModel                  src/ql-with-tensorflow/src/ml_model/model.rs:29-77
 *   SelfDrivingQLearner / Parameter     src/ql-with-tensorflow/src/learn/self_driving_tf_q_learner.rs:20-139
 *   BallGameTestEnvironment (2nd env)   src/ql/src/test/ballgame_test_environment.rs:12-262,
 *                                        src/ql-with-tensorflow/src/test/ballgame_test_env_addons.rs:7-50,
 *                                        src/ql-with-tensorflow/python_model/create_ql_model_ballgame_3x3x4_5_512.py
 *
 * Conventions
 *   - Opaque handles; every call returns int32_t status (QLX_OK = 0, < 0 = error) and
 *     qlx_last_error() returns a thread-local message.  This replaces the reference's
 *     panic!/anyhow::Result (q_learning_model.rs:125,147; mechanics.rs:265,284,303,511).
 *   - Host pointers are caller-owned.  Functions with a `_dev` suffix take device pointers and
 *     enqueue on the object's HIP stream without synchronising (chain them; qlx_*_sync to wait).
 *   - Calls on one handle are externally synchronised (the reference is single-threaded: Rc +
 *     ThreadRng are !Send).
 *   - Observation layout exposed to callers is the reference tensor view [n][x][y][slot] u8
 *     (breakout_environment.rs:44-50: H axis = x, channel = ring slot, raw 0..255).
 *   - No PyTorch/TF types; plain pointers and sizes only.
 */
#ifndef QLX_H
#define QLX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define QLX_OK 0
#define QLX_E_INVALID (-1)
#define QLX_E_HIP (-2)
#define QLX_E_OOM (-3)
#define QLX_E_STATE (-4)
#define QLX_E_COMM (-5)
#define QLX_E_IO (-6)

#define QLX_ENV_BREAKOUT 1
#define QLX_ENV_BALLGAME 2
/* Conv(32,8,s4)-Conv(64,4,s2)-Conv(64,3,s1)-Dense512-Dense3 in fp32: the reference's arithmetic, every reduction a
 * single fmaf chain in the order DESIGN.md §6 defines (bit-exact against the CPU oracle) */
#define QLX_ARCH_NATURE_DQN 1
/* the same net with bf16 MFMA operands, fp32 accumulation and fp32 master weights (the labelled fast path) */
#define QLX_ARCH_NATURE_DQN_BF16 2
/* fp32 weight gradients of the conv layers: per-chunk fmaf chains over this many samples, chunks summed in order */
#ifndef QLX_F32_WGRAD_CHUNK_CONV1   /* (overridable only for A/B timing builds; the oracle follows 2) */
#define QLX_F32_WGRAD_CHUNK_CONV1 2   /* round 6: 4 -> 2 (twice the conv1 weight-gradient blocks: 36.2 -> 31.1 us at B = 1024) */
#endif
#define QLX_F32_WGRAD_CHUNK_CONV2 16
#define QLX_F32_WGRAD_CHUNK_CONV3 16

const char* qlx_last_error(void);
int32_t qlx_version(void);

/* ---------------- Environment (ql::Environment for Breakout, batched) ---------------- */

/* Mechanics snapshot of one env, for parity checks (BreakoutMechanics, mechanics.rs:46-54). */
typedef struct qlx_breakout_state {
  float ball_x, ball_y, dir_x, dir_y;
  float panel_min_x, panel_min_y, panel_max_x, panel_max_y, panel_speed;
  uint32_t score, finished, next_slot, fault, reset_count;
  uint64_t bricks; /* bit i = brick i (creation order) still present */
} qlx_breakout_state;

typedef struct qlx_env qlx_env;

/* Action::ACTION_SPACE (breakout_environment.rs:103; BallGame 5, ballgame_test_environment.rs:239) */
int32_t qlx_env_action_space(int32_t kind);
/* Environment::episode_reward_goal_mean (breakout_environment.rs:203-206): bricks - 1 = 59; BallGame 9.5 (:88) */
float qlx_env_reward_goal_mean(int32_t kind);

/* BreakoutEnvironment::new x n_envs on `device`; env i draws its ball launch angle from the
 * build's counter-based stream (seed, i, reset_count) instead of thread_rng (mechanics.rs:103). */
int32_t qlx_env_create(int32_t kind, uint32_t n_envs, uint64_t seed, int32_t device, qlx_env** out);
int32_t qlx_env_destroy(qlx_env* env);
uint32_t qlx_env_count(const qlx_env* env);
/* Environment::reset (breakout_environment.rs:177-180) for every env, or where mask[i] != 0. */
int32_t qlx_env_reset(qlx_env* env, const uint8_t* mask_or_null);
/* Environment::step (breakout_environment.rs:184-201) for all envs; host arrays of n_envs.
 * Invalid actions (>= 3) fail with QLX_E_INVALID like Action::try_from_numeric. */
int32_t qlx_env_step(qlx_env* env, const uint8_t* actions, float* rewards, uint8_t* dones);
/* Device-pointer form: actions/rewards/dones are device arrays of n_envs. */
int32_t qlx_env_step_dev(qlx_env* env, const uint8_t* d_actions, float* d_rewards, uint8_t* d_dones);
/* ToMultiDimArray::batch_to_multi_dim_array view of the current states: out[n][84][84][4] (x,y,slot). */
int32_t qlx_env_obs(qlx_env* env, uint8_t* out);
int32_t qlx_env_states(qlx_env* env, qlx_breakout_state* out /* [n_envs] */);
/* Running per-env checksum of every step (state + new frame), see DESIGN.md §parity. */
int32_t qlx_env_hashes(qlx_env* env, uint64_t* out /* [n_envs] */);
int32_t qlx_env_sync(qlx_env* env);

/* ---------------- Replay buffer (ReplayBuffer, HBM-resident) ---------------- */

typedef struct qlx_replay qlx_replay;

/* FIFO of `capacity` transitions (history_buffer_len); logical index 0 = oldest (VecDeque). Frames
 * are stored once (s' of step t is s of step t+1), 7,056 B per transition + metadata. */
int32_t qlx_replay_create(uint64_t capacity, uint32_t n_envs, int32_t device, qlx_replay** out);
int32_t qlx_replay_destroy(qlx_replay* rb);
uint64_t qlx_replay_len(const qlx_replay* rb);
/* ReplayBuffer::add for the transition each env of `env` just made (actions = device array used for
 * that step, rewards/dones = its outputs).  Call once after every qlx_env_step[_dev]. */
int32_t qlx_replay_push_dev(qlx_replay* rb, qlx_env* env, const uint8_t* d_actions, const float* d_rewards,
                            const uint8_t* d_dones);
/* Host-array form of qlx_replay_push_dev (synchronises). */
int32_t qlx_replay_push(qlx_replay* rb, qlx_env* env, const uint8_t* actions, const float* rewards,
                        const uint8_t* dones);
/* generate_distinct_random_ids::<B>(rng, 0..len) from stream (seed, update_idx, rank); host out[B]. */
int32_t qlx_replay_sample_distinct(qlx_replay* rb, uint64_t seed, uint32_t update_idx, uint32_t rank, uint32_t batch,
                                   uint64_t* out_indices);
/* ReplayBuffer::get_many + batch_to_multi_dim_array: host outputs, any may be NULL. */
int32_t qlx_replay_get_many(qlx_replay* rb, const uint64_t* indices, uint32_t batch, uint8_t* s /*[B][84][84][4]*/,
                            uint8_t* s_next, uint8_t* actions, float* rewards, uint8_t* dones);

/* ---------------- Q-network (DeepQLearningModel) ---------------- */

typedef struct qlx_model qlx_model;

/* Nature-DQN (arch QLX_ARCH_NATURE_DQN = fp32, QLX_ARCH_NATURE_DQN_BF16 = bf16 MFMA operands) with GlorotUniform
 * weights from stream (seed, var, 0) and zero biases; fp32 master weights + Adam slots in HBM.  lr 2.5e-4, beta
 * 0.9/0.999, eps 1e-7, clipnorm 1. */
int32_t qlx_model_create(int32_t arch, uint64_t seed, int32_t device, qlx_model** out);
int32_t qlx_model_destroy(qlx_model* m);
int32_t qlx_model_num_vars(void);
/* The optimizer hyperparameters every model is created with, out[5] = {learning_rate, beta_1, beta_2, epsilon, clipnorm}
 * (float32; the reference's Keras optimizer_config, keras_metadata.pb; no device needed). */
int32_t qlx_model_hparams(float* out);
int64_t qlx_model_var_size(int32_t var);
/* which: 0 = weights, 1 = Adam m, 2 = Adam v.  Layout = Keras HWIO / [in,out]. */
int32_t qlx_model_get_var(qlx_model* m, int32_t var, int32_t which, float* out);
int32_t qlx_model_set_var(qlx_model* m, int32_t var, int32_t which, const float* in);
int64_t qlx_model_iterations(qlx_model* m);
int32_t qlx_model_copy_weights(qlx_model* dst, const qlx_model* src);
/* predict_action for n states (model.rs:39-42): q_out [n][3] (may be NULL), actions [n] = argmax. */
int32_t qlx_model_predict(qlx_model* m, const uint8_t* obs /*[n][84][84][4]*/, uint32_t n, float* q_out,
                          uint8_t* actions);
/* batch_predict_max_future_reward (model.rs:44-47). */
int32_t qlx_model_batch_max_q(qlx_model* m, const uint8_t* obs, uint32_t n, float* out);
/* train (model.rs:49-65): forward, Huber(1) mean, backward, clip_by_norm(1) per variable, Adam.
 * loss_out (may be NULL) gets the batch loss; grads_out (may be NULL) the raw gradients of all vars
 * concatenated; norms_out (may be NULL) the 10 per-variable L2 norms before clipping. */
int32_t qlx_model_train(qlx_model* m, const uint8_t* obs, const uint8_t* actions, const float* y, uint32_t batch,
                        float* loss_out, float* grads_out, float* norms_out);
// Test hook of the data-parallel update tail (round 6): clip_by_norm(grads * scale) per variable + legacy Adam
// (ResourceApplyAdam, iterations + 1) on host gradients [1,685,667] in the flat variable order, as learner_update runs the
// tail after an all-reduce with scale = 1 / world (self_driving_tf_q_learner.rs:201 train -> q_learning_model.rs:165-189,
// split by the build's DP).  norms_out [10] (or NULL): the clip norms of the scaled gradient.
int32_t qlx_model_apply_gradient(qlx_model* m, const float* grads, float scale, float* norms_out);
/* Load a TF SavedModel / checkpoint bundle of the reference Breakout model (layer_with_weights-0..4 kernel /
 * bias, OPTIMIZER_SLOT m / v, optimizer/iter; shapes checked against saved/ql_model_breakout_84x84x4_3_32). */
int32_t qlx_model_load_tf(qlx_model* m, const char* bundle_prefix);
/* Debug view of intermediate activations of the last predict: layer 1..4 as fp32 host arrays. */
int32_t qlx_model_last_activation(qlx_model* m, int32_t layer, float* out);
/* write_checkpoint (model.rs:67-70): weights + Adam slots + iterations in a flat file. */
int32_t qlx_model_write_checkpoint(qlx_model* m, const char* path);
int32_t qlx_model_read_checkpoint(qlx_model* m, const char* path);
int32_t qlx_model_sync(qlx_model* m);

/* ---------------- Learner (SelfDrivingQLearner) ---------------- */

typedef struct qlx_params { /* Parameter (self_driving_tf_q_learner.rs:20-67) + build fields */
  float gamma;
  float lowest_episode_reward_goal_threshold_pct;
  double epsilon_max;
  double epsilon_min;
  double epsilon_greedy_steps;
  uint64_t max_steps_per_episode;
  uint64_t epsilon_pure_random_steps;
  uint64_t history_buffer_len;
  uint64_t update_after_actions;
  uint64_t target_sync_steps; /* 0 = never (reference behaviour) */
  uint64_t episode_reward_history_buffer_len;
  uint32_t n_envs;
  uint32_t batch_size;
  uint64_t env_seed;
  uint64_t learner_seed;
  uint64_t init_seed;
  uint32_t rank;
  uint32_t flags;     /* QLX_LEARNER_* extensions beyond the reference (0 = the reference algorithm) */
  float per_alpha;    /* prioritized replay: P(i) ~ p_i^alpha, p_i = |td_i| + per_eps */
  float per_beta;     /* importance-sampling exponent, w_i = (len P(i))^-beta / max_batch w */
  float per_eps;
  uint32_t qnet_precision;     /* QLX_PREC_F32 (0, the reference's arithmetic) or QLX_PREC_BF16 */
  uint64_t stats_after_steps;  /* every this many env-steps: checkpoint + learning_update_log (0 = never) */
  char checkpoint_file[256];   /* write_checkpoint target of those events and of solved() (empty = not written) */
  float episode_reward_goal;   /* goal solved() tests (Environment::episode_reward_goal_mean, prelude.rs); NaN (the
                                  qlx_params_default value) = the env's own (Breakout: bricks - 1,
                                  breakout_environment.rs:203-206); any other value, 0 included, mocks it.
                                  ABI semantics change in round 4: 0 used to select the env's goal; a zero-filled
                                  struct now mocks a goal of 0 (qlx_learner_create warns on stderr) */
} qlx_params;

#define QLX_PREC_F32 0u
#define QLX_PREC_BF16 1u

/* qlx_params.flags */
#define QLX_LEARNER_DOUBLE_DQN 1u  /* y = r + gamma Q_target(s', argmax_a Q_online(s')) (van Hasselt et al. 2016) */
#define QLX_LEARNER_PER 2u         /* proportional prioritized replay on an HBM sum tree (Schaul et al. 2016) */

void qlx_params_default(qlx_params* p);

typedef struct qlx_learner qlx_learner;

typedef struct qlx_learner_stats {
  uint64_t step_count, vec_steps, update_count, episode_count, replay_len, solved;
  double epsilon;
  float running_reward, last_loss;
} qlx_learner_stats;

/* SelfDrivingQLearner::new: owns a batched env, replay, online + target ("stabilized") model. */
int32_t qlx_learner_create(const qlx_params* p, int32_t device, qlx_learner** out);
int32_t qlx_learner_destroy(qlx_learner* l);
/* One vector step (n_envs env-steps + the updates they trigger), enqueued asynchronously. */
int32_t qlx_learner_vector_step(qlx_learner* l);
int32_t qlx_learner_run(qlx_learner* l, uint64_t n_vector_steps);
/* Vector steps without updates (act, env step, replay push, episode books; epsilon and step_count advance): fills the
 * replay before a measurement or a parity check at a given replay occupancy.  Not in the reference loop. */
int32_t qlx_learner_prefill(qlx_learner* l, uint64_t n_vector_steps);
/* End the current episode of every env with mask[e] != 0 now, as reaching max_steps_per_episode does (learn_episode
 * :214-224: the episode's reward enters the reward history, episode_count advances, the env resets); no transition is
 * added.  mask: host array [n_envs].  Lets a measurement start the envs' episodes at staggered steps (all envs launch
 * together, so with a short-lived policy their episodes otherwise end in waves).  Not in the reference loop.  Data
 * parallel: a collective (the global solved() statistics are all-reduced), so every rank calls it. */
int32_t qlx_learner_end_episodes(qlx_learner* l, const uint8_t* mask);
/* learn_till_mastered (self_driving_tf_q_learner.rs:127-132): vector steps until solved() or max_vector_steps. */
int32_t qlx_learner_learn_till_mastered(qlx_learner* l, uint64_t max_vector_steps, uint64_t* steps_run);
/* Statistics events so far (write_checkpoint + learning_update_log every stats_after_steps env-steps and on solved,
 * :204-212,226-230); the last event's log text; a callback receiving each log text (the reference's log::info!). */
uint64_t qlx_learner_stats_events(const qlx_learner* l);
int32_t qlx_learner_last_log(qlx_learner* l, char* buf, size_t cap, size_t* len);
int32_t qlx_learner_set_log_callback(qlx_learner* l, void (*cb)(const char* text, void* user), void* user);
int32_t qlx_learner_sync(qlx_learner* l);
int32_t qlx_learner_stats_get(qlx_learner* l, qlx_learner_stats* out);
/* Outputs of the last vector step (host copies; synchronises): actions/rewards/dones [n_envs],
 * losses [n_updates], indices [n_updates][B], targets [n_updates][B]; any may be NULL. Returns the
 * number of updates of that step in *n_updates. */
int32_t qlx_learner_last(qlx_learner* l, uint8_t* actions, float* rewards, uint8_t* dones, float* losses,
                         uint64_t* indices, float* targets, uint32_t* n_updates);
/* Prioritized replay state (learner created with QLX_LEARNER_PER): IS weights of the last vector step's batches
 * [n_updates][B], the sum tree's leaves [history_buffer_len] (priority^alpha per physical replay slot), the
 * priority new transitions enter with; any may be NULL. */
int32_t qlx_learner_priorities(qlx_learner* l, float* is_weights, float* leaves, float* per_max);
/* Frame sparsity of the last vector step (diagnostic, not on the hot path; synchronises): the fractions of the fp32
 * conv work the exact zero skips leave out, in the kernels' own units - out[0..3] over the step's sampled training
 * states (NaN when the step ran no update), out[4..7] over the current acting frames (the observations the next
 * vector step acts on: after this step's env step and resets), each {conv1 forward all-zero steps,
 * conv1 weight-gradient all-zero steps, conv2 background rows, conv3 background rows}. */
int32_t qlx_learner_frame_sparsity(qlx_learner* l, double* out);
/* Learning statistics (learning_update_log, self_driving_tf_q_learner.rs:235-273): per-action counts over the
 * replay's actions [3] (device histogram), the episode reward history oldest first (n = entries, up to cap
 * copied), and the log text itself (UTF-8; *len = full length, buf gets up to cap - 1 bytes + NUL).  Actions are
 * listed in numeric order (the reference iterates a hash map). */
int32_t qlx_learner_action_counts(qlx_learner* l, uint64_t* counts);
int32_t qlx_learner_episode_rewards(qlx_learner* l, float* out, uint64_t cap, uint64_t* n);
int32_t qlx_learner_update_log(qlx_learner* l, char* buf, size_t cap, size_t* len);
qlx_env* qlx_learner_env(qlx_learner* l);
qlx_replay* qlx_learner_replay(qlx_learner* l);
qlx_model* qlx_learner_model(qlx_learner* l, int32_t which /* 0 online, 1 target */);
/* Data-parallel: RCCL communicator over world ranks (one process per GPU); gradients are
 * all-reduced (mean) before clip_by_norm + Adam. uid from qlx_dist_unique_id on rank 0. */
int32_t qlx_dist_unique_id(uint8_t out[128]);
int32_t qlx_learner_dist_init(qlx_learner* l, int32_t world, int32_t rank, const uint8_t uid[128]);
/* Rank count of the learner's RCCL communicator as RCCL reports it (ncclCommCount); 1 without dist_init.  At world W
 * every update averages W per-rank batches of batch_size samples: the global batch per update is W x batch_size. */
int32_t qlx_learner_comm_size(qlx_learner* l, int32_t* world);
/* Kernel timing with HIP events on the learner stream.  Scopes are named per kernel ("conv1_fwd",
 * "conv1_wgrad", "fc1_fwd", "adam", "env_step", "replay_push", ...) or per phase ("act_forward",
 * "gather", "sample"); each carries its algorithmic work (FLOPs for GEMM kernels, bytes for
 * HBM-bound ones).  filter = one scope name records only that scope (NULL = all). */
int32_t qlx_learner_profile(qlx_learner* l, int32_t enable);
int32_t qlx_learner_profile_filter(qlx_learner* l, const char* name_or_null);
/* filter + sampling: record every stride-th launch of that scope (dispatch-bound events, see profiler.h) */
int32_t qlx_learner_profile_sample(qlx_learner* l, const char* name_or_null, uint32_t stride);
int32_t qlx_learner_profile_get(qlx_learner* l, const char* name, double* total_us, double* total_work,
                                uint64_t* launches);
int32_t qlx_learner_profile_names(qlx_learner* l, char* buf, size_t cap);

/* ---------------- DBSCAN over f32 (src/ql/src/util/dbscan.rs:209-341) ----------------
 * cluster_analysis(values, max_neighbor_distance, core_point_min_neighbors) with Distance = |a - b|, exact, in
 * O(n log n): labels[i] = cluster position (clusters ordered by lowest member index, as the reference returns
 * them) or -1 for noise.  _format renders the reference's Display ("Yx(B..C), ..., Yx(noise)", :91-133).
 * Values and max_neighbor_distance must be finite, max_neighbor_distance >= 0. */
int32_t qlx_dbscan_f32(const float* values, uint64_t n, float max_neighbor_distance, uint64_t core_point_min_neighbors,
                       int32_t* labels, uint64_t* n_clusters);
int32_t qlx_dbscan_f32_format(const float* values, uint64_t n, float max_neighbor_distance, uint64_t core_point_min_neighbors,
                              char* buf, size_t cap, size_t* len);

/* ---------------- prioritized-replay sum tree (beyond the reference) ----------------
 * The learner's HBM sum tree as a standalone object: leaves = priorities of `capacity` slots, proportional
 * sampling of n_updates batches of `batch` draws (draw b of update u: stream (seed, first_update + u, rank,
 * purpose 7, word b)), IS weights (len P(i))^-beta normalised per batch, and last-writer-wins priority
 * updates p = (|td| + eps)^alpha.  Oracle: oracle/learner_ref.h SumTree / per_sample. */
typedef struct qlx_sumtree qlx_sumtree;
int32_t qlx_sumtree_create(uint64_t capacity, int32_t device, qlx_sumtree** out);
int32_t qlx_sumtree_destroy(qlx_sumtree* t);
int32_t qlx_sumtree_set_leaves(qlx_sumtree* t, const float* leaves /* [capacity], finite >= 0 */);
int32_t qlx_sumtree_get(qlx_sumtree* t, float* leaves, float* total, float* per_max);
int32_t qlx_sumtree_sample(qlx_sumtree* t, uint64_t seed, uint32_t first_update, uint32_t n_updates, uint32_t rank, uint64_t len,
                           float beta, uint32_t batch, uint64_t* slots /* [n_updates][batch] */, float* weights);
int32_t qlx_sumtree_update(qlx_sumtree* t, const uint64_t* slots, const float* td_abs, uint32_t n, float alpha, float eps);

/* ---------------- BallGame (BallGameTestEnvironment + its 3x3x4 -> 5 Q-model) ----------------
 * The reference's second Environment / DeepQLearningModel pair, batched on the GPU.  Same conventions as
 * above; actions West 0, North 1, East 2, South 3, Nothing 4 (ballgame_test_environment.rs:240-249). */

typedef struct qlx_ballgame_state { /* BallGameState (:92-97) */
  uint8_t field[9];                  /* index x * 3 + y: 0 empty, 1 goal, 2 ball, 3 obstacle */
  uint8_t ball_x, ball_y, pad;
  uint32_t steps;
  uint32_t reset_count;
} qlx_ballgame_state;

typedef struct qlx_bg_env qlx_bg_env;
/* BallGameTestEnvironment::new x n_envs: env i's random_initial_state (:100-123) draws gen_range(0..3) from
 * the build's stream (seed, i, reset_count, purpose 6) instead of thread_rng. */
int32_t qlx_bg_env_create(uint32_t n_envs, uint64_t seed, int32_t device, qlx_bg_env** out);
int32_t qlx_bg_env_destroy(qlx_bg_env* env);
int32_t qlx_bg_env_reset(qlx_bg_env* env, const uint8_t* mask_or_null);
/* Environment::step (:69-86) for all envs (host arrays of n_envs; actions >= 5 fail with QLX_E_INVALID). */
int32_t qlx_bg_env_step(qlx_bg_env* env, const uint8_t* actions, float* rewards, uint8_t* dones);
/* to_multi_dim_array: out[n][3][3][4] u8 one-hot (x, y, channel = entry). */
int32_t qlx_bg_env_obs(qlx_bg_env* env, uint8_t* out);
int32_t qlx_bg_env_states(qlx_bg_env* env, qlx_ballgame_state* out);
int32_t qlx_bg_env_set_states(qlx_bg_env* env, const qlx_ballgame_state* in);

typedef struct qlx_bg_model qlx_bg_model;
/* Conv(32, 2x2 same)-Conv(32, 1x1)-Dense512-Dense5 in fp32; GlorotUniform from stream (seed, var, 1);
 * 8 variables k0 [2,2,4,32] b0 k1 [1,1,32,32] b1 k2 [288,512] b2 k3 [512,5] b3. */
int32_t qlx_bg_model_create(uint64_t seed, int32_t device, qlx_bg_model** out);
/* as qlx_model_hparams, for the BallGame model (create_ql_model_ballgame_3x3x4_5_512.py's Adam) */
int32_t qlx_bg_model_hparams(float* out);
int32_t qlx_bg_model_destroy(qlx_bg_model* m);
int64_t qlx_bg_model_var_size(int32_t var);
int32_t qlx_bg_model_get_var(qlx_bg_model* m, int32_t var, int32_t which, float* out);
int32_t qlx_bg_model_set_var(qlx_bg_model* m, int32_t var, int32_t which, const float* in);
int64_t qlx_bg_model_iterations(qlx_bg_model* m);
int32_t qlx_bg_model_predict(qlx_bg_model* m, const uint8_t* obs /*[n][3][3][4]*/, uint32_t n, float* q_out, uint8_t* actions);
int32_t qlx_bg_model_batch_max_q(qlx_bg_model* m, const uint8_t* obs, uint32_t n, float* out);
/* train_model (.py:71-85): MSE of q_a, backward, clip_by_norm(1) per variable, Adam. */
int32_t qlx_bg_model_train(qlx_bg_model* m, const uint8_t* obs, const uint8_t* actions, const float* y, uint32_t batch,
                           float* loss_out, float* grads_out, float* norms_out);

/* Load a TF SavedModel / checkpoint bundle of the reference model (variables/variables.index + .data, e.g.
 * python_model/saved/ql_model_ballgame_3x3x4_5_512/variables/variables): weights, Adam m / v and iterations. */
int32_t qlx_bg_model_load_tf(qlx_bg_model* m, const char* bundle_prefix);

typedef struct qlx_bg_learner qlx_bg_learner;
/* SelfDrivingQLearner over BallGame (same qlx_params and vector-step semantics as qlx_learner). */
int32_t qlx_bg_learner_create(const qlx_params* p, int32_t device, qlx_bg_learner** out);
int32_t qlx_bg_learner_destroy(qlx_bg_learner* l);
int32_t qlx_bg_learner_run(qlx_bg_learner* l, uint64_t n_vector_steps);
int32_t qlx_bg_learner_sync(qlx_bg_learner* l);
int32_t qlx_bg_learner_stats_get(qlx_bg_learner* l, qlx_learner_stats* out);
int32_t qlx_bg_learner_last(qlx_bg_learner* l, uint8_t* actions, float* rewards, uint8_t* dones, float* losses,
                            uint64_t* indices, float* targets, uint32_t* n_updates);
/* prioritized replay state of a learner created with QLX_LEARNER_PER (as qlx_learner_priorities) */
int32_t qlx_bg_learner_priorities(qlx_bg_learner* l, float* is_weights, float* leaves, float* per_max);
/* learning_update_log for BallGame: counts [5] by numeric action, reward history, log text (qlx_learner_* above) */
int32_t qlx_bg_learner_action_counts(qlx_bg_learner* l, uint64_t* counts);
int32_t qlx_bg_learner_episode_rewards(qlx_bg_learner* l, float* out, uint64_t cap, uint64_t* n);
int32_t qlx_bg_learner_update_log(qlx_bg_learner* l, char* buf, size_t cap, size_t* len);
qlx_bg_env* qlx_bg_learner_env(qlx_bg_learner* l);
qlx_bg_model* qlx_bg_learner_model(qlx_bg_learner* l, int32_t which /* 0 online, 1 target */);

/* ---------------- TF tensor bundles (the reference's model / checkpoint storage) ----------------
 * Host-only reader of variables.index (SSTable of BundleEntryProto) + variables.data-*; block and tensor
 * crc32c are verified.  Replaces SavedModelBundle::load's variable restore (q_learning_model.rs:47-52). */
typedef struct qlx_tf_bundle qlx_tf_bundle;
int32_t qlx_tf_bundle_open(const char* prefix /* ".../variables/variables" */, qlx_tf_bundle** out);
int32_t qlx_tf_bundle_close(qlx_tf_bundle* b);
int32_t qlx_tf_bundle_count(const qlx_tf_bundle* b);
/* dtype: TF DataType enum (1 = float, 9 = int64); dims: up to 8 */
int32_t qlx_tf_bundle_entry(const qlx_tf_bundle* b, int32_t i, char* name, size_t cap, int32_t* dtype, int64_t* dims,
                            int32_t* ndims, int64_t* nbytes);
int32_t qlx_tf_bundle_read(const qlx_tf_bundle* b, const char* name, void* out, size_t cap);

#ifdef __cplusplus
}
#endif
#endif /* QLX_H */
