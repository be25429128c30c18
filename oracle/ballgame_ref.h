// ORACLE — TEST INFRASTRUCTURE ONLY (see rng_ref.h header).  Never linked into the product.
//
// CPU restatement of the reference's second environment + model pair:
//   BallGameTestEnvironment  /root/reference/src/ql/src/test/ballgame_test_environment.rs:12-262
//     3x3 field (x, y), y = 0 north; goal on a random column of row 0, ball on a random column of row 2,
//     obstacles at (1,1) and one random free field (:100-123); step (:69-86): +10 done on reaching the goal,
//     -10 done once steps >= MAX_STEPS = 16 (:12, :77), -0.02 legal move, -1 illegal move; do_move
//     (:155-190); actions West 0, North 1, East 2, South 3, Nothing 4 (:240-249); goal mean 9.5 (:88).
//   State tensor     /root/reference/src/ql-with-tensorflow/src/test/ballgame_test_env_addons.rs:7-50
//     one-hot [x][y][channel] with channel Empty 0, Goal 1, Ball 2, Obstacle 3.
//   Q-model          /root/reference/src/ql-with-tensorflow/python_model/create_ql_model_ballgame_3x3x4_5_512.py
//     :24-31 Conv2D(32, 2x2, stride 1, 'same', relu) -> Conv2D(32, 1x1, relu) -> Flatten -> Dense(512, relu)
//     -> Dense(5, linear); :35-40 Adam(lr 2.5e-4, clipnorm 1.0), MeanSquaredError; :71-85 train_model:
//     q_a = sum(Q(s) * one_hot(a)), loss = MSE(y, q_a) (mean over the batch).  TF 'same' padding of a 2x2
//     kernel at stride 1 pads one row / column AFTER the data (pad_before = 0, pad_after = 1).
// The bit source is the build's Philox stream (purpose P_BALLGAME: c1 = env id, c2 = reset count); the
// rand 0.8.5 derivation of `rng.gen_range(0..3)` for usize (UniformInt::sample_single_inclusive with the
// "(range << leading_zeros) - 1" zone, one u64 per draw) is restated exactly.
#pragma once
#include <cstdint>
#include <deque>
#include <vector>

#include "learner_ref.h"
#include "rng_ref.h"

namespace orc {

constexpr uint32_t P_BALLGAME = 6;
constexpr int kBgActions = 5;
constexpr int kBgMaxSteps = 16;
constexpr int kBgObs = 36;   // [3][3][4] u8 one-hot
enum BgEntry : uint8_t { BG_EMPTY = 0, BG_GOAL = 1, BG_BALL = 2, BG_OBSTACLE = 3 };

struct BgState {   // layout mirrored by qlx_ballgame_state (include/qlx.h)
  uint8_t field[9];   // index x * 3 + y
  uint8_t ball_x, ball_y, pad;
  uint32_t steps;
  uint32_t reset_count;
};

struct BgEnv {
  BgState s;
  uint64_t seed;
  uint32_t id;
};

// rand 0.8.5 UniformInt<usize>::sample_single_inclusive(0, n - 1) - `rng.gen_range(0..n)` on a usize range
uint64_t gen_range_usize_single(Stream& s, uint64_t n);

void bg_random_initial_state(BgState& st, Stream& s);          // :100-123
void bg_env_init(BgEnv& e, uint64_t seed, uint32_t id);        // BallGameTestEnvironment::new
void bg_env_reset(BgEnv& e);                                   // Environment::reset (:65)
void bg_env_step(BgEnv& e, uint8_t action, float* reward, bool* done);   // Environment::step (:69-86)
void bg_obs(const BgState& st, uint8_t* out /*[36]*/);         // to_multi_dim_array

// ---------------- Q-model (fp32) ----------------
constexpr int kBgVars = 8;
extern const int kBgVarSize[kBgVars];   // k0 [2,2,4,32] b0 [32] k1 [1,1,32,32] b1 [32] k2 [288,512] b2 [512] k3 [512,5] b3 [5]

struct BgNet {
  std::vector<float> w[kBgVars], m[kBgVars], v[kBgVars];
  int64_t iterations = 0;
  float lr = 0.00025f, beta1 = 0.9f, beta2 = 0.999f, eps = 1e-7f, clipnorm = 1.0f;
};
struct BgActs { std::vector<float> a1, a2, a3, q; };   // [B,9,32] [B,9,32] [B,512] [B,5] (post-ReLU)
struct BgGrads { std::vector<float> g[kBgVars]; };

void bg_net_init_glorot(BgNet& n, uint64_t seed);       // stream (seed, var, 1, P_INIT)
void bg_net_forward(const BgNet& n, const uint8_t* x /*[B][36]*/, int B, BgActs& a);
// MSE, raw gradients; weights (optional) per-sample loss weights, td_abs (optional) |q_a - y| out
float bg_net_loss_backward(const BgNet& n, const uint8_t* x, const uint8_t* actions, const float* y, int B, const BgActs& a,
                           BgGrads& g, const float* weights = nullptr, float* td_abs = nullptr);
void bg_net_apply_adam(BgNet& n, const BgGrads& g, float* norms_out /*[8] or null*/);

// ---------------- learner (the vectorised SelfDrivingQLearner of learner_ref.h over BallGame) -------------
struct BgParams {   // field layout = qlx_params (include/qlx.h)
  float gamma;
  float lowest_episode_reward_goal_threshold_pct;
  double epsilon_max;
  double epsilon_min;
  double epsilon_greedy_steps;
  uint64_t max_steps_per_episode;
  uint64_t epsilon_pure_random_steps;
  uint64_t history_buffer_len;
  uint64_t update_after_actions;
  uint64_t target_sync_steps;
  uint64_t episode_reward_history_buffer_len;
  uint32_t n_envs;
  uint32_t batch_size;
  uint64_t env_seed;
  uint64_t learner_seed;
  uint64_t init_seed;
  uint32_t rank;
  uint32_t flags;      // bit 0 double DQN, bit 1 prioritized replay (qlx.h QLX_LEARNER_*)
  float per_alpha, per_beta, per_eps;
  uint32_t qnet_precision;     // 0 fp32 (qnet32_ref.cpp, bit-exact definition), 1 bf16 product (double-accumulating oracle)
  uint64_t stats_after_steps;  // learning_update_log + write_checkpoint every this many env-steps (0 = never)
  char checkpoint_file[256];
};

struct BgTransition { uint8_t action; BgState s, s_next; float reward; bool done; };

struct BgLearner {
  BgParams p;
  std::vector<BgEnv> envs;
  std::vector<float> ep_reward;
  std::vector<uint64_t> ep_steps;
  std::deque<BgTransition> replay;
  uint64_t total_pushed = 0;   // prioritized replay (flags bit 1): SumTree over physical slots (learner_ref.h)
  SumTree tree;
  float per_max = 1.0f;
  BgNet online, target;
  uint64_t step_count = 0, vec_steps = 0, update_count = 0, episode_count = 0;
  double epsilon;
  float running_reward = 0.0f;
  std::deque<float> episode_rewards;
  std::vector<uint8_t> last_actions, last_dones;
  std::vector<float> last_rewards, last_losses, last_targets;
  std::vector<uint64_t> last_indices;

  explicit BgLearner(const BgParams& prm);
  void vector_step();
  void targets(const uint64_t* idx, float* y) const;
  void update(const uint64_t* idx, const float* isw, const float* y);
  bool solved() const;
};

}  // namespace orc
