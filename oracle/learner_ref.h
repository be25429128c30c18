// ORACLE — TEST INFRASTRUCTURE ONLY (see rng_ref.h header).
//
// Restatement of the reference agent loop, replay buffer and sampler:
//   /root/reference/src/ql-with-tensorflow/src/learn/self_driving_tf_q_learner.rs:20-67 (Parameter),
//     :94-116 (new: online + "stabilized" model from the same init), :134-139 (solved),
//     :141-233 (learn_episode), :276-296 (generate_distinct_random_ids), :298-315 (add/mul arrays)
//   /root/reference/src/ql-with-tensorflow/src/learn/replay_buffer.rs:21-38,85-137 (FIFO, index 0 = oldest)
//
// Vectorised generalisation (defined by this build; N = 1 is exactly the reference loop):
//   one "vector step" = for e in 0..N: step_count += 1, epsilon-greedy action (Q from the weights at the
//   start of the vector step), epsilon decay;  then for e in 0..N: env step, replay push, episode
//   bookkeeping (+ reset on done / max_steps_per_episode);  then one update per multiple of
//   update_after_actions crossed by step_count, if replay.len > batch.
//   Target network: never synced when target_sync_steps == 0 (the reference: the sync is commented
//   out at :205-210 and update_target_network_after_num_steps is never read).
//   All U batches of a vector step are sampled, and their Bellman targets computed, before its first update.
// Beyond the reference (flags): double DQN targets (a* = argmax of the online net as it stands
//   before the vector step's updates) and proportional prioritized replay (SumTree below).
#pragma once
#include <cstdint>
#include <deque>
#include <memory>
#include <vector>

#include "breakout_ref.h"
#include "qnet_ref.h"

namespace orc {

constexpr int kStateBytes = kFramePix * kSlots;   // 28,224

struct LearnerParams {   // layout mirrored by tests/oracle.py (ctypes)
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
  float episode_reward_goal;   // NaN = the env's own (kNumBricks - 1); any other value mocks it (qlx.h)
};

using StateRef = std::shared_ptr<std::vector<uint8_t>>;   // Rc<BreakoutState> tensor view [x][y][slot]

struct Transition { uint8_t action; StateRef s, s_next; float reward; bool done; };

struct Replay {   // replay_buffer.rs: five parallel VecDeques share one FIFO position
  size_t cap;
  std::deque<Transition> buf;
  explicit Replay(size_t c) : cap(c) {}
  void add(const Transition& t) { if (buf.size() >= cap) buf.pop_front(); buf.push_back(t); }
  size_t len() const { return buf.size(); }
};

constexpr uint32_t P_PER = 7;   // prioritized-replay draws: c1 = update index, c2 = rank, word = sample

// Proportional prioritized replay (Schaul et al. 2016) - beyond the reference.
// Leaves = replay slots (physical FIFO positions), values p^alpha; every internal node = left + right in f32
// (so the tree is a pure function of the leaves).  Batch b of B draws u = (T / B) * (b + r_b), r_b =
// gen_range_f32(0, 1) from Stream(seed, update, rank, P_PER, word b), and descends: left iff u < left sum
// (or the right subtree is empty), else u -= left sum.  IS weights w = (len * leaf / T)^-beta / max over the
// batch.
struct SumTree {
  uint32_t L = 1;   // leaves (power of two >= capacity)
  std::vector<float> t;
  explicit SumTree(uint64_t cap) { while (L < cap) L <<= 1; t.assign(2 * (size_t)L, 0.0f); }
  void set(uint64_t leaf, float v) {
    size_t i = L + leaf;
    t[i] = v;
    for (i >>= 1; i >= 1; i >>= 1) t[i] = t[2 * i] + t[2 * i + 1];
  }
  uint64_t find(float u) const {
    size_t i = 1;
    while (i < L) {
      const float left = t[2 * i];
      if (u < left || t[2 * i + 1] == 0.0f) i = 2 * i;
      else { u -= left; i = 2 * i + 1; }
    }
    return i - L;
  }
};
// x^y of the prioritized replay (priorities (|td| + eps)^alpha, IS weights (len p)^-beta) as the build defines it
// (the product's per.hip per_powf follows the same steps): exp(y ln x) evaluated in binary64 with IEEE basic
// operations only (ln m by the atanh series in f = (m - 1) / (m + 1), exp by argument reduction + a degree-15 Taylor
// polynomial, every multiply-add an explicit fma), rounded once to binary32.  Not the library powf: glibc and the device
// libm each round their own way in the last bit, and one ulp in a leaf moves the sum tree's partial sums.
float det_powf(float x, float y);
// one prioritized batch: physical slots and normalised IS weights
void per_sample(const SumTree& st, uint64_t seed, uint32_t update_idx, uint32_t rank, uint64_t len, float beta, int B,
                uint64_t* slots, float* weights);

// self_driving_tf_q_learner.rs:276-296 with the build's counter-based stream
void generate_distinct_random_ids(uint64_t seed, uint32_t update_idx, uint32_t rank, uint64_t len, int B, uint64_t* out);

struct Learner {
  LearnerParams p;
  std::vector<Env> envs;
  std::vector<StateRef> state;
  std::vector<float> ep_reward;
  std::vector<uint64_t> ep_steps;
  Replay replay;
  uint64_t total_pushed = 0;   // FIFO position of the next push (prioritized replay maps slots <-> logical indices)
  SumTree tree;
  float per_max = 1.0f;        // largest leaf value so far (new transitions enter at it)
  QNet online, target;
  uint64_t step_count = 0;
  double epsilon;
  uint64_t vec_steps = 0;
  uint64_t update_count = 0;
  uint64_t episode_count = 0;
  float running_reward = 0.0f;
  std::deque<float> episode_rewards;   // episode_reward_history (cap episode_reward_history_buffer_len)
  // outputs of the last vector step (for parity tests)
  std::vector<uint8_t> last_actions;
  std::vector<float> last_rewards;
  std::vector<uint8_t> last_dones;
  std::vector<float> last_losses;
  std::vector<uint64_t> last_indices;   // [n_updates][B]
  std::vector<float> last_q;            // [N][3] acting Q values (if computed)
  std::vector<float> last_targets;      // [n_updates][B] y
  std::vector<float> last_weights;      // [n_updates][B] IS weights (1 without prioritized replay)

  uint64_t stats_events = 0;            // write_checkpoint + learning_update_log events so far

  // CPU baseline only (oracle/cpu_baseline): also build the reference's f32 input tensors element by element, as
  // BreakoutState::batch_to_multi_dim_array / to_multi_dim_array do (breakout_environment.rs:36-77), for s' of every
  // target pass, s of every train step and each greedy acting state; the restated Q-net reads the u8 view (same values),
  // so the tensors feed a checksum only.  Off for parity runs (no effect on any result).
  bool pack_like_reference = false;
  double pack_sink = 0.0;
  void pack_reference(const std::vector<StateRef>& states) ;

  explicit Learner(const LearnerParams& prm);
  // train = false: act, step, push and keep the books only (replay prefill: no updates, no update_count)
  void vector_step(bool train = true);
  void fwd(const QNet& q, const uint8_t* x, int B, Acts& a) const;
  void targets(const uint64_t* idx, float* y) const;
  // logical indices of the batch, IS weights (or null), Bellman targets
  void update(const uint64_t* idx, const float* isw, const float* y);
  bool solved() const;
};

}  // namespace orc
