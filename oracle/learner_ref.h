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
  uint32_t pad;
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

// self_driving_tf_q_learner.rs:276-296 with the build's counter-based stream
void generate_distinct_random_ids(uint64_t seed, uint32_t update_idx, uint32_t rank, uint64_t len, int B, uint64_t* out);

struct Learner {
  LearnerParams p;
  std::vector<Env> envs;
  std::vector<StateRef> state;
  std::vector<float> ep_reward;
  std::vector<uint64_t> ep_steps;
  Replay replay;
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

  explicit Learner(const LearnerParams& prm);
  void vector_step();
  void update();
  bool solved() const;
};

}  // namespace orc
