// Host-side definitions of the opaque ABI objects (internal).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "qlx_internal.h"

struct qlx_env {
  int device = 0;
  uint32_t n = 0;
  uint64_t seed = 0;
  uint32_t id_offset = 0;         // global id of env 0 (data-parallel ranks own disjoint ids)
  hipStream_t stream = nullptr;   // owned unless adopted by a learner
  bool own_stream = true;
  qlx_breakout_state* d_state = nullptr;
  uint32_t* d_ep_steps = nullptr;  // [n] steps taken in the current episode
  uint8_t* d_obs = nullptr;        // [n][4][7056] ring frames, s2d layout
  uint64_t* d_hash = nullptr;      // [n] running parity checksum
  uint32_t* d_flags = nullptr;     // [4] bad-action flag
  uint8_t* d_tmp_u8 = nullptr;     // [n] staging
  uint8_t* d_tmp_u8b = nullptr;    // [n]
  float* d_tmp_f32 = nullptr;      // [n]
  uint8_t* d_obs_view = nullptr;   // [n][84][84][4] qlx_env_obs's tensor view (allocated on its first call, kept)
  float acos_thr = 0.0f;
  bool hashing = true;
};

struct qlx_replay {
  int device = 0;
  uint64_t cap = 0;
  uint32_t n = 0;
  uint64_t F = 0;        // frame slots = cap + 4 n
  uint64_t total = 0;    // transitions pushed so far
  hipStream_t stream = nullptr;
  bool own_stream = true;
  uint8_t* d_frames = nullptr;
  uint8_t* d_action = nullptr;
  float* d_reward = nullptr;
  uint8_t* d_done = nullptr;
  uint32_t* d_epstep = nullptr;
  uint64_t* d_idx = nullptr;    // scratch for sampling [max_batch]
  uint32_t idx_cap = 0;
  uint64_t len() const { return total < cap ? total : cap; }
};

namespace qlx {
// episode bookkeeping state of a learner (learner.hip k_episode_book)
struct Book {
  uint64_t episode_count;
  float running_reward;
  uint32_t hist_len;     // current entries in the episode reward ring
  uint32_t hist_head;    // index of the oldest entry
};
// shared launchers of the learner loop (learner.hip / replay.hip), used by both environments' learners
void launch_episode_book(hipStream_t s, uint32_t n, const float* rewards, const uint8_t* dones, const uint32_t* ep_steps,
                         uint64_t max_steps, float* ep_reward, float* hist, uint32_t hist_cap, Book* book, uint8_t* reset_mask);
void launch_select_actions(hipStream_t s, uint32_t n, uint32_t n_actions, uint64_t step_before, uint64_t pure_random,
                           const double* eps_table, uint64_t eps_len, double eps_min, uint64_t seed, uint32_t id_offset,
                           uint32_t vec_step, const float* q, uint8_t* actions);
void launch_sample_distinct(hipStream_t s, uint64_t seed, uint32_t first_update, uint32_t n_updates, uint32_t rank, uint64_t len,
                            uint32_t batch, uint64_t* d_out);
// epsilon after k decrements, k = 0 .. until epsilon_min (repeated f64 subtraction, learn_episode :164-167)
std::vector<double> epsilon_table(const qlx_params& p);
// solved() over the episode reward ring (self_driving_tf_q_learner.rs:134-139)
void learner_book_stats(const Book& b, const float* ring, uint32_t ring_cap, float goal, float pct, float* running, uint64_t* solved);

// Reads the Keras SavedModel variables of `n_layers` weight layers (kernel, bias, Adam m / v) from a TF bundle
// into host arrays laid out like the flat parameter vector (variable 2L = kernel L, 2L + 1 = bias L) and the
// optimizer iteration count.  Shapes must multiply to var_sizes.  (tf_bundle.cpp)
void load_keras_bundle(const char* prefix, int n_layers, const int* var_sizes, std::vector<float>& w, std::vector<float>& m,
                       std::vector<float>& v, int64_t* iterations);

void env_launch_step(qlx_env* env, const uint8_t* d_actions, float* d_rewards, uint8_t* d_dones);
void env_launch_reset(qlx_env* env, const uint8_t* d_mask, int bump);
void replay_launch_push(qlx_replay* rb, qlx_env* env, hipStream_t s, const uint8_t* d_actions, const float* d_rewards,
                        const uint8_t* d_dones);
void replay_launch_sample(qlx_replay* rb, hipStream_t s, uint64_t seed, uint32_t first_update, uint32_t n_updates,
                          uint32_t rank, uint32_t batch, uint64_t* d_out);
}  // namespace qlx
