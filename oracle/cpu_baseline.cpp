// ORACLE — TEST INFRASTRUCTURE ONLY.  CPU baseline driver: the restated reference loop
// (SelfDrivingQLearner::learn_episode with Parameter::default(), one env, B = 32) timed on host cores.
// Usage: cpu_baseline <env_steps> [n_envs] [batch]   -> one JSON line on stdout.
// The reference itself cannot be built here (no Rust toolchain, no libtensorflow); see DESIGN.md.
#include <chrono>
#include <cstdio>
#include <cmath>
#include <cstdlib>
#include <omp.h>

#include "learner_ref.h"

using namespace orc;

int main(int argc, char** argv) {
  const uint64_t steps = argc > 1 ? strtoull(argv[1], nullptr, 10) : 2000;
  const uint32_t n_envs = argc > 2 ? (uint32_t)atoi(argv[2]) : 1;
  const uint32_t batch = argc > 3 ? (uint32_t)atoi(argv[3]) : 32;
  LearnerParams p{};
  p.gamma = 0.99f;
  p.lowest_episode_reward_goal_threshold_pct = 0.9f;
  p.epsilon_max = 1.0; p.epsilon_min = 0.1; p.epsilon_greedy_steps = 1000000.0;
  p.max_steps_per_episode = 10000; p.epsilon_pure_random_steps = 50000;
  p.history_buffer_len = 1000000; p.update_after_actions = 4; p.target_sync_steps = 0;
  p.episode_reward_history_buffer_len = 100;
  p.n_envs = n_envs; p.batch_size = batch;
  p.env_seed = 0x51A5EED; p.learner_seed = 1; p.init_seed = 2; p.rank = 0;
  p.episode_reward_goal = NAN;   // the env's own goal
  Learner l(p);
  l.pack_like_reference = true;   // the reference's per-element f32 tensor packing (learner_ref.h)
  const auto t0 = std::chrono::steady_clock::now();
  uint64_t done_steps = 0;
  while (done_steps < steps) { l.vector_step(); done_steps += n_envs; }
  const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  printf("{\"env_steps\": %llu, \"updates\": %llu, \"seconds\": %.6f, \"env_steps_per_sec\": %.3f, "
         "\"updates_per_sec\": %.3f, \"threads\": %d, \"episodes\": %llu, \"pack_sink\": %.1f}\n",
         (unsigned long long)done_steps, (unsigned long long)l.update_count, sec, done_steps / sec,
         l.update_count / sec, omp_get_max_threads(), (unsigned long long)l.episode_count, l.pack_sink);
  return 0;
}
