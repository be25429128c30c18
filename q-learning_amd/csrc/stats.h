// Learning statistics (stats.hip): action histogram over the replay, 1-D DBSCAN, learning_update_log text.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

namespace qlx {

// counts[a] = occurrences of action a in the first len bytes of d_actions (device), for a < n_actions
void action_counts(hipStream_t s, const uint8_t* d_actions, uint64_t len, uint32_t n_actions, std::vector<uint64_t>& out);
// labels[i] = cluster position (clusters ordered by lowest member index) or -1 (noise); returns the cluster count
uint64_t dbscan_1d(const float* v, uint64_t n, float eps, uint64_t min_neighbors, int32_t* labels);
std::string dbscan_1d_text(const float* v, uint64_t n, float eps, uint64_t min_neighbors);

struct LogInputs {
  uint64_t episode_count, step_count;
  float gamma;
  double epsilon;
  float goal_mean, goal_pct;
  std::vector<float> rewards;   // episode reward history, oldest first
  std::vector<uint64_t> counts; // per action
  const char* const* action_names;
};
std::string learning_log(const LogInputs& in);
int32_t copy_text(const std::string& s, char* buf, size_t cap, size_t* len);

}  // namespace qlx
