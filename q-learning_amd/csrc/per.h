// Prioritized replay state and launchers (per.hip), shared by the learner and the standalone qlx_sumtree.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace qlx {

struct PerState {
  uint64_t cap = 0;
  uint32_t L = 0;               // leaves (power of two >= cap); node i of the heap at d_tree[i], leaves at d_tree + L
  float* d_tree = nullptr;      // [2L]
  uint32_t* d_owner = nullptr;  // [L] last-writer claims of the priority write (zero between launches)
  float* d_max = nullptr;       // largest priority so far (new transitions enter with it), starts at 1
  float* d_w = nullptr;         // [max samples] IS weights of the sampled batches
  float* d_td = nullptr;        // [max samples] |TD error| of the sampled transitions
  void init(uint64_t capacity, size_t max_samples);
  void release();
  float* leaves() const { return d_tree + L; }
};

uint32_t per_leaves(uint64_t cap);
void per_launch_build(hipStream_t s, float* tree, uint32_t L);
// n_updates batches of B draws; out: logical replay indices ((slot - start) mod cap) and normalised IS weights
void per_launch_sample(hipStream_t s, const float* tree, uint32_t L, uint64_t seed, uint32_t first_update, uint32_t n_updates,
                       uint32_t rank, uint64_t len, float beta, uint32_t B, uint64_t cap, uint64_t start, uint64_t* idx_out,
                       float* w_out);
void per_launch_push(hipStream_t s, float* leaves, uint64_t cap, uint64_t first, uint32_t n, const float* per_max);
void per_launch_update(hipStream_t s, const uint64_t* idx, const float* td_abs, uint32_t n, uint64_t cap, uint64_t start,
                       float alpha, float eps, uint32_t* owner, float* leaves, float* per_max);

}  // namespace qlx
