// Device-side view of the HBM replay ring (shared by replay.hip and learner.hip).
//
// Layout (frame dedup; ReplayBuffer semantics of replay_buffer.rs:52-138 are preserved):
//   transitions are pushed n_envs at a time, env order, so push position p = vector_step * n + env.
//   frames[F][7056]   F = capacity + 4 * n_envs   the frame each transition produced (s2d layout)
//   action/reward/done/epstep [capacity]          epstep k = 1-based step of the env's episode
// Transition p's states are rebuilt from the frames of the same env at positions p - d * n:
//   s'  slot j : d = (k - 1 - j) mod 4, valid iff k - d >= 1
//   s   slot j : d = 1 + ((k - 2 - j) mod 4), valid iff k - d >= 1          (invalid -> zero frame)
// which is exactly the FrameRingBuffer content (ring slot = (episode step - 1) mod 4, zeros after reset).
#pragma once
#include <cstdint>

#include "qlx_internal.h"

namespace qlx {

struct ReplayView {
  const uint8_t* frames;
  const uint8_t* action;
  const float* reward;
  const uint8_t* done;
  const uint32_t* epstep;
  uint64_t cap, F, total, len;
  uint32_t n;
};

// frame pointers of transition at logical index i (0 = oldest); which: 0 = s, 1 = s'
__device__ __forceinline__ void replay_frames(const ReplayView& r, uint64_t i, int which, const uint8_t* out[4]) {
  const uint64_t p = r.total - r.len + i;
  const int k = (int)r.epstep[p % r.cap];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int d = which ? ((k - 1 - j) & 3) : 1 + ((k - 2 - j) & 3);
    out[j] = (k - d >= 1) ? r.frames + ((p - (uint64_t)d * r.n) % r.F) * kFramePix : nullptr;
  }
}

}  // namespace qlx
