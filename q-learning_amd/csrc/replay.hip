// HBM-resident replay ring with on-GPU distinct sampling (gfx950).
//
// Reference behaviour (restated): ReplayBuffer::add / get_many (replay_buffer.rs:21-38, 85-98, 126-137),
// generate_distinct_random_ids (self_driving_tf_q_learner.rs:276-296) with rand 0.8.5's
// Uniform<usize> zone rejection.  Layout and state reconstruction: replay_dev.h.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "objects.h"
#include "replay_dev.h"

namespace qlx {

// push: one workgroup (256 threads) per env copies the env's newest frame (28 x 16 B per thread-pass)
// and thread 0 writes the transition metadata.
__global__ __launch_bounds__(256) void k_replay_push(const uint8_t* obs, const qlx_breakout_state* st,
                                                     const uint32_t* ep_steps, uint32_t n, const uint8_t* actions,
                                                     const float* rewards, const uint8_t* dones, uint8_t* frames,
                                                     uint8_t* r_action, float* r_reward, uint8_t* r_done,
                                                     uint32_t* r_epstep, uint64_t total, uint64_t cap, uint64_t F) {
  const uint32_t e = blockIdx.x;
  const uint64_t p = total + e;
  const int slot = (st[e].next_slot + 3) & 3;
  const uint4* src = reinterpret_cast<const uint4*>(obs + ((size_t)e * kSlots + slot) * kFramePix);
  uint4* dst = reinterpret_cast<uint4*>(frames + (p % F) * kFramePix);
  for (int i = threadIdx.x; i < kFramePix / 16; i += blockDim.x) dst[i] = src[i];
  if (threadIdx.x == 0) {
    const uint64_t t = p % cap;
    r_action[t] = actions[e];
    r_reward[t] = rewards[e];
    r_done[t] = dones[e];
    r_epstep[t] = ep_steps[e];
  }
}

__device__ __forceinline__ uint64_t umulhi64(uint64_t a, uint64_t b, uint64_t* lo) {
  const unsigned __int128 m = (unsigned __int128)a * b;
  *lo = (uint64_t)m;
  return (uint64_t)(m >> 64);
}

// generate_distinct_random_ids, one 256-thread block per update.  256 consecutive u64 draws are evaluated in
// parallel per round; a draw is kept iff it passes the zone test and no earlier draw (an earlier round's keep,
// or an earlier draw of this round) has the same value - the sequential loop's result.  Every accepted draw
// claims its value's slot of an LDS hash set (keys u32: values < len < 2^32 - 1) and atomicMin's its draw
// index into the slot's owner word; after a barrier a draw is kept iff it owns its slot (an earlier round's
// keep owns it with a smaller index).  Kept draws are compacted in draw order by a block prefix count.
constexpr int kSampleThreads = 256;
__global__ __launch_bounds__(kSampleThreads) void k_sample_distinct(uint64_t seed, uint32_t first_update, uint32_t rank,
                                                                    uint64_t len, uint32_t B, uint32_t log2_table,
                                                                    uint64_t* out) {
  extern __shared__ uint32_t sh[];
  const uint32_t tsize = 1u << log2_table;
  uint32_t* keys = sh;
  uint32_t* owner = sh + tsize;
  __shared__ uint32_t wave_cnt[kSampleThreads / 64];
  const uint32_t u = first_update + blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t EMPTY = 0xFFFFFFFFu;
  for (uint32_t i = tid; i < tsize; i += kSampleThreads) { keys[i] = EMPTY; owner[i] = EMPTY; }
  __syncthreads();
  const uint64_t zone = ~0ull - ((~0ull - len + 1) % len);
  uint64_t* dst = out + (size_t)blockIdx.x * B;
  uint32_t count = 0;
  for (uint64_t round = 0; count < B; ++round) {
    const uint64_t d = round * kSampleThreads + tid;
    RngStream rs(seed, u, rank, P_SAMPLE, 2 * d);
    const uint64_t v = rs.u64();
    uint64_t lo;
    const uint32_t hi = (uint32_t)umulhi64(v, len, &lo);
    const bool acc = lo <= zone;
    uint32_t h = 0;
    if (acc) {
      h = (uint32_t)(((uint64_t)hi * 0x9E3779B97F4A7C15ull) >> (64 - log2_table));
      for (;;) {
        const uint32_t t = atomicCAS(&keys[h], EMPTY, hi);
        if (t == EMPTY || t == hi) break;
        h = (h + 1) & (tsize - 1);
      }
      atomicMin(&owner[h], (uint32_t)d);
    }
    __syncthreads();
    const bool ok = acc && owner[h] == (uint32_t)d;
    const unsigned long long bal = __ballot(ok);
    if (lane == 0) wave_cnt[wave] = (uint32_t)__popcll(bal);
    __syncthreads();
    uint32_t before = 0, total = 0;
#pragma unroll
    for (int w = 0; w < kSampleThreads / 64; ++w) {
      before += w < wave ? wave_cnt[w] : 0u;
      total += wave_cnt[w];
    }
    const uint32_t pos = count + before + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull));
    if (ok && pos < B) dst[pos] = hi;
    count = min(B, count + total);
    __syncthreads();   // wave_cnt / owner reads done before the next round writes them
  }
}

// get_many + batch_to_multi_dim_array: out [B][84][84][4] (x, y, slot)
__global__ void k_replay_view(ReplayView r, const uint64_t* idx, uint32_t B, int which, uint8_t* out) {
  const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= (size_t)B * kFramePix) return;
  const uint32_t b = (uint32_t)(g / kFramePix);
  const int xy = (int)(g - (size_t)b * kFramePix);
  const int x = xy / kFrame, y = xy - x * kFrame;
  const uint8_t* f[4];
  replay_frames(r, idx[b], which, f);
  const int off = s2d_offset(x, y);
  uchar4 v;
  v.x = f[0] ? f[0][off] : 0;
  v.y = f[1] ? f[1][off] : 0;
  v.z = f[2] ? f[2][off] : 0;
  v.w = f[3] ? f[3][off] : 0;
  reinterpret_cast<uchar4*>(out)[g] = v;
}

__global__ void k_replay_meta(ReplayView r, const uint64_t* idx, uint32_t B, uint8_t* a, float* rw, uint8_t* d) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const uint64_t t = (r.total - r.len + idx[b]) % r.cap;
  a[b] = r.action[t];
  rw[b] = r.reward[t];
  d[b] = r.done[t];
}

ReplayView replay_view(const qlx_replay* rb) {
  ReplayView v;
  v.frames = rb->d_frames; v.action = rb->d_action; v.reward = rb->d_reward; v.done = rb->d_done;
  v.epstep = rb->d_epstep; v.cap = rb->cap; v.F = rb->F; v.total = rb->total; v.len = rb->len(); v.n = rb->n;
  return v;
}

void replay_launch_push(qlx_replay* rb, qlx_env* env, hipStream_t s, const uint8_t* d_actions, const float* d_rewards,
                        const uint8_t* d_dones) {
  hipLaunchKernelGGL(k_replay_push, dim3(env->n), dim3(256), 0, s, env->d_obs, env->d_state, env->d_ep_steps, env->n,
                     d_actions, d_rewards, d_dones, rb->d_frames, rb->d_action, rb->d_reward, rb->d_done, rb->d_epstep,
                     rb->total, rb->cap, rb->F);
  QLX_HIP(hipGetLastError());
  rb->total += env->n;
}

// the set holds at most B + 255 keys (the last round may claim slots past B): keep it at most half full
static uint32_t table_log2(uint32_t batch) {
  uint32_t l = 8;
  while ((1u << l) < 2 * (batch + kSampleThreads)) ++l;
  return l;
}

void launch_sample_distinct(hipStream_t s, uint64_t seed, uint32_t first_update, uint32_t n_updates, uint32_t rank, uint64_t len,
                            uint32_t batch, uint64_t* d_out) {
  const uint32_t l2 = table_log2(batch);
  QLX_CHECK(len < 0xFFFFFFFFull, QLX_E_INVALID, "replay sampling keys are 32-bit: len must be < 2^32 - 1");
  QLX_CHECK(len >= batch, QLX_E_INVALID, "cannot draw more distinct indices than the replay holds");
  set_lds_limit((const void*)k_sample_distinct, 128 * 1024);   // up to 128 KB of hash set at B = 4096
  hipLaunchKernelGGL(k_sample_distinct, dim3(n_updates), dim3(kSampleThreads), (size_t)8 << l2, s, seed, first_update, rank, len,
                     batch, l2, d_out);
  QLX_HIP(hipGetLastError());
}

void replay_launch_sample(qlx_replay* rb, hipStream_t s, uint64_t seed, uint32_t first_update, uint32_t n_updates,
                          uint32_t rank, uint32_t batch, uint64_t* d_out) {
  launch_sample_distinct(s, seed, first_update, n_updates, rank, (uint64_t)rb->len(), batch, d_out);
}

}  // namespace qlx

using namespace qlx;

extern "C" {

int32_t qlx_replay_create(uint64_t capacity, uint32_t n_envs, int32_t device, qlx_replay** out) {
  return guard([&] {
    QLX_CHECK(capacity > 0 && n_envs > 0 && out, QLX_E_INVALID, "capacity and n_envs must be > 0");
    current_device_checked(device);
    auto* r = new qlx_replay;
    try {   // a failure part-way releases what was built
      r->device = device;
      r->cap = capacity;
      r->n = n_envs;
      r->F = capacity + 4ull * n_envs;
      QLX_HIP(hipStreamCreateWithFlags(&r->stream, hipStreamNonBlocking));
      const hipError_t e = hipMalloc(&r->d_frames, r->F * kFramePix);
      if (e != hipSuccess) { delete r; throw Error{QLX_E_OOM, "replay frame store allocation failed"}; }
      QLX_HIP(hipMalloc(&r->d_action, capacity));
      QLX_HIP(hipMalloc(&r->d_reward, capacity * sizeof(float)));
      QLX_HIP(hipMalloc(&r->d_done, capacity));
      QLX_HIP(hipMalloc(&r->d_epstep, capacity * sizeof(uint32_t)));
    } catch (...) {
      qlx_replay_destroy(r);
      throw;
    }
    *out = r;
  });
}

int32_t qlx_replay_destroy(qlx_replay* r) {
  return guard([&] {
    if (!r) return;
    (void)hipSetDevice(r->device);
    (void)hipStreamSynchronize(r->stream);
    (void)hipFree(r->d_frames); (void)hipFree(r->d_action); (void)hipFree(r->d_reward); (void)hipFree(r->d_done);
    (void)hipFree(r->d_epstep); (void)hipFree(r->d_idx);
    if (r->own_stream) (void)hipStreamDestroy(r->stream);
    delete r;
  });
}

uint64_t qlx_replay_len(const qlx_replay* r) { return r ? r->len() : 0; }

int32_t qlx_replay_push_dev(qlx_replay* r, qlx_env* env, const uint8_t* d_actions, const float* d_rewards,
                            const uint8_t* d_dones) {
  return guard([&] {
    QLX_CHECK(r && env && d_actions && d_rewards && d_dones, QLX_E_INVALID, "null argument");
    QLX_CHECK(env->n == r->n, QLX_E_INVALID, "replay n_envs differs from env");
    QLX_HIP(hipSetDevice(r->device));
    replay_launch_push(r, env, env->stream, d_actions, d_rewards, d_dones);
  });
}

int32_t qlx_replay_push(qlx_replay* r, qlx_env* env, const uint8_t* actions, const float* rewards,
                        const uint8_t* dones) {
  return guard([&] {
    QLX_CHECK(r && env && actions && rewards && dones, QLX_E_INVALID, "null argument");
    QLX_CHECK(env->n == r->n, QLX_E_INVALID, "replay n_envs differs from env");
    QLX_HIP(hipSetDevice(r->device));
    QLX_HIP(hipMemcpyAsync(env->d_tmp_u8, actions, env->n, hipMemcpyHostToDevice, env->stream));
    QLX_HIP(hipMemcpyAsync(env->d_tmp_f32, rewards, env->n * sizeof(float), hipMemcpyHostToDevice, env->stream));
    QLX_HIP(hipMemcpyAsync(env->d_tmp_u8b, dones, env->n, hipMemcpyHostToDevice, env->stream));
    replay_launch_push(r, env, env->stream, env->d_tmp_u8, env->d_tmp_f32, env->d_tmp_u8b);
    QLX_HIP(hipStreamSynchronize(env->stream));
  });
}

int32_t qlx_replay_sample_distinct(qlx_replay* r, uint64_t seed, uint32_t update_idx, uint32_t rank, uint32_t batch,
                                   uint64_t* out) {
  return guard([&] {
    QLX_CHECK(r && out, QLX_E_INVALID, "null argument");
    QLX_CHECK(batch > 0 && batch <= 4096, QLX_E_INVALID, "batch must be in 1..4096");
    QLX_CHECK(r->len() >= batch, QLX_E_INVALID, "replay holds fewer transitions than the batch");
    QLX_HIP(hipSetDevice(r->device));
    QLX_HIP(hipDeviceSynchronize());
    if (r->idx_cap < batch) {
      (void)hipFree(r->d_idx);
      QLX_HIP(hipMalloc(&r->d_idx, batch * sizeof(uint64_t)));
      r->idx_cap = batch;
    }
    replay_launch_sample(r, r->stream, seed, update_idx, 1, rank, batch, r->d_idx);
    QLX_HIP(hipMemcpyAsync(out, r->d_idx, batch * sizeof(uint64_t), hipMemcpyDeviceToHost, r->stream));
    QLX_HIP(hipStreamSynchronize(r->stream));
  });
}

int32_t qlx_replay_get_many(qlx_replay* r, const uint64_t* indices, uint32_t B, uint8_t* s, uint8_t* s_next,
                            uint8_t* actions, float* rewards, uint8_t* dones) {
  return guard([&] {
    QLX_CHECK(r && indices && B > 0, QLX_E_INVALID, "null argument");
    for (uint32_t b = 0; b < B; ++b) QLX_CHECK(indices[b] < r->len(), QLX_E_INVALID, "index out of range");
    QLX_HIP(hipSetDevice(r->device));
    QLX_HIP(hipDeviceSynchronize());
    uint64_t* d_idx = nullptr;
    uint8_t* d_out = nullptr;
    float* d_r = nullptr;
    uint8_t *d_a = nullptr, *d_d = nullptr;
    const size_t bytes = (size_t)B * kFramePix * kSlots;
    QLX_HIP(hipMalloc(&d_idx, B * sizeof(uint64_t)));
    QLX_HIP(hipMalloc(&d_out, bytes));
    QLX_HIP(hipMalloc(&d_r, B * sizeof(float)));
    QLX_HIP(hipMalloc(&d_a, B));
    QLX_HIP(hipMalloc(&d_d, B));
    QLX_HIP(hipMemcpyAsync(d_idx, indices, B * sizeof(uint64_t), hipMemcpyHostToDevice, r->stream));
    const ReplayView v = replay_view(r);
    const size_t total = (size_t)B * kFramePix;
    for (int which = 0; which < 2; ++which) {
      uint8_t* dst = which ? s_next : s;
      if (!dst) continue;
      hipLaunchKernelGGL(k_replay_view, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, r->stream, v, d_idx, B, which, d_out);
      QLX_HIP(hipGetLastError());
      QLX_HIP(hipMemcpyAsync(dst, d_out, bytes, hipMemcpyDeviceToHost, r->stream));
      QLX_HIP(hipStreamSynchronize(r->stream));
    }
    hipLaunchKernelGGL(k_replay_meta, dim3((B + 255) / 256), dim3(256), 0, r->stream, v, d_idx, B, d_a, d_r, d_d);
    QLX_HIP(hipGetLastError());
    if (actions) QLX_HIP(hipMemcpyAsync(actions, d_a, B, hipMemcpyDeviceToHost, r->stream));
    if (rewards) QLX_HIP(hipMemcpyAsync(rewards, d_r, B * sizeof(float), hipMemcpyDeviceToHost, r->stream));
    if (dones) QLX_HIP(hipMemcpyAsync(dones, d_d, B, hipMemcpyDeviceToHost, r->stream));
    QLX_HIP(hipStreamSynchronize(r->stream));
    (void)hipFree(d_idx); (void)hipFree(d_out); (void)hipFree(d_r); (void)hipFree(d_a); (void)hipFree(d_d);
  });
}

}  // extern "C"
