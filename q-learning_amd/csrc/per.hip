// Proportional prioritized replay on the device (SURVEY §8f #3, config C5 - beyond the reference, whose replay
// is uniform: replay_buffer.rs:85-137 via self_driving_tf_q_learner.rs:276-296).  Oracle: oracle/learner_ref.h
// SumTree / per_sample and Learner::update's priority write.
//
// Layout: one f32 heap of 2L nodes (L = next power of two >= capacity), leaves t[L + slot] = priority^alpha
// of replay slot `slot` (physical FIFO position), node i = t[2i] + t[2i + 1].  Internal nodes are a pure function
// of the leaves, so instead of walking every changed leaf's path the tree is rebuilt bottom-up once per vector
// step, right before it is sampled: ceil(log2 L / 11) launches, each block reducing 2048 nodes of one level
// through 11 levels in LDS (L = 2^20: 8 MB read + 4 MB written, two launches).
//
// Sampling (one block per update, B draws): u_b = (T / B) * (b + r_b) with r_b = gen_range_f32(0, 1) from
// stream (seed, update, rank, P_PER, word b), descending left iff u < left sum or the right subtree is empty;
// IS weight (len * leaf / T)^-beta, normalised by the batch max.  The slot is returned as the logical replay
// index (0 = oldest) the gather kernels take.
//
// Priority write after a vector step's updates: the |TD| errors of all U*B samples, in (update, sample) order;
// a slot drawn more than once keeps the LAST value (as the oracle's sequential writes do): a claim pass keeps the
// highest flat index per slot with atomicMax, the write pass lets only that index store (and clears its claim).
// per_max (the priority new transitions enter with) is the max over every written value: an integer atomicMax on
// the bits of a positive float.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>

#include "objects.h"
#include "per.h"

namespace qlx {

constexpr uint32_t kTreeChunk = 2048;

// x^y for the priorities (|td| + eps)^alpha and the IS weights (len p)^-beta, as the build defines it (DESIGN.md §6;
// oracle/learner_ref.cpp det_powf restates it): exp(y ln x) in binary64 from IEEE basic operations only (+ - * / fma,
// rint, frexp / ldexp), rounded once to binary32.  Library powf differs between the device (OCML) and glibc in the last
// bit now and then, and a one-ulp leaf changes the sum tree's partial sums and so, rarely, a draw; with this definition
// the prioritized learner is bit-exact against the oracle.  Accuracy: relative error ~1e-15 in binary64 before the
// final rounding (within one float ulp of the correctly rounded powf; tests/test_oracle_per.py).
__device__ __forceinline__ float per_powf(float xf, float yf) {
#pragma clang fp contract(off)
  if (__builtin_isnan(yf)) return __builtin_nanf("");   // a NaN exponent: NaN on both sides (no rint of NaN below)
  if (!(xf > 0.0f)) return xf == 0.0f ? (yf > 0.0f ? 0.0f : (yf < 0.0f ? __builtin_inff() : 1.0f)) : __builtin_nanf("");
  if (__builtin_isinf(xf)) return yf > 0.0f ? __builtin_inff() : (yf < 0.0f ? 0.0f : 1.0f);
  int e;
  double m = frexp((double)xf, &e);   // [0.5, 1)
  if (m < 0.70710678118654752440) { m = m * 2.0; e -= 1; }
  const double f = (m - 1.0) / (m + 1.0), s = f * f;
  // ln m = 2 f (1 + s / 3 + s^2 / 5 + ...), |f| <= 0.1716: 12 terms
  double p = 1.0 / 23.0;
#pragma unroll
  for (int i = 10; i >= 0; --i) p = fma(p, s, 1.0 / (double)(2 * i + 1));
  const double lnx = fma((double)e, 0.69314718055994530942, (f * p) * 2.0);
  const double z = (double)yf * lnx;
  if (z > 700.0) return __builtin_inff();
  if (z < -745.0) return 0.0f;
  const double kd = rint(z * 1.44269504088896340736);
  double r = fma(-kd, 6.93147180369123816490e-01, z);   // ln 2 = hi + lo (hi: 32 significant bits)
  r = fma(-kd, 1.90821492927058770002e-10, r);
  double q = 1.0 / 1307674368000.0;                      // 1 / 15!
  double fact = 1307674368000.0;
#pragma unroll
  for (int i = 14; i >= 0; --i) {
    fact = fact / (double)(i + 1);                       // i! (exact: integers < 2^53)
    q = fma(q, r, 1.0 / fact);
  }
  return (float)ldexp(q, (int)kd);
}

// block j reduces nodes [W + j S, W + (j + 1) S) of one level up log2(S) levels, storing every parent
__global__ __launch_bounds__(256) void k_tree_build(float* t, uint32_t W, uint32_t S) {
  __shared__ float cur[kTreeChunk];
  const uint32_t tid = threadIdx.x;
  const uint32_t off = blockIdx.x * S;
  for (uint32_t i = tid; i < S; i += 256) cur[i] = t[W + off + i];
  __syncthreads();
  uint32_t n = S, w = W, o = off;
  while (n > 1) {
    n >>= 1; w >>= 1; o >>= 1;
    float v[kTreeChunk / 2 / 256];
#pragma unroll
    for (uint32_t k = 0; k < kTreeChunk / 2 / 256; ++k) {
      const uint32_t i = tid + k * 256;
      if (i < n) v[k] = cur[2 * i] + cur[2 * i + 1];
    }
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < kTreeChunk / 2 / 256; ++k) {
      const uint32_t i = tid + k * 256;
      if (i < n) { cur[i] = v[k]; t[w + o + i] = v[k]; }
    }
    __syncthreads();
  }
}

void per_launch_build(hipStream_t s, float* tree, uint32_t L) {
  for (uint32_t W = L; W > 1;) {
    const uint32_t S = std::min(W, kTreeChunk);
    hipLaunchKernelGGL(k_tree_build, dim3(W / S), dim3(256), 0, s, tree, W, S);
    W /= S;
  }
  QLX_HIP(hipGetLastError());
}

__global__ __launch_bounds__(256) void k_per_sample(const float* t, uint32_t L, uint64_t seed, uint32_t first_update,
                                                    uint32_t rank, uint64_t len, float beta, uint32_t B, uint64_t cap,
                                                    uint64_t start, uint64_t* idx_out, float* w_out) {
  __shared__ float red[4];
  const uint32_t u = blockIdx.x, tid = threadIdx.x;
  const float T = t[1];
  const float seg = T / (float)B;
  float wmax = 0.0f;
  for (uint32_t b = tid; b < B; b += 256) {
    RngStream s(seed, first_update + u, rank, P_PER, b);
    const float r = uniform_f32(s, 0.0f, 1.0f);
    float x = seg * ((float)b + r);
    uint32_t i = 1;
    while (i < L) {
      const float left = t[2 * i], right = t[2 * i + 1];
      if (x < left || right == 0.0f) {
        i = 2 * i;
      } else {
        x -= left;
        i = 2 * i + 1;
      }
    }
    const uint64_t slot = i - L;
    const float p = t[i] / T;
    const float w = per_powf((float)len * p, -beta);
    idx_out[(size_t)u * B + b] = (slot + cap - start) % cap;
    w_out[(size_t)u * B + b] = w;
    wmax = fmaxf(wmax, w);
  }
  for (int o = 32; o > 0; o >>= 1) wmax = fmaxf(wmax, __shfl_xor(wmax, o));
  if ((tid & 63) == 0) red[tid >> 6] = wmax;
  __syncthreads();
  wmax = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  for (uint32_t b = tid; b < B; b += 256) w_out[(size_t)u * B + b] = w_out[(size_t)u * B + b] / wmax;
}

void per_launch_sample(hipStream_t s, const float* tree, uint32_t L, uint64_t seed, uint32_t first_update, uint32_t n_updates,
                       uint32_t rank, uint64_t len, float beta, uint32_t B, uint64_t cap, uint64_t start, uint64_t* idx_out,
                       float* w_out) {
  QLX_CHECK(len > 0 && len <= cap && cap <= L && start < cap, QLX_E_INVALID, "prioritized sample: bad replay range");
  hipLaunchKernelGGL(k_per_sample, dim3(n_updates), dim3(256), 0, s, tree, L, seed, first_update, rank, len, beta, B, cap, start,
                     idx_out, w_out);
  QLX_HIP(hipGetLastError());
}

// new transitions (FIFO positions first .. first + n - 1) enter at the largest priority so far
__global__ void k_per_push(float* leaves, uint64_t cap, uint64_t first, uint32_t n, const float* per_max) {
  const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e < n) leaves[(first + e) % cap] = *per_max;
}

void per_launch_push(hipStream_t s, float* leaves, uint64_t cap, uint64_t first, uint32_t n, const float* per_max) {
  hipLaunchKernelGGL(k_per_push, dim3((n + 255) / 256), dim3(256), 0, s, leaves, cap, first, n, per_max);
  QLX_HIP(hipGetLastError());
}

__global__ void k_per_claim(const uint64_t* idx, uint32_t n, uint64_t cap, uint64_t start, uint32_t* owner) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) atomicMax(&owner[(start + idx[k]) % cap], k + 1);
}

__global__ void k_per_write(const uint64_t* idx, const float* td_abs, uint32_t n, uint64_t cap, uint64_t start, float alpha,
                            float eps, uint32_t* owner, float* leaves, float* per_max) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const uint64_t slot = (start + idx[k]) % cap;
  const float pr = per_powf(td_abs[k] + eps, alpha);
  if (owner[slot] == k + 1) {
    leaves[slot] = pr;
    owner[slot] = 0;
  }
  atomicMax(reinterpret_cast<uint32_t*>(per_max), f32_bits(pr));
}

void per_launch_update(hipStream_t s, const uint64_t* idx, const float* td_abs, uint32_t n, uint64_t cap, uint64_t start,
                       float alpha, float eps, uint32_t* owner, float* leaves, float* per_max) {
  if (n == 0) return;
  hipLaunchKernelGGL(k_per_claim, dim3((n + 255) / 256), dim3(256), 0, s, idx, n, cap, start, owner);
  hipLaunchKernelGGL(k_per_write, dim3((n + 255) / 256), dim3(256), 0, s, idx, td_abs, n, cap, start, alpha, eps, owner, leaves,
                     per_max);
  QLX_HIP(hipGetLastError());
}

uint32_t per_leaves(uint64_t cap) {
  uint32_t L = 1;
  while (L < cap) L <<= 1;
  return L;
}

void PerState::init(uint64_t capacity, size_t max_samples) {
  QLX_CHECK(capacity >= 1 && capacity <= (1ull << 30), QLX_E_INVALID, "prioritized replay: capacity out of range");
  cap = capacity;
  L = per_leaves(capacity);
  QLX_HIP(hipMalloc(&d_tree, 2 * (size_t)L * sizeof(float)));
  QLX_HIP(hipMemset(d_tree, 0, 2 * (size_t)L * sizeof(float)));
  QLX_HIP(hipMalloc(&d_owner, (size_t)L * sizeof(uint32_t)));
  QLX_HIP(hipMemset(d_owner, 0, (size_t)L * sizeof(uint32_t)));
  QLX_HIP(hipMalloc(&d_max, sizeof(float)));
  const float one = 1.0f;
  QLX_HIP(hipMemcpy(d_max, &one, sizeof(float), hipMemcpyHostToDevice));
  if (max_samples) {
    QLX_HIP(hipMalloc(&d_w, max_samples * sizeof(float)));
    QLX_HIP(hipMalloc(&d_td, max_samples * sizeof(float)));
  }
}

void PerState::release() {
  for (void* p : {(void*)d_tree, (void*)d_owner, (void*)d_max, (void*)d_w, (void*)d_td})
    if (p) (void)hipFree(p);
  d_tree = nullptr; d_owner = nullptr; d_max = nullptr; d_w = nullptr; d_td = nullptr;
}

}  // namespace qlx

// ---------------- standalone sum tree (C ABI, include/qlx.h) ----------------
using namespace qlx;

struct qlx_sumtree {
  int device = 0;
  hipStream_t stream = nullptr;
  PerState st;
  uint64_t* d_idx = nullptr;
  float* d_w = nullptr;
  float* d_td = nullptr;
  size_t scratch = 0;
  void need(size_t n) {
    if (n <= scratch) return;
    for (void* p : {(void*)d_idx, (void*)d_w, (void*)d_td})
      if (p) (void)hipFree(p);
    QLX_HIP(hipMalloc(&d_idx, n * 8));
    QLX_HIP(hipMalloc(&d_w, n * 4));
    QLX_HIP(hipMalloc(&d_td, n * 4));
    scratch = n;
  }
};

extern "C" {

int32_t qlx_sumtree_create(uint64_t capacity, int32_t device, qlx_sumtree** out) {
  return guard([&] {
    QLX_CHECK(out, QLX_E_INVALID, "null out");
    auto* t = new qlx_sumtree;
    try {
      t->device = current_device_checked(device);
      QLX_HIP(hipStreamCreateWithFlags(&t->stream, hipStreamNonBlocking));
      t->st.init(capacity, 0);
    } catch (...) {
      t->st.release();
      if (t->stream) (void)hipStreamDestroy(t->stream);
      delete t;
      throw;
    }
    *out = t;
  });
}

int32_t qlx_sumtree_destroy(qlx_sumtree* t) {
  return guard([&] {
    if (!t) return;
    (void)hipStreamSynchronize(t->stream);
    t->st.release();
    for (void* p : {(void*)t->d_idx, (void*)t->d_w, (void*)t->d_td})
      if (p) (void)hipFree(p);
    (void)hipStreamDestroy(t->stream);
    delete t;
  });
}

int32_t qlx_sumtree_set_leaves(qlx_sumtree* t, const float* leaves) {
  return guard([&] {
    QLX_CHECK(t && leaves, QLX_E_INVALID, "null argument");
    for (uint64_t i = 0; i < t->st.cap; ++i)
      QLX_CHECK(leaves[i] >= 0.0f && std::isfinite(leaves[i]), QLX_E_INVALID, "leaves must be finite and >= 0");
    QLX_HIP(hipMemcpyAsync(t->st.d_tree + t->st.L, leaves, t->st.cap * 4, hipMemcpyHostToDevice, t->stream));
    per_launch_build(t->stream, t->st.d_tree, t->st.L);
    QLX_HIP(hipStreamSynchronize(t->stream));
  });
}

int32_t qlx_sumtree_get(qlx_sumtree* t, float* leaves, float* total, float* per_max) {
  return guard([&] {
    QLX_CHECK(t, QLX_E_INVALID, "null tree");
    per_launch_build(t->stream, t->st.d_tree, t->st.L);
    if (leaves) QLX_HIP(hipMemcpyAsync(leaves, t->st.d_tree + t->st.L, t->st.cap * 4, hipMemcpyDeviceToHost, t->stream));
    if (total) QLX_HIP(hipMemcpyAsync(total, t->st.d_tree + 1, 4, hipMemcpyDeviceToHost, t->stream));
    if (per_max) QLX_HIP(hipMemcpyAsync(per_max, t->st.d_max, 4, hipMemcpyDeviceToHost, t->stream));
    QLX_HIP(hipStreamSynchronize(t->stream));
  });
}

int32_t qlx_sumtree_sample(qlx_sumtree* t, uint64_t seed, uint32_t first_update, uint32_t n_updates, uint32_t rank, uint64_t len,
                           float beta, uint32_t batch, uint64_t* slots, float* weights) {
  return guard([&] {
    QLX_CHECK(t && slots && weights && batch > 0 && n_updates > 0, QLX_E_INVALID, "bad arguments");
    QLX_CHECK(len >= 1 && len <= t->st.cap, QLX_E_INVALID, "len out of range");
    const size_t n = (size_t)n_updates * batch;
    t->need(n);
    float total = 0.0f;
    QLX_HIP(hipMemcpyAsync(&total, t->st.d_tree + 1, 4, hipMemcpyDeviceToHost, t->stream));
    QLX_HIP(hipStreamSynchronize(t->stream));
    QLX_CHECK(total > 0.0f, QLX_E_STATE, "sum tree is empty");
    per_launch_sample(t->stream, t->st.d_tree, t->st.L, seed, first_update, n_updates, rank, len, beta, batch, t->st.cap, 0,
                      t->d_idx, t->d_w);
    QLX_HIP(hipMemcpyAsync(slots, t->d_idx, n * 8, hipMemcpyDeviceToHost, t->stream));
    QLX_HIP(hipMemcpyAsync(weights, t->d_w, n * 4, hipMemcpyDeviceToHost, t->stream));
    QLX_HIP(hipStreamSynchronize(t->stream));
  });
}

int32_t qlx_sumtree_update(qlx_sumtree* t, const uint64_t* slots, const float* td_abs, uint32_t n, float alpha, float eps) {
  return guard([&] {
    QLX_CHECK(t && (n == 0 || (slots && td_abs)), QLX_E_INVALID, "bad arguments");
    for (uint32_t k = 0; k < n; ++k) QLX_CHECK(slots[k] < t->st.cap, QLX_E_INVALID, "slot out of range");
    t->need(n);
    QLX_HIP(hipMemcpyAsync(t->d_idx, slots, (size_t)n * 8, hipMemcpyHostToDevice, t->stream));
    QLX_HIP(hipMemcpyAsync(t->d_td, td_abs, (size_t)n * 4, hipMemcpyHostToDevice, t->stream));
    per_launch_update(t->stream, t->d_idx, t->d_td, n, t->st.cap, 0, alpha, eps, t->st.d_owner, t->st.d_tree + t->st.L,
                      t->st.d_max);
    per_launch_build(t->stream, t->st.d_tree, t->st.L);
    QLX_HIP(hipStreamSynchronize(t->stream));
  });
}

}  // extern "C"
