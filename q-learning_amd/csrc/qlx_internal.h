// Internal helpers of libqlx (HIP for gfx950).  Not part of the ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <string>

#include "../../include/qlx.h"

namespace qlx {

void set_error(const std::string& msg);

struct Error {
  int32_t code;
  std::string msg;
};

#define QLX_HIP(expr)                                                                        \
  do {                                                                                        \
    hipError_t e__ = (expr);                                                                  \
    if (e__ != hipSuccess)                                                                    \
      throw ::qlx::Error{QLX_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e__) +     \
                                        " (" + __FILE__ + ":" + std::to_string(__LINE__) + ")"}; \
  } while (0)

#define QLX_CHECK(cond, code, msg)                                   \
  do {                                                               \
    if (!(cond)) throw ::qlx::Error{(code), std::string(msg)};       \
  } while (0)

// Runs f(), converting exceptions into a status code + thread-local message.
template <class F>
int32_t guard(F&& f) {
  try {
    f();
    return QLX_OK;
  } catch (const Error& e) {
    set_error(e.msg);
    return e.code;
  } catch (const std::bad_alloc&) {
    set_error("host out of memory");
    return QLX_E_OOM;
  } catch (const std::exception& e) {
    set_error(e.what());
    return QLX_E_STATE;
  }
}

// ---- geometry of the frame store ----------------------------------------------------
constexpr int kFrame = 84;
constexpr int kFramePix = 84 * 84;     // 7,056 bytes per frame
constexpr int kSlots = 4;              // 4-frame stack (ring slots)
constexpr int kBlocks = 21;            // 84 / 4: space-to-depth blocks per axis
constexpr int kActions = 3;
constexpr int kNumBricks = 60;
// Frame layout in HBM (space-to-depth): pixel (x, y) of the reference image lives at
//   ((x >> 2) * 21 + (y >> 2)) * 16 + (x & 3) * 4 + (y & 3)
// so a 4x4 pixel block is one 16-byte chunk, and conv1 (8x8 stride 4) becomes a 2x2 stride-1
// conv over [21][21][slot*16] with 8-byte aligned MFMA fragments.
__host__ __device__ inline int s2d_offset(int x, int y) { return ((x >> 2) * kBlocks + (y >> 2)) * 16 + (x & 3) * 4 + (y & 3); }

// ---- Philox4x32-10 counter-based RNG (build-defined stream) ------------
enum Purpose : uint32_t { P_BALL = 1, P_ACT = 2, P_SAMPLE = 3, P_INIT = 4, P_SYNTH = 5, P_BALLGAME = 6, P_PER = 7 };

__host__ __device__ inline void philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1,
                                       uint32_t out[4]) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
    const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c1 = (uint32_t)p1;
    c3 = (uint32_t)p0;
    c0 = n0;
    c2 = n2;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

// Word stream: word j = output (j & 3) of block ctr {j >> 2, c1, c2, purpose}, key = seed.
struct RngStream {
  uint32_t k0, k1, c1, c2, purpose;
  uint64_t word;
  uint32_t buf[4];
  uint64_t blk;
  __host__ __device__ RngStream(uint64_t seed, uint32_t c1_, uint32_t c2_, uint32_t purpose_, uint64_t start = 0)
      : k0((uint32_t)seed), k1((uint32_t)(seed >> 32)), c1(c1_), c2(c2_), purpose(purpose_), word(start), blk(~0ull) {}
  __host__ __device__ uint32_t u32() {
    const uint64_t b = word >> 2;
    if (b != blk) { philox((uint32_t)b, c1, c2, purpose, k0, k1, buf); blk = b; }
    const uint32_t v = buf[word & 3];
    ++word;
    return v;
  }
  __host__ __device__ uint64_t u64() {
    const uint64_t lo = u32();
    const uint64_t hi = u32();
    return lo | (hi << 32);
  }
};

__host__ __device__ inline float bits_f32(uint32_t b) { return __builtin_bit_cast(float, b); }
__host__ __device__ inline uint32_t f32_bits(float f) { return __builtin_bit_cast(uint32_t, f); }

// rand 0.8.5 UniformFloat<f32>::sample_single
__host__ __device__ inline float uniform_f32(RngStream& s, float low, float high) {
  float scale = high - low;
  for (;;) {
    const float v01 = bits_f32((s.u32() >> 9) | 0x3F800000u) - 1.0f;
    const float res = v01 * scale + low;
    if (res < high) return res;
    scale = bits_f32(f32_bits(scale) - 1u);
  }
}
// rand 0.8.5 gen_range(0_f64..1_f64)
__host__ __device__ inline double uniform_f64_01(RngStream& s) {
  for (;;) {
    const double v01 = __builtin_bit_cast(double, (s.u64() >> 12) | 0x3FF0000000000000ull) - 1.0;
    const double res = v01 * 1.0 + 0.0;
    if (res < 1.0) return res;
  }
}
// rand 0.8.5 UniformInt<u8>::sample_single(0, n)
__host__ __device__ inline uint32_t uniform_u8(RngStream& s, uint32_t n) {
  const uint32_t zone = 0xFFFFFFFFu - (0xFFFFFFFFu - n + 1u) % n;
  for (;;) {
    const uint64_t m = (uint64_t)s.u32() * n;
    if ((uint32_t)m <= zone) return (uint32_t)(m >> 32);
  }
}

// rand 0.8.5 UniformInt<usize>::sample_single_inclusive(0, n - 1) (`rng.gen_range(0..n)` on usize): u64 draws,
// zone = (range << leading_zeros(range)) - 1
__host__ __device__ inline uint64_t uniform_usize_single(RngStream& s, uint64_t n) {
  const uint64_t zone = (n << __builtin_clzll(n)) - 1;
  for (;;) {
    const unsigned __int128 m = (unsigned __int128)s.u64() * n;
    if ((uint64_t)m <= zone) return (uint64_t)(m >> 64);
  }
}

// ---- the linear per-step checksum (shared definition with the oracle) ----
constexpr uint64_t kH1 = 0x9E3779B97F4A7C15ull, kH2 = 0xC2B2AE3D27D4EB4Full, kH3 = 0x100000001B3ull;

int current_device_checked(int device);
// hipFuncAttributeMaxDynamicSharedMemorySize for `kernel` on the current device, once per (device, kernel, size)
void set_lds_limit(const void* kernel, size_t bytes);
// QLX_DEBUG_SYNC=1: synchronise `s` and throw naming `what` if a launch before it failed (no-op otherwise)
void debug_sync(hipStream_t s, const char* what);

}  // namespace qlx
