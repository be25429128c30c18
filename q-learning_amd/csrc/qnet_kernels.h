// Shared device helpers for the Nature-DQN kernels on gfx950 (bf16 MFMA operands, fp32 accumulation):
// bf16 vector types, u8 -> bf16 pixel conversion, LDS-only barrier, fixed-order partial-slab reductions.
//
// Math follows the reference Keras graph (create_ql_model_breakout_84x84x4_3_32.py:20-33,63-82):
// 'valid' convs NHWC/HWIO with ReLU, Flatten (h,w,c), Dense 512 ReLU, Dense 3 linear.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "qlx_internal.h"

namespace qlx {
namespace qn {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// bf16 a3 row pitch: columns 0..3135 the flattened conv3 output, column 3136 = 1.0 and 3137..3143 = 0 (written once per
// workspace, k_a3_pad), so the fc1 weight gradient a3^T dz4 over 3137 rows yields db3 as its last row (bgemm.h)
constexpr int kA3Ld = 3144;

// wave index as a scalar: keeps wave-derived loop bounds and branches uniform (SCC, not EXEC masks)
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

// workgroup barrier ordering LDS only: unlike __syncthreads() it does not drain outstanding global loads
// (vmcnt), so register prefetches of the next tile / sample stay in flight across it
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// MFMA-fragment-major layout of a bf16 [rows][K] operand: element (row, k) of 16-row slice row >> 4 and
// 32-wide k step k >> 5 sits at lane (k >> 3 & 3) * 16 + (row & 15), element k & 7, so one wave's fragment
// (16 rows x 32 k) is 1 KB contiguous: ld8(base + frag_offset(slice, s, K) + lane * 8).
__host__ __device__ constexpr int frag_index(int row, int k, int K) {
  return (((row >> 4) * (K / 32) + (k >> 5)) * 64 + ((k >> 3) & 3) * 16 + (row & 15)) * 8 + (k & 7);
}

__device__ __forceinline__ bf16x8 zero8() {
  const uint4 z = {0, 0, 0, 0};
  return __builtin_bit_cast(bf16x8, z);
}
__device__ __forceinline__ bf16x8 ld8(const bf16* p) { return __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(p)); }
__device__ __forceinline__ bf16x8 ldfrag(const bf16* base, int slice, int s, int K, int lane) {
  return ld8(base + ((slice * (K / 32) + s) * 64 + lane) * 8);
}

// u8 pixel -> bf16 is exact (integers <= 256 have <= 8 significant bits): the f32's top half.
__device__ __forceinline__ uint32_t u8pair_bf16(uint32_t w, int s) {
  const uint32_t lo = __builtin_bit_cast(uint32_t, (float)((w >> s) & 0xFFu)) >> 16;
  const uint32_t hi = __builtin_bit_cast(uint32_t, (float)((w >> (s + 8)) & 0xFFu)) & 0xFFFF0000u;
  return lo | hi;
}
__device__ __forceinline__ bf16x8 u8x8_to_bf16(uint2 v) {
  uint4 r;
  r.x = u8pair_bf16(v.x, 0);
  r.y = u8pair_bf16(v.x, 16);
  r.z = u8pair_bf16(v.y, 0);
  r.w = u8pair_bf16(v.y, 16);
  return __builtin_bit_cast(bf16x8, r);
}

// ------------------------------------------------------------------------------------------
// Fixed-order reductions of per-block fp32 partial slabs.

// out[dst(i)] = sum_c slab[c][i] (deterministic): block = 64 outputs x 4 waves; wave w sums chunk quarter w
// (8 loads in flight per lane), the quarters are added in fixed order through LDS.  grid = ceil(count/64).
// CONV1: i < 8192 is conv1's s2d-ordered [k][oc] weight gradient, stored to its HWIO index (the bias
// partials that follow are stored in place).
__device__ __forceinline__ int conv1_hwio_from_s2d(int i) {   // i = k * 32 + oc, k = ((ij*4 + c)*16) + dx*4 + dy
  const int oc = i & 31, k = i >> 5;
  const int dy = k & 3, dx = (k >> 2) & 3, c = (k >> 4) & 3, j = (k >> 6) & 1, ii = (k >> 7) & 1;
  return (((4 * ii + dx) * 8 + 4 * j + dy) * 4 + c) * 32 + oc;
}

// sq (optional): the block's sum of squares of its 64 outputs -> sq[blk] (the layer's weight blocks come
// first; a block past them holds the bias)
__device__ __forceinline__ void slab_reduce_block(const float* slab, size_t zstride, int chunks, size_t count, float* out,
                                                  bool conv1, int blk, float* sq = nullptr) {
  __shared__ float part[4][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t i = (size_t)blk * 64 + lane;
  const int q = (chunks + 3) / 4, c0 = wave * q, c1 = min(chunks, c0 + q);
  float s = 0.0f;
  if (i < count) {
    int c = c0;
    // up to 32 loads in flight per lane before the in-order sum (conv1's 64 partials per wave: 2 memory
    // round trips instead of 8); the addition order is unchanged
    for (; c + 32 <= c1; c += 32) {
      float v[32];
#pragma unroll
      for (int u = 0; u < 32; ++u) v[u] = slab[(size_t)(c + u) * zstride + i];
#pragma unroll
      for (int u = 0; u < 32; ++u) s += v[u];
    }
    for (; c + 8 <= c1; c += 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = slab[(size_t)(c + u) * zstride + i];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; c < c1; ++c) s += slab[(size_t)c * zstride + i];
  }
  part[wave][lane] = s;
  __syncthreads();
  if (wave == 0) {
    const float v = ((part[0][lane] + part[1][lane]) + part[2][lane]) + part[3][lane];
    if (i < count) {
      const size_t d = conv1 && i < 8192 ? (size_t)conv1_hwio_from_s2d((int)i) : i;
      out[d] = v;
    }
    if (sq) {
      float q = i < count ? v * v : 0.0f;
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) q += __shfl_xor(q, off);
      if (lane == 0) sq[blk] = q;
    }
  }
}

template <bool CONV1 = false>
__global__ __launch_bounds__(256) void k_slab_reduce(const float* slab, size_t zstride, int chunks, size_t count,
                                                     float* out) {
  slab_reduce_block(slab, zstride, chunks, count, out, CONV1, blockIdx.x);
}

// three independent slab reductions in one launch (segment i owns blocks [first_block[i], first_block[i+1]))
struct SlabSeg {
  const float* slab;
  size_t zstride;
  int chunks;
  size_t count;
  float* out;
  int conv1;
  float* sq;   // per-block square sums (nullable): block b of the segment -> sq[b]
};
struct SlabSegs3 {
  SlabSeg seg[3];
  int first_block[4];
};
__global__ __launch_bounds__(256) void k_slab_reduce3(SlabSegs3 a) {
  const int b = blockIdx.x;
  const int i = b < a.first_block[1] ? 0 : (b < a.first_block[2] ? 1 : 2);
  const SlabSeg& g = a.seg[i];
  slab_reduce_block(g.slab, g.zstride, g.chunks, g.count, g.out, g.conv1 != 0, b - a.first_block[i], g.sq);
}

__global__ void k_slab_reduce_bias_relu(const float* slab, size_t zstride, int chunks, int M, int N,
                                        const float* bias, bf16* out) {
  const size_t count = (size_t)M * N;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (size_t)gridDim.x * blockDim.x) {
    float s = 0.0f;
    for (int c = 0; c < chunks; ++c) s += slab[c * zstride + i];
    const float t = s + bias[i % N];
    out[i] = (bf16)(t > 0.0f ? t : 0.0f);
  }
}

}  // namespace qn
}  // namespace qlx
