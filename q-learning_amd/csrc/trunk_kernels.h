// Per-sample fused conv-trunk kernels for gfx950 (Nature-DQN conv1 -> conv2 -> conv3).
//
// One persistent 512-thread block (8 waves, one block per CU by LDS) walks the batch sample by sample.
// A sample's four space-to-depth frames (4 x 7056 B) are staged ONCE into LDS as bf16 [441 pos][64 ch]
// (ch = ring slot * 16 + 4x4 sub-pixel), so conv1's 2x2 s2d convolution reads its im2col rows straight
// from LDS; conv1 writes A1 into LDS for conv2, conv2 writes A2 for conv3.  Activations leave the CU
// with 16-byte coalesced stores (they are needed by the backward pass and fc1).  All conv weights stay
// in VGPRs as MFMA B fragments for the block's lifetime: each wave owns one 16-column output slice of
// every layer (conv1 32 + conv2 64 + conv3 72 VGPRs per lane), so the weights cross L2 once per block.
//
// The conv1 weight-gradient kernel reuses the staging: dW0[k][n] = sum_m X(m,k) dz1[m][n] with the
// m-reduction in the MFMA k slot, both operands read with ds_read_b64_tr_b16 (4 rows x 16 columns per
// 16-lane group, per-lane row addresses = the im2col gather for free).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "qnet_kernels.h"

namespace qlx {
namespace qn {

constexpr int kTrunkThreads = 512;
// Row strides: 40 dwords (80 bf16) puts the 16 (row, k-group) 16-byte windows of every ds_read_b128 lane group
// of a 16x16x32 fragment, and the 8 rows a 32-lane half reads with ds_read_b64_tr_b16, in distinct banks.
constexpr int kXS = 80;                  // staged input row stride (bf16): 64 channels + 16 pad
constexpr int kA1S = 40;                 // A1 [400][32] row stride
constexpr int kA2S = 80;                 // A2 [81][64]
constexpr int kA3S = 80;                 // A3 [49][64]
constexpr int kDZS = 48;                 // dz1 [416][32] row stride (tr-read conflict-free, see k_wgrad)
constexpr int kLdsX = 441 * kXS;         // bf16 elements
constexpr int kLdsA1 = 400 * kA1S;
constexpr int kLdsDZ = 416 * kDZS;
constexpr int kLdsA3 = 49 * kA3S;
// Forward images use row pitches (in positions) chosen so that the 16-lane im2col read groups stay
// bank-conflict-free when their positions wrap to the next image row: with the 40-dword (X, A2) / 20-dword
// (A1, stride-2 reads) position strides the bank window repeats every 8 position steps, and a wrap must
// advance it like one ordinary step: X pitch 28 (20 output columns), A1 25 (9 columns at stride 2),
// A2 15 (7 columns).
constexpr int kXW = 28, kA1W = 25, kA2W = 15;
constexpr int kLdsXf = 21 * kXW * kXS;
constexpr int kLdsA1f = 20 * kA1W * kA1S;
static_assert(9 * kA2W * kA2S <= kLdsXf, "A2 aliases X");
// A2 aliases X (dead after conv1); A3 has its own region because its copy-out is deferred past the next
// sample's staging (see k_trunk_fwd)
constexpr size_t kTrunkFwdLds = (size_t)(kLdsXf + kLdsA1f + kLdsA3) * 2;
constexpr size_t kConv1WgradLds = (size_t)(kLdsX + kLdsDZ) * 2;
constexpr int kFrameChunks = 4 * 441;    // 16-byte s2d blocks per sample
constexpr int kPf = (kFrameChunks + kTrunkThreads - 1) / kTrunkThreads;

// 16 u8 -> 16 bf16 (exact) as two 16-byte halves
__device__ __forceinline__ void u8x16_to_bf16(uint4 v, uint4& lo, uint4& hi) {
  lo.x = u8pair_bf16(v.x, 0);
  lo.y = u8pair_bf16(v.x, 16);
  lo.z = u8pair_bf16(v.y, 0);
  lo.w = u8pair_bf16(v.y, 16);
  hi.x = u8pair_bf16(v.z, 0);
  hi.y = u8pair_bf16(v.z, 16);
  hi.z = u8pair_bf16(v.w, 0);
  hi.w = u8pair_bf16(v.w, 16);
}

template <int NT>
constexpr int pf_chunks() { return (kFrameChunks + NT - 1) / NT; }

// register prefetch of one sample's frames: chunk c = slot * 441 + pos (nullptr frame = zeros); NT threads
template <int NT = kTrunkThreads>
__device__ __forceinline__ void frames_prefetch(const uint8_t* const* table, int b, int B, uint4 (&pf)[pf_chunks<NT>()]) {
#pragma unroll
  for (int u = 0; u < pf_chunks<NT>(); ++u) {
    const int c = threadIdx.x + u * NT;
    pf[u] = uint4{0, 0, 0, 0};
    if (b < B && c < kFrameChunks) {
      const int slot = c / 441, pos = c - slot * 441;
      const uint8_t* f = table[b * 4 + slot];
      // global (not flat) load: a flat load also counts on lgkmcnt, so every LDS wait in the conv phases
      // would wait for this prefetch too
      typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
      if (f) pf[u] = __builtin_bit_cast(uint4, *(const __attribute__((address_space(1))) u32x4*)(f + pos * 16));
    }
  }
}

// the same with the sample's 4 frame pointers already in LDS (fptr[slot]): no dependent pointer load in the
// issuing wave's path (the table entry is fetched a sample earlier, see k_trunk_fwd)
template <int NT = kTrunkThreads>
__device__ __forceinline__ void frames_prefetch_ptrs(const uint8_t* const* fptr, bool valid, uint4 (&pf)[pf_chunks<NT>()]) {
#pragma unroll
  for (int u = 0; u < pf_chunks<NT>(); ++u) {
    const int c = threadIdx.x + u * NT;
    pf[u] = uint4{0, 0, 0, 0};
    if (valid && c < kFrameChunks) {
      const int slot = c / 441, pos = c - slot * 441;
      const uint8_t* f = fptr[slot];
      typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
      if (f) pf[u] = __builtin_bit_cast(uint4, *(const __attribute__((address_space(1))) u32x4*)(f + pos * 16));
    }
  }
}

// Slot-major variant for the forward trunk: thread tid < 441 owns s2d block pos = tid of all 4 slots, so the
// frame pointer of each load is wave-uniform (read from LDS, fptr[slot]) and the per-lane address is one
// 32-bit offset - no 64-bit per-chunk addresses to keep live across the sample.
__device__ __forceinline__ void frames_prefetch_slots(const uint8_t* const* fptr, bool valid, uint4 (&pf)[4]) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  const int pos = threadIdx.x;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    pf[u] = uint4{0, 0, 0, 0};
    const unsigned long long fv = (unsigned long long)fptr[u];   // uniform: one LDS broadcast -> SGPRs
    const uint8_t* f = (const uint8_t*)(((unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((int)(fv >> 32)) << 32) |
                                        (unsigned)__builtin_amdgcn_readfirstlane((int)fv));
    if (valid && f && pos < 441) pf[u] = __builtin_bit_cast(uint4, *(const __attribute__((address_space(1))) u32x4*)(f + pos * 16));
  }
}
template <int PITCH = 21>   // X row pitch in positions
__device__ __forceinline__ void frames_stage_slots(bf16* X, const uint4 (&pf)[4]) {
  const int pos = threadIdx.x;
  if (pos < 441) {
    const int row = PITCH == 21 ? pos : (pos / 21) * PITCH + pos % 21;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      uint4 lo, hi;
      u8x16_to_bf16(pf[u], lo, hi);
      uint4* d = reinterpret_cast<uint4*>(X + row * kXS + u * 16);
      d[0] = lo;
      d[1] = hi;
    }
  }
}

// u8 -> bf16 into the staged image X [441][XS] (ch = slot * 16 + sub-pixel)
template <int NT = kTrunkThreads, int XS = kXS>
__device__ __forceinline__ void frames_stage(bf16* X, const uint4 (&pf)[pf_chunks<NT>()]) {
#pragma unroll
  for (int u = 0; u < pf_chunks<NT>(); ++u) {
    const int c = threadIdx.x + u * NT;
    if (c < kFrameChunks) {
      const int slot = c / 441, pos = c - slot * 441;
      uint4 lo, hi;
      u8x16_to_bf16(pf[u], lo, hi);
      uint4* d = reinterpret_cast<uint4*>(X + pos * XS + slot * 16);
      d[0] = lo;
      d[1] = hi;
    }
  }
}

// LDS rows [rows][stride] -> global contiguous [rows][cols] with 16-byte chunks
template <int ROWS, int COLS, int STRIDE, int NT = kTrunkThreads>
__device__ __forceinline__ void lds_copy_out(const bf16* src, bf16* dst) {
  constexpr int CPR = COLS / 8;
  for (int c = threadIdx.x; c < ROWS * CPR; c += NT) {
    const int row = c / CPR, col = (c - row * CPR) * 8;
    *reinterpret_cast<uint4*>(dst + row * COLS + col) = *reinterpret_cast<const uint4*>(src + row * STRIDE + col);
  }
}

// LDS image rows of W valid positions at pitch PW -> global contiguous [ROWS][COLS]
template <int ROWS, int COLS, int STRIDE, int W, int PW>
__device__ __forceinline__ void lds_copy_out_pitched(const bf16* src, bf16* dst) {
  constexpr int CPR = COLS / 8;
  for (int c = threadIdx.x; c < ROWS * CPR; c += kTrunkThreads) {
    const int row = c / CPR, col = (c - row * CPR) * 8, lrow = (row / W) * PW + row % W;
    *reinterpret_cast<uint4*>(dst + row * COLS + col) = *reinterpret_cast<const uint4*>(src + lrow * STRIDE + col);
  }
}

__device__ __forceinline__ bf16x8 lds8(const bf16* p) { return *reinterpret_cast<const bf16x8*>(p); }

__device__ __forceinline__ bf16 relu_bf16(float v) { return (bf16)(v > 0.0f ? v : 0.0f); }

// One wave's share of a per-sample conv GEMM in the D^T = W X^T orientation: the lane's weight registers
// w[s] (row = output channel lane & 15 of the wave's 16-channel slice, k = 8 (lane >> 4) + j) are the A
// operand, the activation rows (column = output position lane & 15) the B operand, so each lane ends with
// 4 consecutive channels 4 (lane >> 4) + e of one position: one 8-byte LDS store per tile.  The B-fragment
// LDS reads run D deep ahead of their MFMAs across tile boundaries (ring slot s % D), so a tile's epilogue
// overlaps the next tile's reads.  addr(t, s) -> LDS pointer of k-step s of tile t for this lane.
// pre(t) runs at the start of tile t, before the tile's refill reads are issued, and its result is handed to
// epi(t, acc, pre_value): an LDS value the epilogue needs (e.g. a ReLU mask) is then older than the ring
// reads in flight, so waiting for it is lgkmcnt(D) instead of a drain of the whole ring.
template <int KS, int D, class Addr, class Pre, class Epi>
__device__ __forceinline__ void conv_tiles(int t0, int dt, int nt, const bf16x8 (&w)[KS], Addr addr, Pre pre, Epi epi) {
  static_assert(KS % D == 0, "ring depth must divide the k-steps");
  if (t0 >= nt) return;
  bf16x8 a[D];
#pragma unroll
  for (int d = 0; d < D; ++d) a[d] = lds8(addr(t0, d));
  for (int t = t0; t < nt; t += dt) {
    f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
    const bool more = t + dt < nt;
    const auto pv = pre(t);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[s], a[s % D], acc, 0, 0, 0);
      // unconditional refill (the last tile re-reads its own rows): equal LDS-read counts on every path let
      // the compiler wait with lgkmcnt(D - 1) instead of draining the queue before each MFMA
      if (s + D < KS) a[s % D] = lds8(addr(t, s + D));
      else a[s % D] = lds8(addr(more ? t + dt : t, s + D - KS));
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // keep the order: this MFMA, then its refill read
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
    epi(t, acc, pv);
  }
}

typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint2 pack4_bf16(float a, float b, float c, float d) {
  const bf16x4 v = {(bf16)a, (bf16)b, (bf16)c, (bf16)d};
  return __builtin_bit_cast(uint2, v);
}

__device__ __forceinline__ float relu(float v) { return v > 0.0f ? v : 0.0f; }

// a1 [B][400][32], a2 [B][81][64] (written when STORE12), a3 [B][49][64] (always)
// TIMING (development only): wave 0 accumulates s_memtime cycles per phase (staging, conv1, conv2, conv3)
// into timing[blockIdx.x * 4 + phase]
template <bool STORE12, bool TIMING = false>
__global__ __launch_bounds__(kTrunkThreads, 1) void k_trunk_fwd(const uint8_t* const* __restrict__ table, int B,
                                                                const bf16* __restrict__ wf0, const bf16* __restrict__ wf1,
                                                                const bf16* __restrict__ wf2, const float* __restrict__ bias0,
                                                                const float* __restrict__ bias1,
                                                                const float* __restrict__ bias2, bf16* __restrict__ a1,
                                                                bf16* __restrict__ a2, bf16* __restrict__ a3,
                                                                unsigned long long* __restrict__ timing = nullptr) {
  unsigned long long ph[4] = {0, 0, 0, 0}, tm = 0;
  auto mark = [&](int i) {
    if constexpr (TIMING) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      if (i >= 0) ph[i] += t - tm;
      tm = t;
    }
  };
  extern __shared__ __attribute__((aligned(16))) bf16 lds[];
  bf16* X = lds;
  bf16* A1 = lds + kLdsXf;
  bf16* A2 = lds;               // aliases X
  bf16* A3 = lds + kLdsXf + kLdsA1f;
  const int wave = wave_id(), lane = threadIdx.x & 63;
  const int r = lane & 15, g = lane >> 4;
  const int c1 = (wave & 1) * 16, c2 = (wave & 3) * 16;   // the wave's output-channel slice, conv1 / conv2+3
  bf16x8 w1[8], w2[16], w3[18];
  // fragment-major weight copies (frag_index): each fragment load is 1 KB contiguous per wave
#pragma unroll
  for (int s = 0; s < 8; ++s) w1[s] = ldfrag(wf0, c1 >> 4, s, 256, lane);
#pragma unroll
  for (int s = 0; s < 16; ++s) w2[s] = ldfrag(wf1, c2 >> 4, s, 512, lane);
#pragma unroll
  for (int s = 0; s < 18; ++s) w3[s] = ldfrag(wf2, c2 >> 4, s, 576, lane);
  // biases staged in LDS (12 resident VGPRs would spill the weight fragments; a global load in the epilogue
  // would make the compiler drain vmcnt, i.e. wait for the next sample's frame prefetch)
  __shared__ __attribute__((aligned(16))) float sbias[160];
  if (threadIdx.x < 160)
    sbias[threadIdx.x] = threadIdx.x < 32 ? bias0[threadIdx.x] : (threadIdx.x < 96 ? bias1[threadIdx.x - 32] : bias2[threadIdx.x - 96]);
  auto bias_relu4 = [](float4 bv, f32x4 acc) {
    return pack4_bf16(relu(acc[0] + bv.x), relu(acc[1] + bv.y), relu(acc[2] + bv.z), relu(acc[3] + bv.w));
  };
  // Loads and stores share vmcnt: waiting for a prefetch also waits for every store issued before the wait.
  // Each sample's frames are therefore staged BEFORE the previous sample's a3 copy-out is issued, so the wait
  // never covers fresh stores (a1 / a2 go out during the conv2 / conv3 phases, long before).
  // Frame pointers run one sample ahead of the frame data: threads 0-3 load sample b + 2 grid's table entries
  // while sample b computes and park them in LDS at the next staging, so the data prefetch of sample
  // b + grid never waits on a dependent pointer load.
  __shared__ const uint8_t* sptr[4];
  const uint8_t* pnext = nullptr;   // threads 0-3: table entry (slot = tid) of sample b + grid
  uint4 pf[4];
  if (threadIdx.x < 4) sptr[threadIdx.x] = (int)blockIdx.x < B ? table[blockIdx.x * 4 + threadIdx.x] : nullptr;
  if (threadIdx.x < 4 && (int)(blockIdx.x + gridDim.x) < B) pnext = table[(blockIdx.x + gridDim.x) * 4 + threadIdx.x];
  lds_barrier();
  frames_prefetch_slots(sptr, (int)blockIdx.x < B, pf);
  for (int b = blockIdx.x; b < B; b += gridDim.x) {
    mark(-1);
    lds_barrier();   // previous sample's conv phases are done with X / A2 (and the pointer slots)
    frames_stage_slots<kXW>(X, pf);
    if (threadIdx.x < 4) sptr[threadIdx.x] = pnext;
    if (b != (int)blockIdx.x) lds_copy_out<49, 64, kA3S>(A3, a3 + (size_t)(b - gridDim.x) * kA3Ld);
    lds_barrier();
    mark(0);
    frames_prefetch_slots(sptr, b + (int)gridDim.x < B, pf);
    if (threadIdx.x < 4 && b + 2 * (int)gridDim.x < B) pnext = table[(b + 2 * gridDim.x) * 4 + threadIdx.x];
    // conv1: M = 400 (25 tiles of 16), N = 32, K = 256: k-step s covers tap (i, j) = (s >> 2, (s >> 1) & 1)
    conv_tiles<8, 4>(
        wave >> 1, 4, 25, w1,
        [&](int t, int s) {
          const int m = t * 16 + r, ox = m / 20, oy = m - ox * 20;
          return X + ((ox + (s >> 2)) * kXW + oy + ((s >> 1) & 1)) * kXS + 32 * (s & 1) + 8 * g;
        },
        [&](int) { return *reinterpret_cast<const float4*>(sbias + c1 + 4 * g); },
        [&](int t, f32x4 acc, float4 bv) {
          const int m = t * 16 + r, ox = m / 20;
          *reinterpret_cast<uint2*>(A1 + (ox * kA1W + m - ox * 20) * kA1S + c1 + 4 * g) = bias_relu4(bv, acc);
        });
    lds_barrier();
    mark(1);
    if (STORE12) lds_copy_out_pitched<400, 32, kA1S, 20, kA1W>(A1, a1 + (size_t)b * 12800);
    // conv2: 4x4 stride 2 over A1 [20][20][32]; M = 81 (6 tiles), k-step s = tap (kh, kw) = (s >> 2, s & 3)
    conv_tiles<16, 4>(
        wave >> 2, 2, 6, w2,
        [&](int t, int s) {
          const int m = min(t * 16 + r, 80), p = m / 9, q = m - p * 9;
          return A1 + ((2 * p + (s >> 2)) * kA1W + 2 * q + (s & 3)) * kA1S + 8 * g;
        },
        [&](int) { return *reinterpret_cast<const float4*>(sbias + 32 + c2 + 4 * g); },
        [&](int t, f32x4 acc, float4 bv) {
          const int m = t * 16 + r, p = m / 9;
          if (m < 81) *reinterpret_cast<uint2*>(A2 + (p * kA2W + m - p * 9) * kA2S + c2 + 4 * g) = bias_relu4(bv, acc);
        });
    lds_barrier();
    mark(2);
    if (STORE12) lds_copy_out_pitched<81, 64, kA2S, 9, kA2W>(A2, a2 + (size_t)b * 5184);
    // conv3: 3x3 stride 1 over A2 [9][9][64]; M = 49 (4 tiles), k-step s: tap s >> 1, channel half s & 1
    conv_tiles<18, 3>(
        wave >> 2, 2, 4, w3,
        [&](int t, int s) {
          const int m = min(t * 16 + r, 48), p = m / 7, q = m - p * 7;
          const int tap = s >> 1, kh = tap / 3, kw = tap - kh * 3;
          return A2 + ((p + kh) * kA2W + q + kw) * kA2S + 32 * (s & 1) + 8 * g;
        },
        [&](int) { return *reinterpret_cast<const float4*>(sbias + 96 + c2 + 4 * g); },
        [&](int t, f32x4 acc, float4 bv) {
          const int m = t * 16 + r;
          if (m < 49) *reinterpret_cast<uint2*>(A3 + m * kA3S + c2 + 4 * g) = bias_relu4(bv, acc);
        });
    mark(3);
  }
  if constexpr (TIMING) {
    if (threadIdx.x == 0)
      for (int i = 0; i < 4; ++i) timing[blockIdx.x * 4 + i] = ph[i];
  }
  lds_barrier();
  const int last = (int)blockIdx.x + ((B - 1 - (int)blockIdx.x) / (int)gridDim.x) * (int)gridDim.x;
  if ((int)blockIdx.x < B) lds_copy_out<49, 64, kA3S>(A3, a3 + (size_t)last * kA3Ld);
}

// conv1 weight gradient: per block fp32 partial dW[256 (s2d k)][32] followed by the bias partial db[32] in
// slab[blockIdx.x] (stride kConv1SlabStride); reduced over blocks in fixed order by k_slab_reduce<true>.
constexpr int kConv1SlabStride = 8192 + 32;
// Wave w owns k tiles 2w, 2w+1 (one s2d tap (i, j) = ((w >> 1) >> 1, (w >> 1) & 1), 32 channels) x both
// 16-column n tiles.  m-steps of 32 im2col rows (13 per sample, rows 400..415 have dz = 0).
__global__ __launch_bounds__(kTrunkThreads, 1) void k_conv1_wgrad(const uint8_t* const* __restrict__ table,
                                                                  const bf16* __restrict__ dz1, int B, float* slab) {
  extern __shared__ __attribute__((aligned(16))) bf16 lds[];
  bf16* X = lds;
  bf16* DZ = lds + kLdsX;
  __shared__ float bred[16][32];
  const int tid = threadIdx.x, wave = wave_id(), lane = tid & 63;
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  const int ij = wave >> 1, ti = ij >> 1, tj = ij & 1;
  const int col0 = (wave & 1) * 32 + 4 * p;   // channel of this lane's first k tile (second: +16)
  for (int i = tid; i < 16 * kDZS / 8; i += kTrunkThreads)
    *reinterpret_cast<uint4*>(DZ + 400 * kDZS + i * 8) = uint4{0, 0, 0, 0};
  f32x4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int c = 0; c < 2; ++c) acc[a][c] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
  float bsum = 0.0f;
  const int bn = tid & 31, brg = tid >> 5;   // bias: column bn, rows brg + 16 i
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  auto tr = [](const bf16* pp) { return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(pp)); };
  uint4 pf[4], dv[4];
  // dz1 sample block [400][32] -> registers (1600 chunks), one sample ahead like the frames
  auto dz_prefetch = [&](int b) {
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int c = tid + u * kTrunkThreads;
      dv[u] = uint4{0, 0, 0, 0};
      if (b < B && c < 1600)
        dv[u] = __builtin_bit_cast(uint4, *(const __attribute__((address_space(1))) u32x4*)(dz1 + (size_t)b * 12800 + c * 8));
    }
  };
  // frame pointers one sample ahead of the frame data (as in k_trunk_fwd)
  __shared__ const uint8_t* sptr[4];
  const uint8_t* pnext = nullptr;
  if (tid < 4) sptr[tid] = (int)blockIdx.x < B ? table[blockIdx.x * 4 + tid] : nullptr;
  if (tid < 4 && (int)(blockIdx.x + gridDim.x) < B) pnext = table[(blockIdx.x + gridDim.x) * 4 + tid];
  lds_barrier();
  frames_prefetch_slots(sptr, (int)blockIdx.x < B, pf);
  dz_prefetch(blockIdx.x);
  for (int b = blockIdx.x; b < B; b += gridDim.x) {
    lds_barrier();   // previous sample's readers are done
    frames_stage_slots(X, pf);
    if (tid < 4) sptr[tid] = pnext;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int c = tid + u * kTrunkThreads;
      if (c < 1600) *reinterpret_cast<uint4*>(DZ + (c >> 2) * kDZS + (c & 3) * 8) = dv[u];
    }
    lds_barrier();
    frames_prefetch_slots(sptr, b + (int)gridDim.x < B, pf);
    if (tid < 4 && b + 2 * (int)gridDim.x < B) pnext = table[(b + 2 * gridDim.x) * 4 + tid];
    dz_prefetch(b + gridDim.x);
    for (int ms = 0; ms < 13; ++ms) {
      const int m0 = ms * 32;
      // rows of this lane's tr reads: m0 + 4g + q and m0 + 16 + 4g + q
      int mA = min(m0 + 4 * g + q, 399), mB = min(m0 + 16 + 4 * g + q, 399);
      const int oxA = mA / 20, oyA = mA - oxA * 20, oxB = mB / 20, oyB = mB - oxB * 20;
      const bf16* xa = X + ((oxA + ti) * 21 + oyA + tj) * kXS + col0;
      const bf16* xb = X + ((oxB + ti) * 21 + oyB + tj) * kXS + col0;
      typedef short s16x8 __attribute__((ext_vector_type(8)));
      bf16x8 af[2], bf[2];
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        const s16x4 v0 = tr(xa + 16 * a), v1 = tr(xb + 16 * a);
        af[a] = __builtin_bit_cast(bf16x8, (s16x8){v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]});
      }
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const s16x4 v0 = tr(DZ + (m0 + 4 * g + q) * kDZS + c * 16 + 4 * p);
        const s16x4 v1 = tr(DZ + (m0 + 16 + 4 * g + q) * kDZS + c * 16 + 4 * p);
        bf[c] = __builtin_bit_cast(bf16x8, (s16x8){v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]});
      }
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int c = 0; c < 2; ++c) acc[a][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[a], bf[c], acc[a][c], 0, 0, 0);
    }
    for (int m = brg; m < 400; m += 16) bsum += (float)DZ[m * kDZS + bn];
  }
  // D tile (a, c): row k = ij * 64 + (wave & 1) * 32 + a * 16 + 4g + e, col n = c * 16 + li
  float* out = slab + (size_t)blockIdx.x * kConv1SlabStride;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e) out[(ij * 64 + (wave & 1) * 32 + a * 16 + 4 * g + e) * 32 + c * 16 + li] = acc[a][c][e];
  bred[brg][bn] = bsum;
  lds_barrier();
  if (tid < 32) {
    float s = 0.0f;
    for (int i = 0; i < 16; ++i) s += bred[i][tid];
    out[8192 + tid] = s;
  }
}

// Channel-half variant of k_conv1_wgrad (the shipped one): block i = sample chunk i % G1 x half hh = i / G1 of the
// 64 s2d channels (ring slots 2hh, 2hh + 1).  The half image X [441][kXHS] + DZ fit two blocks per CU, so two
// per-sample chains interleave on every CU (the one-block kernel is latency-bound); each block stages half the
// frames and all of dz1.  Wave w owns tap ij = w >> 1 and k tile a = w & 1 (16 channels) x both n tiles.  Every
// dW element sees the same MFMA operands in the same order as in k_conv1_wgrad (bit-identical slab rows);
// half 0 also sums the bias partial.
constexpr int kXHS = 40;
constexpr size_t kConv1WgradHLds = (size_t)(441 * kXHS + kLdsDZ) * 2;
static_assert(2 * (kConv1WgradHLds + 16 * 32 * 4 + 64) <= 160 * 1024, "k_conv1_wgrad_h: two blocks per CU");
__global__ __launch_bounds__(kTrunkThreads, 2) void k_conv1_wgrad_h(const uint8_t* const* __restrict__ table,
                                                                    const bf16* __restrict__ dz1, int B, int G1,
                                                                    float* slab) {
  extern __shared__ __attribute__((aligned(16))) bf16 lds[];
  bf16* X = lds;
  bf16* DZ = lds + 441 * kXHS;
  __shared__ float bred[16][32];
  __shared__ const uint8_t* sptr[2];
  const int tid = threadIdx.x, wave = wave_id(), lane = tid & 63;
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  const int chunk = (int)blockIdx.x % G1, hh = (int)blockIdx.x / G1;
  const int ij = wave >> 1, ti = ij >> 1, tj = ij & 1, ka = wave & 1;
  const int col0 = ka * 16 + 4 * p;
  for (int i = tid; i < 16 * kDZS / 8; i += kTrunkThreads)
    *reinterpret_cast<uint4*>(DZ + 400 * kDZS + i * 8) = uint4{0, 0, 0, 0};
  f32x4 acc[2] = {f32x4{0.0f, 0.0f, 0.0f, 0.0f}, f32x4{0.0f, 0.0f, 0.0f, 0.0f}};
  float bsum = 0.0f;
  const int bn = tid & 31, brg = tid >> 5;
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  auto tr = [](const bf16* pp) { return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(pp)); };
  uint4 pf[2], dv[4];
  auto dz_prefetch = [&](int b) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int c = tid + u * kTrunkThreads;
      dv[u] = uint4{0, 0, 0, 0};
      if (b < B && c < 1600)
        dv[u] = __builtin_bit_cast(uint4, *(const __attribute__((address_space(1))) u32x4*)(dz1 + (size_t)b * 12800 + c * 8));
    }
  };
  // this half's two frames (pointers from LDS, wave-uniform), thread pos < 441 owns s2d block pos
  auto frames_prefetch = [&](bool valid) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      pf[u] = uint4{0, 0, 0, 0};
      const unsigned long long fv = (unsigned long long)sptr[u];
      const uint8_t* f = (const uint8_t*)(((unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((int)(fv >> 32)) << 32) |
                                          (unsigned)__builtin_amdgcn_readfirstlane((int)fv));
      if (valid && f && tid < 441) pf[u] = __builtin_bit_cast(uint4, *(const __attribute__((address_space(1))) u32x4*)(f + tid * 16));
    }
  };
  const uint8_t* pnext = nullptr;
  if (tid < 2) sptr[tid] = chunk < B ? table[chunk * 4 + 2 * hh + tid] : nullptr;
  if (tid < 2 && chunk + G1 < B) pnext = table[(chunk + G1) * 4 + 2 * hh + tid];
  lds_barrier();
  frames_prefetch(chunk < B);
  dz_prefetch(chunk);
  for (int b = chunk; b < B; b += G1) {
    lds_barrier();   // previous sample's readers are done
    if (tid < 441) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        uint4 lo, hi;
        u8x16_to_bf16(pf[u], lo, hi);
        uint4* d = reinterpret_cast<uint4*>(X + tid * kXHS + u * 16);
        d[0] = lo;
        d[1] = hi;
      }
    }
    if (tid < 2) sptr[tid] = pnext;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int c = tid + u * kTrunkThreads;
      if (c < 1600) *reinterpret_cast<uint4*>(DZ + (c >> 2) * kDZS + (c & 3) * 8) = dv[u];
    }
    lds_barrier();
    frames_prefetch(b + G1 < B);
    if (tid < 2 && b + 2 * G1 < B) pnext = table[(b + 2 * G1) * 4 + 2 * hh + tid];
    dz_prefetch(b + G1);
    for (int ms = 0; ms < 13; ++ms) {
      const int m0 = ms * 32;
      int mA = min(m0 + 4 * g + q, 399), mB = min(m0 + 16 + 4 * g + q, 399);
      const int oxA = mA / 20, oyA = mA - oxA * 20, oxB = mB / 20, oyB = mB - oxB * 20;
      typedef short s16x8 __attribute__((ext_vector_type(8)));
      const s16x4 x0 = tr(X + ((oxA + ti) * 21 + oyA + tj) * kXHS + col0);
      const s16x4 x1 = tr(X + ((oxB + ti) * 21 + oyB + tj) * kXHS + col0);
      const bf16x8 af = __builtin_bit_cast(bf16x8, (s16x8){x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]});
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const s16x4 v0 = tr(DZ + (m0 + 4 * g + q) * kDZS + c * 16 + 4 * p);
        const s16x4 v1 = tr(DZ + (m0 + 16 + 4 * g + q) * kDZS + c * 16 + 4 * p);
        const bf16x8 bfr = __builtin_bit_cast(bf16x8, (s16x8){v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]});
        acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr, acc[c], 0, 0, 0);
      }
    }
    if (hh == 0)
      for (int m = brg; m < 400; m += 16) bsum += (float)DZ[m * kDZS + bn];
  }
  // D tile (ka, c): row k = ij * 64 + hh * 32 + ka * 16 + 4g + e, col n = c * 16 + li (k_conv1_wgrad's rows)
  float* out = slab + (size_t)chunk * kConv1SlabStride;
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int e = 0; e < 4; ++e) out[(ij * 64 + hh * 32 + ka * 16 + 4 * g + e) * 32 + c * 16 + li] = acc[c][e];
  if (hh == 0) {
    bred[brg][bn] = bsum;
    lds_barrier();
    if (tid < 32) {
      float t = 0.0f;
      for (int i = 0; i < 16; ++i) t += bred[i][tid];
      out[8192 + tid] = t;
    }
  }
}

// Backward data through conv3 and conv2, fused per sample:
//   dz2 = convT(dz3, W2) * (a2 > 0)        M = 81 rows (ih, iw), N = 64, K = 576 = (kh*3+kw)*64 + oc
//   dz1 = convT(dz2, W1) * (a1 > 0)        by output parity class p = (ih & 1, iw & 1): rows (i, j) of
//                                          10 x 10, N = 128 = p*32 + c, K = 256 = (th*2+tw)*64 + oc
// dz3 is staged into a zero-bordered [11][11] LDS image (interior at +2) and dz2 into another (interior
// at +1), so every transposed-conv gather is an unconditional 16-byte LDS read.  W2^T (72 VGPRs) and the
// parity-packed W1^T (32 VGPRs) are this lane's B fragments for the block's lifetime.
constexpr int kPadS = 80;                  // padded image row stride (bf16)
// Padded images are 11 rows of kW3 / kW2 positions (11 used): the im2col rows a 16-lane read group gathers
// run along an image row and wrap to the next one; with a row pitch of 17 (dz3, 9 output columns) / 18
// (dz2, 10 columns) a wrap advances the position index by 1 mod 8, exactly like a step inside a row, so
// the fragment reads stay bank-conflict-free across wraps (the 40-dword position stride repeats its
// banks every 8 positions).
constexpr int kW3 = 17, kW2 = 18;
constexpr int kLdsPad3 = 11 * kW3 * kPadS, kLdsPad2 = 11 * kW2 * kPadS;
constexpr int kLdsPad = kLdsPad3 + kLdsPad2;   // both images
constexpr int kLdsA2M = 81 * 72;           // staged a2 (ReLU mask of dz2), row stride 72
constexpr size_t kTrunkBwdLds = (size_t)(kLdsPad + kLdsA2M + kLdsA1) * 2;

// TIMING (development only): wave 0's s_memtime cycles per phase (staging + dz1 copy-out, dz2, dz1) ->
// timing[blockIdx.x * 4 + phase]
template <bool TIMING = false>
__global__ __launch_bounds__(kTrunkThreads, 1) void k_trunk_bwd_data(const bf16* __restrict__ dz3, const bf16* __restrict__ a2,
                                                                     const bf16* __restrict__ a1, int B,
                                                                     const bf16* __restrict__ wb2, const bf16* __restrict__ wb1,
                                                                     bf16* __restrict__ dz2, bf16* __restrict__ dz1,
                                                                     unsigned long long* __restrict__ timing) {
  unsigned long long ph[4] = {0, 0, 0, 0}, tm = 0;
  auto mark = [&](int i) {
    if constexpr (TIMING) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      if (i >= 0) ph[i] += t - tm;
      tm = t;
    }
  };
  extern __shared__ __attribute__((aligned(16))) bf16 lds[];
  bf16* P3 = lds;                   // dz3, interior (oh + 2, ow + 2)
  bf16* P2 = lds + kLdsPad3;        // dz2 (masked), interior (oh + 1, ow + 1)
  bf16* M2 = lds + kLdsPad;         // a2
  bf16* D1 = M2 + kLdsA2M;          // dz1 parity rows before masking: [400][32] in natural (ih, iw) order
  const int tid = threadIdx.x, wave = wave_id(), lane = tid & 63;
  const int r = lane & 15, g = lane >> 4;
  for (int i = tid; i < kLdsPad / 8; i += kTrunkThreads) *reinterpret_cast<uint4*>(lds + i * 8) = uint4{0, 0, 0, 0};
  const int c3 = (wave & 3) * 16;       // phase A: the wave's 16 channels of dz2
  bf16x8 w3[18], w2[8];                 // A operands (row = lane & 15 of the wave's channel slice)
#pragma unroll
  for (int s = 0; s < 18; ++s) w3[s] = ldfrag(wb2, c3 >> 4, s, 576, lane);
#pragma unroll
  for (int s = 0; s < 8; ++s) w2[s] = ldfrag(wb1, wave, s, 256, lane);
  // prefetch: dz3 392 chunks + a2 648 chunks = 1040 -> 3 per thread (staged to LDS); the sample's a1 (the
  // dz1 ReLU mask, 1600 chunks -> 4 per thread) stays in registers in the mapping of the dz1 copy-out.
  // Loads and stores share vmcnt, so a sample's dz1 copy-out is deferred until after the next sample's
  // staging wait: no fresh stores are outstanding when a prefetch is awaited.
  constexpr int kC3 = 392, kCA = 648, kCT = kC3 + kCA, kPB = (kCT + kTrunkThreads - 1) / kTrunkThreads;
  constexpr int kPA = (1600 + kTrunkThreads - 1) / kTrunkThreads;
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  typedef const __attribute__((address_space(1))) u32x4 gvec;
  uint4 pf[kPB], pa[kPA];
  auto prefetch = [&](int b) {
#pragma unroll
    for (int u = 0; u < kPB; ++u) {
      const int c = tid + u * kTrunkThreads;
      pf[u] = uint4{0, 0, 0, 0};
      if (b < B && c < kCT)
        pf[u] = __builtin_bit_cast(uint4, c < kC3 ? *(gvec*)(dz3 + (size_t)b * 3136 + c * 8)
                                                  : *(gvec*)(a2 + (size_t)b * 5184 + (c - kC3) * 8));
    }
  };
  auto prefetch_mask = [&](int b) {
#pragma unroll
    for (int u = 0; u < kPA; ++u) {
      const int c = tid + u * kTrunkThreads;
      pa[u] = uint4{0, 0, 0, 0};
      if (b < B && c < 1600) pa[u] = __builtin_bit_cast(uint4, *(gvec*)(a1 + (size_t)b * 12800 + c * 8));
    }
  };
  // dz1 = D1 * (a1 > 0) -> global, coalesced (D1 and pa hold sample b)
  auto dz1_out = [&](int b) {
#pragma unroll
    for (int u = 0; u < kPA; ++u) {
      const int c = tid + u * kTrunkThreads;
      if (c < 1600) {
        const int row = c >> 2, col = (c & 3) * 8;
        const bf16x8 act = __builtin_bit_cast(bf16x8, pa[u]);
        bf16x8 v = lds8(D1 + row * kA1S + col);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = (float)act[e] > 0.0f ? v[e] : (bf16)0.0f;
        *reinterpret_cast<bf16x8*>(dz1 + (size_t)b * 12800 + row * 32 + col) = v;
      }
    }
  };
  prefetch(blockIdx.x);
  lds_barrier();   // borders zeroed
  for (int b = blockIdx.x; b < B; b += gridDim.x) {
    mark(-1);
    lds_barrier();   // previous sample's readers are done
#pragma unroll
    for (int u = 0; u < kPB; ++u) {
      const int c = tid + u * kTrunkThreads;
      if (c < kC3) {
        const int row = c >> 3, col = (c & 7) * 8, oh = row / 7, ow = row - oh * 7;
        *reinterpret_cast<uint4*>(P3 + ((oh + 2) * kW3 + ow + 2) * kPadS + col) = pf[u];
      } else if (c < kCT) {
        const int cc = c - kC3, row = cc >> 3, col = (cc & 7) * 8;
        *reinterpret_cast<uint4*>(M2 + row * 72 + col) = pf[u];
      }
    }
    if (b != (int)blockIdx.x) dz1_out(b - gridDim.x);
    lds_barrier();
    mark(0);
    prefetch(b + gridDim.x);
    prefetch_mask(b);
    // phase A: dz2 (wave: channel slice c3, tiles wave >> 2, +2, ...)
    conv_tiles<18, 3>(
        wave >> 2, 2, 6, w3,
        [&](int t, int s) {
          const int m = min(t * 16 + r, 80), ih = m / 9, iw = m - ih * 9;
          const int tap = s >> 1, kh = tap / 3, kw = tap - kh * 3;
          return P3 + ((ih + 2 - kh) * kW3 + iw + 2 - kw) * kPadS + 32 * (s & 1) + 8 * g;
        },
        [&](int t) { return *reinterpret_cast<const bf16x4*>(M2 + min(t * 16 + r, 80) * 72 + c3 + 4 * g); },
        [&](int t, f32x4 acc, bf16x4 act) {
          const int m = t * 16 + r;
          if (m < 81) {
            const int oh = m / 9, ow = m - oh * 9;
            *reinterpret_cast<uint2*>(P2 + ((oh + 1) * kW2 + ow + 1) * kPadS + c3 + 4 * g) =
                pack4_bf16((float)act[0] > 0.0f ? acc[0] : 0.0f, (float)act[1] > 0.0f ? acc[1] : 0.0f,
                           (float)act[2] > 0.0f ? acc[2] : 0.0f, (float)act[3] > 0.0f ? acc[3] : 0.0f);
          }
        });
    lds_barrier();
    mark(1);
    // dz2 -> global (81 x 64)
    for (int c = tid; c < 648; c += kTrunkThreads) {
      const int row = c >> 3, col = (c & 7) * 8, oh = row / 9, ow = row - oh * 9;
      *reinterpret_cast<uint4*>(dz2 + (size_t)b * 5184 + row * 64 + col) =
          *reinterpret_cast<const uint4*>(P2 + ((oh + 1) * kW2 + ow + 1) * kPadS + col);
    }
    // phase B: dz1 parity classes; wave = 16-column slice of N = p*32 + c (p = wave >> 1)
    {
      const int p = wave >> 1, ph = p >> 1, pw = p & 1, c0 = (wave & 1) * 16;
      conv_tiles<8, 4>(
          0, 1, 7, w2,
          [&](int t, int s) {
            const int m = min(t * 16 + r, 99), i = m / 10, j = m - i * 10;
            const int tp = s >> 1, th = tp >> 1, tw = tp & 1;
            return P2 + ((i + 1 - th) * kW2 + j + 1 - tw) * kPadS + 32 * (s & 1) + 8 * g;
          },
          [](int) { return 0; },
          [&](int t, f32x4 acc, int) {
            const int m = t * 16 + r;
            if (m < 100) {
              const int i = m / 10, j = m - i * 10;
              *reinterpret_cast<uint2*>(D1 + ((2 * i + ph) * 20 + 2 * j + pw) * kA1S + c0 + 4 * g) =
                  pack4_bf16(acc[0], acc[1], acc[2], acc[3]);
            }
          });
    }
    lds_barrier();
    mark(2);
  }
  if constexpr (TIMING) {
    if (threadIdx.x == 0)
      for (int i = 0; i < 4; ++i) timing[blockIdx.x * 4 + i] = ph[i];
  }
  lds_barrier();
  const int last = (int)blockIdx.x + ((B - 1 - (int)blockIdx.x) / (int)gridDim.x) * (int)gridDim.x;
  if ((int)blockIdx.x < B) dz1_out(last);
}

}  // namespace qn
}  // namespace qlx

namespace qlx {
namespace qn {

// Weight gradient of conv2 / conv3, per sample from LDS:
//   dW[(kh*KS + kw)*C + c][n] = sum_samples sum_(oh,ow) in[oh*S + kh][ow*S + kw][c] * dz[oh][ow][n]
//   db[n] = sum dz[..][n]
// Block (8 waves) = one group of TG taps (TG*C rows of dW) x one chunk of samples; per sample the input
// activation [IH*IW][C] and dz [OH*OW][64] are staged into LDS once (prefetched one sample ahead), and
// the m-reduction (output positions, 32 per MFMA) reads both operands with ds_read_b64_tr_b16: each lane
// supplies the LDS row of its own im2col position, so the im2col is never materialised.  Wave w owns
// KTW k-tiles (16 rows of dW each) x NTW of the four 16-column n-tiles.
// Output: slab[chunk][TAPS*C*64 + 64] rows of [dW partial | db partial] (db from tap group 0 only).
// Launched as k_conv23_wgrad (conv3 and conv2 blocks in one grid).
template <int IH, int IW, int C, int KS, int S, int OH, int OW, int TG, int KTW, int NTW, int NS_ = 1>
struct ConvWgradCfg {
  static constexpr int NS = NS_;   // samples staged per LDS round (round 5: one sample per round left 2 m-steps of MFMA
                                   // work (conv3) between each pair of barriers)
  static constexpr int M = OH * OW, MP = (M + 31) / 32 * 32;   // positions, padded to the 32-row m-step
  static constexpr int XS = C + (C == 32 ? 8 : 16);            // input row stride (bf16): 20 / 40 dwords
  static constexpr int DS = 64 + 16;                            // dz row stride: 40 dwords
  static constexpr int LX = IH * IW * XS, LD = MP * DS;
  static constexpr size_t LDS = (size_t)NS * (LX + LD) * 2;
  static constexpr int KTILES = TG * C / 16;                    // 16-row k tiles per block
  static_assert(4 % NTW == 0 && (KTILES / KTW) * (4 / NTW) == 8 && KTILES % KTW == 0,
                "KTW k tiles x NTW n tiles per wave must cover the block's KTILES x 4 tiles with 8 waves");
  static constexpr int CHX = IH * IW * C / 8, CHD = M * 64 / 8;  // 16-byte chunks per sample
  static constexpr int PF = (NS * (CHX + CHD) + kTrunkThreads - 1) / kTrunkThreads;
  static constexpr int TAPS = KS * KS;
  static constexpr size_t ZS = (size_t)TAPS * C * 64 + 64;      // slab row
};

template <int IH, int IW, int C, int KS, int S, int OH, int OW, int TG, int KTW, int NTW, int NS>
__device__ __forceinline__ void conv_wgrad_body(const bf16* __restrict__ in, const bf16* __restrict__ dz, int B, int per_chunk,
                                                float* slab, int chunk, int tg) {
  using Cf = ConvWgradCfg<IH, IW, C, KS, S, OH, OW, TG, KTW, NTW, NS>;
  constexpr int M = Cf::M, MP = Cf::MP, XS = Cf::XS, DS = Cf::DS;
  constexpr int CHX = Cf::CHX, CHD = Cf::CHD, PF = Cf::PF;
  extern __shared__ __attribute__((aligned(16))) bf16 lds[];
  bf16* X = lds;                   // NS images [IH * IW][XS]
  bf16* DZ = lds + NS * Cf::LX;    // NS images [MP][DS]
  const int tid = threadIdx.x, wave = wave_id(), lane = tid & 63;
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  const int b0 = chunk * per_chunk, b1 = min(B, b0 + per_chunk);
  // wave's tiles: k tiles kt0 .. kt0+KTW-1, n tiles nt0 .. nt0+NTW-1
  constexpr int NGROUPS = 4 / NTW;                  // waves sharing a k-tile set
  const int kt0 = (wave / NGROUPS) * KTW, nt0 = (wave % NGROUPS) * NTW;
  for (int i = tid; i < NS * (MP - M) * DS / 8; i += kTrunkThreads) {   // zero the dz pad rows once
    const int s = i / ((MP - M) * DS / 8), r = i - s * ((MP - M) * DS / 8);
    *reinterpret_cast<uint4*>(DZ + s * Cf::LD + M * DS + r * 8) = uint4{0, 0, 0, 0};
  }
  f32x4 acc[KTW][NTW];
#pragma unroll
  for (int a = 0; a < KTW; ++a)
#pragma unroll
    for (int c = 0; c < NTW; ++c) acc[a][c] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
  float bsum = 0.0f;
  const int bn = tid & 63, brg = tid >> 6;          // bias: column bn, rows brg + 8 i
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  typedef const __attribute__((address_space(1))) u32x4 gvec;
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  uint4 pf[PF];
  // chunk c of a round: sample s = c / (CHX + CHD) of the round, then its input chunks, then its dz chunks
  auto prefetch = [&](int b) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const int c = tid + u * kTrunkThreads, s = c / (CHX + CHD), cc = c - s * (CHX + CHD);
      pf[u] = uint4{0, 0, 0, 0};
      if (b + s < b1 && s < NS)
        pf[u] = __builtin_bit_cast(uint4, cc < CHX ? *(gvec*)(in + (size_t)(b + s) * (IH * IW * C) + cc * 8)
                                                   : *(gvec*)(dz + (size_t)(b + s) * (M * 64) + (cc - CHX) * 8));
    }
  };
  auto tr = [](const bf16* pp) { return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(pp)); };
  prefetch(b0);
  for (int b = b0; b < b1; b += NS) {
    lds_barrier();   // previous round's readers are done
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const int c = tid + u * kTrunkThreads, s = c / (CHX + CHD), cc = c - s * (CHX + CHD);
      if (s < NS) {   // samples past the chunk stage zeros (their dz rows contribute nothing)
        if (cc < CHX) {
          const int row = cc / (C / 8), col = (cc - row * (C / 8)) * 8;
          *reinterpret_cast<uint4*>(X + s * Cf::LX + row * XS + col) = pf[u];
        } else {
          const int cd = cc - CHX, row = cd >> 3, col = (cd & 7) * 8;
          *reinterpret_cast<uint4*>(DZ + s * Cf::LD + row * DS + col) = pf[u];
        }
      }
    }
    lds_barrier();
    prefetch(b + NS);
#pragma unroll 1
    for (int sm = 0; sm < NS * MP; sm += 32) {
      const int s = sm / MP, m0 = sm - s * MP;
      const bf16* X = lds + s * Cf::LX;
      const bf16* DZ = lds + NS * Cf::LX + s * Cf::LD;
      // this lane's two tr-read rows: m0 + 4g + q and m0 + 16 + 4g + q (clamped; their dz rows are zero)
      const int mA = min(m0 + 4 * g + q, M - 1), mB = min(m0 + 16 + 4 * g + q, M - 1);
      const int ohA = mA / OW, owA = mA - ohA * OW, ohB = mB / OW, owB = mB - ohB * OW;
      bf16x8 bf[NTW];
#pragma unroll
      for (int c = 0; c < NTW; ++c) {
        const s16x4 v0 = tr(DZ + (m0 + 4 * g + q) * DS + (nt0 + c) * 16 + 4 * p);
        const s16x4 v1 = tr(DZ + (m0 + 16 + 4 * g + q) * DS + (nt0 + c) * 16 + 4 * p);
        bf[c] = __builtin_bit_cast(bf16x8, (s16x8){v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]});
      }
#pragma unroll
      for (int a = 0; a < KTW; ++a) {
        const int kr = (tg * Cf::KTILES + kt0 + a) * 16;   // first dW row of this k tile
        const int tap = kr / C, c0 = kr - tap * C, kh = tap / KS, kw = tap - kh * KS;
        const bf16* xa = X + ((ohA * S + kh) * IW + owA * S + kw) * XS + c0 + 4 * p;
        const bf16* xb = X + ((ohB * S + kh) * IW + owB * S + kw) * XS + c0 + 4 * p;
        const s16x4 v0 = tr(xa), v1 = tr(xb);
        const bf16x8 af = __builtin_bit_cast(bf16x8, (s16x8){v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]});
#pragma unroll
        for (int c = 0; c < NTW; ++c) acc[a][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf[c], acc[a][c], 0, 0, 0);
      }
    }
    if (tg == 0)
      for (int s = 0; s < NS; ++s)
        for (int m = brg; m < M; m += 8) bsum += (float)DZ[s * Cf::LD + m * DS + bn];
  }
  // D tile (a, c): row k = (tg * KTILES + kt0 + a) * 16 + 4g + e, col n = (nt0 + c) * 16 + li
  float* out = slab + (size_t)chunk * Cf::ZS;
#pragma unroll
  for (int a = 0; a < KTW; ++a)
#pragma unroll
    for (int c = 0; c < NTW; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        out[(size_t)((tg * Cf::KTILES + kt0 + a) * 16 + 4 * g + e) * 64 + (nt0 + c) * 16 + li] = acc[a][c][e];
  if (tg == 0) {
    __shared__ float bred[8][64];
    bred[brg][bn] = bsum;
    lds_barrier();
    if (tid < 64) {
      float sb = 0.0f;
      for (int i = 0; i < 8; ++i) sb += bred[i][tid];
      out[(size_t)Cf::TAPS * C * 64 + tid] = sb;
    }
  }
}

// Block -> (chunk, tap group) of a G-group layer whose blocks start at grid offset t0: blocks b and b + 8 share an
// XCD (round-robin dispatch), so the G tap groups of one sample chunk are blocks 8 G k + 8 g + x (consecutive
// dispatch, one XCD) - each sample's activations and dz come from HBM once and from that XCD's L2 for the
// other groups.  Returns false for the padding blocks of the last round.
template <int G>
__device__ __forceinline__ bool wgrad_chunk_group(int t, int used, int& chunk, int& group) {
  const int x = t & 7, r = t >> 3;
  group = r % G;
  chunk = (r / G) * 8 + x;
  return chunk < used;
}
__host__ __device__ __forceinline__ int wgrad_blocks(int groups, int used) { return (used + 7) / 8 * 8 * groups; }

// samples per LDS round (the chunk sizes are multiples of these, qnet.hip).  Measured at C3 (bf16, gpurun_out/a8): conv3 4 and
// conv2 2 samples per round (95 KB of LDS) took the launch 25.8 -> 34.3 us; one sample per round is kept
constexpr int kWg3Samples = 1, kWg2Samples = 1;
// conv3 (blocks [0, wgrad_blocks(3, used3))) and conv2 (the rest) in one launch
__global__ __launch_bounds__(kTrunkThreads, 1) void k_conv23_wgrad(const bf16* __restrict__ a2, const bf16* __restrict__ dz3,
                                                                   int per3, int used3, float* slab3, const bf16* __restrict__ a1,
                                                                   const bf16* __restrict__ dz2, int per2, int used2,
                                                                   float* slab2, int B) {
  const int t = blockIdx.x, n3 = wgrad_blocks(3, used3);
  int chunk, group;
  if (t < n3) {
    if (wgrad_chunk_group<3>(t, used3, chunk, group))
      conv_wgrad_body<9, 9, 64, 3, 1, 7, 7, 3, 3, 2, kWg3Samples>(a2, dz3, B, per3, slab3, chunk, group);
  } else if (wgrad_chunk_group<2>(t - n3, used2, chunk, group)) {
    conv_wgrad_body<20, 20, 32, 4, 2, 9, 9, 8, 2, 4, kWg2Samples>(a1, dz2, B, per2, slab2, chunk, group);
  }
}

}  // namespace qn
}  // namespace qlx
