// Nature-DQN kernels for gfx950: implicit-GEMM convolutions / dense layers on MFMA (bf16 inputs,
// fp32 accumulation), LDS-staged weight-gradient GEMMs with hardware transposed reads.
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

__device__ __forceinline__ bf16x8 zero8() {
  const uint4 z = {0, 0, 0, 0};
  return __builtin_bit_cast(bf16x8, z);
}
__device__ __forceinline__ bf16x8 ld8(const bf16* p) { return __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(p)); }

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
// A-operand loaders: load(m, k0) returns A[m][k0 .. k0+7] as 8 bf16 (zero outside the matrix).

// conv1 over space-to-depth frames: rows m = (b, oh, ow) of [B][20][20]; k = ((i*2+j)*4+c)*16 + dx*4 + dy
// with kh = 4i + dx, kw = 4j + dy, c = ring slot.  A 16-byte s2d block holds (dx, dy) of one 4x4 pixel
// block, so 8 consecutive k are 8 bytes of one block.
struct LoadConv1 {
  const uint8_t* const* frames;   // [B][4] frame pointers (nullptr = zero frame)
  int M;
  __device__ __forceinline__ bf16x8 load(int m, int k0) const {
    if (m >= M) return zero8();
    const int b = m / 400, pos = m - b * 400;
    const int oh = pos / 20, ow = pos - oh * 20;
    const int h = (k0 >> 3) & 1, c = (k0 >> 4) & 3, j = (k0 >> 6) & 1, i = (k0 >> 7) & 1;
    const uint8_t* f = frames[b * 4 + c];
    if (!f) return zero8();
    const uint2 v = *reinterpret_cast<const uint2*>(f + ((oh + i) * kBlocks + (ow + j)) * 16 + h * 8);
    return u8x8_to_bf16(v);
  }
};

// NHWC im2col: rows m = (b, oh, ow) of [B][OH][OW]; k = (kh*KS + kw)*C + c
template <int H, int W, int C, int KS, int S, int OH, int OW>
struct LoadIm2col {
  const bf16* in;
  int M;
  __device__ __forceinline__ bf16x8 load(int m, int k0) const {
    if (m >= M) return zero8();
    const int b = m / (OH * OW), pos = m - b * (OH * OW);
    const int oh = pos / OW, ow = pos - oh * OW;
    const int tap = k0 / C, c = k0 - tap * C;
    const int kh = tap / KS, kw = tap - kh * KS;
    return ld8(in + (((size_t)b * H + oh * S + kh) * W + ow * S + kw) * C + c);
  }
};

// plain row-major [M][K]
template <int K>
struct LoadRows {
  const bf16* in;
  int M;
  __device__ __forceinline__ bf16x8 load(int m, int k0) const {
    if (m >= M) return zero8();
    return ld8(in + (size_t)m * K + k0);
  }
};

// transposed conv (backward data): rows m = (b, ih, iw) of the layer INPUT [B][IH][IW];
// k = (kh*KS + kw)*OC + oc; A = dOut[b][(ih-kh)/S][(iw-kw)/S][oc] where that is an output position.
template <int IH, int IW, int OH, int OW, int OC, int KS, int S>
struct LoadConvT {
  const bf16* dout;
  int M;
  __device__ __forceinline__ bf16x8 load(int m, int k0) const {
    if (m >= M) return zero8();
    const int b = m / (IH * IW), pos = m - b * (IH * IW);
    const int ih = pos / IW, iw = pos - ih * IW;
    const int tap = k0 / OC, oc = k0 - tap * OC;
    const int kh = tap / KS, kw = tap - kh * KS;
    const int th = ih - kh, tw = iw - kw;
    if (th < 0 || tw < 0 || th % S || tw % S) return zero8();
    const int oh = th / S, ow = tw / S;
    if (oh >= OH || ow >= OW) return zero8();
    return ld8(dout + (((size_t)b * OH + oh) * OW + ow) * OC + oc);
  }
};

// conv2 backward data (4x4 stride 2, 20x20x32 <- 9x9x64) split by output parity class p = blockIdx.y:
// (ih, iw) = (2i + ph, 2j + pw), rows m = (b*10 + i)*10 + j of one class; only taps kh = ph + 2th,
// kw = pw + 2tw reach the class, so k = (th*2 + tw)*64 + oc (K = 256 instead of 1024 mostly-zero taps).
struct LoadConv2T {
  const bf16* dout;   // dz2 [B][9][9][64]
  int M;              // B * 100 rows per class
  __device__ __forceinline__ bf16x8 load(int m, int k0) const {
    if (m >= M) return zero8();
    const int b = m / 100, pos = m - b * 100;
    const int i = pos / 10, j = pos - i * 10;
    const int tap = k0 >> 6, oc = k0 & 63;
    const int oh = i - (tap >> 1), ow = j - (tap & 1);
    if (oh < 0 || ow < 0 || oh >= 9 || ow >= 9) return zero8();
    return ld8(dout + (((size_t)b * 9 + oh) * 9 + ow) * 64 + oc);
  }
};

// ------------------------------------------------------------------------------------------
// Epilogues: consume acc tile element (m, n, value).

struct EpiBiasRelu {   // forward: out[m][n] = relu(v + bias[n]) as bf16
  bf16* out;
  const float* bias;
  int ldo;
  __device__ __forceinline__ void operator()(int m, int n, float v) const {
    const float t = v + bias[n];
    out[(size_t)m * ldo + n] = (bf16)(t > 0.0f ? t : 0.0f);
  }
};

struct EpiReluMask {   // backward data: dz[m][n] = v * (act[m][n] > 0)
  bf16* out;
  const bf16* act;
  int ldo;
  __device__ __forceinline__ void operator()(int m, int n, float v) const {
    const size_t i = (size_t)m * ldo + n;
    out[i] = (bf16)((float)act[i] > 0.0f ? v : 0.0f);
  }
};

struct EpiReluMaskConv2T {   // parity-class rows -> dz1[b][2i+ph][2j+pw][c] * (a1 > 0); n = p*32 + c
  bf16* out;
  const bf16* act;
  __device__ __forceinline__ void operator()(int m, int n, float v) const {
    const int p = n >> 5, c = n & 31;
    const int b = m / 100, pos = m - b * 100;
    const int i = pos / 10, j = pos - i * 10;
    const size_t idx = (((size_t)b * 20 + 2 * i + (p >> 1)) * 20 + 2 * j + (p & 1)) * 32 + c;
    out[idx] = (bf16)((float)act[idx] > 0.0f ? v : 0.0f);
  }
};

struct EpiSlab {   // split-K partial: slab[z][m][n] (fp32)
  float* slab;
  int ldo;
  size_t zstride;
  __device__ __forceinline__ void operator()(int m, int n, float v) const {
    slab[blockIdx.z * zstride + (size_t)m * ldo + n] = v;
  }
};

// ------------------------------------------------------------------------------------------
// C[m][n] = sum_k A(m,k) * Bt[n][k].  Block = 4 waves laid out WM x WN; wave tile (TM*16) x (TN*16);
// grid = (ceil(M/BM), N/BN, ksplit).  A and B fragments go straight from global/L2 to registers with
// a one-step register prefetch; the 16x16x32 bf16 MFMA accumulates in fp32.
template <int TM, int TN, int WM, int WN, class LoadA, class Epi>
__global__ __launch_bounds__(256) void k_igemm(LoadA la, const bf16* __restrict__ Bt, int M, int K, int k_per_split,
                                               Epi epi) {
  static_assert(WM * WN == 4, "4 waves");
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wm = wave / WN, wn = wave - wm * WN;
  const int m0 = blockIdx.x * (WM * TM * 16) + wm * TM * 16;
  const int n0 = blockIdx.y * (WN * TN * 16) + wn * TN * 16;
  const int kb = blockIdx.z * k_per_split;
  const int ke = min(K, kb + k_per_split);
  const int r = lane & 15, h = lane >> 4;
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
  bf16x8 a[TM], b[TN];
#pragma unroll
  for (int i = 0; i < TM; ++i) a[i] = la.load(m0 + i * 16 + r, kb + 8 * h);
#pragma unroll
  for (int j = 0; j < TN; ++j) b[j] = ld8(Bt + (size_t)(n0 + j * 16 + r) * K + kb + 8 * h);
  for (int k0 = kb; k0 < ke; k0 += 32) {
    bf16x8 an[TM], bn[TN];
    const int kn = k0 + 32 < ke ? k0 + 32 : k0;
#pragma unroll
    for (int i = 0; i < TM; ++i) an[i] = la.load(m0 + i * 16 + r, kn + 8 * h);
#pragma unroll
    for (int j = 0; j < TN; ++j) bn[j] = ld8(Bt + (size_t)(n0 + j * 16 + r) * K + kn + 8 * h);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < TM; ++i) a[i] = an[i];
#pragma unroll
    for (int j = 0; j < TN; ++j) b[j] = bn[j];
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + i * 16 + h * 4 + e;
        if (m < M) epi(m, n0 + j * 16 + r, acc[i][j][e]);
      }
}

// ------------------------------------------------------------------------------------------
// Implicit GEMM v2 for the conv-shaped layers (N = 32 / 64 per block, K <= 576):
//   C[m][n] = sum_k A(m,k) Bt[n][k] with v_mfma_f32_32x32x16_bf16.
// The block's B panel [BN][K] is staged once into LDS (row stride K+8 bf16: 16-B slot rotation makes the
// 32-row ds_read_b128 fragment reads conflict-free) and reused by every M tile the persistent block
// walks.  Each wave owns WMT x 32 rows x BN columns; A fragments (32 rows x 16 k, 16 B per lane) are
// gathered by the loader straight into a depth-4 register ring, issued 4 k-steps ahead of their MFMAs.
// Fragment maps (gfx950): A lane l = (row l&31, k 8(l>>5)+j); B lane l = (col l&31, k 8(l>>5)+j);
// D reg i of lane l = (row (i&3) + 8(i>>2) + 4(l>>5), col l&31).
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int BN, int WMT, int K, class LoadA, class Epi>
__global__ __launch_bounds__(256, 2) void k_igemm2(LoadA la, const bf16* __restrict__ Bt, int M, int n_mtiles, Epi epi) {
  constexpr int KP = K + 8;
  constexpr int NT = BN / 32;
  constexpr int BM = 4 * WMT * 32;
  constexpr int KS = K / 16;
  constexpr int D = 4;
  static_assert(KS % D == 0, "K/16 must be a multiple of the pipeline depth");
  extern __shared__ __attribute__((aligned(16))) bf16 lds_b[];
  const int n0 = blockIdx.y * BN;
  for (int i = threadIdx.x; i < BN * (K / 8); i += 256) {
    const int row = i / (K / 8), c = i - row * (K / 8);
    *reinterpret_cast<uint4*>(lds_b + row * KP + c * 8) = *reinterpret_cast<const uint4*>(Bt + (size_t)(n0 + row) * K + c * 8);
  }
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;
  const bf16* bbase = lds_b + r * KP + 8 * h;
  for (int tile = blockIdx.x; tile < n_mtiles; tile += gridDim.x) {
    const int m0 = tile * BM + wave * WMT * 32;
    f32x16 acc[WMT][NT];
#pragma unroll
    for (int t = 0; t < WMT; ++t)
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[t][j][e] = 0.0f;
    bf16x8 a[D][WMT];
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
      for (int t = 0; t < WMT; ++t) a[d][t] = la.load(m0 + t * 32 + r, d * 16 + 8 * h);
#pragma unroll 1
    for (int ks = 0; ks < KS; ks += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const int k0 = (ks + d) * 16;
        bf16x8 b[NT];
#pragma unroll
        for (int j = 0; j < NT; ++j) b[j] = *reinterpret_cast<const bf16x8*>(bbase + j * 32 * KP + k0);
#pragma unroll
        for (int t = 0; t < WMT; ++t)
#pragma unroll
          for (int j = 0; j < NT; ++j) acc[t][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[d][t], b[j], acc[t][j], 0, 0, 0);
        if (ks + d + D < KS) {
#pragma unroll
          for (int t = 0; t < WMT; ++t) a[d][t] = la.load(m0 + t * 32 + r, k0 + D * 16 + 8 * h);
        }
      }
    }
#pragma unroll
    for (int t = 0; t < WMT; ++t)
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int m = m0 + t * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
          if (m < M) epi(m, n0 + j * 32 + r, acc[t][j][e]);
        }
  }
}

// ------------------------------------------------------------------------------------------
// Weight gradient: dW[k][n] = sum_m X(m,k) dY[m][n]  (+ optional bias gradient db[n] = sum_m dY[m][n]).
// Block = 4 waves, output tile 64 (k) x NB (n); grid = (KIN/64, N/NB, chunks); each block reduces its
// m-chunk in steps of 32 rows staged in LDS, and writes an fp32 partial slab (reduced in fixed order
// by k_slab_reduce -> deterministic).  MFMA operands are read with ds_read_b64_tr_b16 (4 rows x 16
// columns per 16-lane group, delivered column-major), so the m-reduction lands in the MFMA k slot.
// Row permutation inside a 32-row step: MFMA k = 8g + e  <->  m = (e < 4 ? 4g + e : 16 + 4g + e - 4),
// which makes each 32-lane half read 8 consecutive rows; with row strides of 160 B (64 cols) or 96 B
// (32 cols) those 8 rows fall on disjoint 8-dword bank windows: conflict-free.
template <int NB>
struct WgradLds {
  static constexpr int XS = 80;                    // X tile row stride (bf16), 160 B
  static constexpr int YS = NB == 64 ? 80 : 48;    // dY tile row stride (bf16)
};

__device__ __forceinline__ bf16x8 tr_pair(const bf16* lds_base, int stride, int g, int p, int q, int col) {
  // rows for e = 0..3: 4g + q ; e = 4..7: 16 + 4g + q ; columns col + 4p .. col + 4p + 3
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  const bf16* p0 = lds_base + (4 * g + q) * stride + col + 4 * p;
  const bf16* p1 = lds_base + (16 + 4 * g + q) * stride + col + 4 * p;
  const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p0));
  const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p1));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 r = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
  return __builtin_bit_cast(bf16x8, r);
}

template <int NB, class LoadX>
__global__ __launch_bounds__(256) void k_wgrad(LoadX lx, const bf16* __restrict__ dY, int M, int N, int m_chunk,
                                               float* slab, int slab_ld, size_t slab_zstride, float* bias_slab) {
  constexpr int XS = WgradLds<NB>::XS, YS = WgradLds<NB>::YS;
  constexpr int TN = NB / 16;
  __shared__ __attribute__((aligned(16))) bf16 lds[32 * XS + 32 * YS];
  bf16* xl = lds;
  bf16* yl = lds + 32 * XS;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int k0 = blockIdx.x * 64, n0 = blockIdx.y * NB;
  const int mb = blockIdx.z * m_chunk, me = min(M, mb + m_chunk);
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  f32x4 acc[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) acc[j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
  float bsum = 0.0f;
  const bool do_bias = bias_slab != nullptr && blockIdx.x == 0;
  // cooperative tile loads: X 32 rows x 64 cols = 256 chunks of 8; dY 32 x NB = 4*NB chunks
  const int xr = tid >> 3, xc = (tid & 7) * 8;
  const int yr = NB == 64 ? (tid >> 3) : (tid >> 2), yc = NB == 64 ? (tid & 7) * 8 : (tid & 3) * 8;
  const bool yact = NB == 64 || tid < 128;
  for (int m = mb; m < me; m += 32) {
    const bf16x8 xv = lx.load(m + xr < me ? m + xr : M, k0 + xc);
    bf16x8 yv = zero8();
    if (yact && m + yr < me) yv = ld8(dY + (size_t)(m + yr) * N + n0 + yc);
    __syncthreads();   // previous step's reads are done
    *reinterpret_cast<uint4*>(xl + xr * XS + xc) = __builtin_bit_cast(uint4, xv);
    if (yact) *reinterpret_cast<uint4*>(yl + yr * YS + yc) = __builtin_bit_cast(uint4, yv);
    __syncthreads();
    const bf16x8 af = tr_pair(xl, XS, g, p, q, wave * 16);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const bf16x8 bfr = tr_pair(yl, YS, g, p, q, j * 16);
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr, acc[j], 0, 0, 0);
    }
    if (do_bias && tid < NB) {
#pragma unroll 8
      for (int rr = 0; rr < 32; ++rr) bsum += (float)yl[rr * YS + tid];
    }
  }
  float* out = slab + blockIdx.z * slab_zstride;
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) out[(size_t)(k0 + wave * 16 + g * 4 + e) * slab_ld + n0 + j * 16 + li] = acc[j][e];
  if (do_bias && tid < NB) bias_slab[(size_t)blockIdx.z * N + n0 + tid] = bsum;
}

// Weight gradient v2: block tile KT (k) x NB (n) with KT = 4 waves x KW rows (KW = 16 * KWT); 64 m-rows
// per LDS fill (two MFMA k-slices of 32), the global loads of fill i+1 in flight while fill i computes.
// Row strides are padded by 16 bf16 so the 8 consecutive rows a 32-lane half reads with
// ds_read_b64_tr_b16 land on disjoint 8-dword bank windows (same row permutation as k_wgrad).
template <int KWT, int NB, class LoadX>
__global__ __launch_bounds__(256) void k_wgrad2(LoadX lx, const bf16* __restrict__ dY, int M, int N, int m_chunk,
                                                float* slab, int slab_ld, size_t slab_zstride, float* bias_slab) {
  constexpr int KT = 4 * 16 * KWT;
  constexpr int XS = KT + 16, YS = NB + 16;
  constexpr int TN = NB / 16;
  constexpr int XCH = 64 * KT / 8 / 256;        // 16-byte X chunks per thread per fill
  constexpr int YCH = (64 * NB / 8 + 255) / 256;
  static_assert(XCH >= 1 && (64 * KT / 8) % 256 == 0, "X tile must split evenly over 256 threads");
  __shared__ __attribute__((aligned(16))) bf16 lds[64 * XS + 64 * YS];
  bf16* xl = lds;
  bf16* yl = lds + 64 * XS;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int k0 = blockIdx.x * KT, n0 = blockIdx.y * NB;
  const int mb = blockIdx.z * m_chunk, me = min(M, mb + m_chunk);
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  f32x4 acc[KWT][TN];
#pragma unroll
  for (int i = 0; i < KWT; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
  float bsum = 0.0f;
  const bool do_bias = bias_slab != nullptr && blockIdx.x == 0;
  bf16x8 xv[XCH], yv[YCH];
  auto fetch = [&](int m) {
#pragma unroll
    for (int c = 0; c < XCH; ++c) {
      const int idx = tid + c * 256, row = idx / (KT / 8), col = (idx - row * (KT / 8)) * 8;
      xv[c] = lx.load(m + row < me ? m + row : M, k0 + col);
    }
#pragma unroll
    for (int c = 0; c < YCH; ++c) {
      const int idx = tid + c * 256, row = idx / (NB / 8), col = (idx - row * (NB / 8)) * 8;
      yv[c] = (idx < 64 * NB / 8 && m + row < me) ? ld8(dY + (size_t)(m + row) * N + n0 + col) : zero8();
    }
  };
  fetch(mb);
  for (int m = mb; m < me; m += 64) {
    __syncthreads();   // readers of the previous fill are done
#pragma unroll
    for (int c = 0; c < XCH; ++c) {
      const int idx = tid + c * 256, row = idx / (KT / 8), col = (idx - row * (KT / 8)) * 8;
      *reinterpret_cast<uint4*>(xl + row * XS + col) = __builtin_bit_cast(uint4, xv[c]);
    }
#pragma unroll
    for (int c = 0; c < YCH; ++c) {
      const int idx = tid + c * 256, row = idx / (NB / 8), col = (idx - row * (NB / 8)) * 8;
      if (idx < 64 * NB / 8) *reinterpret_cast<uint4*>(yl + row * YS + col) = __builtin_bit_cast(uint4, yv[c]);
    }
    __syncthreads();
    if (m + 64 < me) fetch(m + 64);
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const bf16* xh = xl + half * 32 * XS;
      const bf16* yh = yl + half * 32 * YS;
      bf16x8 bfr[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = tr_pair(yh, YS, g, p, q, j * 16);
#pragma unroll
      for (int i = 0; i < KWT; ++i) {
        const bf16x8 af = tr_pair(xh, XS, g, p, q, (wave * KWT + i) * 16);
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr[j], acc[i][j], 0, 0, 0);
      }
    }
    if (do_bias && tid < NB) {
#pragma unroll 8
      for (int rr = 0; rr < 64; ++rr) bsum += (float)yl[rr * YS + tid];
    }
  }
  float* out = slab + blockIdx.z * slab_zstride;
#pragma unroll
  for (int i = 0; i < KWT; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        out[(size_t)(k0 + (wave * KWT + i) * 16 + g * 4 + e) * slab_ld + n0 + j * 16 + li] = acc[i][j][e];
  if (do_bias && tid < NB) bias_slab[(size_t)blockIdx.z * N + n0 + tid] = bsum;
}

// out[i] = sum_c slab[c][i] (deterministic): block = 64 outputs x 4 waves; wave w sums chunk quarter w
// (8 loads in flight per lane), the quarters are added in fixed order through LDS.  grid = ceil(count/64)
__global__ __launch_bounds__(256) void k_slab_reduce(const float* slab, size_t zstride, int chunks, size_t count,
                                                     float* out) {
  __shared__ float part[4][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t i = (size_t)blockIdx.x * 64 + lane;
  const int q = (chunks + 3) / 4, c0 = wave * q, c1 = min(chunks, c0 + q);
  float s = 0.0f;
  if (i < count) {
    int c = c0;
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
  if (wave == 0 && i < count) out[i] = ((part[0][lane] + part[1][lane]) + part[2][lane]) + part[3][lane];
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
