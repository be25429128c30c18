// LDS-tiled bf16 GEMM for the dense layer fc1 (3136 <-> 512) on gfx950.
//
//   C[m][n] = sum_k A(m, k) B(n, k), fp32 accumulation with v_mfma_f32_32x32x16_bf16.
//   Operand layouts (per operand): row-major  [rows][ld], k contiguous   (AK / BK = false)
//                                  k-major    [K][ld], rows contiguous  (AK / BK = true)
//   fc1 forward  : A = a3 [B][3136]           B = W3 [3136][512] k-major (the Keras [in][out] layout)
//   fc1 dgrad    : A = dz4 [B][512]           B = W3 [3136][512] row-major (n = in, k = out)
//   fc1 wgrad    : A = a3 [B][3136] k-major   B = dz4 [B][512] k-major (k = batch)
// Block tile 128 x 128 (4 waves as 2 x 2, each 64 x 64 = 2 x 2 MFMA tiles), K stepped by 64 through a
// double-buffered LDS image fed from two register stages (global loads run two k-steps ahead); 80 KB of
// LDS per block, so two blocks share a CU and hide each other's barriers.  Row-major images [128][64 + 8]
// are read with ds_read_b128 (the 8-bf16 pad makes the 32-row fragment reads conflict-free); k-major images [64][128 + 32] with ds_read_b64_tr_b16 (4 k-rows x 64 B
// per 32-lane half land in disjoint bank windows at the 80-dword row stride).  Both deliver k in natural
// order, so the layouts mix freely.  The MFMA computes C^T (B fragment as the A operand): each lane ends
// with 4 consecutive n of one m, so epilogues move 8 (bf16) or 16 (fp32) bytes per access.
// A problem has ceil(M/128) x ceil(N/128) x splits tiles (one block each); split z covers k in
// [z*kps, min(K, (z+1)*kps)).
// Row-major operands need K % 64 == 0 and kps % 64 == 0.
// ones_m >= 0 (a multiple of 8, k-major A only) makes A row ones_m all ones, so C row ones_m = sum_k B(n, k)
// (the bias gradient of a dense layer rides along as one extra output row).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "qnet_kernels.h"

namespace qlx {
namespace qn {

struct GemmCfg {
  static constexpr int BM = 128, BN = 128, KT = 64;
  static constexpr int SR = KT + 8;                 // row-major image row stride (bf16)
  static constexpr int SK = 128 + 32;               // k-major image row stride (bf16)
  static constexpr int IMG = KT * SK;               // >= 128 * SR; one operand image (bf16 elements)
  static constexpr size_t LDS = (size_t)2 * 2 * IMG * 2;
  static constexpr int CH = 128 * KT / 8 / 256;     // 16-byte chunks per thread per operand (4)
};

// Buffer-resource loads: an out-of-range tile element gets an offset past the descriptor's range and reads
// as zero, so the loads are branch-free and the compiler can count them (vmcnt(N) instead of vmcnt(0)) -
// the second register stage stays in flight while the first is stored.
constexpr int kOobOffset = 0x7FFFFFF0;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

template <bool KM>
struct GemmOperand {
  // global 16-byte chunk idx of the tile at (row0, k0) -> registers
  __device__ __forceinline__ static uint4 load(__amdgpu_buffer_rsrc_t r, int ld, int row0, int rows, int k0, int ke, int idx,
                                               int ones) {
    if (!KM) {
      const int row = idx >> 3, col = (idx & 7) * 8;
      const int off = row0 + row < rows ? ((row0 + row) * ld + k0 + col) * 2 : kOobOffset;
      return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
    }
    const int kr = idx >> 4, col = (idx & 15) * 8;
    const bool in = k0 + kr < ke && row0 + col < rows;
    const int off = in ? ((k0 + kr) * ld + row0 + col) * 2 : kOobOffset;
    uint4 v = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
    if (row0 + col == ones && k0 + kr < ke) v = uint4{0x3F80u, 0u, 0u, 0u};   // bf16 1.0 in element 0
    return v;
  }
  __device__ __forceinline__ static void store(bf16* img, int idx, uint4 v) {
    const int row = KM ? idx >> 4 : idx >> 3, col = KM ? (idx & 15) * 8 : (idx & 7) * 8;
    *reinterpret_cast<uint4*>(img + row * (KM ? GemmCfg::SK : GemmCfg::SR) + col) = v;
  }
  // MFMA fragment: 32 rows (base + lane & 31) x 16 k (k16 + 8 (lane >> 5) + j, natural order)
  __device__ __forceinline__ static bf16x8 frag(const bf16* img, int base, int k16, int lane) {
    const int h = lane >> 5;
    if (!KM) return *reinterpret_cast<const bf16x8*>(img + (base + (lane & 31)) * GemmCfg::SR + k16 + 8 * h);
    typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    const int gh = (lane >> 4) & 1, q = (lane & 15) >> 2, p = lane & 3;
    const bf16* p0 = img + (k16 + 8 * h + q) * GemmCfg::SK + base + 16 * gh + 4 * p;
    const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p0));
    const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p0 + 4 * GemmCfg::SK));
    return __builtin_bit_cast(bf16x8, (s16x8){v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]});
  }
};

// Epilogues: operator()(m, n, v, z) for C[m][n .. n+3] = v[0..3] of k split z (n % 4 == 0, n + 3 < N when n < N)
// kSq: the epilogue also yields this tile's sum of squares of the stored values (split by the ones_m row),
// the clip_by_norm partials of a weight gradient written straight to its final place (see gemm_tile)
struct Epi4Slab {   // split-K partial: slab[z][m][n] (fp32)
  static constexpr bool kSq = false;
  float* slab;
  int ldo;
  size_t zstride;
  __device__ __forceinline__ void operator()(int m, int n, f32x4 v, int z) const {
    *reinterpret_cast<f32x4*>(slab + z * zstride + (size_t)m * ldo + n) = v;
  }
};

struct Epi4StoreF32 {   // out[m][n] = v (fp32); sq (optional): [tiles] partials of rows != ones_m, then [tiles] of row ones_m
  static constexpr bool kSq = true;
  float* out;
  int ldo;
  float* sq;
  __device__ __forceinline__ void operator()(int m, int n, f32x4 v, int) const {
    *reinterpret_cast<f32x4*>(out + (size_t)m * ldo + n) = v;
  }
};

// sum of squares of 4 values with explicit roundings: a tile's clip_by_norm partial does not depend on where
// the compiler chooses to contract into FMAs
__device__ __forceinline__ float sq4(f32x4 v) {
  return __fadd_rn(__fadd_rn(__fadd_rn(__fmul_rn(v[0], v[0]), __fmul_rn(v[1], v[1])), __fmul_rn(v[2], v[2])),
                   __fmul_rn(v[3], v[3]));
}

__device__ __forceinline__ uint2 pack4(float a, float b, float c, float d) {
  typedef __bf16 bf16x4v __attribute__((ext_vector_type(4)));
  const bf16x4v v = {(bf16)a, (bf16)b, (bf16)c, (bf16)d};
  return __builtin_bit_cast(uint2, v);
}

struct Epi4BiasRelu {   // out[m][n] = relu(v + bias[n]) as bf16
  static constexpr bool kSq = false;
  bf16* out;
  const float* bias;
  int ldo;
  __device__ __forceinline__ void operator()(int m, int n, f32x4 v, int) const {
    const float4 b = *reinterpret_cast<const float4*>(bias + n);
    auto r = [](float x) { return x > 0.0f ? x : 0.0f; };
    *reinterpret_cast<uint2*>(out + (size_t)m * ldo + n) = pack4(r(v[0] + b.x), r(v[1] + b.y), r(v[2] + b.z), r(v[3] + b.w));
  }
};

struct Epi4ReluMask {   // dz[m][n] = v * (act[m][n] > 0) as bf16 (act rows act_ld apart)
  static constexpr bool kSq = false;
  bf16* out;
  const bf16* act;
  int ldo;
  int act_ld;
  // every field named: a form without act_ld (the old three-field aggregate) does not compile
  __host__ __device__ Epi4ReluMask(bf16* out_, const bf16* act_, int ldo_, int act_ld_) : out(out_), act(act_), ldo(ldo_), act_ld(act_ld_) {}
  __device__ __forceinline__ void operator()(int m, int n, f32x4 v, int) const {
    const size_t i = (size_t)m * ldo + n;
    typedef __bf16 bf16x4v __attribute__((ext_vector_type(4)));
    const bf16x4v a = *reinterpret_cast<const bf16x4v*>(act + (size_t)m * act_ld + n);
    *reinterpret_cast<uint2*>(out + i) = pack4((float)a[0] > 0.0f ? v[0] : 0.0f, (float)a[1] > 0.0f ? v[1] : 0.0f,
                                               (float)a[2] > 0.0f ? v[2] : 0.0f, (float)a[3] > 0.0f ? v[3] : 0.0f);
  }
};

// One problem C[M][N] (+ split z of K); a launch covers ceil(M/128) x ceil(N/128) x splits tiles.  Tile
// order: split slowest, then n-tiles, m fastest - or n fastest (n_fastest) when the tiles of one m-panel
// should share an XCD (the m-panel operand is the big one, e.g. the wgrad's a3).
template <class Epi>
struct GemmProblem {
  const bf16* A;
  int lda;
  const bf16* B;
  int ldb;
  int M, N, K, kps, ones_m;
  int tiles_m, tiles_n, splits;
  int n_fastest;
  int remap;        // XCD-grouped tile order (xcd_tile); grid = xcd_grid(tiles) either way
  Epi epi;
  __host__ __device__ int tiles() const { return tiles_m * tiles_n * splits; }
};

// Blocks b and b + 8 share an XCD (round-robin dispatch, MI355X_MICROARCH.md): block b runs logical tile
// (b % 8) * (grid / 8) + b / 8, so each XCD owns one contiguous range of the tile order and the operand
// panels its tiles share are fetched into its own L2 once.  grid is a multiple of 8.
__device__ __forceinline__ int xcd_tile(int b, int grid) { return (b & 7) * (grid >> 3) + (b >> 3); }
__host__ __forceinline__ int xcd_grid(int tiles) { return (tiles + 7) / 8 * 8; }

// S register stages (S = 2 or 3): the 16-byte global loads of k-step j land in set j % S and are stored to
// LDS S steps of MFMA work later.  Step it computes LDS buffer it % 2, stores set (it + 1) % S (k-step
// it + 1) into the other buffer, then reloads that set with k-step it + 1 + S.
// DBG (development timing only): 1 = no global loads inside the k loop, 2 = no MFMAs
template <bool AK, bool BK, int S, class Epi, int DBG = 0>
__device__ __forceinline__ void gemm_tile(const GemmProblem<Epi>& P, int tile) {
  static_assert(S == 2 || S == 3, "2 or 3 register stages");
  const bf16* __restrict__ A = P.A;
  const bf16* __restrict__ Bm = P.B;
  const int lda = P.lda, ldb = P.ldb, M = P.M, N = P.N, K = P.K, kps = P.kps, ones_m = P.ones_m;
  const Epi& epi = P.epi;
  const int mn = tile % (P.tiles_m * P.tiles_n), bz = tile / (P.tiles_m * P.tiles_n);
  const int bx = P.n_fastest ? mn / P.tiles_n : mn % P.tiles_m;
  const int by = P.n_fastest ? mn % P.tiles_n : mn / P.tiles_m;
  using C = GemmCfg;
  constexpr int KT = C::KT, IMG = C::IMG, CH = C::CH;
  using OA = GemmOperand<AK>;
  using OB = GemmOperand<BK>;
  extern __shared__ __attribute__((aligned(16))) bf16 lds[];
  const int tid = threadIdx.x, wave = wave_id(), lane = tid & 63;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = bx * C::BM, n0 = by * C::BN;
  const int kb = bz * kps, ke = min(K, kb + kps);
  // descriptor ranges: row-major operands [rows][ld], k-major ones [K][ld]
  const __amdgpu_buffer_rsrc_t rA = make_rsrc(A, (uint32_t)((AK ? K : M) * lda * 2));
  const __amdgpu_buffer_rsrc_t rB = make_rsrc(Bm, (uint32_t)((BK ? K : N) * ldb * 2));
  uint4 ra[S][CH], rb[S][CH];
  auto gload = [&](int set, int k0) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      ra[set][c] = OA::load(rA, lda, m0, M, k0, ke, tid + c * 256, ones_m);
      rb[set][c] = OB::load(rB, ldb, n0, N, k0, ke, tid + c * 256, -1);
    }
  };
  auto sstore = [&](int set, int buf) {
    bf16* la = lds + buf * 2 * IMG;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      OA::store(la, tid + c * 256, ra[set][c]);
      OB::store(la + IMG, tid + c * 256, rb[set][c]);
    }
  };
  f32x16 acc[2][2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[t][j][e] = 0.0f;
  const int nk = (ke - kb + KT - 1) / KT;
  // Loads past the split's k range hit real memory or the descriptor's zero range and are never consumed,
  // so every stage is issued unconditionally: with static register sets (the loop is unrolled by the
  // period lcm(2, S)) the body is branch-free and the compiler waits with vmcnt for the oldest set only.
#pragma unroll
  for (int j = 0; j < S; ++j) gload(j, kb + j * KT);
  sstore(0, 0);
  lds_barrier();
  gload(0, kb + S * KT);
  auto step = [&](auto phase, int it) {
    constexpr int buf = decltype(phase)::value % 2, set = (decltype(phase)::value + 1) % S;
    const bf16* la = lds + buf * 2 * IMG;
    const bf16* lb = la + IMG;
#pragma unroll
    for (int ks = 0; ks < KT / 16; ++ks) {
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) af[t] = OA::frag(la, wm * 64 + t * 32, ks * 16, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j) bfr[j] = OB::frag(lb, wn * 64 + j * 32, ks * 16, lane);
      if constexpr (DBG == 2) {
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[t][j][0] += (float)af[t][0] * (float)bfr[j][0];
      } else {
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[t][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bfr[j], af[t], acc[t][j], 0, 0, 0);
      }
    }
    // the other LDS buffer was last read in step it - 1, before the previous barrier
    sstore(set, buf ^ 1);
    lds_barrier();
    if constexpr (DBG != 1) gload(set, kb + (it + 1 + S) * KT);
    // keep the loads here: left alone the scheduler sinks them past the next step's stores (register
    // pressure), which shortens the prefetch distance by a step
    __builtin_amdgcn_sched_barrier(0);
  };
  using P0 = std::integral_constant<int, 0>;
  using P1 = std::integral_constant<int, 1>;
  using P2 = std::integral_constant<int, 2>;
  using P3 = std::integral_constant<int, 3>;
  using P4 = std::integral_constant<int, 4>;
  using P5 = std::integral_constant<int, 5>;
  constexpr int L = S == 2 ? 2 : 6;
  int it = 0;
  for (; it + L <= nk; it += L) {
    step(P0{}, it);
    step(P1{}, it + 1);
    if constexpr (L == 6) {
      step(P2{}, it + 2);
      step(P3{}, it + 3);
      step(P4{}, it + 4);
      step(P5{}, it + 5);
    }
  }
  // tail (< L steps), nested so each phase is reached only after the previous one
  if (it < nk) {
    step(P0{}, it);
    if (it + 1 < nk) {
      step(P1{}, it + 1);
      if constexpr (L == 6) {
        if (it + 2 < nk) {
          step(P2{}, it + 2);
          if (it + 3 < nk) {
            step(P3{}, it + 3);
            if (it + 4 < nk) step(P4{}, it + 4);
          }
        }
      }
    }
  }
  // C^T tile: lane = m (lane & 31), reg e = n offset (e & 3) + 8 (e >> 2) + 4 (lane >> 5)
  const int h = lane >> 5;
  float sq_main = 0.0f, sq_ones = 0.0f;
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int m = m0 + wm * 64 + t * 32 + (lane & 31);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int n = n0 + wn * 64 + j * 32 + 8 * u + 4 * h;
        if (m < M && n < N) {
          const f32x4 v = {acc[t][j][4 * u], acc[t][j][4 * u + 1], acc[t][j][4 * u + 2], acc[t][j][4 * u + 3]};
          epi(m, n, v, bz);
          if constexpr (Epi::kSq) {
            const float q = sq4(v);
            if (m == ones_m) sq_ones = __fadd_rn(sq_ones, q);
            else sq_main = __fadd_rn(sq_main, q);
          }
        }
      }
    }
  if constexpr (Epi::kSq) {
    if (epi.sq) {   // fixed-order block reduction: xor butterfly per wave, then the 4 waves in order
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) {
        sq_main += __shfl_xor(sq_main, off);
        sq_ones += __shfl_xor(sq_ones, off);
      }
      float* red = reinterpret_cast<float*>(lds);   // the k loop ended on a barrier: LDS is free
      if (lane == 0) { red[2 * wave] = sq_main; red[2 * wave + 1] = sq_ones; }
      __syncthreads();
      if (tid == 0) {
        epi.sq[tile] = ((red[0] + red[2]) + red[4]) + red[6];
        epi.sq[P.tiles() + tile] = ((red[1] + red[3]) + red[5]) + red[7];
      }
    }
  }
}

constexpr int kGemmStages = 2;

// single problem; grid = xcd_grid(P.tiles())
template <bool AK, bool BK, class Epi>
__global__ __launch_bounds__(256, 2) void k_gemm(GemmProblem<Epi> P) {
  const int t = P.remap ? xcd_tile(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  if (t < P.tiles()) gemm_tile<AK, BK, kGemmStages>(P, t);
}

// two independent problems in one launch (blocks [0, P1.tiles()) -> P1, the rest -> P2): concurrency without
// cross-stream events, whose dependency latency costs more than a small kernel
template <bool AK1, bool BK1, class E1, bool AK2, bool BK2, class E2>
__device__ __forceinline__ void gemm_pair_block(const GemmProblem<E1>& P1, const GemmProblem<E2>& P2, int t) {
  if (t < P1.tiles()) gemm_tile<AK1, BK1, kGemmStages>(P1, t);
  else if (t < P1.tiles() + P2.tiles()) gemm_tile<AK2, BK2, kGemmStages>(P2, t - P1.tiles());
}

}  // namespace qn
}  // namespace qlx
