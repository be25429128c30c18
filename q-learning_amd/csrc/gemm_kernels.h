// LDS-tiled bf16 GEMM for the dense layer fc1 (3136 <-> 512) on gfx950.
//
//   C[m][n] = sum_k A(m, k) B(n, k), fp32 accumulation with v_mfma_f32_32x32x16_bf16.
//   NT (TN = false): A stored [M][lda] and B stored [N][ldb], k contiguous   (fc1 forward, fc1 dgrad)
//   TN (TN = true) : A stored [K][lda] and B stored [K][ldb], m / n contiguous (fc1 wgrad: k = batch)
// Block tile 128 x 128 (4 waves as 2 x 2, each 64 x 64 = 2 x 2 MFMA tiles), K stepped by 64 through a
// double-buffered LDS image (next step's 16-byte global loads in flight in registers during the MFMAs).
// NT images: [128 rows][64 + 8] (the 8-bf16 pad makes the 32-row ds_read_b128 fragment reads
// conflict-free); TN images: [64 k][128 + 32], read with ds_read_b64_tr_b16 (4 k-rows x 64 B per 32-lane
// half land in disjoint bank windows at the 80-dword row stride).  grid = (ceil(M/128), ceil(N/128),
// splits); blockIdx.z covers k in [z*kps, min(K, (z+1)*kps)).  NT requires K % 64 == 0.
// TN only: ones_m >= 0 (a multiple of 8) makes A row ones_m an all-ones row, so C row ones_m = sum_k B(n, k)
// (the bias gradient of a dense layer rides along as one extra output row).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "qnet_kernels.h"

namespace qlx {
namespace qn {

template <bool TN>
struct GemmCfg {
  static constexpr int BM = 128, BN = 128, KT = 64;
  static constexpr int S = TN ? 128 + 32 : 64 + 8;          // image row stride (bf16)
  static constexpr int IMG = TN ? KT * S : 128 * S;         // one operand image (bf16 elements)
  static constexpr size_t LDS = (size_t)2 * 2 * IMG * 2;    // 2 buffers x (A, B) x bf16
  static constexpr int CH = 128 * KT / 8 / 256;             // 16-byte chunks per thread per operand (4)
};

template <bool TN, class Epi>
__global__ __launch_bounds__(256, 1) void k_gemm(const bf16* __restrict__ A, int lda, const bf16* __restrict__ Bm, int ldb,
                                                 int M, int N, int K, int kps, int ones_m, Epi epi) {
  using C = GemmCfg<TN>;
  constexpr int KT = C::KT, S = C::S, IMG = C::IMG, CH = C::CH;
  extern __shared__ __attribute__((aligned(16))) bf16 lds[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.x * C::BM, n0 = blockIdx.y * C::BN;
  const int kb = blockIdx.z * kps, ke = min(K, kb + kps);
  uint4 ra[CH], rb[CH];
  // chunk idx -> (row, col) of the 128 x 64 (NT) or 64 x 128 (TN) tile
  auto gload = [&](int k0) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int idx = tid + c * 256;
      if (!TN) {
        const int row = idx >> 3, col = (idx & 7) * 8;
        const int m = m0 + row, n = n0 + row;
        ra[c] = m < M ? *reinterpret_cast<const uint4*>(A + (size_t)m * lda + k0 + col) : uint4{0, 0, 0, 0};
        rb[c] = n < N ? *reinterpret_cast<const uint4*>(Bm + (size_t)n * ldb + k0 + col) : uint4{0, 0, 0, 0};
      } else {
        const int row = idx >> 4, col = (idx & 15) * 8;
        const int k = k0 + row;
        ra[c] = uint4{0, 0, 0, 0};
        if (k < ke && m0 + col == ones_m) ra[c].x = 0x3F80u;   // bf16 1.0 in element 0
        else if (k < ke && m0 + col < M) ra[c] = *reinterpret_cast<const uint4*>(A + (size_t)k * lda + m0 + col);
        rb[c] = (k < ke && n0 + col < N) ? *reinterpret_cast<const uint4*>(Bm + (size_t)k * ldb + n0 + col) : uint4{0, 0, 0, 0};
      }
    }
  };
  auto sstore = [&](int buf) {
    bf16* la = lds + buf * 2 * IMG;
    bf16* lb = la + IMG;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int idx = tid + c * 256;
      const int row = TN ? idx >> 4 : idx >> 3, col = TN ? (idx & 15) * 8 : (idx & 7) * 8;
      *reinterpret_cast<uint4*>(la + row * S + col) = ra[c];
      *reinterpret_cast<uint4*>(lb + row * S + col) = rb[c];
    }
  };
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const int h = lane >> 5, r = lane & 31;
  const int gh = (lane >> 4) & 1, li = lane & 15, q = li >> 2, p = li & 3;
  // operand fragment (32 rows/cols x 16 k) at tile offset `base` (m or n) and k offset k16
  auto frag = [&](const bf16* img, int base, int k16) -> bf16x8 {
    if (!TN) return *reinterpret_cast<const bf16x8*>(img + (base + r) * S + k16 + 8 * h);
    const bf16* p0 = img + (k16 + 8 * h + q) * S + base + 16 * gh + 4 * p;
    const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p0));
    const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p0 + 4 * S));
    return __builtin_bit_cast(bf16x8, (s16x8){v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]});
  };
  f32x16 acc[2][2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[t][j][e] = 0.0f;
  const int nk = (ke - kb + KT - 1) / KT;
  if (nk > 0) {
    gload(kb);
    sstore(0);
  }
  __syncthreads();
  for (int it = 0; it < nk; ++it) {
    const int buf = it & 1;
    if (it + 1 < nk) gload(kb + (it + 1) * KT);
    const bf16* la = lds + buf * 2 * IMG;
    const bf16* lb = la + IMG;
#pragma unroll
    for (int ks = 0; ks < KT / 16; ++ks) {
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) af[t] = frag(la, wm * 64 + t * 32, ks * 16);
#pragma unroll
      for (int j = 0; j < 2; ++j) bfr[j] = frag(lb, wn * 64 + j * 32, ks * 16);
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[t][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[t], bfr[j], acc[t][j], 0, 0, 0);
    }
    if (it + 1 < nk) sstore(buf ^ 1);
    __syncthreads();
  }
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int m = m0 + wm * 64 + t * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
        const int n = n0 + wn * 64 + j * 32 + r;
        if (m < M && n < N) epi(m, n, acc[t][j][e]);
      }
}

struct EpiStoreF32 {   // out[m][n] = v (fp32)
  float* out;
  int ldo;
  __device__ __forceinline__ void operator()(int m, int n, float v) const { out[(size_t)m * ldo + n] = v; }
};

}  // namespace qn
}  // namespace qlx
