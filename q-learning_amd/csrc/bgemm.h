// bf16 GEMM core of the bf16 fast path (round 5): the dense layer fc1 (3136 <-> 512) forward, backward data and weight
// gradient (qnet.hip), replacing the register-staged 128 x 128 core of gemm_kernels.h.
//
//   C[m][n] = sum_k A(m, k) B(n, k), fp32 accumulation on v_mfma_f32_16x16x32_bf16 (16 cycles per MFMA per SIMD).
//   Operands in global memory: row-major  [rows][ld], k contiguous   (KM = false)
//                              k-major    [K][ld], rows contiguous  (KM = true)
//   fc1 forward  : A = a3 [B][ld] row-major          B = W3 [3136][512] k-major (the Keras [in][out] layout)
//   fc1 dgrad    : A = dz4 [B][512] row-major        B = W3 [3136][512] row-major (n = in, k = out)
//   fc1 wgrad    : A = a3 [B][ld] k-major (k = b)    B = dz4 [B][512] k-major; a3's pitch ld > 3136 holds a column of
//                  ones at 3136, so output row 3136 is db3 (the bias gradient rides along as one more row of dW3)
//
// Why this shape (MI355X_MICROARCH.md §LDS, cdna_hip_programming.md §5):
// - operands reach LDS by LDS-DMA (`buffer_load_dwordx4 ... lds`, 1 KB per wave instruction): no VGPR staging and no
//   ds_write pass (ds_write_b128 moves ~79 B/clk per CU, which is what bounded the old core's k-steps), and the buffer
//   descriptor's range check turns rows / k-rows past the operand into zeros (ragged M, N and K need no branches);
// - a 3-stage LDS ring, BK = 32: k-step t + 2 is in flight while t is multiplied; one raw s_barrier per k-step and a
//   counted `s_waitcnt vmcnt` (never __syncthreads, whose fence would drain the DMA in flight);
// - MFMA fragments come from LDS conflict-free: row-major images [rows][32] (64-byte rows) read with ds_read_b128 under
//   the chunk XOR swz_r(r) = ((r >> 3) & 1) * 2; k-major images [32][rows] read with two ds_read_b64_tr_b16 per fragment
//   (the transpose on read) under the chunk XOR of k-row kr: s128(kr) = 2 ((kr & 3) | ((kr & 8) >> 1)) for 128-row
//   images, s64(kr) = 2 (((kr >> 1) & 1) | ((kr >> 3) & 1) << 1) for 64-row ones.  The DMA writes each wave
//   instruction's 1 KB linearly, so the permutation is applied on the SOURCE address (each lane fetches the chunk that
//   belongs at its linear LDS slot; the permutation stays inside one row / k-row, so coalescing is unchanged) and the
//   same XOR on the read (cdna_hip_programming.md §5.4 rule 21).  scripts/lds_banks.py checks both layouts;
// - the MFMA computes C^T (B fragment as the A operand), so each lane ends with 4 consecutive n of one m: the epilogues
//   of gemm_kernels.h (Epi4*) move 16 bytes (fp32) or 8 bytes (bf16) per access.
// Requirements (host-checked): row-major operands have K % 32 == 0; every split's k range is a multiple of 32 but the last.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "gemm_kernels.h"
#include "qnet_kernels.h"

namespace qlx {
namespace qn {

struct BOp {
  const bf16* p;
  int ld;     // elements between rows (row-major) or k-rows (k-major)
  int rows;   // valid rows (M for A, N for B)
};

// DBG_ (development timing only, scripts/ubench_bgemm.hip): 1 = no MFMAs, 2 = no DMA in the k loop, 3 = DMA and barriers
// only, 4 = no k loop (prologue DMA + epilogue), 5 = no epilogue stores
// AG_: void, or the im2col geometry of a gathered A operand (ConvGather: A(m, k) = in[im2col row k][column m], k-major)
template <int BM_, int BN_, int WM_, int WN_, bool AK_, bool BKM_, int S_ = 3, int DBG_ = 0, class AG_ = void>
struct BGemmCfg {
  static constexpr int DBG = DBG_;
  using AG = AG_;
  static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_, NW = WM_ * WN_, T = NW * 64;
  static constexpr int BK = 32, S = S_;   // S LDS stages: S - 1 k-steps in flight ahead of the one multiplied
  static constexpr bool AK = AK_, BKM = BKM_;
  static constexpr int TM = BM / WM, TN = BN / WN;   // wave tile
  static constexpr int FM = TM / 16, FN = TN / 16;   // 16 x 16 MFMA tiles per wave
  static constexpr int ABYTES = BM * BK * 2, BBYTES = BN * BK * 2, STAGE = ABYTES + BBYTES;
  static constexpr size_t LDS = (size_t)S * STAGE;
  static constexpr int LA = ABYTES / 1024, LB = BBYTES / 1024;   // 1 KB DMA instructions per stage and operand
  static constexpr int LPA = LA / NW, LPB = LB / NW;              // per wave
  static_assert(LA % NW == 0 && LB % NW == 0, "every wave issues the same DMA count per operand");
  static_assert(TM % 16 == 0 && TN % 16 == 0, "wave tile of whole 16 x 16 MFMA tiles");
  static_assert(!AK || BM == 64 || BM == 128, "k-major images are 64 or 128 rows");
  static_assert(std::is_void<AG_>::value || (AK_ && BM_ == 128), "a gathered A operand is a 128-row k-major image");
  static_assert(!BKM || BN == 64 || BN == 128, "k-major images are 64 or 128 rows");
  static_assert(S >= 2 && S <= 8 && (S - 1) * (LPA + LPB) <= 63, "vmcnt counts to 63");
};

template <class Epi>
struct BGemmProblem {
  BOp A, B;
  int M, N, K, kps;   // kps: k per split (a multiple of 32)
  int ones_m;         // kSq epilogues: the output row whose square sum goes to its own partial (a bias row), or -1
  int tiles_m, tiles_n, splits;
  int n_fastest;      // tile order: n fastest (the tiles of one m-panel adjacent) or m fastest
  Epi epi;
  __host__ __device__ int tiles() const { return tiles_m * tiles_n * splits; }
};

// chunk XOR of row-major (64-byte-row) images and of k-major images by their row count
__device__ __forceinline__ int bswz_r(int r) { return ((r >> 3) & 1) * 2; }
template <int BR>
__device__ __forceinline__ int bswz_k(int kr) {
  if constexpr (BR == 128) return 2 * ((kr & 3) | ((kr & 8) >> 1));
  else return 2 * (((kr >> 1) & 1) | (((kr >> 3) & 1) << 1));
}

typedef __attribute__((address_space(3))) void* lds_vptr;

// One operand's DMA inside a tile.  Instruction j of this wave covers image bytes [1024 (wave + NW j), + 1024).  The
// descriptor of a k-major operand starts at the tile's first k-row and ends at its last (k-rows past the split read zeros,
// so a split's k range need not be a multiple of BK); a row-major one spans the operand (rows past it read zeros).
template <bool KM, int BR, int NW, int LP>
struct BStage {
  uint32_t voff[LP];   // per-lane source byte offsets (k0 = 0); kOobOffset for rows past the operand
  int first;           // this wave's first instruction index
  __amdgpu_buffer_rsrc_t rs;
  uint32_t base, step;   // soffset of k-step t = base + t * step
  __device__ void init(const BOp& o, int row0, int kb, int ke, int wave, int lane) {
    first = wave;
    if constexpr (KM) {
      rs = make_rsrc(o.p + (size_t)kb * o.ld, (uint32_t)((ke - kb) * o.ld * 2));
      base = 0;
      step = (uint32_t)(32 * o.ld * 2);
    } else {
      rs = make_rsrc(o.p, (uint32_t)(o.rows * o.ld * 2));
      base = (uint32_t)(kb * 2);
      step = 64u;
    }
#pragma unroll
    for (int j = 0; j < LP; ++j) {
      const int ii = wave + NW * j;
      if constexpr (!KM) {   // 16 rows of 64 bytes per instruction
        const int r = ii * 16 + (lane >> 2), gc = (lane & 3) ^ bswz_r(r);
        voff[j] = row0 + r < o.rows ? (uint32_t)(((row0 + r) * o.ld + 8 * gc) * 2) : (uint32_t)kOobOffset;
      } else {   // 1024 / (2 BR) k-rows per instruction
        constexpr int CPR = BR / 8;   // 16-byte chunks per k-row
        const int kr = ii * (64 / CPR) + lane / CPR, gc = (lane % CPR) ^ bswz_k<BR>(kr);
        const int row = row0 + 8 * gc;
        voff[j] = row < o.rows ? (uint32_t)((kr * o.ld + row) * 2) : (uint32_t)kOobOffset;
      }
    }
  }
  // issue this wave's DMA of k-step t into the operand image at img (LDS byte address of the image)
  __device__ void issue(int t, char* img) const {
    const uint32_t soff = base + (uint32_t)t * step;
#pragma unroll
    for (int j = 0; j < LP; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_vptr)(img + 1024 * (first + NW * j)), 16, voff[j], soff, 0, 0);
  }
};

// im2col geometry of a conv weight gradient's gathered operand: input in [B][IH][IW][C] (bf16), reduction index
// k = b * P + oh * OW + ow (P = OH * OW output positions per sample), row m = (kh * KS + kw) * C + c (the HWIO row of dW).
// Element offset of (m, k) = kbase(k) + roff(m); 8 consecutive rows (one 16-byte chunk, 8 | C) are contiguous.
template <int IH_, int IW_, int C_, int KS_, int S_, int OH_, int OW_>
struct ConvGather {
  static constexpr int IH = IH_, IW = IW_, C = C_, KS = KS_, S = S_, OH = OH_, OW = OW_, P = OH_ * OW_, M = KS_ * KS_ * C_;
  static_assert(C % 8 == 0, "16-byte chunks of one tap");
  __device__ static uint32_t kbase(int k) {
    const int b = k / P, p = k - b * P, oh = p / OW, ow = p - oh * OW;
    return (uint32_t)(((b * IH + oh * S) * IW + ow * S) * C);
  }
  __device__ static uint32_t roff(int m) {
    const int tap = m / C, c = m - tap * C, kh = tap / KS, kw = tap - kh * KS;
    return (uint32_t)((kh * IW + kw) * C + c);
  }
};

// The gathered (im2col) A operand as a 128-row k-major image: lane chunk -> rows m0 + 8 gc .. + 7 of k-row kr, fetched from
// in + kbase(k) + roff(m).  kbase is evaluated per k-step (a few VALU per DMA instruction); roff is fixed per lane.
template <class G, int NW, int LP>
struct BStageGather {
  uint32_t roff[LP];
  int kr[LP];
  int first, kstart;
  __amdgpu_buffer_rsrc_t rs;
  __device__ void init(const BOp& o, int row0, int kb, int ke, int wave, int lane) {
    first = wave;
    kstart = kb;
    rs = make_rsrc(o.p, (uint32_t)((size_t)o.ld * 2));   // gathered operand: o.ld = elements of the whole input tensor
#pragma unroll
    for (int j = 0; j < LP; ++j) {
      const int ii = wave + NW * j, k = ii * 4 + (lane >> 4), gc = (lane & 15) ^ bswz_k<128>(k);
      const int m = row0 + 8 * gc;
      kr[j] = k;
      roff[j] = m < o.rows ? G::roff(m) : 0xFFFFFFFFu;
    }
  }
  __device__ void issue(int t, char* img) const {
    const int k0 = kstart + 32 * t;
#pragma unroll
    for (int j = 0; j < LP; ++j) {
      const uint32_t v = roff[j] == 0xFFFFFFFFu ? (uint32_t)kOobOffset : (G::kbase(k0 + kr[j]) + roff[j]) * 2u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_vptr)(img + 1024 * (first + NW * j)), 16, v, 0, 0, 0);
    }
  }
};

template <class C, bool IS_A>
struct BStageOf {
  using type = BStage<IS_A ? C::AK : C::BKM, IS_A ? C::BM : C::BN, C::NW, IS_A ? C::LPA : C::LPB>;
};
template <class C>
struct BStageA {
  using type = std::conditional_t<std::is_void<typename C::AG>::value, typename BStageOf<C, true>::type,
                                  BStageGather<std::conditional_t<std::is_void<typename C::AG>::value, ConvGather<1, 1, 8, 1, 1, 1, 1>,
                                                                  typename C::AG>,
                                               C::NW, C::LPA>>;
};

// fragment read addresses (byte offsets inside an operand image) for fragment f of a wave whose rows start at r0
template <bool KM, int BR>
__device__ __forceinline__ int bfrag_off(int r0, int f, int lane) {
  const int rb = r0 + 16 * f;
  if constexpr (!KM) {
    const int r = rb + (lane & 15);
    return r * 64 + 16 * ((lane >> 4) ^ bswz_r(r));
  } else {
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3, kr = 8 * g + q;
    const int c = (rb >> 3) + (p >> 1);
    return kr * (BR * 2) + 16 * (c ^ bswz_k<BR>(kr)) + 8 * (p & 1);
  }
}

// The fragment reads are inline asm: the compiler's wait-count pass makes every LDS read it can see wait for all LDS-DMA in
// flight (s_waitcnt vmcnt(0) before the first ds_read of each k-step - measured in the .s of this core), which would
// drain the ring each step.  The asm reads are invisible to it, so the kernel counts lgkmcnt itself (bfrag_wait) and
// fences the MFMAs behind each wait with a scheduling barrier (cdna_hip_programming.md §5.4 rule 18).
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
template <bool KM>
constexpr int bfrag_insts() { return KM ? 2 : 1; }   // LDS instructions per fragment
// one LDS read at addr + OFF (OFF an immediate; the ds offset field is 16 bits, so 64 KB moves into the address)
template <int OFF>
__device__ __forceinline__ u32x4 ds_b128(uint32_t addr) {
  if constexpr (OFF >= 65536) {
    return ds_b128<OFF - 65536>(addr + 65536u);
  } else {
    u32x4 r;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "n"(OFF));
    return r;
  }
}
template <int OFF>
__device__ __forceinline__ u32x2 ds_tr16(uint32_t addr) {
  if constexpr (OFF >= 65536) {
    return ds_tr16<OFF - 65536>(addr + 65536u);
  } else {
    u32x2 r;
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "n"(OFF));
    return r;
  }
}
// addr: the fragment's lane address inside the operand image (VGPR); OFF: the image's byte offset in LDS (immediate)
template <bool KM, int BR, int OFF>
__device__ __forceinline__ bf16x8 bfrag_read(uint32_t addr) {
  if constexpr (!KM) {
    return __builtin_bit_cast(bf16x8, ds_b128<OFF>(addr));
  } else {
    const u32x2 v0 = ds_tr16<OFF>(addr), v1 = ds_tr16<OFF + 4 * BR * 2>(addr);
    return __builtin_bit_cast(bf16x8, u32x4{v0[0], v0[1], v1[0], v1[1]});
  }
}
template <int N>
__device__ __forceinline__ void bfrag_wait() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
  __builtin_amdgcn_sched_barrier(0);
}

template <int I, int N, class F>
__device__ __forceinline__ void static_for_impl(F& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for_impl<I + 1, N>(f);
  }
}
template <int N, class F>
__device__ __forceinline__ void static_for(F f) { static_for_impl<0, N>(f); }

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// s_waitcnt vmcnt(L * n) for a wave-uniform n in [0, NMAX]
template <int L, int NMAX>
__device__ __forceinline__ void wait_vm_n(int n) {
  if constexpr (NMAX <= 0) {
    wait_vm<0>();
  } else {
    if (n >= NMAX) wait_vm<L * NMAX>();
    else wait_vm_n<L, NMAX - 1>(n);
  }
}

// One output tile (m-panel, n-panel, k split) of problem P; lds = the block's dynamic LDS (C::LDS bytes).
template <class C, class Epi>
__device__ __forceinline__ void bgemm_tile(const BGemmProblem<Epi>& P, int tile, char* lds) {
  const int mn = tile % (P.tiles_m * P.tiles_n), bz = tile / (P.tiles_m * P.tiles_n);
  const int bx = P.n_fastest ? mn / P.tiles_n : mn % P.tiles_m;
  const int by = P.n_fastest ? mn % P.tiles_n : mn / P.tiles_m;
  const int tid = threadIdx.x, wave = wave_id(), lane = tid & 63;
  const int wm = wave / C::WN, wn = wave - wm * C::WN;
  const int m0 = bx * C::BM, n0 = by * C::BN;
  const int kb = bz * P.kps, ke = min(P.K, kb + P.kps);
  const int nk = (ke - kb + C::BK - 1) / C::BK;
  typename BStageA<C>::type sa;
  typename BStageOf<C, false>::type sb;
  sa.init(P.A, m0, kb, ke, wave, lane);
  sb.init(P.B, n0, kb, ke, wave, lane);
  auto issue = [&](int t, int stage) {
    char* st = lds + stage * C::STAGE;
    sa.issue(t, st);
    sb.issue(t, st + C::ABYTES);
  };
  const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)lds;
  uint32_t offA[C::FM], offB[C::FN];
#pragma unroll
  for (int f = 0; f < C::FM; ++f) offA[f] = lds_base + bfrag_off<C::AK, C::BM>(wm * C::TM, f, lane);
#pragma unroll
  for (int f = 0; f < C::FN; ++f) offB[f] = lds_base + bfrag_off<C::BKM, C::BN>(wn * C::TN, f, lane);
  f32x4 acc[C::FM][C::FN];
#pragma unroll
  for (int i = 0; i < C::FM; ++i)
#pragma unroll
    for (int j = 0; j < C::FN; ++j) acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
  constexpr int LPW = C::LPA + C::LPB;
  constexpr int S = C::S;
  static_assert(S >= 3, "the fragment prefetch reads stage t + 1 while stage t + 2 .. t + S - 1 land");
  // Fragments of step t + 1 are read while the MFMAs of step t run (two register sets, fr[t % 2]): the LDS latency hides
  // behind the matrix pipe instead of sitting between the barrier and the MFMAs.
  bf16x8 fa[2][C::FM], fb[2][C::FN];
  auto read_frags = [&](auto stage_c, auto par_c) {
    constexpr int stage = decltype(stage_c)::value, par = decltype(par_c)::value;
#pragma unroll
    for (int f = 0; f < C::FM; ++f) fa[par][f] = bfrag_read<C::AK, C::BM, stage * C::STAGE>(offA[f]);
#pragma unroll
    for (int f = 0; f < C::FN; ++f) fb[par][f] = bfrag_read<C::BKM, C::BN, stage * C::STAGE + C::ABYTES>(offB[f]);
  };
#pragma unroll
  for (int s = 0; s < S - 1; ++s)
    if (s < nk) issue(s, s);
  if (nk > 0) {
    wait_vm_n<LPW, S - 2>(min(S - 2, nk - 1));
    __builtin_amdgcn_s_barrier();
    if constexpr (C::DBG != 3) read_frags(std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{});
  }
  auto step = [&](auto u_c, int t) {
    constexpr int u = decltype(u_c)::value, stage = u % S, par = u % 2;
    // k-step t + 1 has landed (this wave's part; t + 2 .. t + S - 2 may stay in flight), then every wave's part
    // (barrier).  The barrier also retires every wave's reads of stage t - 1 (waited for before the MFMAs of step t - 1),
    // which the DMA of step t + S - 1 overwrites next.
    const bool more = t + 1 < nk;
    if (more) {
      wait_vm_n<LPW, S - 3>(min(S - 3, nk - 2 - t));
      __builtin_amdgcn_s_barrier();
      if (t + S - 1 < nk && C::DBG != 2) issue(t + S - 1, (stage + S - 1) % S);
    }
    if constexpr (C::DBG == 3) return;
    bfrag_wait<0>();   // the fragments of step t (read during step t - 1)
    auto col = [&](auto jc) {
      constexpr int j = decltype(jc)::value;
#pragma unroll
      for (int i = 0; i < C::FM; ++i) {
        if constexpr (C::DBG == 1) acc[i][j][0] += (float)fb[par][j][0] * (float)fa[par][i][0];
        else acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[par][j], fa[par][i], acc[i][j], 0, 0, 0);
      }
      if constexpr (j == 0) {   // the next step's reads go out behind the first column of MFMAs
        if (more) read_frags(std::integral_constant<int, (stage + 1) % S>{}, std::integral_constant<int, par ^ 1>{});
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    static_for<C::FN>(col);
  };
  // the loop unrolled by U (a multiple of S and of 2), so every stage offset and register set is static
  constexpr int U = S % 2 == 0 ? S : 2 * S;
  int t = C::DBG == 4 ? nk : 0;
  if constexpr (C::DBG == 4) wait_vm<0>();
  for (; t + U <= nk; t += U) static_for<U>([&](auto uc) { step(uc, t + decltype(uc)::value); });
  static_for<U - 1>([&](auto uc) {
    if (t + decltype(uc)::value < nk) step(uc, t + decltype(uc)::value);
  });
  // Epilogue through LDS: the C^T fragments (lane & 15 = m, 4 consecutive n at 4 (lane >> 4)) are written to a per-wave
  // [rows][TN + 4] fp32 image and read back along the rows, so each store instruction covers whole row segments
  // (TN / 4 lanes per row: 256-byte fp32 / 128-byte bf16 runs) instead of 16 rows x 64 bytes.  Half the wave's rows at
  // a time (LDS), every DMA landed and every k-loop read retired before the image reuses the ring.
  const Epi& epi = P.epi;
  float sq_main = 0.0f, sq_ones = 0.0f;
  wait_vm<0>();
  bfrag_wait<0>();
  __builtin_amdgcn_s_barrier();
  constexpr int HR = C::TM / 2, PITCH = C::TN + 4, LPR = C::TN / 4, RPI = 64 / LPR;   // rows per half, lanes per row
  static_assert((size_t)C::NW * HR * PITCH * 4 <= C::LDS, "epilogue image fits the ring");
  float* img = reinterpret_cast<float*>(lds) + wave * HR * PITCH;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int i = 0; i < C::FM / 2; ++i)
#pragma unroll
      for (int j = 0; j < C::FN; ++j)
        *reinterpret_cast<f32x4*>(img + (16 * i + (lane & 15)) * PITCH + 16 * j + 4 * (lane >> 4)) = acc[h * (C::FM / 2) + i][j];
    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): this wave's image is written (the wave reads only its own)
#pragma unroll
    for (int it = 0; it < HR / RPI; ++it) {
      const int r = it * RPI + lane / LPR, c = 4 * (lane % LPR);
      const f32x4 v = *reinterpret_cast<const f32x4*>(img + r * PITCH + c);
      const int m = m0 + wm * C::TM + h * HR + r, n = n0 + wn * C::TN + c;
      if constexpr (C::DBG == 5) {
        asm volatile("" ::"v"(v));
        continue;
      }
      if (m < P.M && n < P.N) {
        epi(m, n, v, bz);
        if constexpr (Epi::kSq) {
          const float q = sq4(v);
          if (m == P.ones_m) sq_ones = __fadd_rn(sq_ones, q);
          else sq_main = __fadd_rn(sq_main, q);
        }
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);   // the reads are done before the second half overwrites the image
  }
  if constexpr (Epi::kSq) {
    if (epi.sq) {   // fixed-order block reduction: xor butterfly per wave, then the waves in order
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) {
        sq_main += __shfl_xor(sq_main, off);
        sq_ones += __shfl_xor(sq_ones, off);
      }
      float* red = reinterpret_cast<float*>(lds) + C::NW * HR * PITCH;
      static_assert((size_t)C::NW * HR * PITCH * 4 + 2 * C::NW * 4 <= C::LDS, "sq scratch");
      if (lane == 0) { red[2 * wave] = sq_main; red[2 * wave + 1] = sq_ones; }
      __syncthreads();
      if (tid == 0) {
        float a = red[0], b = red[1];
        for (int w = 1; w < C::NW; ++w) { a += red[2 * w]; b += red[2 * w + 1]; }
        epi.sq[tile] = a;
        epi.sq[P.tiles() + tile] = b;
      }
    }
  }
}

template <class C, class Epi>
__global__ __launch_bounds__(C::T, 2) void k_bgemm(BGemmProblem<Epi> P, int remap) {
  extern __shared__ __attribute__((aligned(16))) char bg_lds[];
  const int t = remap ? xcd_tile(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  if (t < P.tiles()) bgemm_tile<C>(P, t, bg_lds);
}

}  // namespace qn
}  // namespace qlx
