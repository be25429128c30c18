// fp32 Nature-DQN kernels for gfx950: the reference's arithmetic (Keras float32 graph,
// create_ql_model_breakout_84x84x4_3_32.py:20-33,37-61) on v_mfma_f32_16x16x4_f32.
//
// Every GEMM-shaped op is one LDS-tiled implicit-GEMM kernel (gemm_body) driven by a per-layer operand policy.
// v_mfma_f32_16x16x4_f32 is bit-for-bit a k-ordered fmaf chain over its four k (lane group 0 first; measured on
// MI355X, scripts/mfma_f32_probe.hip), and each output element keeps ONE accumulator over the whole reduction,
// consumed in ascending k.  So every output is exactly
//     acc = 0; for k in the layer's order: acc = fmaf(x_k, w_k, acc)
// in the order DESIGN.md §6 defines per layer (and oracle/qnet32_ref.cpp restates): the fp32 Q-net is
// bit-exact against the CPU oracle.  The only reductions split across blocks are the conv weight gradients
// (sample chunks of a fixed size, partials summed in chunk order) and the clip_by_norm sums of squares.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "qlx_internal.h"

namespace qlx {
namespace q32 {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int BK = 32;   // reduction depth staged per LDS slab
// background-row lists (C1Lists): regions per list (one per XCD) and the counter stride (128 bytes)
#ifndef QLX_LIST_SLOTS
#define QLX_LIST_SLOTS 8   // (A/B builds only: scripts/build_variant.sh -DQLX_LIST_SLOTS=n)
#endif
constexpr int kListSlots = QLX_LIST_SLOTS;
constexpr int kCntStride = 16;   // [region][layer] at (region * 2 + layer) * kCntStride

// Operand tile in LDS for MFMA shape MF (16: v_mfma_f32_16x16x4_f32, 32: v_mfma_f32_32x32x2_f32).  RMAJ: t[row][k]
// (pitch BK + 4); KMAJ: t[k][row] (pitch = rows padded to MF mod 64, so the MF rows x (64 / MF) k of a fragment read
// hit distinct banks).  Writes are 16-byte float4 along the operand's contiguous source dimension.
// MF 16: the four lane groups of a fragment read k rows 0..3 of the image, i.e. offsets 0, p, 2p, 3p: any p = 16 or
// 48 mod 64 puts them on four disjoint 16-bank ranges; the smallest such p >= rows (32 rows: 48, not 80, which lets
// one more block per CU fit).  MF 32: two lane groups, p = 32 mod 64.
__host__ __device__ constexpr int kmaj_pitch_min(int rows, int mf) { return rows + (((mf - rows % 64) % 64) + 64) % 64; }
__host__ __device__ constexpr int kmaj_pitch(int rows, int mf) {
  return mf == 16 && rows + ((48 - rows % 64) % 64 + 64) % 64 < kmaj_pitch_min(rows, mf)
             ? rows + ((48 - rows % 64) % 64 + 64) % 64
             : kmaj_pitch_min(rows, mf);
}
static_assert(kmaj_pitch(32, 16) == 48 && kmaj_pitch(64, 16) == 80 && kmaj_pitch(128, 16) == 144 && kmaj_pitch(64, 32) == 96,
              "KMAJ pitches");

// RMAJ images of the 16x16x4 MFMA (P8, round 6): lane l of a fragment read needs (row r0 + l % 16, k = 4 kk + l / 16) at
// k step kk, so over one slab a lane reads k = g, g + 4, .., g + 28 (g = l / 16).  The image stores a row's 32 k at the
// permuted positions P(k) = (k % 4) * 8 + k / 4, which puts those eight k of lane group g side by side (P = 8 g + kk):
// two ds_read_b128 (16-byte chunks 2 g and 2 g + 1) fetch a lane's operands of all eight k steps, in the same k order
// as before - the chains, and so every result, are unchanged.  The chunk index is XORed with row & 1 and the pitch is
// 40 floats: with the ds_read_b128 lane groups of MI355X_MICROARCH.md §LDS every fragment read is conflict-free, and so
// are the stores, which become four ds_write_b32 per float4 of k (positions 8 q + j, q = 0..3, for the float4 j of a row)
// (scripts/p8_layout_search.py checks both).  Before: pitch 36 and one ds_read_b32 per k step and fragment, 2-way
// conflicted (rows i and i + 8 share a bank; a k-pair swap for rows 8..15 that removed it measured slower in round 3).
#ifndef QLX_Q32_P8
#define QLX_Q32_P8 1   // (A/B builds: -DQLX_Q32_P8=0 restores the round-5 pitch-36 image and ds_read_b32 fragments)
#endif
template <int ROWS, bool KMAJ, int MF = 16>
struct Opnd {
  static constexpr bool P8 = QLX_Q32_P8 && !KMAJ && MF == 16;
  static constexpr int PITCH = KMAJ ? kmaj_pitch(ROWS, MF) : P8 ? BK + 8 : BK + 4;
  static constexpr int FLOATS = KMAJ ? BK * PITCH : ROWS * PITCH;
  static constexpr int F4 = ROWS * BK / 4;   // float4 per slab
  static constexpr int KG = 64 / MF;         // k per MFMA (lane groups)
  __host__ __device__ static void coord(int idx, int& row, int& k) {
    if (KMAJ) { k = idx / (ROWS / 4); row = (idx % (ROWS / 4)) * 4; }
    else { row = idx >> 3; k = (idx & 7) * 4; }
  }
  // P8: float offset of (row, k) in the image
  __host__ __device__ static constexpr int p8_off(int row, int k) {
    return row * PITCH + 4 * ((((k & 3) * 8 + (k >> 2)) >> 2) ^ (row & 1)) + ((k >> 2) & 3);
  }
  __device__ static void put(float* t, int row, int k, f32x4 v) {
    if constexpr (P8) {   // k = 4 j: the four k of the float4 go to positions 8 q + j
      const int j = k >> 2, o = row * PITCH + (j & 3), x = row & 1;
#pragma unroll
      for (int q = 0; q < 4; ++q) t[o + 4 * ((2 * q + (j >> 2)) ^ x)] = v[q];
    } else {
      *reinterpret_cast<f32x4*>(t + (KMAJ ? k * PITCH + row : row * PITCH + k)) = v;
    }
  }
  __device__ static float at(const float* t, int row, int k) {
    if constexpr (P8) return t[p8_off(row, k)];
    return KMAJ ? t[k * PITCH + row] : t[row * PITCH + k];
  }
  // MFMA operand of the MF rows from r0, k step kk: lane l holds (r0 + l % MF, KG kk + l / MF)
  __device__ static float frag(const float* t, int r0, int kk, int lane) { return at(t, r0 + (lane & (MF - 1)), KG * kk + lane / MF); }
  // P8: the operands of k steps 4 h .. 4 h + 3 of the slab (element q = k step 4 h + q): one ds_read_b128
  __device__ static f32x4 frag4(const float* t, int r0, int h, int lane) {
    const int row = r0 + (lane & 15);
    return *reinterpret_cast<const f32x4*>(t + row * PITCH + 4 * ((2 * (lane >> 4) + h) ^ (lane & 1)));
  }
};

// One slab's MFMA chains of a wave's TM x TN fragments (k steps in ascending order; P8 operands read four k steps per
// ds_read_b128, the others one ds_read_b32 per k step).  bsum (DB): the B fragments' running column sums (bias chains).
template <class OA, class OB, int TM, int TN, bool DB, class Acc>
__device__ __forceinline__ void slab_mfma16(const float* a, const float* b, int wm, int wn, int lane, Acc (&acc)[TM][TN],
                                            float (&bsum)[TN], bool do_bias = true) {
  constexpr int MF = 16;
#pragma unroll
  for (int h = 0; h < BK / 16; ++h) {
    f32x4 a4[TM], b4[TN];
    if constexpr (OA::P8)
#pragma unroll
      for (int i = 0; i < TM; ++i) a4[i] = OA::frag4(a, (wm * TM + i) * MF, h, lane);
    if constexpr (OB::P8)
#pragma unroll
      for (int j = 0; j < TN; ++j) b4[j] = OB::frag4(b, (wn * TN + j) * MF, h, lane);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int kk = 4 * h + q;
      float af[TM], bf[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        if constexpr (OA::P8) af[i] = a4[i][q];
        else af[i] = OA::frag(a, (wm * TM + i) * MF, kk, lane);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        if constexpr (OB::P8) bf[j] = b4[j][q];
        else bf[j] = OB::frag(b, (wn * TN + j) * MF, kk, lane);
      }
      if constexpr (DB) {
        if (do_bias)
#pragma unroll
          for (int j = 0; j < TN; ++j) bsum[j] = __fadd_rn(bsum[j], bf[j]);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
  }
}

// K-split groups of a policy: its member KSPLIT when it has one, else 1 (gemm_body)
template <class P, class = void>
struct KSplitOf : std::integral_constant<int, 1> {};
template <class P>
struct KSplitOf<P, std::void_t<decltype(P::KSPLIT)>> : std::integral_constant<int, P::KSPLIT> {};
template <class P>
constexpr int threads_of() { return P::WM * P::WN * 64 * KSplitOf<P>::value; }
// K-split chains of a policy run one after another in the same waves: its member KSEQ when it has one, else 1
template <class P, class = void>
struct KSeqOf : std::integral_constant<int, 1> {};
template <class P>
struct KSeqOf<P, std::void_t<decltype(P::KSEQ)>> : std::integral_constant<int, P::KSEQ> {};

// MFMA shape of a policy: its member MF when it has one, else 16
template <class P, class = void>
struct MfOf : std::integral_constant<int, 16> {};
template <class P>
struct MfOf<P, std::void_t<decltype(P::MF)>> : std::integral_constant<int, P::MF> {};

typedef float f32x16 __attribute__((ext_vector_type(16)));
template <int MF>
struct MfAcc { typedef f32x4 type; };
template <>
struct MfAcc<32> { typedef f32x16 type; };

__device__ __forceinline__ f32x4 zero4() { return f32x4{0.0f, 0.0f, 0.0f, 0.0f}; }
__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
// Masked operand load for the policies: masked lanes load 16 zero bytes from q32_zero4, so the load is issued on every
// path and nothing waits on its value before it is stored.  A branch around a load makes the compiler's vmcnt
// bookkeeping path-dependent (it then waits for every outstanding load - including the next slab's - before storing
// the current one), and a select on the loaded value pulls the wait up to the select; either collapses gemm_body's
// two-slabs-in-flight register pipeline.
#ifdef QLX_Q32_POLICIES_ONLY
static const float q32_zero4[4] __attribute__((aligned(16))) = {0.0f, 0.0f, 0.0f, 0.0f};
#else
// (global address space, never written: a const variable would live in the constant space and turn the load into a
// flat load, which also counts on lgkmcnt and so joins every LDS wait)
static __attribute__((device)) float q32_zero4[4] __attribute__((aligned(16))) = {0.0f, 0.0f, 0.0f, 0.0f};
#endif
__device__ __forceinline__ f32x4 ld4m(const float* p, bool ok) { return ld4(ok ? p : q32_zero4); }
// a value the caller knows to be equal on every lane, as a wave-uniform (scalar) value; the identity in the host replay of
// the policies (scripts/q32_host_check.hip, QLX_Q32_POLICIES_ONLY)
__device__ __forceinline__ int q32_uniform(int x) {
#ifdef QLX_Q32_POLICIES_ONLY
  return x;
#else
  return __builtin_amdgcn_readfirstlane(x);
#endif
}
__device__ __forceinline__ f32x4 u8x4(uint32_t w) {
  return f32x4{(float)(w & 0xFFu), (float)((w >> 8) & 0xFFu), (float)((w >> 16) & 0xFFu), (float)(w >> 24)};
}
__device__ __forceinline__ float relu(float v) { return v > 0.0f ? v : 0.0f; }

// workgroup barrier ordering LDS only (keeps register prefetches in flight)
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// XCD-aware block order: hardware block b runs on XCD b % 8; logical blocks [x * G / 8, ...) are all given to XCD x,
// so consecutive logical tiles (neighbouring im2col rows, the tiles of one weight-gradient chunk) share an L2.
__device__ __forceinline__ int xcd_logical(int b, int G) {
  const int x = b & 7, i = b >> 3, q = G >> 3, r = G & 7;
  return x * q + (x < r ? x : r) + i;
}

// Scheduling strategy of a policy's slab loop: IGLP = n >= 0 asks the compiler for its MFMA / LDS interleave strategy n
// (__builtin_amdgcn_iglp_opt), -1 leaves the default scheduler.  Default 1: measured in place at C3 (profiles/r02_v6 README),
// conv2 / conv3 forward 61.5 / 46.1 -> 58.0 / 43.7 us, the fc1 / conv2 backward pairs 73.3 / 117.1 -> 69.5 / 112.9 us,
// the chunk-size conv3 forward 281.5 -> 272 us (strategy 0 for all: 1-4 % slower than 1 on these); the fc1 forward runs
// slower with strategy 1 and best with 0 (PFc1FwdT); the conv1 kernels' MFMA loops gain nothing from either.
#ifndef QLX_IGLP_DEFAULT
#define QLX_IGLP_DEFAULT 1   // (A/B builds: the strategy of the policies without an IGLP member)
#endif
template <class P, class = void>
struct IglpOf : std::integral_constant<int, QLX_IGLP_DEFAULT> {};
template <class P>
struct IglpOf<P, std::void_t<decltype(P::IGLP)>> : std::integral_constant<int, P::IGLP> {};


// LOAD_FENCE = false: no scheduling barrier between a slab's global loads and its MFMAs (the scheduler may sink the
// loads); measured per layer with iglp_opt in place: the fc1 forward 39.8 -> 38.3 us, the chunk-size conv2 forward 404 ->
// 389 us, the conv3 backward pair 98.8 -> 97.7 us without it; every other layer 2-5 % slower without it.  Re-measured on
// the stream core (round 4, gpurun_out/w17: every policy with / without it, iglp 0 / none for all): off for the conv2 pair's
// two policies too; strategy 1 stays the best default (re-measured after the round-5 slab-loop fix: strategy 0 / none for all
// 278K / 281K env-steps/s against 288K).
template <class P, class = void>
struct LoadFenceOf : std::true_type {};
template <class P>
struct LoadFenceOf<P, std::void_t<decltype(P::LOAD_FENCE)>> : std::integral_constant<bool, P::LOAD_FENCE> {};


// Optional per-tile A-operand context: a policy with a member type ACtx provides
//   ACtx a_ctx(int z, int row0, int tid) const                       once per tile, per thread (e.g. the frame pointers of its rows)
//   f32x4 ldA_c(const ACtx&, int i, int z, int s, int row, int k) const    instead of ldA (i = the thread's load index)
// so loop-invariant pointer loads (frame tables) leave the slab loop: one memory latency per slab, not two.
template <class P, class = void>
struct HasACtx : std::false_type {};
template <class P>
struct HasACtx<P, std::void_t<typename P::ACtx>> : std::true_type {};
struct NoCtx {};
template <class P, bool = HasACtx<P>::value>
struct ACtxOf { using type = NoCtx; };
template <class P>
struct ACtxOf<P, true> { using type = typename P::ACtx; };

// Optional early epilogue operands (MF 16 policies): a policy with epi_pre(z, row, col) -> f32x4 (e.g. the ReLU mask
// values of its four rows) and epi_post(z, row, col, acc, pre) has epi_pre's loads issued before the slab loop, so the
// epilogue waits on nothing (a load issued after the loop would wait behind every slab load still in flight).
template <class P, class = void>
struct HasEpiPre : std::false_type {};
template <class P>
struct HasEpiPre<P, std::void_t<decltype(std::declval<const P&>().epi_pre(0, 0, 0))>> : std::true_type {};
// the type epi_pre returns (f32x4 unless the policy says otherwise)
template <class P, bool = HasEpiPre<P>::value>
struct PreOf { using type = f32x4; };
template <class P>
struct PreOf<P, true> { using type = decltype(std::declval<const P&>().epi_pre(0, 0, 0)); };

// Optional tile filter: a policy with active(z, row0) skips the tiles it returns false for (rows counted on the device)
template <class P, class = void>
struct HasActive : std::false_type {};
template <class P>
struct HasActive<P, std::void_t<decltype(std::declval<const P&>().active(0, 0))>> : std::true_type {};

// One output tile of a policy P (see the policies below for the members it provides):
//   acc[row][col] = sum over the slabs s = 0 .. nslabs(z) - 1 and k = 0 .. 31 of A(z, s, row, k) * B(z, s, col, k),
// one fmaf chain per output in (s, k) order; then P::epi stores it.  With P::BIAS the tiles of row-tile 0 also
// sum B's columns (bias gradient): four chains over the reduction index mod 4, combined ((C0 + C1) + C2) + C3.
// With P::KSPLIT = G > 1 the block runs G wave groups, group g chaining the slabs [g ns / G, (g + 1) ns / G) into its
// own accumulators (own LDS buffers, the same barriers); the tile is then ((C0 + C1) + ..) + C(G-1), summed by group 0
// through LDS before its epilogue (ns must be a multiple of G).
template <class P>
__device__ __forceinline__ void gemm_body(const P& p, int lb, float* lds) {
  constexpr int MF = MfOf<P>::value;
  using OA = Opnd<P::BM, P::A_KMAJ, MF>;
  using OB = Opnd<P::BN, P::B_KMAJ, MF>;
  using Acc = typename MfAcc<MF>::type;
  constexpr int G = KSplitOf<P>::value;
  static_assert(G == 1 || !P::BIAS, "K-split groups: no bias chains");
  constexpr int T = P::WM * P::WN * 64;   // threads of one K group
  constexpr int TM = P::BM / (P::WM * MF), TN = P::BN / (P::WN * MF);
  static_assert(TM >= 1 && TN >= 1 && TM * P::WM * MF == P::BM && TN * P::WN * MF == P::BN, "tile shape");
  constexpr int NA = (OA::F4 + T - 1) / T, NB = (OB::F4 + T - 1) / T;
  constexpr int GROUP_LDS = 2 * (OA::FLOATS + OB::FLOATS);
  static_assert(G == 1 || TM * TN * (MF * MF / 64) * T <= GROUP_LDS, "K-split hand-off fits the group's LDS");
  const int kg = G > 1 ? __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6) / (P::WM * P::WN)) : 0;
  const int tid = threadIdx.x - kg * T, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % P::WM, wn = wave / P::WM;
  int tm, tn, z;
  p.decode(lb, tm, tn, z);
  const int row0 = tm * P::BM, col0 = tn * P::BN;
  if constexpr (HasActive<P>::value) {
    if (!p.active(z, row0)) return;
  }
  const int ns = p.nslabs(z) / G, s_base = kg * ns;   // this group's slabs: s_base + [0, ns)
  constexpr int Q = KSeqOf<P>::value;   // (KSEQ: see gemm_body_s)
  static_assert(Q == 1 || (Q == 2 && G == 1 && MF == 16 && !P::BIAS), "sequential K split: two chains, 16x16x4, no bias");
  const int s_half = Q > 1 ? ns / 2 : -1;
  typename ACtxOf<P>::type actx{};
  if constexpr (HasACtx<P>::value) actx = p.a_ctx(z, row0, tid);
  lds += kg * GROUP_LDS;
  float* As0 = lds;
  float* As1 = lds + OA::FLOATS;
  float* Bs0 = lds + 2 * OA::FLOATS;
  float* Bs1 = Bs0 + OB::FLOATS;
  // two register sets: slab s + 2 is in flight from global memory while slab s is multiplied from LDS and slab
  // s + 1 waits in registers for its LDS buffer (two slabs of MFMA work cover a load's latency)
  f32x4 ra0[NA], rb0[NB], ra1[NA], rb1[NB];
  auto load = [&](int s, f32x4(&ra)[NA], f32x4(&rb)[NB]) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int idx = tid + i * T;
      if (OA::F4 % T == 0 || idx < OA::F4) {
        int r, k;
        OA::coord(idx, r, k);
        if constexpr (HasACtx<P>::value) ra[i] = p.ldA_c(actx, i, z, s_base + s, row0 + r, k);
        else ra[i] = p.ldA(z, s_base + s, row0 + r, k);
      }
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int idx = tid + i * T;
      if (OB::F4 % T == 0 || idx < OB::F4) {
        int r, k;
        OB::coord(idx, r, k);
        rb[i] = p.ldB(z, s_base + s, col0 + r, k);
      }
    }
  };
  auto store = [&](int s, const f32x4(&ra)[NA], const f32x4(&rb)[NB]) {
    float* as = (s & 1) ? As1 : As0;
    float* bs = (s & 1) ? Bs1 : Bs0;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int idx = tid + i * T;
      if (OA::F4 % T == 0 || idx < OA::F4) {
        int r, k;
        OA::coord(idx, r, k);
        OA::put(as, r, k, ra[i]);
      }
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int idx = tid + i * T;
      if (OB::F4 % T == 0 || idx < OB::F4) {
        int r, k;
        OB::coord(idx, r, k);
        OB::put(bs, r, k, rb[i]);
      }
    }
  };
  Acc acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < MF * MF / 64; ++e) acc[i][j][e] = 0.0f;
  Acc first[Q > 1 ? TM : 1][Q > 1 ? TN : 1];   // KSEQ: the finished first chain
  // bias (BIAS policies, row-tile 0): column sums of B as KG interleaved chains - lane group q of the wave's B fragments
  // chains the k = q mod KG rows - combined in group order at the end
  float bsum[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) bsum[j] = 0.0f;
  const bool do_bias = P::BIAS && tm == 0 && wm == 0;
  auto compute = [&](int s) {
    const float* a = (s & 1) ? As1 : As0;
    const float* b = (s & 1) ? Bs1 : Bs0;
    if constexpr (Q > 1) {
      if (s == s_half) {   // (wave-uniform) the first chain is done: keep it, start the second from zero
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            first[i][j] = acc[i][j];
            acc[i][j] = zero4();
          }
      }
    }
    if constexpr (IglpOf<P>::value >= 0) __builtin_amdgcn_iglp_opt(IglpOf<P>::value);
    if constexpr (MF == 16) {
      slab_mfma16<OA, OB, TM, TN, P::BIAS>(a, b, wm, wn, lane, acc, bsum, do_bias);
    } else {
#pragma unroll
      for (int kk = 0; kk < BK / OA::KG; ++kk) {
        float af[TM], bf[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) af[i] = OA::frag(a, (wm * TM + i) * MF, kk, lane);
#pragma unroll
        for (int j = 0; j < TN; ++j) bf[j] = OB::frag(b, (wn * TN + j) * MF, kk, lane);
        if (P::BIAS && do_bias)
#pragma unroll
          for (int j = 0; j < TN; ++j) bsum[j] = __fadd_rn(bsum[j], bf[j]);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i], bf[j], acc[i][j], 0, 0, 0);
      }
    }
  };
  // iteration s: x holds slab s + 1, y is free.  Every iteration issues its loads unconditionally (the last slab again
  // past the end), so the number of loads in flight is the same on every path and the store of slab s + 1 waits only
  // for slab s + 1's loads (vmcnt = this iteration's NA + NB), never for slab s + 2's (see ld4m)
  auto iter = [&](int s, f32x4(&xa)[NA], f32x4(&xb)[NB], f32x4(&ya)[NA], f32x4(&yb)[NB]) {
    load(s + 2 < ns ? s + 2 : ns - 1, ya, yb);
    if constexpr (LoadFenceOf<P>::value) __builtin_amdgcn_sched_barrier(0);   // the loads stay ahead of the slab's MFMAs
    compute(s);
    store(s + 1, xa, xb);   // unconditional, as in gemm_body_s (past the last slab: the idle buffer, never read)
    lds_barrier();
  };
  constexpr bool PRE = HasEpiPre<P>::value && MF == 16;
  typename PreOf<P>::type pre[TM][TN];
  if constexpr (PRE) {
    if (kg == 0) {   // (K groups: group 0 runs the epilogue)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          pre[i][j] = p.epi_pre(z, row0 + (wm * TM + i) * 16 + (lane >> 4) * 4, col0 + (wn * TN + j) * 16 + (lane & 15));
    }
  }
  if (ns > 0) {
    load(0, ra1, rb1);
    store(0, ra1, rb1);
    load(ns > 1 ? 1 : 0, ra0, rb0);
    lds_barrier();
    int s = 0;
    for (; s + 1 < ns; s += 2) {
      iter(s, ra0, rb0, ra1, rb1);
      iter(s + 1, ra1, rb1, ra0, rb0);
    }
    if (s < ns) iter(s, ra0, rb0, ra1, rb1);
  }
  if constexpr (Q > 1) {   // C0 + C1
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[i][j][e] = __fadd_rn(ns > s_half ? first[i][j][e] : acc[i][j][e], ns > s_half ? acc[i][j][e] : 0.0f);
  }
  if constexpr (G > 1) {   // groups 1 .. G - 1 hand their accumulators to group 0 through their own LDS (free now)
    constexpr int E = MF * MF / 64;
    if (kg > 0) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int e = 0; e < E; ++e) lds[((i * TN + j) * E + e) * T + tid] = acc[i][j][e];
    }
    __syncthreads();
    if (kg > 0) return;
#pragma unroll
    for (int g = 1; g < G; ++g)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int e = 0; e < E; ++e) acc[i][j][e] = __fadd_rn(acc[i][j][e], lds[g * GROUP_LDS + ((i * TN + j) * E + e) * T + tid]);
  }
  // accumulator layout: MF 16: lane l holds rows 4 (l / 16) .. + 3 of column l % 16; MF 32: element 4 q + e is row
  // 8 q + 4 (l / 32) + e of column l % 32
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      if constexpr (PRE) {
        p.epi_post(z, row0 + (wm * TM + i) * 16 + (lane >> 4) * 4, col0 + (wn * TN + j) * 16 + (lane & 15), acc[i][j], pre[i][j]);
      } else if constexpr (MF == 16) {
        p.epi(z, row0 + (wm * TM + i) * 16 + (lane >> 4) * 4, col0 + (wn * TN + j) * 16 + (lane & 15), acc[i][j]);
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q)
          p.epi(z, row0 + (wm * TM + i) * 32 + 8 * q + 4 * (lane >> 5), col0 + (wn * TN + j) * 32 + (lane & 31),
                f32x4{acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]});
      }
    }
  if constexpr (P::BIAS) {
    if (do_bias) {
      static_assert(MF == 16, "bias chains: 16x16x4 fragments");
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const float c1 = __shfl(bsum[j], lane + 16), c2 = __shfl(bsum[j], lane + 32), c3 = __shfl(bsum[j], lane + 48);
        if (lane < 16) p.epi_bias(z, col0 + (wn * TN + j) * 16 + lane, __fadd_rn(__fadd_rn(__fadd_rn(bsum[j], c1), c2), c3));
      }
    }
  }
}

// Chained sub-tiles: one block runs the tiles (tm, tn, z_0), (tm, tn, z_1), .. of its group zg = the z grid index
// (P::sub_count(zg) <= P::NSUB sub-tiles, z_i = P::sub_z(zg, i)) as ONE slab pipeline over the concatenated slabs: the
// loads of a sub-tile's first slabs are in flight while the previous sub-tile's last slabs are multiplied, and at a
// sub-tile's last slab its accumulators go through P::epi and restart from zero.  Each output is still one chain over its
// own tile's slabs in order, so the results equal gemm_body's on the same tiles bit for bit.  For short-K tiles (pixel-major
// backward data: 1..9 valid taps) this removes the per-tile pipeline ramp and epilogue wait that dominate a short tile.
// The sub-tile queue is kept as shifting scalars (no runtime-indexed arrays or captured references: those end up in
// scratch memory): a load cursor and an epilogue cursor each advance through (z_i, end slab e_i) in order.
// (gemm_body_chain) the streams type of a policy, or an empty placeholder
template <class P, class = void>
struct HasStreamsC : std::false_type {};
#ifndef QLX_Q32_NO_STREAMS
template <class P>
struct HasStreamsC<P, std::void_t<typename P::Streams>> : std::bool_constant<!std::is_void_v<typename P::Streams>> {};
#endif
struct NoStreams { struct Regs {}; };
template <class P, bool = HasStreamsC<P>::value>
struct StreamsOf { using type = NoStreams; };
template <class P>
struct StreamsOf<P, true> { using type = typename P::Streams; };
template <class P>
struct StreamsRegsOf { using type = typename StreamsOf<P>::type::Regs; };

struct ChainQ {
  int z0, e0, z1, e1, z2, e2, z3, e3;
  __device__ __forceinline__ void pop() { z0 = z1; e0 = e1; z1 = z2; e1 = e2; z2 = z3; e2 = e3; }
};
template <class P>
__device__ __forceinline__ void gemm_body_chain(const P& p, int lb, float* lds) {
  constexpr int MF = 16;
  using OA = Opnd<P::BM, P::A_KMAJ, MF>;
  using OB = Opnd<P::BN, P::B_KMAJ, MF>;
  static_assert(KSplitOf<P>::value == 1 && !P::BIAS && !HasACtx<P>::value, "chained tiles: plain policies");
  static_assert(P::NSUB == 4, "chained tiles: up to four sub-tiles");
  constexpr int T = P::WM * P::WN * 64;
  constexpr int TM = P::BM / (P::WM * MF), TN = P::BN / (P::WN * MF);
  static_assert(TM >= 1 && TN >= 1 && TM * P::WM * MF == P::BM && TN * P::WN * MF == P::BN, "tile shape");
  constexpr int NA = (OA::F4 + T - 1) / T, NB = (OB::F4 + T - 1) / T;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % P::WM, wn = wave / P::WM;
  int tm, tn, zg;
  p.decode(lb, tm, tn, zg);
  const int row0 = tm * P::BM, col0 = tn * P::BN;
  const int nsub = p.sub_count(zg);
  ChainQ q;
  q.z0 = p.sub_z(zg, 0);
  q.z1 = nsub > 1 ? p.sub_z(zg, 1) : q.z0;
  q.z2 = nsub > 2 ? p.sub_z(zg, 2) : q.z0;
  q.z3 = nsub > 3 ? p.sub_z(zg, 3) : q.z0;
  q.e0 = p.nslabs(q.z0);
  q.e1 = q.e0 + (nsub > 1 ? p.nslabs(q.z1) : 0);
  q.e2 = q.e1 + (nsub > 2 ? p.nslabs(q.z2) : 0);
  q.e3 = q.e2 + (nsub > 3 ? p.nslabs(q.z3) : 0);
  const int ns = q.e3;
  ChainQ lq = q, fq = q;   // load cursor, epilogue cursor
  int lbase = 0;           // first slab of lq's current sub-tile
  float* As0 = lds;
  float* As1 = lds + OA::FLOATS;
  float* Bs0 = lds + 2 * OA::FLOATS;
  float* Bs1 = Bs0 + OB::FLOATS;
  // slab staging: the policy's streams (lane offsets per block; a sub-tile's slab offsets on the scalar unit) or ldA / ldB
  constexpr bool STR = HasStreamsC<P>::value;
  using St = typename StreamsOf<P>::type;
  St st{};
  if constexpr (STR) st = p.streams(0, row0, col0, tid);
  struct RegsL { f32x4 a[NA], b[NB]; };
  using Regs = std::conditional_t<STR, typename StreamsRegsOf<P>::type, RegsL>;
  Regs x0, x1;
  // slab s of the concatenation (s never decreases between calls; past the end the last slab again)
  auto load = [&](int s, Regs& x) {
    if (s >= lq.e0 && s < ns) {
      lbase = lq.e0;
      lq.pop();
    }
    const int z = lq.z0, sl = s - lbase;
    if constexpr (STR) {
      st.load_z(z, sl, x);
    } else {
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int idx = tid + i * T;
        if (OA::F4 % T == 0 || idx < OA::F4) {
          int r, k;
          OA::coord(idx, r, k);
          x.a[i] = p.ldA(z, sl, row0 + r, k);
        }
      }
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int idx = tid + i * T;
        if (OB::F4 % T == 0 || idx < OB::F4) {
          int r, k;
          OB::coord(idx, r, k);
          x.b[i] = p.ldB(z, sl, col0 + r, k);
        }
      }
    }
  };
  auto store = [&](int s, const Regs& x) {
    float* as = (s & 1) ? As1 : As0;
    float* bs = (s & 1) ? Bs1 : Bs0;
    if constexpr (STR) {
      st.store(as, bs, x);
    } else {
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int idx = tid + i * T;
        if (OA::F4 % T == 0 || idx < OA::F4) {
          int r, k;
          OA::coord(idx, r, k);
          OA::put(as, r, k, x.a[i]);
        }
      }
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int idx = tid + i * T;
        if (OB::F4 % T == 0 || idx < OB::F4) {
          int r, k;
          OB::coord(idx, r, k);
          OB::put(bs, r, k, x.b[i]);
        }
      }
    }
  };
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = zero4();
  auto compute = [&](int s) {
    const float* a = (s & 1) ? As1 : As0;
    const float* b = (s & 1) ? Bs1 : Bs0;
    if constexpr (IglpOf<P>::value >= 0) __builtin_amdgcn_iglp_opt(IglpOf<P>::value);
    float nobias[TN];
    slab_mfma16<OA, OB, TM, TN, false>(a, b, wm, wn, lane, acc, nobias);
  };
  constexpr bool PRE = HasEpiPre<P>::value;
  f32x4 pre[TM][TN];
  auto fetch_pre = [&](int z) {
    if constexpr (PRE) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          pre[i][j] = p.epi_pre(z, row0 + (wm * TM + i) * 16 + (lane >> 4) * 4, col0 + (wn * TN + j) * 16 + (lane & 15));
    }
  };
  // after slab s: the epilogue of a sub-tile ending there, fresh accumulators (and the next sub-tile's early operands)
  auto flush = [&](int s) {
    if (s + 1 != fq.e0) return;
    const int z = fq.z0;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = row0 + (wm * TM + i) * 16 + (lane >> 4) * 4, col = col0 + (wn * TN + j) * 16 + (lane & 15);
        if constexpr (PRE) p.epi_post(z, row, col, acc[i][j], pre[i][j]);
        else p.epi(z, row, col, acc[i][j]);
        acc[i][j] = zero4();
      }
    fq.pop();
    if (s + 1 < ns) fetch_pre(fq.z0);
  };
  auto iter = [&](int s, Regs& xs, Regs& ys) {
    load(s + 2 < ns ? s + 2 : ns - 1, ys);
    if constexpr (LoadFenceOf<P>::value) __builtin_amdgcn_sched_barrier(0);
    compute(s);
    flush(s);
    if (s + 1 < ns) store(s + 1, xs);
    lds_barrier();
  };
  fetch_pre(q.z0);
  if (ns > 0) {
    load(0, x1);
    store(0, x1);
    load(ns > 1 ? 1 : 0, x0);
    lds_barrier();
    for (int s = 0; s < ns; s += 2) {
      iter(s, x0, x1);
      if (s + 1 < ns) iter(s + 1, x1, x0);
    }
  }
}

// a policy with RAW_ORDER = true takes its blocks in hardware order (no XCD grouping)
template <class P, class = void>
struct RawOrder : std::false_type {};
template <class P>
struct RawOrder<P, std::void_t<decltype(P::RAW_ORDER)>> : std::integral_constant<bool, P::RAW_ORDER> {};
template <class P>
__device__ __forceinline__ int block_order(int h, int G) { return RawOrder<P>::value ? h : xcd_logical(h, G); }



// grid layout shared by the policies: tile index fastest (col tile, then row tile), then z
struct Grid {
  int tiles_m, tiles_n, nz;
  __host__ __device__ void decode(int lb, int& tm, int& tn, int& z) const {
    tn = lb % tiles_n;
    const int q = lb / tiles_n;
    tm = q % tiles_m;
    z = q / tiles_m;
  }
  __host__ __device__ int blocks() const { return tiles_m * tiles_n * nz; }
};

// ---------------------------------------------------------------------------------------------------------------
// Operand streams: slab staging with no per-slab vector address arithmetic.
//
// On gfx950 the fp32 MFMA and the VALU do not overlap: an MFMA loop and a VALU loop on one SIMD take the sum of their
// times (scripts/coexec_probe.hip), so every vector instruction of a slab loop is MFMA time lost.  The ldA / ldB form of
// the policies recomputes each load's 64-bit address per slab (divisions, masks, selects: 40 to 100 VALU instructions per
// slab of 32 MFMAs).  A stream computes its per-lane byte offsets once per tile; per slab it adds a wave-uniform offset
// (SALU) and issues raw buffer loads, whose range check returns zeros for a lane offset past the buffer (rows past the
// batch) or for a whole-slab descriptor of zero records (gather rows past a chunk).
//   load(s, regs)  - issue the slab's loads (s wave-uniform)
//   store(t, regs) - write them into the operand's LDS image t (the Opnd layout the fragment reads use)
constexpr uint32_t kOob = 0x80000000u;   // lane offset past any buffer: the load returns zeros

__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, uint32_t bytes) {
  // descriptor words from provably wave-uniform inputs (otherwise each load is wrapped in a waterfall loop)
  const uint64_t a = (uint64_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0,
                                           (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
__device__ __forceinline__ f32x4 buf_ld4(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}
__device__ __forceinline__ float buf_ld1(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
}

// Affine stream over an Opnd<ROWS, KMAJ> image: element (row, k) of slab s at lane_off(row, k) + slab_off(s) bytes.
// RMAJ: k runs along memory (16-byte chunks of 4 k), KMAJ: rows run along memory (chunks of 4 rows).  KMASK: lanes whose
// k is at or past the slab's valid count read zeros (a partial last slab of a reduction along k).
template <int ROWS, bool KMAJ, int T, bool KMASK = false>
struct AffineStream {
  using O = Opnd<ROWS, KMAJ, 16>;
  static constexpr int N = (O::F4 + T - 1) / T;
  using Regs = f32x4[N];
  __amdgpu_buffer_rsrc_t rs;
  uint32_t vo[N];
  int kk[N];        // (KMASK) the lane's k of each load
  int tid;
  template <class F>
  __device__ void init(const void* base, uint32_t bytes, int tid_, F lane_off) {
    rs = buf_rsrc(base, bytes);
    tid = tid_;
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int idx = tid + i * T;
      int r = 0, k = 0;
      if (O::F4 % T == 0 || idx < O::F4) O::coord(idx, r, k);
      vo[i] = lane_off(r, k);
      kk[i] = k;
    }
  }
  // slab s at byte offset soff (wave-uniform); kvalid: k < kvalid are live (KMASK)
  __device__ void load(uint32_t soff, int kvalid, Regs& rg) const {
    if (!KMASK || kvalid >= BK) {   // (wave-uniform: the masked form only in a partial last slab)
#pragma unroll
      for (int i = 0; i < N; ++i)
        if (O::F4 % T == 0 || tid + i * T < O::F4) rg[i] = buf_ld4(rs, vo[i], soff);
    } else {
#pragma unroll
      for (int i = 0; i < N; ++i)
        if (O::F4 % T == 0 || tid + i * T < O::F4) rg[i] = buf_ld4(rs, kk[i] < kvalid ? vo[i] : kOob, soff);
    }
  }
  __device__ void store(float* t, const Regs& rg) const {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int idx = tid + i * T;
      if (O::F4 % T == 0 || idx < O::F4) {
        int r, k;
        O::coord(idx, r, k);
        O::put(t, r, k, rg[i]);
      }
    }
  }
};

// Two affine streams (A, B) whose slab offsets are s * the policies' per-slab strides
template <class SA, class SB, uint32_t DA, uint32_t DB, bool KMASK = false>
struct PairStreams {
  SA a;
  SB b;
  int kmax;   // (KMASK) the reduction length: slab s has kmax - s * BK live k
  struct Regs {
    typename SA::Regs a;
    typename SB::Regs b;
  };
  __device__ void load(int s, Regs& x) const {
    const int kv = kmax - s * BK;
    a.load((uint32_t)s * DA, kv, x.a);
    b.load((uint32_t)s * DB, kv, x.b);
  }
  __device__ void store(float* as, float* bs, const Regs& x) const {
    a.store(as, x.a);
    b.store(bs, x.b);
  }
};

// Gather stream for a KMAJ image whose reduction index k is not affine in memory (the conv weight gradient's im2col
// operand: k = (b, oh, ow)): a per-tile table in LDS holds each k's byte offset (kOob past the valid count), written once
// by the block before its slab loop (prepare); per slab a thread reads its two k's offsets (two broadcast ds_read_b32)
// and adds its row offset - no per-slab division or scalar offset arithmetic.  A thread stages 4 consecutive rows (a float4)
// of one k; the 64 lanes of a wave instruction cover 4 consecutive k (16 lanes each): wave w stages k = 4 w + g and
// 16 + 4 w + g.  (Measured slower and removed: the same offsets generated per slab on the scalar unit, 4 per wave load.)
// (SHIFT / MASK / MUL: an entry packs more than one offset - the lane's byte offset is ((entry >> SHIFT) & MASK) * MUL;
// kOob must stay past the buffer's end under that map)
template <int T, bool PADS = true, int SHIFT = 0, uint32_t MASK = 0xFFFFFFFFu, uint32_t MUL = 1u>
struct TableK4Stream {
  static_assert(T == 256, "table gather stream: four waves");
  using O = Opnd<64, true, 16>;
  static constexpr int N = 2;   // float4 loads per thread per slab
  using Regs = f32x4[N];
  __amdgpu_buffer_rsrc_t rs;
  uint32_t vo;   // the lane's row-group offset
  int tid, g, k0;
  const uint32_t* tbl;   // LDS: byte offset of each k of the tile's reduction (kOob past its end), in the operand images' pads
  // entry r of the table: 16-entry segment r / 16 in the pad columns 64 .. 79 of k-row (r / 16) % 32 of image r / 512 (the
  // four 64-row KMAJ images - A and B, two buffers each - are contiguous, 2,560 floats each; no fragment read or slab store
  // touches a pad), so the table costs no LDS and the launch keeps four blocks per CU
  static constexpr int IMG = Opnd<64, true, 16>::FLOATS, PITCH = Opnd<64, true, 16>::PITCH;
  static_assert(PITCH == 80, "table stream: 16 pad columns per k-row");
  // (PADS = false: the table follows the four images, entry r at 4 IMG + r - the launch then needs EXTRA_LDS)
  __host__ __device__ static int slot(int r) { return PADS ? (r >> 9) * IMG + ((r >> 4) & 31) * PITCH + 64 + (r & 15) : 4 * IMG + r; }
  __device__ void init(const void* base, uint32_t bytes, int tid_, uint32_t row_off) {
    rs = buf_rsrc(base, bytes);
    tid = tid_;
    g = (tid & 63) >> 4;
    k0 = __builtin_amdgcn_readfirstlane(tid >> 6) * 4;
    vo = row_off;
  }
  __device__ void load(int kbase, Regs& rg) const {
#pragma unroll
    for (int i = 0; i < N; ++i) rg[i] = buf_ld4(rs, vo + ((tbl[slot(kbase + k0 + 16 * i + g)] >> SHIFT) & MASK) * MUL, 0u);
  }
  __device__ void store(float* t, const Regs& rg) const {
#pragma unroll
    for (int i = 0; i < N; ++i) O::put(t, (tid & 15) * 4, k0 + 16 * i + g, rg[i]);
  }
};

// a policy's LDS beyond its operand images (EXTRA_LDS bytes, after them)
template <class P, class = void>
struct ExtraLdsOf : std::integral_constant<size_t, 0> {};
template <class P>
struct ExtraLdsOf<P, std::void_t<decltype(P::EXTRA_LDS)>> : std::integral_constant<size_t, P::EXTRA_LDS> {};

// streams with a per-tile prepare(lds, ns) (tables written into LDS before the slab loop)
template <class S, class = void>
struct HasPrepare : std::false_type {};
template <class S>
struct HasPrepare<S, std::void_t<decltype(std::declval<S&>().prepare((float*)nullptr, 0))>> : std::true_type {};

template <class P>
constexpr size_t gemm_lds_bytes() {
  return (size_t)KSplitOf<P>::value * 2 *
             (size_t)(Opnd<P::BM, P::A_KMAJ, MfOf<P>::value>::FLOATS + Opnd<P::BN, P::B_KMAJ, MfOf<P>::value>::FLOATS) * sizeof(float) +
         ExtraLdsOf<P>::value;
}

// Stream form of gemm_body (policies with a member type Streams): the same pipeline, fragments, MFMA chains, bias chains
// and epilogue, with the slab staging done by the policy's streams:
//   typename P::Streams st = p.streams(z, row0, col0, tid);   per tile
//   st.load(s, x) / st.store(s, x, As, Bs)                    x: a P::Streams::Regs register set
template <class P, class = void>
struct HasStreams : std::false_type {};
#ifndef QLX_Q32_NO_STREAMS   // (A/B builds of the measurement harnesses: every policy on the ldA / ldB core)
template <class P>
struct HasStreams<P, std::void_t<typename P::Streams>> : std::bool_constant<!std::is_void_v<typename P::Streams>> {};
#endif

// K split (round 6, policies with KSPLIT = G > 1 or KSEQ = Q > 1): the reduction is G (Q) chains over consecutive equal
// slab ranges, combined ((C0 + C1) + ..) before the epilogue - the same value either way: KSPLIT runs the chains in G
// wave groups of the block at once (group 0 sums them through LDS), KSEQ one after another in the same waves (the
// finished chains wait in registers).  ns must be a multiple of G (Q).
template <class P>
__device__ __forceinline__ void gemm_body_s(const P& p, int lb, float* lds) {
  constexpr int MF = 16;
  using OA = Opnd<P::BM, P::A_KMAJ, MF>;
  using OB = Opnd<P::BN, P::B_KMAJ, MF>;
  using Acc = f32x4;
  constexpr int TM = P::BM / (P::WM * MF), TN = P::BN / (P::WN * MF);
  static_assert(TM >= 1 && TN >= 1 && TM * P::WM * MF == P::BM && TN * P::WN * MF == P::BN, "tile shape");
  constexpr int G = KSplitOf<P>::value, Q = KSeqOf<P>::value;
  static_assert((G == 1 && Q <= 2) || (Q == 1 && !P::BIAS), "K split: two sequential chains, or wave groups without bias");
  static_assert(G == 1 || TM * TN * 4 * P::WM * P::WN * 64 <= 2 * (OA::FLOATS + OB::FLOATS), "K-split hand-off fits a group's LDS");
  constexpr int T = P::WM * P::WN * 64;   // threads of one K group
  constexpr int GROUP_LDS = 2 * (OA::FLOATS + OB::FLOATS);
  using St = typename P::Streams;
  using Regs = typename St::Regs;
  const int kg = G > 1 ? __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6) / (P::WM * P::WN)) : 0;
  const int tid = threadIdx.x - kg * T, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % P::WM, wn = wave / P::WM;
  int tm, tn, z;
  p.decode(lb, tm, tn, z);
  const int row0 = tm * P::BM, col0 = tn * P::BN;
  if constexpr (HasActive<P>::value) {
    if (!p.active(z, row0)) return;
  }
  const int ns = p.nslabs(z) / G, s_base = kg * ns;   // this group's slabs: s_base + [0, ns)
  const int s_half = Q > 1 ? ns / 2 : -1;              // KSEQ: the second chain starts at this slab
  St st = p.streams(z, row0, col0, tid);
  lds += kg * GROUP_LDS;
  float* As0 = lds;
  float* As1 = lds + OA::FLOATS;
  float* Bs0 = lds + 2 * OA::FLOATS;
  float* Bs1 = Bs0 + OB::FLOATS;
  if constexpr (HasPrepare<St>::value) {   // the streams' per-tile LDS tables, complete before the first slab load
    st.prepare(lds, ns);
    __syncthreads();
  }
  Regs x0, x1;
  Acc acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = zero4();
  Acc first[Q > 1 ? TM : 1][Q > 1 ? TN : 1];   // KSEQ: the finished first chain
  float bsum[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) bsum[j] = 0.0f;
  // the bias chains run in the waves that own them only: the slab loop is compiled twice (a runtime test per k step
  // keeps the B fragments' registers and the adds in every wave's loop)
  const bool do_bias = P::BIAS && tm == 0 && wm == 0;
  auto slab_loop = [&](auto bias_tag) {
    constexpr bool DB = decltype(bias_tag)::value;
    auto compute = [&](int s) {
      const float* a = (s & 1) ? As1 : As0;
      const float* b = (s & 1) ? Bs1 : Bs0;
      if constexpr (Q > 1) {
        if (s == s_half) {   // (wave-uniform) the first chain is done: keep it, start the second from zero
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) {
              first[i][j] = acc[i][j];
              acc[i][j] = zero4();
            }
        }
      }
      if constexpr (IglpOf<P>::value >= 0) __builtin_amdgcn_iglp_opt(IglpOf<P>::value);
      slab_mfma16<OA, OB, TM, TN, DB>(a, b, wm, wn, lane, acc, bsum);
    };
    // (the store of slab s + 1 is unconditional: past the last slab it writes the idle buffer with the reloaded last slab,
    // which nothing reads.  Skipped there, its registers' loads stayed pending on that path, and the compiler - which does
    // not see that the path leaves the loop - waited for them at the top of every other slab step: the two register sets
    // degenerated to one.)
    auto iter = [&](int s, Regs& xs, Regs& ys) {
      st.load(s_base + (s + 2 < ns ? s + 2 : ns - 1), ys);
      if constexpr (LoadFenceOf<P>::value) __builtin_amdgcn_sched_barrier(0);
      compute(s);
      st.store((s + 1) & 1 ? As1 : As0, (s + 1) & 1 ? Bs1 : Bs0, xs);
      lds_barrier();
    };
    if (ns > 0) {
      st.load(s_base, x1);
      st.store(As0, Bs0, x1);
      st.load(s_base + (ns > 1 ? 1 : 0), x0);
      lds_barrier();
      // (the odd last step after the loop: a conditional second step inside it was, to the compiler, a path back to the
      // loop head with a register set still loading - see iter)
      int s = 0;
      for (; s + 1 < ns; s += 2) {
        iter(s, x0, x1);
        iter(s + 1, x1, x0);
      }
      if (s < ns) iter(s, x0, x1);
    }
  };
  constexpr bool PRE = HasEpiPre<P>::value;
  typename PreOf<P>::type pre[TM][TN];
  if constexpr (PRE) {
    if (kg == 0) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          pre[i][j] = p.epi_pre(z, row0 + (wm * TM + i) * 16 + (lane >> 4) * 4, col0 + (wn * TN + j) * 16 + (lane & 15));
    }
  }
  if constexpr (P::BIAS) {
    if (do_bias) slab_loop(std::true_type{});
    else slab_loop(std::false_type{});
  } else {
    slab_loop(std::false_type{});
  }
  if constexpr (Q > 1) {   // C0 + C1
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[i][j][e] = __fadd_rn(ns > s_half ? first[i][j][e] : acc[i][j][e], ns > s_half ? acc[i][j][e] : 0.0f);
  }
  if constexpr (G > 1) {   // groups 1 .. G - 1 hand their chains to group 0 through their own LDS (free now); ((C0 + C1) + ..)
    if (kg > 0) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) lds[((i * TN + j) * 4 + e) * T + tid] = acc[i][j][e];
    }
    __syncthreads();
    if (kg > 0) return;
#pragma unroll
    for (int g = 1; g < G; ++g)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[i][j][e] = __fadd_rn(acc[i][j][e], lds[g * GROUP_LDS + ((i * TN + j) * 4 + e) * T + tid]);
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int row = row0 + (wm * TM + i) * 16 + (lane >> 4) * 4, col = col0 + (wn * TN + j) * 16 + (lane & 15);
      if constexpr (PRE) p.epi_post(z, row, col, acc[i][j], pre[i][j]);
      else p.epi(z, row, col, acc[i][j]);
    }
  if constexpr (P::BIAS) {
    if (do_bias) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const float c1 = __shfl(bsum[j], lane + 16), c2 = __shfl(bsum[j], lane + 32), c3 = __shfl(bsum[j], lane + 48);
        if (lane < 16) p.epi_bias(z, col0 + (wn * TN + j) * 16 + lane, __fadd_rn(__fadd_rn(__fadd_rn(bsum[j], c1), c2), c3));
      }
    }
  }
}

// a policy with NSUB (chained sub-tiles per block) runs gemm_body_chain
template <class P, class = void>
struct HasChain : std::false_type {};
template <class P>
struct HasChain<P, std::void_t<decltype(P::NSUB)>> : std::true_type {};
template <class P>
__device__ __forceinline__ void body(const P& p, int lb, float* lds) {
  if constexpr (HasChain<P>::value) gemm_body_chain(p, lb, lds);
  else if constexpr (HasStreams<P>::value) gemm_body_s(p, lb, lds);
  else gemm_body(p, lb, lds);
}

template <class P>
__global__ __launch_bounds__(threads_of<P>()) void k_gemm32(const P p) {
  extern __shared__ float lds[];
  body(p, block_order<P>(blockIdx.x, gridDim.x), lds);
}

// two independent GEMMs in one grid (hardware blocks [side.blocks(), side.blocks() + G1) run P1), plus `side` leading
// blocks running S and `tail` trailing blocks running T (independent work that fills CU slots beside / after the tiles)
// Occupancy floor of a pair launch (waves per SIMD the register allocation must allow): the larger of QLX_PAIR_MINW and
// the policies' MINW members.  Round 6: the P8 fragments' b128 reads let the compiler hoist a whole slab's operands; at
// the default allocation the conv2 pair grew 112 -> 154 VGPRs (3 waves / SIMD, 95.0 -> 98.0 us); held to 4 waves it
// takes 106 VGPRs (93.4 us).
#ifndef QLX_PAIR_MINW
#define QLX_PAIR_MINW 4
#endif
template <class P, class = void>
struct MinWOf : std::integral_constant<int, 1> {};
template <class P>
struct MinWOf<P, std::void_t<decltype(P::MINW)>> : std::integral_constant<int, P::MINW> {};
template <class P, class = void>
struct HasMinW : std::false_type {};
template <class P>
struct HasMinW<P, std::void_t<decltype(P::MINW)>> : std::true_type {};
// the policies' own floors when either declares one (the larger), else QLX_PAIR_MINW
template <class P1, class P2>
constexpr int pair_minw() {
  return (HasMinW<P1>::value || HasMinW<P2>::value)
             ? (MinWOf<P1>::value > MinWOf<P2>::value ? MinWOf<P1>::value : MinWOf<P2>::value)
             : QLX_PAIR_MINW;
}
template <class P1, class P2, class S, class T>
__global__ __launch_bounds__(256, (pair_minw<P1, P2>())) void k_gemm32_pair(const P1 p1, const P2 p2, const S side, const T tail) {
  static_assert(KSplitOf<P1>::value == 1 && KSplitOf<P2>::value == 1, "pair launches: 256 threads");
  extern __shared__ float lds[];
  const int b = blockIdx.x, ns = side.blocks();
  if (b < ns) { side.run(b, lds); return; }
  // the problems take consecutive hardware blocks (so both spread over all eight XCDs, P1 - the longer weight-gradient
  // tiles - dispatched first); inside each problem the XCD-grouped tile order
  const int h = b - ns;
  const int g1 = p1.g.blocks(), g2 = p2.g.blocks();
  if (h < g1) body(p1, block_order<P1>(h, g1), lds);
  else if (h < g1 + g2) body(p2, block_order<P2>(h - g1, g2), lds);
  else tail.run(h - g1 - g2, lds);
}

// one GEMM plus `side` leading blocks running S (the background rows of a list forward)
template <class P, class S>
__global__ __launch_bounds__(threads_of<P>()) void k_gemm32_side(const P p, const S side) {
  extern __shared__ float lds[];
  const int b = blockIdx.x, ns = side.blocks();
  if (b < ns) { side.run(b, lds); return; }
  body(p, block_order<P>(b - ns, (int)gridDim.x - ns), lds);
}

// A conv layer's background-row dz sums per sample chunk z (PConvWgrad CMP, SC = 16; conv2: P = 81, conv3: P = 49):
// S[z][oc] = ((T0 + T1) + T2) + T3, Tq = chain over p in [Q q, min(P, Q q + Q)) ascending of pbg[z][p][oc], Q = ceil(P / 4)
// (the per-chunk partials of the backward-data epilogue that produced dz).  Leading blocks of the layer's backward
// launch, one per chunk.
template <int P = 81>
struct SideBgSum {
  static constexpr size_t LDS = 4 * 64 * sizeof(float);
  static constexpr int Q = (P + 3) / 4;   // positions per chain
  const float* pbg;   // [nz][P][64]
  float* S;           // [nz][64]
  int nz;
  __host__ __device__ int blocks() const { return nz; }
  __device__ void run(int z, float* lds) const {
    const int oc = threadIdx.x & 63, q = threadIdx.x >> 6, p0 = Q * q, n = q < 3 ? Q : P - 3 * Q;
    float v[Q];
#pragma unroll
    for (int i = 0; i < Q; ++i) v[i] = i < n ? pbg[((size_t)z * P + p0 + i) * 64 + oc] : 0.0f;
    float t = 0.0f;
#pragma unroll
    for (int i = 0; i < Q; ++i)
      if (i < n) t = __fadd_rn(t, v[i]);
    lds[q * 64 + oc] = t;
    __syncthreads();
    if (q == 0) S[(size_t)z * 64 + oc] = __fadd_rn(__fadd_rn(__fadd_rn(lds[oc], lds[64 + oc]), lds[128 + oc]), lds[192 + oc]);
  }
};

struct NoSide {
  static constexpr size_t LDS = 0;
  __host__ __device__ int blocks() const { return 0; }
  __device__ void run(int, float*) const {}
};

// ---------------------------------------------------------------------------------------------------------------
// Layer policies.  Chain orders (oracle/qnet32_ref.cpp):
//   conv forward    k = (kh, kw, c)  (conv1: k_conv1_fwd32 below)                          fc1 forward k = h, w, c
//   conv dgrad      k = (kh, kw, oc) over the valid taps                                   fc1 dgrad   k = n
//   weight grads    r = (b, oh, ow) ascending inside a sample chunk; fc1 / fc2 over b ascending, no chunks

// conv2 / conv3 forward chains: z = C0 + C1, Ch = chain over the k = (kh, kw, c) half h (conv2: taps
// 0..7 / 8..15; conv3: k < 288 / the rest), so that the training-batch list launch can run the two chains in two wave groups
// of a block (KSPLIT); the chunk-batch launches run them one after the other (KSEQ)
#ifndef QLX_CONV_FWD_CHAINS
#define QLX_CONV_FWD_CHAINS 1   // (2 measured slower, round 6: conv3 forward 26.4 -> 29.5 us in wave groups, the chunk pass 166 -> 175 us in turn; the oracle follows this value)
#endif
constexpr int kConvFwdChains = QLX_CONV_FWD_CHAINS;
// conv2 / conv3 forward on fp32 NHWC input: out = relu(conv + bias); slab s: tap = 32 s / C, c0 = 32 s % C
template <int H, int W, int C, int KS, int S, int OH, int OW, int OC, int BM_ = 64, int BN_ = 64, int WM_ = 2, int WN_ = 2,
          int MF_ = 16>
struct PConvFwd {
  static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_, MF = MF_;
  static constexpr int KSEQ = kConvFwdChains;
  static constexpr int MINW = 3;   // (pair launches of the dense forward: the finished first chain's registers, no spill)
  static_assert(MF_ == 16, "conv forward chains: 16x16x4");
  static constexpr bool LOAD_FENCE = !(H == 20 && BN_ == 64);   // the chunk-size conv2 forward runs without it
  static constexpr bool A_KMAJ = false, B_KMAJ = true, BIAS = false;
  Grid g;
  const float* in;
  const float* w;    // [KS][KS][C][OC]
  const float* bias;
  float* out;        // [M][OC]
  int M;             // B * OH * OW
  __host__ __device__ void decode(int lb, int& tm, int& tn, int& z) const { g.decode(lb, tm, tn, z); }
  __host__ __device__ int nslabs(int) const { return KS * KS * C / BK; }
  __device__ f32x4 ldA(int, int s, int row, int k) const {
    const bool ok = row < M;
    const int rr = ok ? row : 0;
    const int tap = (s * BK) / C, c0 = (s * BK) % C, kh = tap / KS, kw = tap % KS;
    const int b = rr / (OH * OW), p = rr - b * (OH * OW), oh = p / OW, ow = p - oh * OW;
    return ld4m(in + ((size_t)(b * H + oh * S + kh) * W + ow * S + kw) * C + c0 + k, ok);
  }
  __device__ f32x4 ldB(int, int s, int col, int k) const { return ld4(w + (size_t)(s * BK + k) * OC + col); }
  __device__ void epi(int, int row, int col, f32x4 v) const {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (row + r < M) out[(size_t)(row + r) * OC + col] = relu(v[r] + bias[col]);
  }
  // the bias, loaded before the slab loop (HasEpiPre: a load after the loop waits behind the pipeline's last loads)
  __device__ f32x4 epi_pre(int, int, int col) const {
    const float b = bias[col];
    return f32x4{b, b, b, b};
  }
  __device__ void epi_post(int, int row, int col, f32x4 v, f32x4 b) const {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (row + r < M) out[(size_t)(row + r) * OC + col] = relu(v[r] + b[r]);
  }
};
using PConv2Fwd = PConvFwd<20, 20, 32, 4, 2, 9, 9, 64>;
using PConv3Fwd = PConvFwd<9, 9, 64, 3, 1, 7, 7, 64>;
// training-batch (B <= 2048) tile shapes: more, narrower blocks (scripts/ubench32.hip sweep at B = 1024)
using PConv2FwdS = PConvFwd<20, 20, 32, 4, 2, 9, 9, 64, 64, 32, 2, 2>;
using PConv3FwdS = PConvFwd<9, 9, 64, 3, 1, 7, 7, 64, 64, 32, 2, 2>;
// Balanced grids (f32_forward): whole 64 x 64 tiles in a multiple of the CU count, then the rows left over as 16 x 64
// tiles (RowShift: row tiles counted past the whole ones) in the same launch, so every CU gets the same work instead of
// a few CUs running one more whole tile at the end.  A 16 x 64 tile is four waves with one chain each (the same k order).
template <class Base>
struct RowShift : Base {
  int tm0;
  __host__ __device__ void decode(int lb, int& tm, int& tn, int& z) const {
    Base::decode(lb, tm, tn, z);
    tm += tm0;
  }
};
using PConv2FwdR = RowShift<PConvFwd<20, 20, 32, 4, 2, 9, 9, 64, 16, 64, 1, 4>>;
using PConv3FwdR = RowShift<PConvFwd<9, 9, 64, 3, 1, 7, 7, 64, 16, 64, 1, 4>>;

// conv2 / conv3 forward over the non-background rows (see C1Lists).  Row tile 0 holds one row, the constant row: its input
// is the constant vector cx at every tap (conv2: relu(0 + b0); conv3: c2) and its output goes to cbuf (c2; c3) - the
// background rows' value, computed by the GEMM's own chain (ConstRows runs these as the first block of the conv2 launch).
// Row tile 1 + t * kListSlots + x is tile t of list region x, whose row lr is output row list[x][lr] (chunk-local
// b * OH * OW + p, bits 0..19) for lr < the region's count (device memory); tiles past it return at once.  Tiles run in
// hardware block order (the live ones first, spread over the XCDs).  SEL (conv3): the taps whose input position is
// background in the layer below (list entry bits 20..28, written by conv1) read cx = that layer's constant row instead of
// `in` (those rows are written by this launch's side blocks).
template <int H, int W, int C, int KS, int S, int OH, int OW, int OC, int BM_ = 64, int BN_ = 64, int WM_ = 2, int WN_ = 2,
          bool SEL = false, int KS_ = 1>
struct PConvFwdL {
  static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_;
  static constexpr int KSPLIT = KS_, KSEQ = kConvFwdChains / KS_;   // the two chains in wave groups (KS_ = 2) or in turn
  static_assert(KSPLIT * KSEQ == kConvFwdChains, "conv forward: the chain definition");
  static constexpr bool A_KMAJ = false, B_KMAJ = true, BIAS = false, RAW_ORDER = true;
  // (with the slab loop's wait fixed, round 5: the fence on for conv2 too - the 8,192-sample pass 131 -> 127 us)
  static constexpr bool LOAD_FENCE = true;
  static constexpr int R = OH * OW;
  using OA = Opnd<BM, false, 16>;
  static constexpr int T = WM * WN * 64, NA = (OA::F4 + T - 1) / T;   // (T: threads of one K group)
  Grid g;            // tiles_m = 1 + kListSlots * tiles per region
  const float* in;
  const float* w;    // [KS][KS][C][OC]
  const float* bias;
  float* out;        // [rows][OC]
  const int* list;   // [kListSlots][cap]
  int cap;
  const unsigned long long* cnt;   // this layer's counter of region 0 (region x at x * 2 * kCntStride)
  const float* cx;   // constant input row [C]
  float* cbuf;       // constant output row [OC]
  // the epilogue rows' entries batched per call (entries()) or row by row, per launch: measured at C3, batched: conv3
  // 28.0 -> 27.5 us, the 8,192-sample conv2 / conv3 passes 137 / 180 -> 128 / 171 us, but the B = 1024 conv2 23.9 -> 25.6 us
  // (that launch sets it false)
  bool pre_batched = true;
  struct ACtx { int off[NA]; uint32_t m[NA]; };   // input offset (-1: no row), taps read from cx
  struct Pre { float b; int o[4]; };   // o: the rows' raw list entries

  __host__ __device__ void decode(int lb, int& tm, int& tn, int& z) const { g.decode(lb, tm, tn, z); }
  __host__ __device__ int nslabs(int) const { return KS * KS * C / BK; }
  __device__ int count(int x) const { return (int)(cnt[x * 2 * kCntStride] >> 32); }
  // list entry of a GEMM row: >= 0 a row (SEL: with its constant-tap mask << 20), -1 none, -2 the constant row
  // List entries of N rows of one row tile (the callers' rows all lie in one tile, so the tile index is read as
  // wave-uniform): one scalar branch for the constant-row tile, the region counter as a scalar load, and the N entry loads -
  // unconditional, at clamped addresses - all in flight at once.  (Row by row with a per-lane tile index the compiler put
  // each row's loads behind an exec-masked branch and a vmcnt(0): one memory round trip per row in the tile prologue.)
  template <int N>
  __device__ void entries(const int (&row)[N], int (&out)[N]) const {
    const int tm = q32_uniform(row[0] / BM);
    if (tm == 0) {
#pragma unroll
      for (int i = 0; i < N; ++i) out[i] = row[i] == 0 ? -2 : -1;
      return;
    }
    const int x = (tm - 1) % kListSlots, base = ((tm - 1) / kListSlots) * BM;
    const int n = count(x);
    int v[N];
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] = list[x * cap + min(base + row[i] % BM, cap - 1)];
#pragma unroll
    for (int i = 0; i < N; ++i) out[i] = base + row[i] % BM < n ? v[i] : -1;
  }
  __device__ bool active(int, int row0) const {   // (row tile 0 only where the constant row has somewhere to go)
    const int tm = row0 / BM;
    return tm == 0 ? cbuf != nullptr : ((tm - 1) / kListSlots) * BM < count((tm - 1) % kListSlots);
  }
  __device__ ACtx a_ctx(int, int row0, int tid) const {
    ACtx c;
    int rows[NA], raws[NA];
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      int r, k;
      OA::coord(tid + i * T, r, k);
      rows[i] = row0 + r;
    }
    entries(rows, raws);
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int raw = raws[i], e = raw >= 0 ? raw & 0xFFFFF : raw;
      const int b = e / R, p = e - b * R, oh = p / OW, ow = p - oh * OW;
      c.off[i] = e >= 0 ? ((b * H + oh * S) * W + ow * S) * C : -1;
      c.m[i] = e == -2 ? 0xFFFFFFFFu : (SEL && raw >= 0 ? (uint32_t)raw >> 20 : 0u);
    }
    return c;
  }
  __device__ f32x4 ldA_c(const ACtx& c, int i, int, int s, int, int k) const {
    const int tap = (s * BK) / C, c0 = (s * BK) % C, kh = tap / KS, kw = tap % KS;
    const int o = c.off[i];
    const bool cst = (c.m[i] >> tap) & 1u;
    const float* src = cst ? cx + c0 + k : in + (size_t)(o < 0 ? 0 : o) + (kh * W + kw) * C + c0 + k;
    return ld4m(src, cst || o >= 0);
  }
  __device__ f32x4 ldB(int, int s, int col, int k) const { return ld4(w + (size_t)(s * BK + k) * OC + col); }
  __device__ Pre epi_pre(int, int row, int col) const {
    Pre q;
    q.b = bias[col];
    if (!pre_batched) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int tm = (row + r) / BM;
      if (tm == 0) { q.o[r] = row + r == 0 ? -2 : -1; continue; }
      const int x = (tm - 1) % kListSlots, lr = ((tm - 1) / kListSlots) * BM + (row + r) % BM;
      q.o[r] = lr < count(x) ? list[x * cap + lr] : -1;
    }
    } else {
    const int rows[4] = {row, row + 1, row + 2, row + 3};
    entries(rows, q.o);   // raw entries: decoded in the epilogue, so nothing waits for these loads before the slab loop
    }
    return q;
  }
  __device__ void epi_post(int, int, int col, f32x4 v, const Pre& q) const {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#ifdef QLX_LIST_CHECK
      if (q.o[r] >= 0 && (q.o[r] & 0xFFFFF) >= kListSlots * cap) printf("LISTCHK epi o %d cap %d\n", q.o[r], cap);
#endif
      if (q.o[r] >= 0) out[(size_t)(q.o[r] & 0xFFFFF) * OC + col] = relu(v[r] + q.b);
      else if (q.o[r] == -2) cbuf[col] = relu(v[r] + q.b);
    }
  }
  // streams (gemm_body_s; the list tiles, row tile >= 1 - the constant-row tile runs in ConstRows on the ldA core): A =
  // the listed rows' im2col windows (rows past the list read zeros), a slab's tap and channel offset wave-uniform; SEL:
  // a row's background taps read the constant row cx instead (one buffer spans `in` and cx: both live in the model's
  // workspace), a per-lane select per slab.  B = the weight rows, affine.
  struct StreamsImpl {
    __amdgpu_buffer_rsrc_t ra;
    uint32_t vo[NA], cxo[NA], msk[NA];
    int tid;
    AffineStream<BN_, true, T> b;
    struct Regs {
      f32x4 a[NA];
      typename AffineStream<BN_, true, T>::Regs b;
    };
    __device__ void load(int s, Regs& x) const {
      const int tap = (s * BK) / C, c0 = (s * BK) % C, kh = tap / KS, kw = tap - kh * KS;
      const uint32_t so = (uint32_t)((kh * W + kw) * C + c0) * 4u;
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        if (OA::F4 % T == 0 || tid + i * T < OA::F4) {
          if constexpr (SEL) {
            const bool cst = (msk[i] >> tap) & 1u;
            x.a[i] = buf_ld4(ra, cst ? cxo[i] + (uint32_t)c0 * 4u : vo[i] + so, 0u);
          } else {
            x.a[i] = buf_ld4(ra, vo[i], so);
          }
        }
      }
      b.load((uint32_t)s * BK * OC * 4u, 0, x.b);
    }
    __device__ void store(float* as, float* bs, const Regs& x) const {
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int idx = tid + i * T;
        if (OA::F4 % T == 0 || idx < OA::F4) {
          int r, k;
          OA::coord(idx, r, k);
          OA::put(as, r, k, x.a[i]);
        }
      }
      b.store(bs, x.b);
    }
  };
  using Streams = StreamsImpl;
  __device__ Streams streams(int, int row0, int col0, int tid) const {
    Streams st;
    st.tid = tid;
    // one descriptor over [min(in, cx), max end): both in the model's workspace (f32_forward)
    const char* lo = (const char*)in;
    const char* base = SEL && (const char*)cx < lo ? (const char*)cx : lo;
    const uint32_t in_off = (uint32_t)(lo - base), cx_off = SEL ? (uint32_t)((const char*)cx - base) : 0u;
    st.ra = buf_rsrc(base, 0x7FFFFFF0u);   // (row offsets are bounded by the list entries: b * R + p of this chunk)
    int rows[NA], raws[NA];
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      int r = 0, k = 0;
      OA::coord(tid + i * T, r, k);
      rows[i] = row0 + r;
    }
    entries(rows, raws);
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      int r = 0, k = 0;
      OA::coord(tid + i * T, r, k);
      const int raw = raws[i], e = raw >= 0 ? raw & 0xFFFFF : -1;
      const int bb = e / R, pp = e - bb * R, oh = pp / OW, ow = pp - oh * OW;
      st.vo[i] = e >= 0 ? in_off + (uint32_t)(((bb * H + oh * S) * W + ow * S) * C + k) * 4u : kOob;
      st.cxo[i] = cx_off + (uint32_t)k * 4u;
      st.msk[i] = SEL && raw >= 0 ? (uint32_t)raw >> 20 : 0u;
    }
    st.b.init(w, (uint32_t)KS * KS * C * OC * 4u, tid, [col0](int r, int k) { return (uint32_t)(k * OC + col0 + r) * 4u; });
    return st;
  }
};
template <int BM, int BN, int WM, int WN, int KS_ = 1>
using PConv2FwdL = PConvFwdL<20, 20, 32, 4, 2, 9, 9, 64, BM, BN, WM, WN, false, KS_>;
template <int BM, int BN, int WM, int WN, int KS_ = 1>
using PConv3FwdL = PConvFwdL<9, 9, 64, 3, 1, 7, 7, 64, BM, BN, WM, WN, true, KS_>;

// The constant rows as the first block of the conv2 launch: the conv2 constant row (input relu(0 + b0) -> c2), then, from
// c2, the conv3 constant row (-> c3), each as the constant-row tile of a 16 x 64 list policy (4 waves x 16 channels, the
// GEMM's chains).  Both are ready when the conv3 launch starts, so its side blocks can write the background rows of a2
// and a3 and the fc1 forward reads a complete a3.
template <class PA, class PB>
struct ConstRows {
  static constexpr size_t LDS = gemm_lds_bytes<PA>() > gemm_lds_bytes<PB>() ? gemm_lds_bytes<PA>() : gemm_lds_bytes<PB>();
  PA pa;
  PB pb;
  __host__ __device__ int blocks() const { return 1; }
  __device__ void run(int, float* lds) const {
    gemm_body(pa, 0, lds);
    __syncthreads();
    __threadfence();   // c2 (stored by this block's epilogue) is pb's constant input
    gemm_body(pb, 0, lds);
  }
};

// Leading blocks of a list launch (its block size: 256 or 512 threads): the layer below's background rows get its constant row
// c_in, 16 lanes (256 bytes) per row, 8 list entries per lane loaded together (the back ends of the list regions).
struct BgRows {
  static constexpr size_t LDS = 64 * sizeof(float);
  static constexpr int U = 8;
  int nblk;
  const int* list;         // [kListSlots][cap]
  const unsigned long long* cnt;   // that layer's counter of region 0
  int cap;                 // rows per region
  const float* c_in;       // [64]
  float* out;              // [rows][64]
  __host__ __device__ int blocks() const { return nblk; }
  __device__ void run(int blk, float* lds) const {
    const int tid = threadIdx.x, q = tid & 15, RB = (int)blockDim.x >> 4;   // RB rows per pass (the launch's block size)
    const f32x4 v = ld4(c_in + 4 * q);
    for (int x = 0; x < kListSlots; ++x) {
      const int nbg = (int)(uint32_t)cnt[x * 2 * kCntStride];
#ifdef QLX_LIST_CHECK
      if (tid == 0 && blk == 0 && (nbg > cap || (int)(cnt[x * 2 * kCntStride] >> 32) + nbg > cap))
        printf("LISTCHK bgrows region %d nbg %d non %d cap %d\n", x, nbg, (int)(cnt[x * 2 * kCntStride] >> 32), cap);
#endif
      const int* back = list + (size_t)(x + 1) * cap - 1;
      for (int i0 = blk * RB * U + (tid >> 4); i0 < nbg; i0 += nblk * RB * U) {
        int e[U];
#pragma unroll
        for (int u = 0; u < U; ++u) e[u] = i0 + RB * u < nbg ? back[-(i0 + RB * u)] : -1;
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (e[u] >= 0) {
#ifdef QLX_LIST_CHECK
            if (e[u] >= kListSlots * cap && q == 0) printf("LISTCHK bgrows e %d cap %d region %d i %d\n", e[u], cap, x, i0 + RB * u);
#endif
            *reinterpret_cast<f32x4*>(out + (size_t)e[u] * 64 + 4 * q) = v;
          }
      }
    }
  }
};
struct BgRows2 {   // two background-row jobs (a2 and a3) in one launch's leading blocks
  static constexpr size_t LDS = BgRows::LDS;
  BgRows a, b;
  __host__ __device__ int blocks() const { return a.nblk + b.nblk; }
  __device__ void run(int blk, float* lds) const {
    if (blk < a.nblk) a.run(blk, lds);
    else b.run(blk - a.nblk, lds);
  }
};

// fc1 forward: a4 [B][512] = relu(a3 [B][3136] W3 + b3), the reduction as kFc1Chains chains over consecutive k halves
// (C0 + C1; round 6): at the training batch the two chains run in two wave groups of a block at once (KS_ =
// 2: twice the waves on the chip for the same 512 output tiles), at chunk batches one after the other (KQ_ = 2)
#ifndef QLX_FC1_CHAINS
#define QLX_FC1_CHAINS 2   // (A/B timing builds only: 1 = the round-5 single chain, which the oracle no longer follows)
#endif
constexpr int kFc1Chains = QLX_FC1_CHAINS;
template <int BM_ = 32, int BN_ = 64, int WM_ = 2, int WN_ = 2, int MF_ = 16, int KS_ = 1, int KQ_ = kFc1Chains>
struct PFc1FwdT {
  static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_, MF = MF_;
  static constexpr int KSPLIT = KS_, KSEQ = KQ_;
  static_assert(KS_ * KQ_ == kFc1Chains && MF_ == 16, "fc1 forward: the chain definition");
  static constexpr bool LOAD_FENCE = false;   // (round 5: with it 35.3 / 209.8 us against 33.8 / 203.4)
  // strategy 0 at the training batch (default scheduler 40.4, strategy 1 42.2, 0 39.8 us at B = 1024; round 5: 1 39.3 against
  // 33.8), strategy 1 for the chunk-batch tiles (round 5: 196.7 against 203.4 us)
  static constexpr int IGLP = BM_ == 64 ? 1 : 0;
  static constexpr bool A_KMAJ = false, B_KMAJ = true, BIAS = false;
  Grid g;
  const float* a3;
  const float* w3;
  const float* b3;
  float* a4;
  int M;
  __host__ __device__ void decode(int lb, int& tm, int& tn, int& z) const { g.decode(lb, tm, tn, z); }
  __host__ __device__ int nslabs(int) const { return 3136 / BK; }
  __device__ f32x4 ldA(int, int s, int row, int k) const {
    return ld4m(a3 + (size_t)(row < M ? row : 0) * 3136 + s * BK + k, row < M);
  }
  __device__ f32x4 ldB(int, int s, int col, int k) const { return ld4(w3 + (size_t)(s * BK + k) * 512 + col); }
  __device__ void epi(int, int row, int col, f32x4 v) const {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (row + r < M) a4[(size_t)(row + r) * 512 + col] = relu(v[r] + b3[col]);
  }
  __device__ f32x4 epi_pre(int, int, int col) const {
    const float b = b3[col];
    return f32x4{b, b, b, b};
  }
  __device__ void epi_post(int, int row, int col, f32x4 v, f32x4 b) const {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (row + r < M) a4[(size_t)(row + r) * 512 + col] = relu(v[r] + b[r]);
  }
  // streams (gemm_body_s; MF 16): a3 rows (rows past M read zeros), W3 k rows
  static constexpr int T = WM_ * WN_ * 64;
  using SA = AffineStream<BM_, false, T>;
  using SB = AffineStream<BN_, true, T>;
  using Streams = std::conditional_t<MF_ == 16, PairStreams<SA, SB, BK * 4u, BK * 512u * 4u>, void>;
  template <class S = Streams>
  __device__ S streams(int, int row0, int col0, int tid) const {
    S st;
    const int m = M;
    st.a.init(a3, (uint32_t)M * 3136u * 4u, tid,
              [row0, m](int r, int k) { return row0 + r < m ? (uint32_t)((row0 + r) * 3136 + k) * 4u : kOob; });
    st.b.init(w3, 3136u * 512u * 4u, tid, [col0](int r, int k) { return (uint32_t)(k * 512 + col0 + r) * 4u; });
    st.kmax = 3136;
    return st;
  }
};
using PFc1Fwd = PFc1FwdT<32, 64, 2, 2, 16, 1, kFc1Chains>;
// chunk-size batches: 64 x 128 tiles on the stream core (in place: 208 us against 228 us for 64 x 64 on
// v_mfma_f32_32x32x2_f32, 212 / 215 us for 64 x 64 / 128 x 64; gpurun_out/w12)
using PFc1FwdB = PFc1FwdT<64, 128, 2, 2, 16, 1, kFc1Chains>;
// (re-checked on the stream core in place: 32 x 64 / 64 x 32 / 16 x 64 ran 35.3 / 35.9 / 40.4 us against 34.1 us, w9)
using PFc1FwdS = PFc1FwdT<32, 32, 2, 2, 16, kFc1Chains, 1>;   // (round 5, after the slab-loop fix: 64 x 32 / 32 x 64 38.4 / 38.9 us against 33.8)

// fc1 backward-data: dz3 [B][3136] = (dz4 [B][512] W3^T) * (a3 > 0); k = n
#ifndef QLX_PB_XCH
#define QLX_PB_XCH 1   // conv1 bias partials: lane exchanges by v_permlane16/32_swap (1) or ds_bpermute (0)
#endif
// (Q0 + Q1) + (Q2 + Q3) of a 16-row MFMA fragment column, Qg = ((d0 + d1) + d2) + d3 of lane group g's four rows, in every
// lane (PConv2DgradPx::pb)
#ifndef QLX_Q32_POLICIES_ONLY
__device__ __forceinline__ float pb_sum16(const float (&d)[4]) {
  float s = __fadd_rn(__fadd_rn(__fadd_rn(d[0], d[1]), d[2]), d[3]);
#if QLX_PB_XCH
  // VALU lane swaps (gfx950): with both operands s, the pair holds the lower and the upper row's (half's) value in every
  // lane, so both partners form the same sum (an fp32 sum of two does not depend on the order)
  const auto r16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(s), __float_as_uint(s), false, false);
  s = __fadd_rn(__uint_as_float(r16[0]), __uint_as_float(r16[1]));
  const auto r32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(s), __float_as_uint(s), false, false);
  return __fadd_rn(__uint_as_float(r32[0]), __uint_as_float(r32[1]));
#else
  s = __fadd_rn(s, __shfl_xor(s, 16));
  return __fadd_rn(s, __shfl_xor(s, 32));
#endif
}
#else
inline float pb_sum16(const float (&d)[4]) { return ((d[0] + d[1]) + d[2]) + d[3]; }   // (host address replay)
#endif

template <int BM_ = 64, int BN_ = 64, int WM_ = 2, int WN_ = 2, int MF_ = 16>
struct PFc1DgradT {
  static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_, MF = MF_;
  static constexpr bool A_KMAJ = false, B_KMAJ = false, BIAS = false;
  Grid g;
  const float* dz4;
  const float* w3;
  const float* a3;
  float* dz3;
  int M;
  // conv3's background-row dz3 sums per 16-sample chunk and position, as PConv3DgradPx::pbg for conv2 (null: none):
  // pbg[g16][p][c], column = 64 p + c, background bytes bg[49][bg_ld]
  float* pbg = nullptr;
  const uint8_t* bg = nullptr;
  int bg_ld = 0;
  struct Pre {
    f32x4 m;
    uint32_t bg;
  };
  __host__ __device__ void decode(int lb, int& tm, int& tn, int& z) const { g.decode(lb, tm, tn, z); }
  __host__ __device__ int nslabs(int) const { return 512 / BK; }
  __device__ f32x4 ldA(int, int s, int row, int k) const {
    return ld4m(dz4 + (size_t)(row < M ? row : 0) * 512 + s * BK + k, row < M);
  }
  __device__ f32x4 ldB(int, int s, int col, int k) const { return ld4(w3 + (size_t)col * 512 + s * BK + k); }
  __device__ void epi(int z, int row, int col, f32x4 v) const { epi_post(z, row, col, v, epi_pre(z, row, col)); }
  // the ReLU mask of the four rows, loaded before the slab loop (HasEpiPre; rows past M read row 0)
  __device__ Pre epi_pre(int, int row, int col) const {
    Pre pr;
#pragma unroll
    for (int r = 0; r < 4; ++r) pr.m[r] = a3[(size_t)(row + r < M ? row + r : 0) * 3136 + col];
    // (row is a multiple of 4 and row + 3 < bg_ld: the four samples' bytes are one aligned dword)
    pr.bg = pbg ? *reinterpret_cast<const uint32_t*>(bg + (size_t)(col >> 6) * bg_ld + row) : 0u;
    return pr;
  }
  __device__ void epi_post(int, int row, int col, f32x4 v, const Pre& pr) const {
    float d[4], e[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      d[r] = row + r < M && pr.m[r] > 0.0f ? v[r] : 0.0f;
      e[r] = ((pr.bg >> (8 * r)) & 0xFFu) != 0u ? d[r] : 0.0f;
      if (row + r < M) dz3[(size_t)(row + r) * 3136 + col] = d[r];
    }
    if (pbg) {   // (uniform: every lane of the wave takes part in the exchanges)
      const float s = pb_sum16(e);
      if ((row & 15) == 0 && row < M) pbg[(size_t)(row >> 4) * 3136 + col] = s;
    }
  }
  // streams (gemm_body_s): dz4 rows (rows past M read zeros), W3 rows (k = n contiguous)
  static constexpr int T = WM_ * WN_ * 64;
  using SA = AffineStream<BM_, false, T>;
  using SB = AffineStream<BN_, false, T>;
  using Streams = std::conditional_t<MF_ == 16, PairStreams<SA, SB, BK * 4u, BK * 4u>, void>;
  template <class S = Streams>
  __device__ S streams(int, int row0, int col0, int tid) const {
    S st;
    const int m = M;
    st.a.init(dz4, (uint32_t)M * 512u * 4u, tid,
              [row0, m](int r, int k) { return row0 + r < m ? (uint32_t)((row0 + r) * 512 + k) * 4u : kOob; });
    st.b.init(w3, 3136u * 512u * 4u, tid, [col0](int r, int k) { return (uint32_t)((col0 + r) * 512 + k) * 4u; });
    st.kmax = 512;
    return st;
  }
};
using PFc1Dgrad = PFc1DgradT<>;
// (64 x 32 on the stream core: 61.4 vs 66.0 us alone in scripts/ubench32.hip sweep, but 67.0 vs 65.2 us in place)
using PFc1DgradS = PFc1DgradT<32, 64, 2, 2>;

// fc1 weight gradient: dW3 [3136][512] = a3^T dz4 over b ascending; db3 = column sums of dz4 (row-tile 0 blocks)
template <int BM_ = 64, int BN_ = 64, int WM_ = 2, int WN_ = 2, int MF_ = 16>
struct PFc1WgradT {
  static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_, MF = MF_;
  // the pair at >= 6 waves per SIMD (78 VGPRs; at the default allocation the P8 fragments took it to 86, 5 waves)
#ifndef QLX_FC1_MINW
#define QLX_FC1_MINW 6
#endif
  static constexpr int MINW = QLX_FC1_MINW;
  static constexpr bool A_KMAJ = true, B_KMAJ = true, BIAS = true;
  Grid g;
  const float* a3;
  const float* dz4;
  float* dw3;
  float* db3;
  int B;
  __host__ __device__ void decode(int lb, int& tm, int& tn, int& z) const { g.decode(lb, tm, tn, z); }
  __host__ __device__ int nslabs(int) const { return (B + BK - 1) / BK; }
  __device__ f32x4 ldA(int, int s, int row, int k) const {
    const int b = s * BK + k;
    const bool ok = b < B && row < 3136;
    return ld4m(a3 + (ok ? (size_t)b * 3136 + row : 0), ok);
  }
  __device__ f32x4 ldB(int, int s, int col, int k) const {
    const int b = s * BK + k;
    return ld4m(dz4 + (size_t)(b < B ? b : 0) * 512 + col, b < B);
  }
  __device__ void epi(int, int row, int col, f32x4 v) const {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (row + r < 3136) dw3[(size_t)(row + r) * 512 + col] = v[r];
  }
  __device__ void epi_bias(int, int col, float v) const { db3[col] = v; }
  // streams (gemm_body_s): a3 and dz4 rows of the slab's samples (k = b; samples past B read zeros)
  static constexpr int T = WM_ * WN_ * 64;
  using SA = AffineStream<BM_, true, T, true>;
  using SB = AffineStream<BN_, true, T, true>;
  using Streams = std::conditional_t<MF_ == 16, PairStreams<SA, SB, BK * 3136u * 4u, BK * 512u * 4u, true>, void>;
  template <class S = Streams>
  __device__ S streams(int, int row0, int col0, int tid) const {
    S st;
    st.a.init(a3, (uint32_t)B * 3136u * 4u, tid, [row0](int r, int k) { return (uint32_t)(k * 3136 + row0 + r) * 4u; });
    st.b.init(dz4, (uint32_t)B * 512u * 4u, tid, [col0](int r, int k) { return (uint32_t)(k * 512 + col0 + r) * 4u; });
    st.kmax = B;
    return st;
  }
};
using PFc1Wgrad = PFc1WgradT<>;
// training batch: 64 x 64 tiles (392 + the fc1 backward-data tiles; in place at C3: 68.6 -> 65.1 us per fc1 backward
// against 64 x 32, 128 x 64 75.3, 64 x 128 77.3, 128 x 128 91.1 - gpurun_out/fc1b, fc1c)
// (on the stream core: 64 x 32, 784 tiles - fc1 backward pair 64.8 -> 61.6 us in place, gpurun_out/w7; with it, backward
// data 64 x 32 / 32 x 32 / 64 x 64 ran 62.6 / 63.2 / 64.3 us against 61.5 us for 32 x 64, w8)
using PFc1WgradS = PFc1WgradT<64, 32, 2, 2>;

// conv3 backward-data: dz2 [B][9][9][64] = convT(dz3, W2) * (a2 > 0); rows (b, ih, iw), k = (kh, kw, oc)
template <int BM_ = 64, int BN_ = 64, int WM_ = 2, int WN_ = 2, int MF_ = 16>
struct PConv3DgradT {
  static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_, MF = MF_;
  static constexpr bool A_KMAJ = false, B_KMAJ = false, BIAS = false;
  Grid g;
  const float* dz3;   // [B][7][7][64]
  const float* w2;    // [3][3][64][64]
  const float* a2;
  float* dz2;
  int M;              // B * 81
  __host__ __device__ void decode(int lb, int& tm, int& tn, int& z) const { g.decode(lb, tm, tn, z); }
  __host__ __device__ int nslabs(int) const { return 18; }
  __device__ f32x4 ldA(int, int s, int row, int k) const {
    const int tap = s >> 1, kh = tap / 3, kw = tap - kh * 3, oc0 = (s & 1) * 32;
    const int rr = row < M ? row : 0;
    const int b = rr / 81, p = rr - b * 81, ih = p / 9, iw = p - ih * 9;
    const int oh = ih - kh, ow = iw - kw;
    const bool ok = row < M && oh >= 0 && oh < 7 && ow >= 0 && ow < 7;
    return ld4m(dz3 + (ok ? ((size_t)(b * 7 + oh) * 7 + ow) * 64 + oc0 + k : 0), ok);
  }
  __device__ f32x4 ldB(int, int s, int col, int k) const {   // W2[kh][kw][c = col][oc]
    return ld4(w2 + ((size_t)(s >> 1) * 64 + col) * 64 + (s & 1) * 32 + k);
  }
  __device__ void epi(int, int row, int col, f32x4 v) const {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (row + r < M) {
        const size_t o = (size_t)(row + r) * 64 + col;
        dz2[o] = a2[o] > 0.0f ? v[r] : 0.0f;
      }
  }
};
using PConv3Dgrad = PConv3DgradT<>;
using PConv3DgradS = PConv3DgradT<32, 64, 2, 2>;

// Pixel-major backward data.  A block owns one input pixel (all samples of a row tile): its valid taps are uniform, so
// the k loop runs over those taps only - the same chain (valid (kh, kw, oc) lexicographic) as the row-major policies
// without their zero taps.  Pixels are numbered heavy first (most valid taps: long tiles start first) and the blocks
// keep the hardware order (RAW_ORDER: every XCD gets its share of the heavy pixels).
// 1-D heavy-first order of the 9 input rows of conv3 dgrad (valid kh: 3 for ih 2..6, 2 for 1 and 7, 1 for 0 and 8)
__host__ __device__ inline int px3_order(int z) { return z < 5 ? z + 2 : (z == 5 ? 1 : (z == 6 ? 7 : (z == 7 ? 0 : 8))); }
// ... and of the 10 class rows of conv2 dgrad (valid th: 2 for i 1..8, 1 for 0 and 9)
__host__ __device__ inline int px2_order(int z) { return z < 8 ? z + 1 : (z == 8 ? 0 : 9); }


#ifndef QLX_BG2_POST
#define QLX_BG2_POST 0
#endif
// conv3 backward-data, pixel-major: z = pixel (ih, iw) of the 9 x 9 grid; rows b; k = valid (kh, kw) x oc
template <int BM_ = 32, int BN_ = 64, int WM_ = 2, int WN_ = 2, bool DIRECT = false>
struct PConv3DgradPx {
  static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_;
  static constexpr bool LOAD_FENCE = false;
  static constexpr bool A_KMAJ = false, B_KMAJ = false, BIAS = false, RAW_ORDER = true;
  Grid g;             // {ceil(B / BM), 64 / BN, 81}
  const float* dz3;   // [B][7][7][64]
  const float* w2;    // [3][3][64][64]
  const float* a2;
  float* dz2;
  int B;
  // conv2's background-row dz2 sums per sample chunk (16 samples: one MFMA fragment's rows) and position (null: none):
  // pbg[g16][p][oc] = (Q0 + Q1) + (Q2 + Q3), Qg = ((d0 + d1) + d2) + d3 over samples 16 g16 + 4 g .. + 3 of the stored dz2
  // where position p of the sample is a background row (bg2, c1_flags), else 0 (PConvWgrad compacted, SideBgSum)
  float* pbg = nullptr;
  const uint8_t* bg2 = nullptr;
  int bg2_ld = 0;
  __host__ __device__ void decode(int lb, int& tm, int& tn, int& z) const { g.decode(lb, tm, tn, z); }
  struct Px {
    int ih, iw, kh0, kw0, nkw, ntap;
  };
  struct Pre {
    f32x4 m;       // a2 of the four rows (the ReLU mask)
    uint32_t bg;   // their background bytes
  };
  __host__ __device__ static Px px(int z) {
    Px q;
    q.ih = DIRECT ? z / 9 : px3_order(z / 9);   // DIRECT: z = ih * 9 + iw
    q.iw = DIRECT ? z % 9 : px3_order(z % 9);
    q.kh0 = q.ih > 6 ? q.ih - 6 : 0;
    q.kw0 = q.iw > 6 ? q.iw - 6 : 0;
    const int kh1 = q.ih < 2 ? q.ih : 2, kw1 = q.iw < 2 ? q.iw : 2;
    q.nkw = kw1 - q.kw0 + 1;
    q.ntap = (kh1 - q.kh0 + 1) * q.nkw;
    return q;
  }
  __host__ __device__ int nslabs(int z) const { return 2 * px(z).ntap; }
  __device__ f32x4 ldA(int z, int s, int row, int k) const {
    const Px q = px(z);
    const int t = s >> 1, kh = q.kh0 + t / q.nkw, kw = q.kw0 + t % q.nkw;
    return ld4m(dz3 + ((size_t)((row < B ? row : 0) * 7 + q.ih - kh) * 7 + q.iw - kw) * 64 + (s & 1) * 32 + k, row < B);
  }
  __device__ f32x4 ldB(int z, int s, int col, int k) const {   // W2[kh][kw][c = col][oc]
    const Px q = px(z);
    const int t = s >> 1, kh = q.kh0 + t / q.nkw, kw = q.kw0 + t % q.nkw;
    return ld4(w2 + ((size_t)(kh * 3 + kw) * 64 + col) * 64 + (s & 1) * 32 + k);
  }
  __device__ void epi(int z, int row, int col, f32x4 v) const { epi_post(z, row, col, v, epi_pre(z, row, col)); }
  __device__ Pre epi_pre(int z, int row, int col) const {
    const Px q = px(z);
    Pre pr;
#pragma unroll
    for (int r = 0; r < 4; ++r) pr.m[r] = a2[((size_t)((row + r < B ? row + r : 0) * 9 + q.ih) * 9 + q.iw) * 64 + col];
    // (row is a multiple of 4 and row + 3 < bg2_ld: the four samples' bytes are one aligned dword)
#if !QLX_BG2_POST
    pr.bg = pbg ? *reinterpret_cast<const uint32_t*>(bg2 + (size_t)(q.ih * 9 + q.iw) * bg2_ld + row) : 0u;
#endif
    return pr;
  }
  __device__ void epi_post(int z, int row, int col, f32x4 v, const Pre& pr0) const {
    const Px q = px(z);
    Pre pr = pr0;
#if QLX_BG2_POST   // (the background bytes loaded in the epilogue: no register held across the slab loop)
    pr.bg = pbg ? *reinterpret_cast<const uint32_t*>(bg2 + (size_t)(q.ih * 9 + q.iw) * bg2_ld + row) : 0u;
#endif
    float d[4], e[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      d[r] = row + r < B && pr.m[r] > 0.0f ? v[r] : 0.0f;
      e[r] = ((pr.bg >> (8 * r)) & 0xFFu) != 0u ? d[r] : 0.0f;
      if (row + r < B) dz2[((size_t)((row + r) * 9 + q.ih) * 9 + q.iw) * 64 + col] = d[r];
    }
    if (pbg) {   // (uniform: every lane of the wave takes part in the exchanges)
      const float s = pb_sum16(e);
      if ((row & 15) == 0 && row < B) pbg[((size_t)(row >> 4) * 81 + q.ih * 9 + q.iw) * 64 + col] = s;
    }
  }
  // streams (gemm_body_s, gemm_body_chain): dz3 rows of the tile's samples (rows past B read zeros), W2 rows of the tile's
  // channels; a slab's pixel tap (kh, kw) and oc half are wave-uniform offsets (per sub-tile z in a chained group)
  static constexpr int T = WM_ * WN_ * 64;
  struct Streams {
    AffineStream<BM_, false, T> a;
    AffineStream<BN_, false, T> b;
    struct Regs {
      typename AffineStream<BM_, false, T>::Regs a;
      typename AffineStream<BN_, false, T>::Regs b;
    };
    int z0;   // (gemm_body_s: the tile's pixel)
    __device__ void load(int s, Regs& x) const { load_z(z0, s, x); }
    __device__ void load_z(int z, int s, Regs& x) const {
      const Px q = px(z);
      const int t = s >> 1, kh = q.kh0 + t / q.nkw, kw = q.kw0 + t % q.nkw, h = (s & 1) * 32;
      a.load((uint32_t)(((q.ih - kh) * 7 + q.iw - kw) * 64 + h) * 4u, 0, x.a);
      b.load((uint32_t)((kh * 3 + kw) * 4096 + h) * 4u, 0, x.b);
    }
    __device__ void store(float* as, float* bs, const Regs& x) const {
      a.store(as, x.a);
      b.store(bs, x.b);
    }
  };
  __device__ Streams streams(int z, int row0, int col0, int tid) const {
    Streams st;
    st.z0 = z;
    const int nb = B;
    st.a.init(dz3, (uint32_t)B * 3136u * 4u, tid,
              [row0, nb](int r, int k) { return row0 + r < nb ? (uint32_t)((row0 + r) * 3136 + k) * 4u : kOob; });
    st.b.init(w2, 9u * 4096u * 4u, tid, [col0](int r, int k) { return (uint32_t)((col0 + r) * 64 + k) * 4u; });
    return st;
  }
};

// conv2 backward-data, pixel-major over the class grid: z = (i, j) of 10 x 10; rows b; cols (py, px, c) = 128 (the four
// output parity classes share the A operand: dz2[b][i - th][j - tw]); k = valid (th, tw) x oc, which is the valid
// (kh = py + 2 th, kw = px + 2 tw, oc) lexicographic order of every class
template <int BM_ = 32, int BN_ = 128, int WM_ = 2, int WN_ = 2, bool DIRECT = false>
struct PConv2DgradPx {
  static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_;
  static constexpr bool LOAD_FENCE = false;   // (stream core, in place: conv2 pair -1.0 us without it, gpurun_out/w18)
  static constexpr bool A_KMAJ = false, B_KMAJ = false, BIAS = false, RAW_ORDER = true;
  Grid g;             // {ceil(B / BM), 128 / BN, 100}
  const float* dz2;   // [B][9][9][64]
  const float* w1;    // [4][4][32][64]
  const float* a1;
  float* dz1;         // [B][20][20][32]
  int B;
  // conv1's bias partials [ceil(B / 16)][20][20][32] (null: none): per 16-sample row group g16 and position,
  // (Q0 + Q1) + (Q2 + Q3), Qg = ((d0 + d1) + d2) + d3 over samples 16 g16 + 4 g .. + 3 of the stored dz1 (0 past B) -
  // the lane's four rows, then its partners in lane groups g ^ 1 and g ^ 2 (k_conv1_wgrad32 chains them)
  float* pb = nullptr;
  // the forward's conv1 step bits as bytes [100][need_ld] (c1_steps; null: every row): dz1 rows of a clear step are not
  // stored - no wave of k_conv1_wgrad32 multiplies them and it does not fetch them (their bias share is in pb all the same)
  const uint8_t* need = nullptr;
  int need_ld = 0;
  __host__ __device__ void decode(int lb, int& tm, int& tn, int& z) const { g.decode(lb, tm, tn, z); }
  struct Px {
    int i, j, th0, tw0, ntw, ntap;
  };
  struct Pre {
    f32x4 m;       // a1 of the four rows (the ReLU mask)
    uint32_t nb;   // their step bytes
  };
  __host__ __device__ static Px px(int z) {
    Px q;
    q.i = DIRECT ? z / 10 : px2_order(z / 10);   // DIRECT: z = i * 10 + j
    q.j = DIRECT ? z % 10 : px2_order(z % 10);
    q.th0 = q.i == 9 ? 1 : 0;
    q.tw0 = q.j == 9 ? 1 : 0;
    const int th1 = q.i == 0 ? 0 : 1, tw1 = q.j == 0 ? 0 : 1;
    q.ntw = tw1 - q.tw0 + 1;
    q.ntap = (th1 - q.th0 + 1) * q.ntw;
    return q;
  }
  __host__ __device__ int nslabs(int z) const { return 2 * px(z).ntap; }
  __device__ f32x4 ldA(int z, int s, int row, int k) const {
    const Px q = px(z);
    const int t = s >> 1, th = q.th0 + t / q.ntw, tw = q.tw0 + t % q.ntw;
    return ld4m(dz2 + ((size_t)((row < B ? row : 0) * 9 + q.i - th) * 9 + q.j - tw) * 64 + (s & 1) * 32 + k, row < B);
  }
  __device__ f32x4 ldB(int z, int s, int col, int k) const {   // W1[kh][kw][c][oc], col = (py, px, c)
    const Px q = px(z);
    const int t = s >> 1, th = q.th0 + t / q.ntw, tw = q.tw0 + t % q.ntw;
    const int cls = col >> 5, kh = (cls >> 1) + 2 * th, kw = (cls & 1) + 2 * tw;
    return ld4(w1 + ((size_t)(kh * 4 + kw) * 32 + (col & 31)) * 64 + (s & 1) * 32 + k);
  }
  __device__ void epi(int z, int row, int col, f32x4 v) const { epi_post(z, row, col, v, epi_pre(z, row, col)); }
  __device__ Pre epi_pre(int z, int row, int col) const {
    const Px q = px(z);
    const int cls = col >> 5, ih = 2 * q.i + (cls >> 1), iw = 2 * q.j + (cls & 1);
    Pre pr;
#pragma unroll
    for (int r = 0; r < 4; ++r) pr.m[r] = a1[((size_t)((row + r < B ? row + r : 0) * 20 + ih) * 20 + iw) * 32 + (col & 31)];
    // (row is a multiple of 4 and row + 3 < need_ld: the four samples' bytes are one aligned dword)
    pr.nb = need ? *reinterpret_cast<const uint32_t*>(need + (size_t)((ih * 20 + iw) >> 2) * need_ld + row) : ~0u;
    return pr;
  }
  __device__ void epi_post(int z, int row, int col, f32x4 v, const Pre& pr) const {
    const Px q = px(z);
    const int cls = col >> 5, ih = 2 * q.i + (cls >> 1), iw = 2 * q.j + (cls & 1);
    float d[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      d[r] = row + r < B && pr.m[r] > 0.0f ? v[r] : 0.0f;
      if (row + r < B && ((pr.nb >> (8 * r)) & 0xFFu) != 0u) dz1[((size_t)((row + r) * 20 + ih) * 20 + iw) * 32 + (col & 31)] = d[r];
    }
    if (pb) {   // (uniform: every lane of the wave takes part in the exchanges)
      const float s = pb_sum16(d);
      if ((row & 15) == 0 && row < B) pb[((size_t)(row >> 4) * 400 + ih * 20 + iw) * 32 + (col & 31)] = s;
    }
  }
  // streams (gemm_body_s): A = dz2 rows of the tile's samples (rows past B read zeros), B = W1 rows of the tile's class
  // channels; a slab's tap (th, tw) and oc half are wave-uniform offsets
  static constexpr int T = WM_ * WN_ * 64;
  struct Streams {
    AffineStream<BM_, false, T> a;
    AffineStream<BN_, false, T> b;
    Px q;
    struct Regs {
      typename AffineStream<BM_, false, T>::Regs a;
      typename AffineStream<BN_, false, T>::Regs b;
    };
    __device__ void load_z(int z, int s, Regs& x) const {   // (chained sub-tiles, PConv2DgradPxG)
      Streams o = *this;
      o.q = px(z);
      o.load(s, x);
    }
    __device__ void load(int s, Regs& x) const {
      const int t = s >> 1, th = q.th0 + t / q.ntw, tw = q.tw0 + t % q.ntw, h = (s & 1) * 32;
      a.load((uint32_t)(((q.i - th) * 9 + q.j - tw) * 64 + h) * 4u, 0, x.a);
      b.load((uint32_t)((8 * th + 2 * tw) * 2048 + h) * 4u, 0, x.b);
    }
    __device__ void store(float* as, float* bs, const Regs& x) const {
      a.store(as, x.a);
      b.store(bs, x.b);
    }
  };
  __device__ Streams streams(int z, int row0, int col0, int tid) const {
    Streams st;
    st.q = px(z);
    const int nb = B;
    st.a.init(dz2, (uint32_t)B * 5184u * 4u, tid,
              [row0, nb](int r, int k) { return row0 + r < nb ? (uint32_t)((row0 + r) * 5184 + k) * 4u : kOob; });
    st.b.init(w1, 16u * 32u * 64u * 4u, tid, [col0](int r, int k) {
      const int col = col0 + r, cls = col >> 5;
      return (uint32_t)((((cls >> 1) * 4 + (cls & 1)) * 32 + (col & 31)) * 64 + k) * 4u;
    });
    return st;
  }
};

// Pixel-major backward data with balanced pixel groups (chained sub-tiles, gemm_body_chain): a block runs a group of
// pixels whose valid taps add up to a full tile's - conv3: 9 taps (interior pixels alone; a 6-tap edge pixel with its
// 3-tap neighbour; per corner quadrant the 4 + 2 + 2 + 1 taps), 49 groups of 18 slabs; conv2: 4 taps over the 10 x 10 class
// grid (interior alone; 2-tap edge pixels in pairs; the four 1-tap corners together), 81 groups of 8 slabs.  Every pixel
// keeps its own chain (valid taps lexicographic), so dz is bit-identical to the one-pixel tiles.
template <int BM_ = 32, int BN_ = 64, int WM_ = 2, int WN_ = 2>
struct PConv3DgradPxG : PConv3DgradPx<BM_, BN_, WM_, WN_, true> {
  static constexpr int NSUB = 4, GROUPS = 49;
  static constexpr bool RAW_ORDER = false;   // groups are equal: XCD-grouped order (a group's tiles share W2 taps in L2)
  __host__ __device__ static int sub_count(int g) { return g < 25 ? 1 : (g < 45 ? 2 : 4); }
  __host__ __device__ static int sub_z(int g, int i) {
    int ih, iw;
    if (g < 25) {
      ih = 2 + g / 5; iw = 2 + g % 5;
    } else if (g < 35) {   // (ih, 1) + (ih, 0) or (ih, 7) + (ih, 8)
      const int t = g - 25;
      ih = 2 + t / 2;
      iw = (t & 1) ? 7 + i : 1 - i;
    } else if (g < 45) {   // (1, iw) + (0, iw) or (7, iw) + (8, iw)
      const int t = g - 35;
      iw = 2 + t / 2;
      ih = (t & 1) ? 7 + i : 1 - i;
    } else {               // quadrant (a, b), (edge, b), (a, edge), (edge, edge)
      const int q = g - 45, a = (q & 2) ? 7 : 1, b = (q & 1) ? 7 : 1;
      ih = (i & 1) ? (a == 1 ? 0 : 8) : a;
      iw = (i & 2) ? (b == 1 ? 0 : 8) : b;
    }
    return ih * 9 + iw;
  }
};
template <int BM_ = 64, int BN_ = 64, int WM_ = 2, int WN_ = 2>
struct PConv2DgradPxG : PConv2DgradPx<BM_, BN_, WM_, WN_, true> {
  static constexpr int NSUB = 4, GROUPS = 81;
  static constexpr bool RAW_ORDER = false;
  __host__ __device__ static int sub_count(int g) { return g < 64 ? 1 : (g < 80 ? 2 : 4); }
  __host__ __device__ static int sub_z(int g, int i) {
    int ci, cj;
    if (g < 64) {
      ci = 1 + g / 8; cj = 1 + g % 8;
    } else if (g < 80) {
      const int t = g - 64, u = t >> 1, side = t & 1;
      if (u < 4) { ci = side ? 9 : 0; cj = 1 + 2 * u + i; }
      else { cj = side ? 9 : 0; ci = 1 + 2 * (u - 4) + i; }
    } else {
      ci = (i & 2) ? 9 : 0; cj = (i & 1) ? 9 : 0;
    }
    return ci * 10 + cj;
  }
};

// conv2 backward-data, all four parity classes in one GEMM: rows (b, i, j) of the 10 x 10 class grid, cols (py, px, c),
// k = (th, tw, oc) with zero taps (the row-major form of PConv2DgradPx)
template <int BM_ = 64, int BN_ = 128, int WM_ = 2, int WN_ = 2>
struct PConv2DgradAll {
  static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_;
  static constexpr bool A_KMAJ = false, B_KMAJ = false, BIAS = false;
  Grid g;             // {ceil(100 B / BM), 128 / BN, 1}
  const float* dz2;
  const float* w1;
  const float* a1;
  float* dz1;
  int M;              // B * 100
  __host__ __device__ void decode(int lb, int& tm, int& tn, int& z) const { g.decode(lb, tm, tn, z); }
  __host__ __device__ int nslabs(int) const { return 8; }
  __device__ f32x4 ldA(int, int s, int row, int k) const {
    const int t = s >> 1, th = t >> 1, tw = t & 1;
    const int rr = row < M ? row : 0;
    const int b = rr / 100, p = rr - b * 100, i = p / 10, j = p - i * 10;
    const int oh = i - th, ow = j - tw;
    const bool ok = row < M && oh >= 0 && oh < 9 && ow >= 0 && ow < 9;
    return ld4m(dz2 + (ok ? ((size_t)(b * 9 + oh) * 9 + ow) * 64 + (s & 1) * 32 + k : 0), ok);
  }
  __device__ f32x4 ldB(int, int s, int col, int k) const {
    const int t = s >> 1, cls = col >> 5, kh = (cls >> 1) + 2 * (t >> 1), kw = (cls & 1) + 2 * (t & 1);
    return ld4(w1 + ((size_t)(kh * 4 + kw) * 32 + (col & 31)) * 64 + (s & 1) * 32 + k);
  }
  __device__ void epi(int, int row, int col, f32x4 v) const {
    const int cls = col >> 5;
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (row + r < M) {
        const int rr = row + r, b = rr / 100, p = rr - b * 100, i = p / 10, j = p - i * 10;
        const size_t o = ((size_t)(b * 20 + 2 * i + (cls >> 1)) * 20 + 2 * j + (cls & 1)) * 32 + (col & 31);
        dz1[o] = a1[o] > 0.0f ? v[r] : 0.0f;
      }
  }
};

// conv2 backward-data by output parity class z = (py, px): rows (b, i, j) with ih = 2 i + py, iw = 2 j + px
// (10 x 10 per class); taps t = (th, tw): kh = py + 2 th, kw = px + 2 tw, source dz2[b][i - th][j - tw];
// k = (t, oc): the valid taps of the lexicographic (kh, kw, oc) order
template <int BM_ = 128, int BN_ = 32, int WM_ = 4, int WN_ = 1, int MF_ = 16>
struct PConv2DgradT {
  static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_, MF = MF_;
  static constexpr bool A_KMAJ = false, B_KMAJ = false, BIAS = false;
  Grid g;
  const float* dz2;   // [B][9][9][64]
  const float* w1;    // [4][4][32][64]
  const float* a1;
  float* dz1;         // [B][20][20][32]
  int M;              // B * 100
  __host__ __device__ void decode(int lb, int& tm, int& tn, int& z) const { g.decode(lb, tm, tn, z); }
  __host__ __device__ int nslabs(int) const { return 8; }
  __device__ f32x4 ldA(int z, int s, int row, int k) const {
    const int t = s >> 1, th = t >> 1, tw = t & 1, oc0 = (s & 1) * 32;
    const int rr = row < M ? row : 0;
    const int b = rr / 100, p = rr - b * 100, i = p / 10, j = p - i * 10;
    const int oh = i - th, ow = j - tw;
    const bool ok = row < M && oh >= 0 && oh < 9 && ow >= 0 && ow < 9;
    (void)z;
    return ld4m(dz2 + (ok ? ((size_t)(b * 9 + oh) * 9 + ow) * 64 + oc0 + k : 0), ok);
  }
  __device__ f32x4 ldB(int z, int s, int col, int k) const {   // W1[kh][kw][c = col][oc]
    const int t = s >> 1, kh = (z >> 1) + 2 * (t >> 1), kw = (z & 1) + 2 * (t & 1);
    return ld4(w1 + ((size_t)(kh * 4 + kw) * 32 + col) * 64 + (s & 1) * 32 + k);
  }
  __device__ void epi(int z, int row, int col, f32x4 v) const {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (row + r < M) {
        const int rr = row + r, b = rr / 100, p = rr - b * 100, i = p / 10, j = p - i * 10;
        const int ih = 2 * i + (z >> 1), iw = 2 * j + (z & 1);
        const size_t o = ((size_t)(b * 20 + ih) * 20 + iw) * 32 + col;
        dz1[o] = a1[o] > 0.0f ? v[r] : 0.0f;
      }
  }
};
using PConv2Dgrad = PConv2DgradT<>;
using PConv2DgradS = PConv2DgradT<64, 32, 4, 1>;

// conv2 / conv3 weight gradient over sample chunk z (samples [z SC, min(B, (z + 1) SC))): rows m = (kh, kw, c),
// cols oc, r = (b, oh, ow) ascending; partial slab[z][M + 1][OC] (row M = bias partial)
// CMP (round 6, conv2): the reduction runs over the chunk's non-background rows only (rows: the forward's row flags,
// c1_flags), in order; a background row's im2col row is the constant u (relu(b0) per channel, the forward's xbg), so
// its share u[m] dz[r][oc] is taken as u[m] S[oc] with S the chunk's background-row dz sum (SideBgSum), in the
// weight-gradient reduction (k_wreduce32): slab[z][m][oc] + u[m] S[z][oc] per chunk.  The table entries
// pack the im2col row offset from the chunk's first sample (bits 0..19) and the chunk row r (bits 20..31), which
// addresses the dz row: one table for both streams.
template <int H, int W, int C, int KS, int S, int OH, int OW, int OC, int SC, int BM_ = 64, int BN_ = 64, int WM_ = 2, int WN_ = 2,
          int MF_ = 16, bool TPADS = true, bool CMP = false>
struct PConvWgrad {
  static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_, MF = MF_;
  static constexpr bool LOAD_FENCE = false;   // (with the conv2 backward data's: conv2 pair 101.3 -> 99.8 us, w18)
  // (XCD-grouped block order kept: hardware order measured conv2 / conv3 pairs +2.3 / +1.0 us, w19)
  static constexpr bool A_KMAJ = true, B_KMAJ = true, BIAS = true;
  static constexpr int MROWS = KS * KS * C, P = OH * OW, CHUNK = SC;
  Grid g;
  const float* in;
  const float* dz;   // [B][OH][OW][OC]
  float* slab;
  int B;
  const uint32_t* rows = nullptr;   // CMP: the samples' non-background row bits [B][4]
  __host__ __device__ void decode(int lb, int& tm, int& tn, int& z) const { g.decode(lb, tm, tn, z); }
  __host__ __device__ int rows_in(int z) const {
    const int b0 = z * SC, b1 = b0 + SC < B ? b0 + SC : B;
    return (b1 - b0) * P;
  }
  static_assert(!CMP || (P <= 96 && SC * P <= 4096 && (size_t)SC * H * W * C * 4 <= 0xFFFFFu - 4 * KS * W * C),
                "compacted weight gradient: packed table entries");
  __host__ __device__ int kept_in(int z) const {   // CMP: the chunk's non-background rows
    int n = 0;
    for (int bl = 0; bl < SC; ++bl) {
      const int b = z * SC + bl;
      if (b < B) n += __builtin_popcount(rows[(size_t)b * 4]) + __builtin_popcount(rows[(size_t)b * 4 + 1]) +
                      __builtin_popcount(rows[(size_t)b * 4 + 2]);
    }
    return n;
  }
  __host__ __device__ int nslabs(int z) const { return ((CMP ? kept_in(z) : rows_in(z)) + BK - 1) / BK; }
  __device__ f32x4 ldA(int z, int s, int row, int k) const {
    const int r0 = s * BK + k;
    const bool ok = r0 < rows_in(z);
    const int r = ok ? r0 : 0;
    const int tap = row / C, c = row - tap * C, kh = tap / KS, kw = tap - kh * KS;
    const int bl = r / P, p = r - bl * P, oh = p / OW, ow = p - oh * OW, b = z * SC + bl;
    return ld4m(in + ((size_t)(b * H + oh * S + kh) * W + ow * S + kw) * C + c, ok);
  }
  __device__ f32x4 ldB(int z, int s, int col, int k) const {
    const int r = s * BK + k;
    const bool ok = r < rows_in(z);
    return ld4m(dz + ((size_t)z * SC * P + (ok ? r : 0)) * OC + col, ok);
  }
  __device__ void epi(int z, int row, int col, f32x4 v) const {
#pragma unroll
    for (int r = 0; r < 4; ++r) slab[((size_t)z * (MROWS + 1) + row + r) * OC + col] = v[r];
  }
  __device__ void epi_bias(int z, int col, float v) const { slab[((size_t)z * (MROWS + 1) + MROWS) * OC + col] = v; }
  // streams (gemm_body_s): A = the im2col rows gathered through the tile's offset table (TableK4Stream: one entry per
  // reduction index r = (b, oh, ow) of the chunk), B = dz rows, affine in r; r past the chunk reads zeros
  static constexpr int T = WM_ * WN_ * 64;
  static constexpr int KMAX = (SC * P + BK - 1) / BK * BK;   // table entries: the chunk's r, padded to whole slabs
  struct StreamsImpl {
    TableK4Stream<T, TPADS> a;
    AffineStream<BN_, true, T, true> b;
    int z, rows;
    struct Regs {
      typename TableK4Stream<T, TPADS>::Regs a;
      typename AffineStream<BN_, true, T, true>::Regs b;
    };
    // the chunk's r -> byte offset of its im2col row base in `in` (kOob past the chunk)
    __device__ void prepare(float* lds, int ns) {
      uint32_t* t = reinterpret_cast<uint32_t*>(lds);
      for (int r = a.tid; r < ns * BK; r += T) {
        uint32_t o = kOob;
        if (r < rows) {
          const int bl = r / P, pp = r - bl * P, oh = pp / OW, ow = pp - oh * OW;
          o = (uint32_t)((((z * SC + bl) * H + oh * S) * W + ow * S) * C) * 4u;
        }
        t[TableK4Stream<T, TPADS>::slot(r)] = o;
      }
      a.tbl = t;
    }
    __device__ void load(int s, Regs& x) const {
      const int kbase = s * BK;
      a.load(kbase, x.a);
      b.load((uint32_t)kbase * OC * 4u, rows - kbase, x.b);
    }
    __device__ void store(float* as, float* bs, const Regs& x) const {
      a.store(as, x.a);
      b.store(bs, x.b);
    }
  };
  // CMP: both operands through one table of the chunk's non-background rows (entry = A offset | r << 20; all ones past them)
  using TA = TableK4Stream<T, TPADS, 0, 0xFFFFFu, 1u>;
  using TB = TableK4Stream<T, TPADS, 20, 0xFFFu, (uint32_t)OC * 4u>;
  struct StreamsCmp {
    TA a;
    TB b;
    int z;
    const uint32_t* rows;
    int B;
    struct Regs {
      typename TA::Regs a;
      typename TB::Regs b;
    };
    __device__ void prepare(float* lds, int ns) {
      uint32_t* t = reinterpret_cast<uint32_t*>(lds);
      int run = 0;   // kept rows of the samples before bl (uniform)
      for (int bl = 0; bl < SC; ++bl) {
        const int b = z * SC + bl;
        if (b >= B) break;
        const uint32_t w0 = rows[(size_t)b * 4], w1 = rows[(size_t)b * 4 + 1], w2 = rows[(size_t)b * 4 + 2];
        for (int pp = a.tid; pp < P; pp += T) {
          const uint32_t w = pp < 32 ? w0 : (pp < 64 ? w1 : w2), bit = 1u << (pp & 31);
          if (w & bit) {
            const int below = (pp >= 32 ? __builtin_popcount(w0) : 0) + (pp >= 64 ? __builtin_popcount(w1) : 0) +
                              __builtin_popcount(w & (bit - 1u));
            const int oh = pp / OW, ow = pp - oh * OW;
            const uint32_t ao = (uint32_t)(((bl * H + oh * S) * W + ow * S) * C) * 4u;
            t[TA::slot(run + below)] = ao | ((uint32_t)(bl * P + pp) << 20);
          }
        }
        run += __builtin_popcount(w0) + __builtin_popcount(w1) + __builtin_popcount(w2);
      }
      for (int r = run + a.tid; r < ns * BK; r += T) t[TA::slot(r)] = 0xFFFFFFFFu;   // past both buffers under both maps
      a.tbl = t;
      b.tbl = t;
    }
    __device__ void load(int s, Regs& x) const {
      a.load(s * BK, x.a);
      b.load(s * BK, x.b);
    }
    __device__ void store(float* as, float* bs, const Regs& x) const {
      a.store(as, x.a);
      b.store(bs, x.b);
    }
  };
  // (the table stream stages 64-row tiles on four waves: other tile shapes keep the ldA / ldB core)
  // (in place against the ldA / ldB core: 262.3K vs 263.0K env-steps/s, conv2 pair 102.0 vs 102.2 us - neutral; kept as the
  // one path: the weight-gradient tiles then issue no per-slab address arithmetic)
  static constexpr bool STREAMED = BM_ == 64 && MF_ == 16 && WM_ * WN_ == 4;
  static_assert(!CMP || STREAMED, "compacted weight gradient: streamed tiles");
  using Streams = std::conditional_t<STREAMED, std::conditional_t<CMP, StreamsCmp, StreamsImpl>, void>;
  static_assert(!TPADS || KMAX <= 4 * 32 * 16, "weight-gradient chunk: the offset table lives in the four images' pads");
  // TableK4Stream::slot() places the table in the pad columns 64..79 of four 64-row KMAJ images (A and B, two buffers):
  // a B tile of another width would put it into B's live data
  static_assert(!STREAMED || !TPADS || BN_ == 64, "streamed weight-gradient tiles with the table in the pads need BN = 64");
  static constexpr size_t EXTRA_LDS = STREAMED && !TPADS ? (size_t)KMAX * 4 : 0;
  template <class ST = Streams>
  __device__ ST streams(int z, int row0, int col0, int tid) const {
    ST st;
    st.z = z;
    const int m = row0 + (tid & 15) * 4, tap = m / C, c = m - tap * C, kh = tap / KS, kw = tap - kh * KS;
    if constexpr (CMP) {
      st.rows = rows;
      st.B = B;
      const int nb = B - z * SC < SC ? B - z * SC : SC;   // the chunk's samples: its A and dz rows end the buffers
      st.a.init(in + (size_t)z * SC * H * W * C, (uint32_t)nb * H * W * C * 4u, tid, (uint32_t)((kh * W + kw) * C + c) * 4u);
      st.b.init(dz + (size_t)z * SC * P * OC, (uint32_t)nb * P * OC * 4u, tid, (uint32_t)(col0 + (tid & 15) * 4) * 4u);
    } else {
      st.rows = rows_in(z);
      st.a.init(in, (uint32_t)B * H * W * C * 4u, tid, (uint32_t)((kh * W + kw) * C + c) * 4u);
      st.b.init(dz + (size_t)z * SC * P * OC, (uint32_t)st.rows * OC * 4u, tid,
                [col0](int r, int k) { return (uint32_t)(k * OC + col0 + r) * 4u; });
    }
    return st;
  }
};

// dW4[k][n] = fmaf chain over b of a4[b][k] dq[b][n]; db4[n] = sum over b of dq[b][n]; loss = (sum over b of h_b) / B.
// Leading blocks of the fc1 backward launch (independent of its GEMM tiles), block t = one 16-row tile of the GEMM
// [a4^T ; 1] [dq | h] on v_mfma_f32_16x16x4_f32 (b on the lane groups, so each output is the b-ordered chain; the
// all-ones row 512 gives db4 and the loss sum, fmaf(1, v, s) = s + v).  Per HB samples the block's four waves load
// the tile's a4 columns and [dq | h] into LDS with every load in flight at once (40 KB),
// then wave 0 runs the chain from LDS: two memory latencies per launch instead of one per few MFMAs.
struct SideFc2 {
  static constexpr int BLOCKS = 33;   // 512 rows of a4^T + the ones row
  __host__ __device__ int blocks() const { return BLOCKS; }
  static constexpr int HB = 512;      // samples per LDS pass (40 KB; 256 measured slower: 73.4 vs 71.2 us per fc1 backward,
                                      // 61.9 vs 61.7 us on the stream core, gpurun_out/w23)
  static constexpr size_t LDS = (size_t)HB * 20 * sizeof(float);
  const float* a4;
  const uint8_t* act;
  const float* gs;
  const float* hs;
  int B;
  float* dw4;
  float* db4;
  float* loss;
  __device__ void run(int t, float* lds) const {
    float* as = lds;              // [HB][16] a4 columns t*16 .. +15
    float* ds = lds + HB * 16;    // [HB][4]  dq0, dq1, dq2, h
    const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, n = lane & 15;
    f32x4 acc = zero4();
    for (int b0 = 0; b0 < B; b0 += HB) {
      __syncthreads();   // the previous pass's LDS reads are done
      if (t < 32) {
#pragma unroll
        for (int j = 0; j < HB * 4 / 256; ++j) {   // HB x 4 float4: row bl = q / 4, quarter q % 4
          const int q = tid + 256 * j, bl = q >> 2, b = b0 + bl;
          f32x4 v = zero4();
          if (b < B) v = ld4(a4 + (size_t)b * 512 + t * 16 + (q & 3) * 4);
          *reinterpret_cast<f32x4*>(as + q * 4) = v;
        }
      }
#pragma unroll
      for (int j = 0; j < HB / 256; ++j) {
        const int bl = tid + 256 * j, b = b0 + bl;
        f32x4 v = zero4();
        if (b < B) {
          const int a = act[b];
          const float gv = gs[b];
          v = f32x4{a == 0 ? gv : 0.0f, a == 1 ? gv : 0.0f, a == 2 ? gv : 0.0f, hs[b]};
        }
        *reinterpret_cast<f32x4*>(ds + bl * 4) = v;
      }
      __syncthreads();
      if (tid < 64) {
        const int S = (min(HB, B - b0) + 3) / 4;   // zero rows past B leave the chains unchanged
#pragma unroll 8
        for (int s = 0; s < S; ++s) {
          const int bl = 4 * s + g;
          const float av = t < 32 ? as[bl * 16 + n] : (n == 0 ? 1.0f : 0.0f);
          const float bv = n < 4 ? ds[bl * 4 + n] : 0.0f;
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc, 0, 0, 0);
        }
      }
    }
    if (tid >= 64) return;
    if (t < 32) {
      if (n < 3)
#pragma unroll
        for (int i = 0; i < 4; ++i) dw4[(t * 16 + 4 * g + i) * 3 + n] = acc[i];
    } else if (g == 0) {
      if (n < 3) db4[n] = acc[0];
      else if (n == 3) *loss = acc[0] / (float)B;
    }
  }
};

#ifndef QLX_Q32_POLICIES_ONLY   // (scripts/q32_host_check.hip replays the policies on the host without the kernels)
// conv1 (8x8 stride 4, 4 -> 32 channels) from the u8 frames, one sample at a time per block with the sample's four
// frames staged in LDS while the next sample's frames are in flight in registers.
// LDS frame layout (rows): slot c, image row x, dword y / 4 holds pixels (x, y .. y + 3) at dword c * 1776 + x * 21 + y / 4.
// Rows of 21 dwords make 16 consecutive output positions (oh, ow) hit 16 consecutive banks (84 = 20 mod 64 dwords per
// oh step), and the slot stride 1,776 = 48 mod 64 puts the four slots (the MFMA lane groups) on disjoint bank ranges.
#ifndef QLX_C1_EXP
#define QLX_C1_EXP 0   // (timing experiments of the conv1 forward only, scripts/build_variant.sh: 1 no a1 stores, 2 no MFMA, 3 no list claims)
#endif
constexpr int kC1SlotDw = 1776;                 // 84 rows x 21 dwords + 12 (bank skew)
constexpr int kC1Frames = 4 * kC1SlotDw * 4;    // 28,416 B of one sample's frames in LDS
constexpr int kC1Chunks = 4 * kFramePix / 16;   // 1,764 s2d uint4 chunks in HBM

// 16 bytes (s2d chunk pos) of a frame from the table; a null entry reads the zero frame.  The load is a global load
// issued on every path: a load through a generic pointer compiles to a flat load, which also counts on lgkmcnt, so
// every LDS wait of the MFMA loop would wait for the next sample's frames too (and a branch around it makes the vmcnt
// bookkeeping conservative)
typedef const __attribute__((address_space(1))) uint8_t gbyte;
typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4v gu4;
__device__ __forceinline__ uint4 ldg_frame(const uint8_t* f, int pos) {
  gbyte* p = f ? (gbyte*)f + pos * 16 : (gbyte*)q32_zero4;   // the byte pointer is cast first, so the load is global
  const u32x4v v = *(gu4*)p;
  return uint4{v.x, v.y, v.z, v.w};
}

// The four frame pointers of sample b (b uniform across the block).  Read through the constant address space, so they
// are scalar loads: a vector load of a per-lane table entry makes every frame load wait for it with vmcnt(0), i.e. for
// every store and load still in flight (a whole sample's a1 stores in the forward), and serialises the prefetch branches
// behind one memory round trip each.
typedef const __attribute__((address_space(4))) unsigned long long cu64;
typedef const __attribute__((address_space(4))) uint32_t cu32;
struct C1Ptrs {
  const uint8_t* p[4];
};
__device__ __forceinline__ C1Ptrs c1_ptrs(const uint8_t* const* table, int b) {
  cu64* t = (cu64*)(table + (size_t)b * 4);
  return C1Ptrs{{(const uint8_t*)t[0], (const uint8_t*)t[1], (const uint8_t*)t[2], (const uint8_t*)t[3]}};
}
// (two levels of selects, so the per-lane choice stays v_cndmask and not a branch)
__device__ __forceinline__ const uint8_t* c1_slot(const C1Ptrs& f, int slot) {
  const uint8_t* lo = (slot & 1) ? f.p[1] : f.p[0];
  const uint8_t* hi = (slot & 1) ? f.p[3] : f.p[2];
  return (slot & 2) ? hi : lo;
}

// next sample's frames into registers (null table entry = the zero frame).  Every lane issues its loads (lanes past the
// frames read the zero page) with no branch around them: a load in a divergent branch makes the compiler wait for all
// loads in flight (vmcnt(0)) before the other path may reuse its registers.
__device__ __forceinline__ void c1_prefetch(const C1Ptrs& f, uint4 (&pf)[7]) {
#pragma unroll
  for (int j = 0; j < 7; ++j) {
    const int q = threadIdx.x + 256 * j;
    const bool ok = q < kC1Chunks;
    const int qq = ok ? q : 0, slot = qq / 441, pos = qq - slot * 441;
    pf[j] = ldg_frame(ok ? c1_slot(f, slot) : nullptr, pos);
  }
}
// s2d chunk (slot, block row bx, block column by) = pixels x = 4 bx + xl, y = 4 by .. 4 by + 3 in component xl
__device__ __forceinline__ void c1_put(uint32_t* dst, int q, const uint4& v) {
  const int slot = q / 441, pos = q - slot * 441, bx = pos / 21, by = pos - bx * 21;
  uint32_t* d = dst + slot * kC1SlotDw + 4 * bx * 21 + by;
  d[0] = v.x;
  d[21] = v.y;
  d[42] = v.z;
  d[63] = v.w;
}
__device__ __forceinline__ void c1_stage(uint32_t* dst, const uint4 (&pf)[7]) {
#pragma unroll
  for (int j = 0; j < 7; ++j) {
    const int q = threadIdx.x + 256 * j;
    if (q < kC1Chunks) c1_put(dst, q, pf[j]);
  }
}
__device__ __forceinline__ float ubyte(uint32_t w, int i) { return (float)((w >> (8 * i)) & 0xFFu); }

// Background rows.  A conv2 output position (i, j) sees the pixels x in [8 i, 8 i + 20), y in [8 j, 8 j + 20) of the four
// frames (conv1 positions 2 i .. 2 i + 3 of 8 x 8 pixels at stride 4); when they are all 0 (the black background), every
// conv1 output it reads is relu(0 + b0), so its input row is the same vector for every such position of every sample and
// its output is the same chain: one constant row c2.  A conv3 position (i, j) whose nine conv2 positions are all
// background (pixels [8 i, 8 i + 36)) likewise has the constant output c3.  So the conv2 / conv3 forward GEMMs run over
// the non-background rows only (PConvFwdL), and the background rows are written with c2 / c3 (BgRows).  Exact: the same
// chains on the same operands, whatever row a GEMM tile holds them in.
// The forward's conv1 kernel classifies each sample while its frames are staged: a 4 x 4 pixel block (one s2d chunk per
// frame) marks bit by of the row mask rm[bx] (21 x 21 blocks) when any of its bytes is non-zero, and a conv2 (conv3) row is
// background when the 5 x 5 (9 x 9) blocks from (2 i, 2 j) are unmarked.  Row lists (entries b * R + p, R = 81 / 49 rows
// per sample) in kListSlots regions, one per XCD (conv1 block g writes region g % kListSlots): a region's non-background rows from
// its front, its background rows from its back, their counts in the region's counter (non-background << 32 |
// background), claimed once per wave after the block's last sample.  One counter per XCD instead of one per list: the
// claims of all blocks arrive together at the end of the launch, and on one address they serialise (measured: +11.5 us
// on a 46 us conv1 launch at B = 1024).  The order of a region's entries varies between runs; the values do not.
struct C1Lists {
  int* rl2;                       // null: no lists (every row computed)
  int* rl3;
  int cap2, cap3;                 // rows per region
  unsigned long long* cnt;        // this forward's counters
  unsigned long long* cnt_next;   // the next forward's (double-buffered by forward parity), zeroed here
  float* xbg;                     // relu(0 + b0) [32]
  uint32_t* steps;                // null, or the samples' conv1 step masks [n][4] (c1_steps)
  uint8_t* need;                  // null, or the same bits as bytes [100][need_ld] (step-major: PConv2DgradPx::need)
  int need_ld;
  // null, or the samples' conv2 row flags (the row lists' classification, also without lists): rows2[n][4] the
  // non-background bits (words 0, 1: rows 0..63, word 2: rows 64..80), bg2[81][need_ld] background as bytes (row-major)
  uint32_t* rows2;
  uint8_t* bg2;
  uint32_t* rows3;                // the same for conv3's 49 rows: rows3[n][4] (words 0, 1), bg3[49][need_ld]
  uint8_t* bg3;
};
constexpr int kC1RmDw = 24;       // one row-mask buffer (21 dwords + pad); three buffers after the frames in LDS

// (the thread index is laundered through an empty asm per call, so the address arithmetic is redone per sample instead
// of being hoisted out of the sample loop into registers the MFMA loop needs: conv1 runs at the 256-VGPR limit)
__device__ __forceinline__ int c1_opaque_tid() {
  int t = threadIdx.x;
  asm volatile("" : "+v"(t));
  return t;
}
__device__ __forceinline__ void c1_mark(uint32_t* rm, const uint4 (&pf)[7]) {
  const int t = c1_opaque_tid();
#pragma unroll
  for (int j = 0; j < 7; ++j) {
    const int q = t + 256 * j;
    if (q < kC1Chunks && (pf[j].x | pf[j].y | pf[j].z | pf[j].w) != 0u) {
      const int pos = q % 441, bx = pos / 21, by = pos - bx * 21;
      atomicOr(&rm[bx], 1u << by);
    }
  }
}

// A sample's conv1 step mask (the weight gradient's 100 steps of 4 output positions r = 4 s .. 4 s + 3, all in row oh = s / 5,
// columns ow = 4 t .. 4 t + 3, t = s % 5): bit s is set when any of the four positions' 8 x 8 x 4 patches holds a non-zero
// byte, i.e. when a block of rows oh, oh + 1 and columns 4 t .. 4 t + 4 is marked.  Bits 100..127 are 0.  One wave: two
// ballots, stored by lanes 0..3 (vector stores).  A clear bit means every wave of k_conv1_wgrad32 skips the step, so its
// dz1 values are neither needed there nor (when the mask is given to the conv2 backward) stored.
__device__ __forceinline__ void c1_steps(const uint32_t* rm, uint32_t* out, uint8_t* need, int need_ld, int b, int lane) {
  bool nd[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int s = lane + 64 * h;
    const bool valid = s < 100;
    const int ss = valid ? s : 0, oh = ss / 5, t = ss - 5 * oh;
    nd[h] = valid && ((((rm[oh] | rm[oh + 1]) >> (4 * t)) & 0x1Fu) != 0u);
    if (need && valid) need[(size_t)s * need_ld + b] = nd[h] ? 1 : 0;
  }
  const unsigned long long m0 = __builtin_amdgcn_ballot_w64(nd[0]), m1 = __builtin_amdgcn_ballot_w64(nd[1]);
  if (lane < 4) {
    const unsigned long long m = lane < 2 ? m0 : m1;
    out[lane] = (uint32_t)(m >> (32 * (lane & 1)));
  }
}
// is step st (0..99) of the mask (lo = bits 0..63, hi = 64..127) set
__device__ __forceinline__ bool c1_step_set(unsigned long long lo, unsigned long long hi, int st) {
  return ((st < 64 ? lo >> st : hi >> (st - 64)) & 1ull) != 0ull;
}

// a sample's row flags, one wave's share (waves 0, 1: conv2 rows p = tid; wave 2: conv3 rows p = tid - 128), as two
// ballots (non-background / background rows) stored in LDS at the end of the sample's iteration; the list entries are
// claimed and written once per wave after the block's last sample (c1_lists_flush), so no atomic's round trip is waited
// for inside the sample loop
__device__ __forceinline__ void c1_flags(const uint32_t* rm, unsigned long long* cl, int wave, const C1Lists& L, int b) {
  const int tid = c1_opaque_tid();
  const int R = wave < 2 ? 81 : 49, p = wave < 2 ? tid : tid - 128;
  const bool valid = p < R;
  const int pp = valid ? p : 0;
  bool nonbg;
  if (wave < 2) {
    const int i = pp / 9, j = pp - 9 * i;
    uint32_t mm = 0;
#pragma unroll
    for (int r = 0; r < 5; ++r) mm |= rm[2 * i + r];
    nonbg = ((mm >> (2 * j)) & 0x1Fu) != 0u;
  } else {
    const int i = pp / 7, j = pp - 7 * i;
    uint32_t mm = 0;
#pragma unroll
    for (int r = 0; r < 9; ++r) mm |= rm[2 * i + r];
    nonbg = ((mm >> (2 * j)) & 0x1FFu) != 0u;
  }
  const unsigned long long bn = __builtin_amdgcn_ballot_w64(valid && nonbg), bb = __builtin_amdgcn_ballot_w64(valid && !nonbg);
  if ((tid & 63) == 0) {
    cl[0] = bn;
    cl[1] = bb;
  }
  if (wave < 2 && L.rows2) {   // (vector stores: lanes 0, 1 of waves 0, 1)
    const int lane = tid & 63;
    if (lane < 2 && (wave == 0 || lane == 0)) L.rows2[(size_t)b * 4 + 2 * wave + lane] = (uint32_t)(bn >> (32 * lane));
    if (wave == 1 && lane == 1) L.rows2[(size_t)b * 4 + 3] = 0u;
    if (valid) L.bg2[(size_t)p * L.need_ld + b] = nonbg ? 0 : 1;
  }
  if (wave == 2 && L.rows3) {
    const int lane = tid & 63;
    if (lane < 4) L.rows3[(size_t)b * 4 + lane] = lane < 2 ? (uint32_t)(bn >> (32 * lane)) : 0u;
    if (valid) L.bg3[(size_t)p * L.need_ld + b] = nonbg ? 0 : 1;
  }
}
// cl: [iteration][3 waves][2]; the block's samples b0, b0 + G, .. (nit of them)
// Called by every wave of the block (it holds a block barrier); waves 0..2 write.  One claim per layer and block: wave 0
// claims the conv2 rows of waves 0 and 1 together and hands wave 1 its start through LDS (xch), wave 2 claims the conv3
// rows (round 6: with one sample per block - k_conv1_fwd32 ONE - the claims doubled, and a claim per wave put 256 of them
// on each region's conv2 counter).
__device__ __forceinline__ void c1_lists_flush(const unsigned long long* cl, int nit, int b0, int G, const C1Lists& L, int wave,
                                               int tid, int B, unsigned long long* xch) {
  const int lane = tid & 63, R = wave < 2 ? 81 : 49, p = wave < 2 ? tid : tid - 128;
  int* rl = wave < 2 ? L.rl2 : L.rl3;
  auto wave_tot = [&](int wv) {   // (non-background << 32 | background) rows of wave wv's share over the block's samples
    unsigned long long t = 0;
    for (int it = 0; it < nit; ++it)
      t += ((unsigned long long)__builtin_popcountll(cl[(it * 3 + wv) * 2]) << 32) |
           (unsigned long long)__builtin_popcountll(cl[(it * 3 + wv) * 2 + 1]);
    return t;
  };
  unsigned long long old = 0;
  const int slot = blockIdx.x % kListSlots, cap = wave < 2 ? L.cap2 : L.cap3;
  rl += slot * cap;
#if QLX_C1_EXP == 3   // (timing experiment: no claim - every block writes a fixed, overlapping range; wrong lists)
  old = ((unsigned long long)((blockIdx.x / kListSlots) % 64) << 32) | (unsigned long long)((blockIdx.x / kListSlots) % 64);
  __syncthreads();
#else
  if ((wave == 0 || wave == 2) && lane == 0) {
    const unsigned long long tot = wave == 0 ? wave_tot(0) + wave_tot(1) : wave_tot(2);
    old = __hip_atomic_fetch_add(L.cnt + (slot * 2 + (wave < 2 ? 0 : 1)) * kCntStride, tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (wave == 0) *xch = old;
  }
  __syncthreads();
  if (wave == 1) old = *xch + wave_tot(0);   // wave 1's rows follow wave 0's in the claimed range
#endif
  if (wave >= 3) return;
  old = __shfl(old, 0);
  int on = (int)(old >> 32), og = (int)(uint32_t)old;
  const unsigned long long below = (1ull << lane) - 1ull;
  for (int it = 0; it < nit; ++it) {
    const unsigned long long bn = cl[(it * 3 + wave) * 2], bb = cl[(it * 3 + wave) * 2 + 1];
    const int e = (b0 + it * G) * R + p;
    int tap = 0;   // conv3 rows: the taps whose conv2 position is background (PConvFwdL SEL), bits 20..28 of the entry
    if (wave == 2) {
      const unsigned long long g0 = cl[(it * 3) * 2 + 1], g1 = cl[(it * 3 + 1) * 2 + 1];   // conv2 background, 0..63, 64..80
      const int i = p / 7, j = p - 7 * (p / 7);
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int q = (i + t / 3) * 9 + j + t % 3;
        tap |= (int)(((q < 64 ? g0 >> q : g1 >> (q - 64)) & 1ull) << t);
      }
    }
#ifdef QLX_LIST_CHECK
    {
      const int i1 = on + __builtin_popcountll(bn & below), i2 = cap - 1 - (og + __builtin_popcountll(bb & below));
      if ((((bn >> lane) & 1ull) && (i1 < 0 || i1 >= cap)) || (((bb >> lane) & 1ull) && (i2 < 0 || i2 >= cap)) || e >= B * R)
        printf("LISTCHK flush blk %d wave %d it %d e %d B %d i1 %d i2 %d cap %d\n", (int)blockIdx.x, wave, it, e, B, i1, i2, cap);
    }
#endif
    if ((bn >> lane) & 1ull) rl[on + __builtin_popcountll(bn & below)] = e | (tap << 20);
    else if ((bb >> lane) & 1ull) rl[cap - 1 - (og + __builtin_popcountll(bb & below))] = e;
    on += __builtin_popcountll(bn);
    og += __builtin_popcountll(bb);
  }
}

// One sample's conv1 forward in one wave (k_conv1_fwd32): its 12 / 13 patch tiles of 16 output channels from the frames fr
// staged in LDS; tile-outer: each tile's chain over (kq, kw) runs to completion and its four rows are stored before the
// next tile's chain, so the sample's a1 stores (51 KB) leave during its MFMAs instead of after the last one; the next
// tile's 16 frame dwords are read while this tile multiplies (against the kq-outer loop over all 13 accumulators: 49.1 ->
// 47.9 us at B = 1024, 320 -> 309 us per 8,192-sample chunk, 256 -> 218 VGPRs; gpurun_out/w4).  One branch per (kq, tile)
// with its four kw steps back to back (a branch per MFMA: 60 vs 46 us at C3)
struct C1NoHook {
  __device__ void operator()(int) const {}
};
// Hook (ONE, staged rows): called by every wave before its first tile of tile row R = 1 .. 4 (t / 5; every wave has tiles in
// every row), so it may hold a block barrier; the next tile's frame dwords are not read ahead across a row boundary
template <class Hook = C1NoHook>
__device__ __forceinline__ void c1_fwd_sample(const uint32_t* fr, const uint32_t (&ob2)[7], int nt, int rp, int g, int col,
                                              const float (&wf)[64], float bias, int skip, float* a1, int b,
                                              const Hook& hook = Hook{}) {
  constexpr bool HOOK = !std::is_same_v<Hook, C1NoHook>;
  {
    uint32_t dn[16];
    auto tile_dwords = [&](int j, uint32_t (&d)[16]) {
      const uint32_t base = (ob2[j >> 1] >> (16 * (j & 1))) & 0xFFFFu;
#pragma unroll
      for (int kq = 0; kq < 16; ++kq) d[kq] = fr[base + (kq >> 1) * 21 + (kq & 1)];   // (kh, kw half): pixels (4 oh + kh, 4 ow + 4 hw ..)
    };
    tile_dwords(0, dn);
#pragma unroll
    for (int j = 0; j < 13; ++j)
      if (j < nt) {
        if constexpr (HOOK) {
          const int row = (rp + 2 * j) / 5;
          if (j > 0 && row != (rp + 2 * (j - 1)) / 5) {   // (wave-uniform) the first tile of tile row `row`
            hook(row);
            tile_dwords(j, dn);
          }
        }
        uint32_t d[16];
#pragma unroll
        for (int kq = 0; kq < 16; ++kq) d[kq] = dn[kq];
        // the tile's 16 step masks are taken before the next tile's LDS reads are issued, so no branch merge of the MFMA
        // chain waits for those reads (masks interleaved with the chain: the compiler put lgkmcnt(0) at the merges, 48.2 vs
        // 46.7 us at B = 1024; with the short-circuit form of the mask, a branch per mask: 46.7 vs 42.7 us)
        bool nz[16];
#pragma unroll
        for (int kq = 0; kq < 16; ++kq) nz[kq] = (__builtin_amdgcn_ballot_w64(d[kq] != 0u) != 0) | (skip == 0);   // wave-uniform, no branch
        if (j + 1 < nt && (!HOOK || (rp + 2 * (j + 1)) / 5 == (rp + 2 * j) / 5)) tile_dwords(j + 1, dn);
        f32x4 acc = zero4();
#if QLX_C1_EXP != 2   // (timing experiments only: 2 = no MFMA, 1 = no a1 stores)
#pragma unroll
        for (int kq = 0; kq < 16; ++kq)
          if (nz[kq])
#pragma unroll
            for (int kw = 0; kw < 4; ++kw) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ubyte(d[kq], kw), wf[kq * 4 + kw], acc, 0, 0, 0);
#endif
        const int t = rp + 2 * j, r0 = (4 * (t / 5) + g) * 20 + 4 * (t % 5);   // rows (oh, ow .. ow + 3) of the patch
#if QLX_C1_EXP == 1
        if (acc[0] == 1234.5f)
#endif
#pragma unroll
        for (int i = 0; i < 4; ++i) a1[((size_t)b * 400 + r0 + i) * 32 + col] = relu(acc[i] + bias);
      }
  }
}

// forward: a1[b][r][oc] = relu(chain over k = (kh, kw, c) of x * W0[kh][kw][c][oc] + b0[oc]), r = (oh, ow).
// Wave w owns output channels (w & 1) * 16 .. + 15 and the tiles t = (w >> 1) + 2 j (13 / 12 of the 25); tile t is the
// 4 x 4 patch of output positions oh = 4 (t / 5) + 0..3, ow = 4 (t % 5) + 0..3 (tile row l = (oh % 4, ow % 4)); one
// v_mfma_f32_16x16x4_f32 per (tile, kh, kw) with c on the lane groups, W0 fragments resident in VGPRs.
// Zero steps (skip != 0): an MFMA whose 64 frame values are all 0 adds +-0 to each of its 16 x 16 chains, which leaves
// every chain as it is (a chain from +0 never holds -0: x + (-x) and +0 + -0 round to +0), so it is not issued.  The
// frames are mostly background (0), and a patch tile's receptive field (20 x 20 pixels per frame) is often all of it
// (~70 % of the steps at C3), where a tile of 16 consecutive positions crosses the side walls.  Exact for finite W0.
// ROLE only names the instantiation (0: training batches, 1: chunk-size target / acting passes), so a kernel trace
// tells the two launch shapes apart.
// ONE (round 6, the training batch): one sample per block, grid = B.  The persistent form (two blocks per CU, each block's
// samples in turn, the next sample's frames in flight in registers) holds 220 VGPRs and two frame buffers (57 KB), so a
// CU runs two samples at a time and a B = 1,024 batch is two samples deep per block: a sample's frame fetch, its
// 13-tile chains and its a1 stores follow each other.  One sample per block needs one frame buffer (28 KB) and no prefetch
// registers, so 4 blocks share a CU and all of a CU's samples run at once (VGPRs held to 128 by the launch bound).
#ifndef QLX_C1_ROWS
#define QLX_C1_ROWS 0   // ONE: stage the frames by tile rows (measured slower, round 6: 37.2 -> 48.1 us at B = 1024 - the four
                        // row barriers cost more than the overlap wins, and the live load registers spill at 4 waves / SIMD)
#endif
#ifndef QLX_C1_ONE_MINW
#define QLX_C1_ONE_MINW 4
#endif
template <int ROLE, bool ONE = false>
__global__ __launch_bounds__(256, ONE ? QLX_C1_ONE_MINW : 2) void k_conv1_fwd32(const uint8_t* const* table, int B, const float* w0,
                                                                           const float* b0, float* a1, int skip, const C1Lists L) {
  extern __shared__ __attribute__((aligned(16))) uint32_t c1w[];   // [2 (ONE: 1)][4 slots][1776 dwords], rm [3][24], flags
  uint32_t* rm = c1w + (ONE ? 1 : 2) * 4 * kC1SlotDw;
  unsigned long long* cl = reinterpret_cast<unsigned long long*>(rm + 3 * kC1RmDw);   // [iteration][3][2] (c1_flags)
  const bool lists = L.rl2 != nullptr;
  const bool marks = lists || L.rows2 != nullptr || L.rows3 != nullptr;   // the samples' row classification (lists, row flags, step masks)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (marks) {
    if (blockIdx.x == 0 && tid < 2 * kListSlots) L.cnt_next[tid * kCntStride] = 0ull;
    if (blockIdx.x == 0 && tid < 32) L.xbg[tid] = relu(0.0f + b0[tid]);   // conv2's constant input row
    if (tid < 3 * kC1RmDw) rm[tid] = 0u;
    __syncthreads();
  }
  const int ct = wave & 1, rp = wave >> 1;
  const int col = ct * 16 + (lane & 15), g = lane >> 4;
  float wf[64];
#pragma unroll
  for (int kk = 0; kk < 64; ++kk) wf[kk] = w0[(kk * 4 + g) * 32 + col];
  const float bias = b0[col];
  // dword offsets of the lane's 13 tile rows (lane group g reads ring slot g), two 16-bit offsets per register
  uint32_t ob2[7];
#pragma unroll
  for (int j = 0; j < 7; ++j) ob2[j] = 0;
#pragma unroll
  for (int j = 0; j < 13; ++j) {
    const int t = rp + 2 * j < 25 ? rp + 2 * j : 0, l = lane & 15;
    const int oh = 4 * (t / 5) + (l >> 2), ow = 4 * (t % 5) + (l & 3);
    ob2[j >> 1] |= (uint32_t)(g * kC1SlotDw + 4 * oh * 21 + ow) << (16 * (j & 1));
  }
  const int nt = rp == 0 ? 13 : 12;
  int b = blockIdx.x;
  if (b >= B) return;
  if constexpr (ONE) {
#if QLX_C1_ROWS
    // Staged by tile rows (round 6): the sample's 1,764 frame chunks in row order (block row bx, slot, block column by), a
    // thread's load j = chunk tid + 256 j; tile row R needs block rows <= 4 R + 4, i.e. loads j < 2, 3, 5, 6, 7 for R = 0..4.
    // Loads 0..2 are issued first and 0, 1 staged; the hook before row R stages what R needs and issues the loads row R + 1
    // needs, so the first tiles multiply while the later rows are in flight (all of a CU's blocks start together: with one
    // stage up front their fetches and their MFMAs did not overlap)
    const C1Ptrs f = c1_ptrs(table, b);
    uint4 pf[7];
    auto issue = [&](int j) {
      const int q = tid + 256 * j;
      const bool ok = q < kC1Chunks;
      const int qq = ok ? q : 0, bx = qq / 84, rem = qq - bx * 84, slot = rem / 21, by = rem - slot * 21;
      pf[j] = ldg_frame(ok ? c1_slot(f, slot) : nullptr, bx * 21 + by);
    };
    auto stage = [&](int j) {
      const int q = tid + 256 * j;
      if (q < kC1Chunks) {
        const int bx = q / 84, rem = q - bx * 84, slot = rem / 21, by = rem - slot * 21;
        c1_put(c1w, slot * 441 + bx * 21 + by, pf[j]);
        if (marks && (pf[j].x | pf[j].y | pf[j].z | pf[j].w) != 0u) atomicOr(&rm[bx], 1u << by);
      }
    };
    issue(0);
    issue(1);
    issue(2);
    stage(0);
    stage(1);
    __syncthreads();
    auto hook = [&](int R) {
      if (R == 1) { stage(2); issue(3); issue(4); }
      else if (R == 2) { stage(3); stage(4); issue(5); }
      else if (R == 3) { stage(5); issue(6); }
      else { stage(6); }
      __syncthreads();
    };
    c1_fwd_sample(c1w, ob2, nt, rp, g, col, wf, bias, skip, a1, b, hook);
#else
    {
      uint4 pf[7];
      c1_prefetch(c1_ptrs(table, b), pf);
      c1_stage(c1w, pf);
      if (marks) c1_mark(rm, pf);
    }
    __syncthreads();
    c1_fwd_sample(c1w, ob2, nt, rp, g, col, wf, bias, skip, a1, b);
#endif
    if (marks) {
      if (wave < 3) c1_flags(rm, cl + wave * 2, wave, L, b);
      else if (L.steps) c1_steps(rm, L.steps + (size_t)b * 4, L.need, L.need_ld, b, lane);
      if (lists) {
        __syncthreads();
        c1_lists_flush(cl, 1, blockIdx.x, gridDim.x, L, wave, tid, B, cl + 6);
      }
    }
    return;
  }
  uint4 pf[7];
  c1_prefetch(c1_ptrs(table, b), pf);
  // frame pointers one sample ahead of the frames (scalar registers)
  C1Ptrs nxt = c1_ptrs(table, b + (int)gridDim.x < B ? b + (int)gridDim.x : b);
  c1_stage(c1w, pf);
  if (marks) c1_mark(rm, pf);
  __syncthreads();
  for (int it = 0; b < B; b += gridDim.x, ++it) {
    const uint32_t* fr = c1w + (it & 1) * (4 * kC1SlotDw);
    const int nb = b + gridDim.x;
    if (nb < B) {
      c1_prefetch(nxt, pf);
      nxt = c1_ptrs(table, nb + (int)gridDim.x < B ? nb + (int)gridDim.x : nb);
    }
    // row masks: buffer it % 3 holds sample b's (complete since the last barrier, read by c1_flags at the end of this
    // iteration); (it + 1) % 3 gets the next sample's at the end of this iteration; (it + 2) % 3, read at the end of
    // it - 1, is cleared for it + 1
    if (marks && wave == 3 && tid - 192 < kC1RmDw) rm[((it + 2) % 3) * kC1RmDw + tid - 192] = 0u;
    c1_fwd_sample(fr, ob2, nt, rp, g, col, wf, bias, skip, a1, b);
    if (marks && wave < 3) c1_flags(rm + (it % 3) * kC1RmDw, cl + it * 6 + wave * 2, wave, L, b);
    if (marks && wave == 3 && L.steps) c1_steps(rm + (it % 3) * kC1RmDw, L.steps + (size_t)b * 4, L.need, L.need_ld, b, lane);
    if (nb < B) {
      c1_stage(c1w + ((it + 1) & 1) * (4 * kC1SlotDw), pf);
      if (marks) c1_mark(rm + ((it + 1) % 3) * kC1RmDw, pf);
    }
    __syncthreads();
  }
  if (lists) {
    const int nit = (B - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
    c1_lists_flush(cl, nit, blockIdx.x, gridDim.x, L, wave, tid, B, cl + nit * 6);
  }
}

// weight gradient over sample chunk z (SC samples): slab[z][m][oc] = chain over r = (b, oh, ow) ascending of
// x[r][m] dz1[r][oc] (steps whose frame values are all 0 skipped when skip != 0, exactly as in the forward; exact for
// finite dz1), m = (kh, kw, c) HWIO; bias slab[z][256][oc] = the chunk's share of the conv2 backward's bias partials
// (PConv2DgradPx::pb) as 16 chains combined in order, so only the dz1 rows of set steps (c1_steps: the rows
// some wave multiplies) are fetched - 27 % of them at C3 - when the forward's step masks are given.  One block per
// chunk, 8 waves: waves 0..3 cover output channels 0..15, waves 4..7 channels 16..31 (round 6: before, one block per
// (chunk, channel half) - both blocks fetched the chunk's frames, 29 of the launch's 110 MB).  Wave w owns kh = 2 (w % 4),
// 2 (w % 4) + 1: lane row rho = (kh low bit, h, c), tile t = kw - 4 h, so one LDS dword (pixels 4 ow + 4 h .. + 3 of image
// row 4 oh + kh) feeds the lane's four MFMAs of a step.  Per sample the frames (row layout, slot stride kC1WgSlotDw) and
// dz1 (all 32 channels) sit in LDS (79,488 B) while the next sample's are in flight in registers.
constexpr int kC1DzChunks = 400 * 32 / 4;   // 3,200 uint4 of one sample's dz1
// frame slot stride of the weight gradient's image: 1,768 = 8 mod 32 dwords puts the four slots of a step's 32-lane half
// (lane l % 4) on distinct banks (1,776 = 16 mod 32, the forward's, pairs slots 0 / 2 and 1 / 3: 2-way)
constexpr int kC1WgSlotDw = 1768;
constexpr int kC1WgradThreads = 512;
constexpr int kC1WgradPf = (kC1Chunks + kC1DzChunks + kC1WgradThreads - 1) / kC1WgradThreads;   // 10 uint4 per thread
constexpr size_t kC1WgradLds = (size_t)4 * kC1WgSlotDw * 4 + (size_t)400 * 32 * 4;          // 79,488 B
__host__ __device__ constexpr int c1_wgrad_blocks(int nz) { return nz; }
__global__ __launch_bounds__(kC1WgradThreads, 2) void k_conv1_wgrad32(const uint8_t* const* table, const float* dz1, int B, int nz,
                                                                       float* slab, int skip, const uint32_t* steps,
                                                                       const float* pb) {
  extern __shared__ __attribute__((aligned(16))) uint32_t c1w[];   // frames [4][1768] dwords, then dz [2 halves][400][16] f32
  float* dzs = reinterpret_cast<float*>(c1w + 4 * kC1WgSlotDw);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int z = blockIdx.x, hh = wave >> 2, wq = wave & 3;
  const int g = lane >> 4, l15 = lane & 15;
  const int b0 = z * QLX_F32_WGRAD_CHUNK_CONV1;
  const int nb = min(QLX_F32_WGRAD_CHUNK_CONV1, B - b0);
  // this lane's A row rho = l15: kh = 2 wq + rho / 8, h = (rho / 4) % 2, c = rho % 4; dword of (x = 4 oh + kh, y / 4 = ow + h)
  const int ao = (l15 & 3) * kC1WgSlotDw + (2 * wq + (l15 >> 3)) * 21 + ((l15 >> 2) & 1);
  const int bo = hh * 16 + l15;   // the lane's dz1 column
  // dz1 in LDS as two [400][16] channel halves: a step's reads (rows r, r + 1 on lane groups g, g + 1; 16 channels each) are
  // 32 consecutive dwords - conflict-free (a [400][32] image puts both rows on the same 16 banks: 2-way)

  // conv1's bias: this chunk's share of the partials pb (rows i = g16 * 400 + position, NR of them, R per chunk), 16
  // chains per channel (chain jb over rows i0 + jb, i0 + jb + 16, ..), combined in jb order at the end.
  // Issued first, four loads in flight per thread, so the chain waits for them only.
  const int boc = tid & 31, bjb = tid >> 5;
  float bt = 0.0f;
  {
    const int NR = ((B + 15) >> 4) * 400, R = (NR + nz - 1) / nz, i0 = z * R, i1 = min(NR, i0 + R);
    for (int i = i0 + bjb; i < i1; i += 64) {
      float v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = i + 16 * u < i1 ? pb[(size_t)(i + 16 * u) * 32 + boc] : 0.0f;
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (i + 16 * u < i1) bt = __fadd_rn(bt, v[u]);
    }
  }
  uint4 pf[kC1WgradPf];
  auto prefetch = [&](int b, uint4 (&pf)[kC1WgradPf]) {
    const C1Ptrs f = c1_ptrs(table, b);
    const uint64_t zp = (uint64_t)(gbyte*)q32_zero4;
    const uint64_t dzb = (uint64_t)(dz1 + (size_t)b * 400 * 32);
    // the sample's step mask (scalar loads; null: every step): a dz1 chunk of a clear step is not fetched - its LDS rows
    // get the zero page, and no wave multiplies them (c1_steps)
    unsigned long long lo = ~0ull, hi = ~0ull;
    if (steps) {
      cu32* sp = (cu32*)(steps + (size_t)b * 4);
      lo = (unsigned long long)sp[0] | ((unsigned long long)sp[1] << 32);
      hi = (unsigned long long)sp[2] | ((unsigned long long)sp[3] << 32);
    }
#pragma unroll
    for (int j = 0; j < kC1WgradPf; ++j) {   // one unconditional 16-byte load per j: a frame chunk, a dz1 chunk or the zero page
      const int q = tid + kC1WgradThreads * j;
      const bool isf = q < kC1Chunks, isd = !isf && q < kC1Chunks + kC1DzChunks;
      const int qf = isf ? q : 0, slot = qf / 441, pos = qf - slot * 441;
      const int e = isd ? q - kC1Chunks : 0;
      const uint64_t fp = (uint64_t)c1_slot(f, slot);
      const uint64_t fa = fp ? fp + (uint64_t)(pos * 16) : zp;
      const uint64_t da = c1_step_set(lo, hi, e >> 5) ? dzb + (uint64_t)e * 16 : zp;
      const u32x4v v = *(gu4*)(isf ? fa : (isd ? da : zp));
      pf[j] = uint4{v.x, v.y, v.z, v.w};
    }
  };
  auto stage = [&](const uint4 (&pf)[kC1WgradPf]) {
#pragma unroll
    for (int j = 0; j < kC1WgradPf; ++j) {
      const int q = tid + kC1WgradThreads * j;
      if (q < kC1Chunks) {
        const int slot = q / 441, pos = q - slot * 441, bx = pos / 21, by = pos - bx * 21;
        uint32_t* d = c1w + slot * kC1WgSlotDw + 4 * bx * 21 + by;
        d[0] = pf[j].x;
        d[21] = pf[j].y;
        d[42] = pf[j].z;
        d[63] = pf[j].w;
      } else if (q < kC1Chunks + kC1DzChunks) {
        const int e = q - kC1Chunks, r = e >> 3, part = e & 7;   // dz1[r][4 part .. 4 part + 3]
        *reinterpret_cast<uint4*>(dzs + (part >> 2) * 6400 + r * 16 + (part & 3) * 4) = pf[j];
      }
    }
  };
  f32x4 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = zero4();
  prefetch(b0, pf);
#pragma unroll
  for (int bl = 0; bl < QLX_F32_WGRAD_CHUNK_CONV1; ++bl) {
    if (bl >= nb) break;
    __syncthreads();   // the previous sample's LDS reads are done
    stage(pf);
    __syncthreads();
    if (bl + 1 < nb) prefetch(b0 + bl + 1, pf);
    // Operand groups of GS steps, software-pipelined: the next group's LDS reads are issued before this group's ballots and
    // MFMAs, and a group's ballots are all taken before its first branch, so no branch merge waits for a read in flight.  (In
    // the per-step form the compiler waits lgkmcnt(0) at every step's branch merge - one LDS round trip per step, 100 per
    // sample: 43.3 -> 39.2 us at B = 1024; groups of 2 / 10 / 25 / 50 steps: 51.5 / 40.1 / 68.5 / 123 us; branch-free
    // masks: 36.4 us.)  Same MFMAs on the same operands in the same order: bit-identical slabs.
    constexpr int GS = 5, NG = 100 / GS;
    static_assert(NG % 2 == 0 && NG * GS == 100, "conv1 weight gradient: operand groups");
    float bA[GS], bB[GS];
    uint32_t xA[GS], xB[GS];
    auto rd = [&](int grp, float (&bv)[GS], uint32_t (&px)[GS]) {
#pragma unroll
      for (int j = 0; j < GS; ++j) {
        const int r = 4 * (grp * GS + j) + g, oh = r / 20, ow = r - oh * 20;
        bv[j] = dzs[hh * 6400 + r * 16 + l15];
        px[j] = c1w[ao + 84 * oh + ow];
      }
    };
    auto run = [&](const float (&bv)[GS], const uint32_t (&px)[GS]) {
      bool nz[GS];
#pragma unroll
      for (int j = 0; j < GS; ++j) nz[j] = (__builtin_amdgcn_ballot_w64(px[j] != 0u) != 0) | (skip == 0);   // wave-uniform, no branch
#pragma unroll
      for (int j = 0; j < GS; ++j) {
        // all 64 x 4 frame values 0: the step adds +-0 (see the forward)
        if (nz[j])
#pragma unroll
          for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(ubyte(px[j], t), bv[j], acc[t], 0, 0, 0);
      }
    };
    rd(0, bA, xA);
    for (int grp = 0; grp < NG; grp += 2) {
      rd(grp + 1, bB, xB);
      run(bA, xA);
      if (grp + 2 < NG) rd(grp + 2, bA, xA);
      run(bB, xB);
    }
  }
  float* out = slab + (size_t)z * 257 * 32;
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) {   // output row rho = 4 g + i of tile t -> HWIO (kh, kw = 4 h + t, c)
      const int rho = 4 * g + i, kh = 2 * wq + (rho >> 3), kw = 4 * ((rho >> 2) & 1) + t, c = rho & 3;
      out[(size_t)((kh * 8 + kw) * 4 + c) * 32 + bo] = acc[t][i];
    }
  // bias row 256: the 16 chains in order, through the dz1 image (every wave is past its last step)
  __syncthreads();
  dzs[bjb * 32 + boc] = bt;
  __syncthreads();
  if (tid < 32) {
    float sb = 0.0f;
#pragma unroll
    for (int j = 0; j < 16; ++j) sb = __fadd_rn(sb, dzs[j * 32 + tid]);
    out[256 * 32 + tid] = sb;
  }
}

#endif  // QLX_Q32_POLICIES_ONLY

}  // namespace q32
}  // namespace qlx
