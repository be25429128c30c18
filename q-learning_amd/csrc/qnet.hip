// DeepQLearningModel on MI355X: Nature-DQN forward / backward / Huber / clip_by_norm / Adam.
//
// Reference (restated): create_ql_model_breakout_84x84x4_3_32.py:20-33 (graph), :36-55 (predict_action,
// batch_predict_max_future_reward), :63-82 (train_model; intended q_a = Q(s)[a] semantics of
// create_ql_model_ballgame_3x3x4_5_512.py:71-78), legacy keras Adam(lr 2.5e-4, clipnorm 1.0) =
// tf.clip_by_norm per variable + ResourceApplyAdam (saved_model.pb op names), Huber(delta=1) mean.
// The reference runs this inside libtensorflow behind Session::run (q_learning_model.rs:107-189).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <vector>

#include "objects.h"
#include "qnet.h"
#include "qnet_kernels.h"
#include "trunk_kernels.h"
#include "gemm_kernels.h"
#include "bgemm.h"
#include "profiler.h"

namespace qlx {

using namespace qn;

extern const int kVarSize[kNumVars];
const int kVarSize[kNumVars] = {8 * 8 * 4 * 32, 32, 4 * 4 * 32 * 64, 64, 3 * 3 * 64 * 64, 64, 3136 * 512, 512, 512 * 3, 3};
static int64_t var_offset(int v) {
  int64_t o = 0;
  for (int i = 0; i < v; ++i) o += kVarSize[i];
  return o;
}

static_assert(8 * 8 * 4 * 32 + 32 + 4 * 4 * 32 * 64 + 64 + 3 * 3 * 64 * 64 + 64 == kVarOffsetDense, "dense bucket offset");

// fused clip_by_norm partial slots per variable: conv W/b from the slab reduction blocks (64 outputs each),
// W3/b3 from the 25 x 4 fc1 wgrad tiles (each writes one W3 and one b3 slot), W4 from the 64 dW4 blocks
constexpr int kFc1WgradTiles = 25 * 4;
static const int kSqSlots[kNumVars] = {128, 1, 512, 1, 576, 1, kFc1WgradTiles, kFc1WgradTiles, 64, 1};
static int sq_first(int v) {
  int o = 0;
  for (int i = 0; i < v; ++i) o += kSqSlots[i];
  return o;
}

// tf.clip_by_norm + ResourceApplyAdam (legacy Keras) for one element
__device__ __forceinline__ float adam_elem(float g, float scale, float clipnorm, float denom, float alpha, float beta1,
                                           float beta2, float eps, float& m, float& v, float w) {
  // explicit roundings (no contraction): the same bits wherever this is inlined, and the oracle's order
  const float gc = (g * scale * clipnorm) / denom;
  m = __fadd_rn(m, __fmul_rn(__fsub_rn(gc, m), 1.0f - beta1));
  v = __fadd_rn(v, __fmul_rn(__fsub_rn(__fmul_rn(gc, gc), v), 1.0f - beta2));
  return __fsub_rn(w, __fmul_rn(m, alpha) / __fadd_rn(sqrtf(v), eps));
}

// ------------------------------------------------------------------------------------------
// weight packing: fp32 master (Keras layouts) -> bf16 MFMA operand layouts

__device__ __forceinline__ int conv1_s2d_k(int kh, int kw, int c) {
  const int i = kh >> 2, dx = kh & 3, j = kw >> 2, dy = kw & 3;
  return (((i * 2 + j) * 4 + c) * 16) + dx * 4 + dy;
}

struct PackPtrs {
  bf16 *wf0, *wf1, *wb1, *wf2, *wb2, *wb3;
};

// writes the bf16 copies of parameter element idx (global flat index) with value w; the conv operand copies
// are MFMA-fragment-major (frag_index), the dense one keeps the Keras [3136][512] layout
__device__ __forceinline__ void pack_one(const PackPtrs& P, int64_t idx, float w) {
  const bf16 v = (bf16)w;
  if (idx < 8192) {   // conv1 kernel [8][8][4][32]
    const int oc = idx & 31, c = (idx >> 5) & 3, kw = (idx >> 7) & 7, kh = (int)(idx >> 10);
    P.wf0[frag_index(oc, conv1_s2d_k(kh, kw, c), 256)] = v;
    return;
  }
  idx -= 8192 + 32;
  if (idx < 0) return;
  if (idx < 32768) {   // conv2 kernel [4][4][32][64]
    const int oc = idx & 63, c = (idx >> 6) & 31, tap = (int)(idx >> 11);   // tap = kh*4 + kw
    P.wf1[frag_index(oc, tap * 32 + c, 512)] = v;
    // backward data by parity class p = (kh&1)*2 + (kw&1): [p*32 + c][(kh>>1)*2 + (kw>>1)][oc]
    const int kh = tap >> 2, kw = tap & 3, p = (kh & 1) * 2 + (kw & 1);
    P.wb1[frag_index(p * 32 + c, ((kh >> 1) * 2 + (kw >> 1)) * 64 + oc, 256)] = v;
    return;
  }
  idx -= 32768 + 64;
  if (idx < 0) return;
  if (idx < 36864) {   // conv3 kernel [3][3][64][64]
    const int oc = idx & 63, c = (idx >> 6) & 63, tap = (int)(idx >> 12);  // tap = kh*3 + kw
    P.wf2[frag_index(oc, tap * 64 + c, 576)] = v;
    P.wb2[frag_index(c, tap * 64 + oc, 576)] = v;
    return;
  }
  idx -= 36864 + 64;
  if (idx < 0) return;
  if (idx < 3136 * 512) P.wb3[idx] = v;   // full_layer kernel [3136][512]: the Keras layout serves fwd and dgrad
}

__global__ void k_pack_all(const float* w, int64_t count, PackPtrs P) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (int64_t)gridDim.x * blockDim.x)
    pack_one(P, i, w[i]);
}

// ------------------------------------------------------------------------------------------
// host obs [B][x][y][slot] -> s2d frames [B*4][7056] + frame pointer table

__global__ void k_pack_obs(const uint8_t* obs, int B, uint8_t* frames) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;   // over B*84*84
  if (i >= (int64_t)B * kFramePix) return;
  const int b = (int)(i / kFramePix), xy = (int)(i - (int64_t)b * kFramePix);
  const int x = xy / kFrame, y = xy - x * kFrame;
  const uchar4 v = reinterpret_cast<const uchar4*>(obs)[i];
  const int off = s2d_offset(x, y);
  frames[((size_t)b * 4 + 0) * kFramePix + off] = v.x;
  frames[((size_t)b * 4 + 1) * kFramePix + off] = v.y;
  frames[((size_t)b * 4 + 2) * kFramePix + off] = v.z;
  frames[((size_t)b * 4 + 3) * kFramePix + off] = v.w;
}

__global__ void k_frame_table(const uint8_t* frames, int B, const uint8_t** table) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < B * 4) table[i] = frames + (size_t)i * kFramePix;
}

// ------------------------------------------------------------------------------------------
// dense 512 -> 3 (linear) on VALU, one wave per sample; optional heads:
//   mode 0: q only; mode 1: argmax actions (predict_action); mode 2: max -> Bellman target
//   (the training head with Huber + dq lives in k_fc2_train)


// this lane's 8 a4 values of sample b (k = 8 lane + e): straight from a4, or finished from the fc1 split-K
// partials (sum over z in order, + b3, ReLU, bf16 - the values k_slab_reduce_bias_relu would store)
__device__ __forceinline__ bf16x8 fc2_load_a4(const Fc2Args& A, int b, int lane) {
  if (A.splits == 0) return ld8(A.a4 + (size_t)b * 512 + lane * 8);
  const size_t i = (size_t)b * 512 + lane * 8;
  float4 s0 = {0.0f, 0.0f, 0.0f, 0.0f}, s1 = s0;
  for (int z = 0; z < A.splits; ++z) {
    const float4 u0 = *reinterpret_cast<const float4*>(A.slab + z * A.zstride + i);
    const float4 u1 = *reinterpret_cast<const float4*>(A.slab + z * A.zstride + i + 4);
    s0.x += u0.x; s0.y += u0.y; s0.z += u0.z; s0.w += u0.w;
    s1.x += u1.x; s1.y += u1.y; s1.z += u1.z; s1.w += u1.w;
  }
  const float4 c0 = *reinterpret_cast<const float4*>(A.b3 + lane * 8);
  const float4 c1 = *reinterpret_cast<const float4*>(A.b3 + lane * 8 + 4);
  const float t[8] = {s0.x + c0.x, s0.y + c0.y, s0.z + c0.z, s0.w + c0.w, s1.x + c1.x, s1.y + c1.y, s1.z + c1.z, s1.w + c1.w};
  bf16x8 v;
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = (bf16)(t[e] > 0.0f ? t[e] : 0.0f);
  *reinterpret_cast<bf16x8*>(A.a4_out + i) = v;
  return v;
}

template <int MODE>
__global__ __launch_bounds__(256) void k_fc2(Fc2Args A) {
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (b >= A.B) return;
  float s0 = 0.0f, s1 = 0.0f, s2 = 0.0f;
  const bf16x8 v = fc2_load_a4(A, b, lane);
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float x = (float)v[e];
    const float* w = A.w4 + (lane * 8 + e) * 3;
    s0 += x * w[0];
    s1 += x * w[1];
    s2 += x * w[2];
  }
  for (int off = 32; off > 0; off >>= 1) {
    s0 += __shfl_xor(s0, off);
    s1 += __shfl_xor(s1, off);
    s2 += __shfl_xor(s2, off);
  }
  if (lane != 0) return;
  const float q0 = s0 + A.b4[0], q1 = s1 + A.b4[1], q2 = s2 + A.b4[2];
  if (A.q) { A.q[b * 3 + 0] = q0; A.q[b * 3 + 1] = q1; A.q[b * 3 + 2] = q2; }
  if (MODE == 1) {   // tf.argmax: first maximal index
    int best = 0;
    float bv = q0;
    if (q1 > bv) { best = 1; bv = q1; }
    if (q2 > bv) { best = 2; }
    A.argmax[b] = (uint8_t)best;
  } else if (MODE == 2) {   // max_a Q_target(s') (or Q_target(s', argmax Q_online(s'))) -> r + v * gamma, or r if done
    float mx;
    if (A.q_select) {
      const float* qs = A.q_select + b * 3;
      int best = 0;
      float bv = qs[0];
      if (qs[1] > bv) { best = 1; bv = qs[1]; }
      if (qs[2] > bv) best = 2;
      mx = best == 0 ? q0 : (best == 1 ? q1 : q2);
    } else {
      mx = fmaxf(fmaxf(q0, q1), q2);
    }
    const float r = A.rewards[b];
    A.y_out[b] = A.dones[b] ? r : __fadd_rn(r, __fmul_rn(mx, A.gamma));   // two roundings, as the reference (add_arrays after array_mul)
  }
}

// Training head, one wave per sample: q = a4 W4 + b4, Huber(delta=1) of e = q_a - y (per-sample value and
// dloss/dq_a = clip(e, -1, 1) / B), and the backward into the dense-512 layer in the same wave:
// dz4[b][k] = g_b * W4[k][a_b] * (a4[b][k] > 0).  The xor butterfly leaves the full dot products in every
// lane, so each lane finishes its own 8 k.
__global__ __launch_bounds__(256) void k_fc2_train(Fc2Args A, bf16* dz4) {
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (b >= A.B) return;
  float s0 = 0.0f, s1 = 0.0f, s2 = 0.0f;
  const bf16x8 v = fc2_load_a4(A, b, lane);
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float x = (float)v[e];
    const float* w = A.w4 + (lane * 8 + e) * 3;
    s0 += x * w[0];
    s1 += x * w[1];
    s2 += x * w[2];
  }
  for (int off = 32; off > 0; off >>= 1) {
    s0 += __shfl_xor(s0, off);
    s1 += __shfl_xor(s1, off);
    s2 += __shfl_xor(s2, off);
  }
  const float q0 = s0 + A.b4[0], q1 = s1 + A.b4[1], q2 = s2 + A.b4[2];
  const int a = A.actions[b];
  const float qa = a == 0 ? q0 : (a == 1 ? q1 : q2);
  const float e = qa - A.y[b];
  const float ae = fabsf(e);
  const float wgt = A.weights ? A.weights[b] : 1.0f;   // prioritized replay: the IS weight scales h and dloss/dq
  const float g = (wgt * (ae <= 1.0f ? e : (e > 0.0f ? 1.0f : -1.0f))) / (float)A.B;
  if (lane == 0) {
    A.q[b * 3 + 0] = q0; A.q[b * 3 + 1] = q1; A.q[b * 3 + 2] = q2;
    A.hsample[b] = wgt * (ae <= 1.0f ? 0.5f * e * e : ae - 0.5f);
    A.gsample[b] = g;
    if (A.td_abs) A.td_abs[b] = ae;
  }
  bf16x8 d;
#pragma unroll
  for (int e8 = 0; e8 < 8; ++e8) d[e8] = (bf16)((float)v[e8] > 0.0f ? g * A.w4[(lane * 8 + e8) * 3 + a] : 0.0f);
  *reinterpret_cast<bf16x8*>(dz4 + (size_t)b * 512 + lane * 8) = d;
}

// dW4[k][a] = sum_b a4[b][k] g_b [a_b == a]: block j < 64 owns k = 8j .. 8j+7 and reads those 16 bytes of every
// a4 row once; block 64 sums db4[a] = sum_b g_b [a_b == a] and the loss = sum_b h_b / B.  Per-thread strided
// sums, an xor butterfly per wave, then the 4 wave sums in order: deterministic.  Runs as trailing blocks of
// the fc1 backward launch (k_fc1_bwd), overlapping its GEMM tiles.
struct Fc2WgradArgs {
  const bf16* a4;
  const uint8_t* actions;
  const float* gs;
  const float* hs;
  int B;
  float* g_w4;
  float* g_b4;
  float* loss;
  float* sq_w4;   // [64] square sums of each block's 24 dW4 values
  float* sq_b4;   // [1]
};
constexpr int kFc2WgradBlocks = 65;

template <int NT>
__device__ __forceinline__ void fc2_wgrad_block(const Fc2WgradArgs& A, int j, float* red /* LDS [NT / 64][24] + 24 */) {
  constexpr int NWV = NT / 64;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float s[24];
#pragma unroll
  for (int i = 0; i < 24; ++i) s[i] = 0.0f;
  if (j == 64) {
    for (int b = tid; b < A.B; b += NT) {
      const int a = A.actions[b];
      const float g = A.gs[b];
      s[0] += a == 0 ? g : 0.0f;
      s[1] += a == 1 ? g : 0.0f;
      s[2] += a == 2 ? g : 0.0f;
      s[3] += A.hs[b];
    }
  } else {
    const int k0 = j * 8;
    for (int b = tid; b < A.B; b += NT) {
      const bf16x8 x = ld8(A.a4 + (size_t)b * 512 + k0);
      const int a = A.actions[b];
      const float g = A.gs[b];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float v = (float)x[e] * g;
        s[e * 3 + 0] += a == 0 ? v : 0.0f;
        s[e * 3 + 1] += a == 1 ? v : 0.0f;
        s[e * 3 + 2] += a == 2 ? v : 0.0f;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 24; ++i)
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s[i] += __shfl_xor(s[i], off);
  if (lane == 0)
#pragma unroll
    for (int i = 0; i < 24; ++i) red[wave * 24 + i] = s[i];
  __syncthreads();
  float t = 0.0f;
  if (tid < 24) {
    t = red[tid];
    for (int w = 1; w < NWV; ++w) t += red[24 * w + tid];   // the wave sums in order
    if (j == 64) {
      if (tid < 3) A.g_b4[tid] = t;
      else if (tid == 3) *A.loss = t / (float)A.B;
    } else {
      A.g_w4[j * 24 + tid] = t;   // [k][a] with k = 8 j + tid / 3
    }
    red[24 * NWV + tid] = (j < 64 || tid < 3) ? t * t : 0.0f;
  }
  __syncthreads();
  if (tid == 0) {
    float q = 0.0f;
    for (int i = 0; i < 24; ++i) q += red[24 * NWV + i];
    if (j < 64) A.sq_w4[j] = q;
    else A.sq_b4[0] = q;
  }
}

// fc1 on the bf16 GEMM core (bgemm.h): the forward at the training batch in kFc1Split k splits (fp32 slabs the head
// reduces), at chunk batches (and for the target net, fc1_single) in one pass with bias + ReLU; the backward as one
// launch of the weight gradient (dW3 | db3 = a3^T dz4, 3137 x 512 x B), the backward data (dz3 = (dz4 W3^T) (a3 > 0),
// B x 3136 x 512) and the dense-3 weight gradient blocks.
// tiles and ring depths from scripts/ubench_bgemm.hip (gpurun_out/a4): forward at B = 1024 on 128 x 64 tiles in 4 k splits
// 8.7 us (128 x 128 in 7 splits: 9.6 us, and twice the slab bytes the head reads), backward data 9.1 us and weight
// gradient 12.5 us on 8-wave 128 x 128 tiles with 4 stages
using CfgFc1Fwd = BGemmCfg<128, 64, 2, 2, false, true, 4>;    // A = a3 (k = feature), B = W3 [3136][512] k-major
using CfgFc1FwdBig = BGemmCfg<128, 128, 2, 4, false, true, 4>;   // chunk batches (one pass, bias + ReLU)
using CfgFc1Wg = BGemmCfg<128, 128, 2, 4, true, true, 4>;     // A = a3 k-major (k = sample), B = dz4 k-major
using CfgFc1Dg = BGemmCfg<128, 128, 2, 4, false, false, 4>;   // A = dz4 (k = out), B = W3 (rows = in, k = out)
static_assert(CfgFc1Wg::T == CfgFc1Dg::T && CfgFc1Wg::LDS == CfgFc1Dg::LDS, "one block shape for the backward launch");
constexpr int kFc1BwdThreads = CfgFc1Wg::T;

// block b runs unit map[b] (weight-gradient tile, backward-data tile, then fc2 wgrad blocks; -1 = idle), see fc1_bwd_map
template <class E1, class E2>
__global__ __launch_bounds__(kFc1BwdThreads, 4) void k_fc1_bwd(BGemmProblem<E1> Pw, BGemmProblem<E2> Pd, Fc2WgradArgs F,
                                                               const int* map) {
  extern __shared__ __attribute__((aligned(16))) char fc1_lds[];
  const int t = map[blockIdx.x], tw = Pw.tiles(), tg = tw + Pd.tiles();
  if (t < 0) return;
  if (t < tw) bgemm_tile<CfgFc1Wg>(Pw, t, fc1_lds);
  else if (t < tg) bgemm_tile<CfgFc1Dg>(Pd, t - tw, fc1_lds);
  else fc2_wgrad_block<kFc1BwdThreads>(F, t - tg, reinterpret_cast<float*>(fc1_lds));
}

template <class Epi>
static BGemmProblem<Epi> bproblem(BOp A, BOp Bo, int M, int N, int K, int splits, int bm, int bn, Epi e, int ones_m = -1) {
  const int kps = ((K + splits - 1) / splits + 31) / 32 * 32;
  return BGemmProblem<Epi>{A, Bo, M, N, K, kps, ones_m, (M + bm - 1) / bm, (N + bn - 1) / bn, (K + kps - 1) / kps, 0, e};
}

// a3's pad columns: 1 at 3136 (the ones row of the weight gradient), 0 at 3137 .. kA3Ld - 1
__global__ void k_a3_pad(bf16* a3, int B) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;   // over B * 8
  if (i >= B * 8) return;
  const int b = i >> 3, c = 3136 + (i & 7);
  a3[(size_t)b * kA3Ld + c] = (bf16)(c == 3136 ? 1.0f : 0.0f);
}

// Block -> unit table of k_fc1_bwd.  Blocks b and b + 8 share an XCD (round-robin dispatch), so the table gives
// each XCD whole operand panels: the dW3 tiles of a3 column panels {x, x + 8, ..} (all 4 dz4 panels each) and
// the dz3 tiles of W3 panels {x + 4, x + 12, ..} (all batch panels each), then its share of the fc2 wgrad
// blocks.  Every a3 / W3 panel is fetched into one L2 instead of up to eight, and both GEMMs (16 vs 8 k-steps
// per tile) spread evenly over the XCDs.
template <class PW, class PD>
static void fc1_bwd_map(qlx_model* m, const PW& Pw, const PD& Pd, int extra, hipStream_t s) {
  if (m->fc1bwd_map_B == Pd.M) return;
  std::vector<int> lists[8];
  auto tile_of = [](const auto& P, int mi, int nj) {
    return P.n_fastest ? mi * P.tiles_n + nj : nj * P.tiles_m + mi;
  };
  for (int mi = 0; mi < Pw.tiles_m; ++mi)
    for (int nj = 0; nj < Pw.tiles_n; ++nj) lists[mi % 8].push_back(tile_of(Pw, mi, nj));
  for (int nj = 0; nj < Pd.tiles_n; ++nj)
    for (int mi = 0; mi < Pd.tiles_m; ++mi) lists[(nj + 4) % 8].push_back(Pw.tiles() + tile_of(Pd, mi, nj));
  const int tg = Pw.tiles() + Pd.tiles();
  for (int j = 0; j < extra; ++j) lists[j % 8].push_back(tg + j);
  size_t per = 0;
  for (auto& l : lists) per = std::max(per, l.size());
  std::vector<int> map(8 * per, -1);
  for (int x = 0; x < 8; ++x)
    for (size_t l = 0; l < lists[x].size(); ++l) map[l * 8 + x] = lists[x][l];
  if ((int)map.size() > m->fc1bwd_cap) {
    QLX_HIP(hipStreamSynchronize(s));
    if (m->d_fc1bwd_map) (void)hipFree(m->d_fc1bwd_map);
    QLX_HIP(hipMalloc(&m->d_fc1bwd_map, map.size() * sizeof(int)));
    m->fc1bwd_cap = (int)map.size();
  }
  QLX_HIP(hipMemcpy(m->d_fc1bwd_map, map.data(), map.size() * sizeof(int), hipMemcpyHostToDevice));
  m->fc1bwd_grid = (int)map.size();
  m->fc1bwd_map_B = Pd.M;
}

void launch_fc2(int mode, const Fc2Args& a, int B, hipStream_t s) {
  if (a.a4f) { f32_head(mode, a, B, s); return; }
  const dim3 g((B + 3) / 4), blk(256);
  switch (mode) {
    case 0: hipLaunchKernelGGL(k_fc2<0>, g, blk, 0, s, a); break;
    case 1: hipLaunchKernelGGL(k_fc2<1>, g, blk, 0, s, a); break;
    default: hipLaunchKernelGGL(k_fc2<2>, g, blk, 0, s, a); break;
  }
  QLX_HIP(hipGetLastError());
}

// ------------------------------------------------------------------------------------------
// clip_by_norm per variable + ResourceApplyAdam

// Per-range sums of squares: block r sums gradient range r (<= 2048 elements of one variable).  The norms
// themselves are finished by every k_adam block from these partials (fixed order, no extra launch).
__global__ __launch_bounds__(256) void k_sumsq(const float* g, const int64_t* range_begin, const int64_t* range_end, float scale,
                                               float* partial) {
  __shared__ float red[256];
  const int64_t b = range_begin[blockIdx.x], e = range_end[blockIdx.x];
  float s = 0.0f;
  for (int64_t i = b + threadIdx.x; i < e; i += 256) {
    const float x = g[i] * scale;
    s += x * x;
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0];
}

constexpr int kAdamMaxPartials = 832;   // norm partials per variable (the largest: W3's 784 k_sumsq ranges)

struct AdamArgs {
  float* w;
  float* m;
  float* v;
  const float* g;
  const float* partial;    // k_sumsq output
  const int* var_first;    // partial range of variable v: [var_first[v], var_first[v + 1])
  float* norms;            // written by block 0 (for the ABI)
  int64_t count;
  float scale;     // 1/world for data-parallel mean
  float alpha;     // lr * sqrt(1 - b2^t) / (1 - b1^t)
  float beta1, beta2, eps, clipnorm;
  PackPtrs pack;
};

// flat offsets of the ten variables (kVarSize running sums); every variable but b4 starts at a multiple of 4
__device__ constexpr int64_t kVarOff[kNumVars + 1] = {0, 8192, 8224, 40992, 41056, 77920, 77984, 1683616, 1684128, 1685664, 1685667};
__device__ __forceinline__ int adam_var_of(int64_t i) {
  int v = 0;
#pragma unroll
  for (int k = 1; k < kNumVars; ++k) v += i >= kVarOff[k] ? 1 : 0;
  return v;
}

// the bf16 operand copies of float4 group i0 (4 consecutive parameters of one variable)
__device__ __forceinline__ void pack_group(const PackPtrs& P, int64_t i0, int var, f32x4 w) {
  if (var == 6) {   // W3: the Keras layout, 8-byte store
    *reinterpret_cast<uint2*>(P.wb3 + (i0 - kVarOff[6])) = pack4(w[0], w[1], w[2], w[3]);
  } else if (var == 0 || var == 2 || var == 4) {   // conv kernels: fragment-major scatter
#pragma unroll
    for (int k = 0; k < 4; ++k) pack_one(P, i0 + k, w[k]);
  }
}

// tf.clip_by_norm per variable + ResourceApplyAdam + the bf16 operand copies.  Two float4 groups per thread, all eight
// loads issued before the norm prologue; every block first finishes the per-variable norms from the partials (wave w
// reduces variables w, w+4, w+8: lane-strided sums + xor tree, the same fixed order in every block).  (Round 5: one
// element per thread over 2048 blocks took 16.6 us per update; 16-byte groups per thread measured slower in round 1 -
// then without the loads issued ahead of the prologue.)
constexpr int kAdamGroups = 2;
__global__ __launch_bounds__(256) void k_adam(AdamArgs A) {
  __shared__ float nrm[kNumVars];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t n4 = A.count / 4, st = (int64_t)gridDim.x * blockDim.x, q0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  f32x4 g[kAdamGroups], w[kAdamGroups], m[kAdamGroups], vs[kAdamGroups];
#pragma unroll
  for (int u = 0; u < kAdamGroups; ++u) {
    const int64_t qq = q0 + u * st, i0 = (qq < n4 ? qq : 0) * 4;
    g[u] = *reinterpret_cast<const f32x4*>(A.g + i0);
    w[u] = *reinterpret_cast<const f32x4*>(A.w + i0);
    m[u] = *reinterpret_cast<const f32x4*>(A.m + i0);
    vs[u] = *reinterpret_cast<const f32x4*>(A.v + i0);
  }
  for (int v = wave; v < kNumVars; v += 4) {
    // all of a lane's partials are loaded before the first add (one memory latency, not one per partial),
    // then summed in the lane-strided order
    const int first = A.var_first[v], last = A.var_first[v + 1];
    float p[kAdamMaxPartials / 64];
#pragma unroll
    for (int k = 0; k < kAdamMaxPartials / 64; ++k) {
      const int r = first + lane + 64 * k;
      p[k] = r < last ? A.partial[r] : 0.0f;
    }
    float t = 0.0f;
#pragma unroll
    for (int k = 0; k < kAdamMaxPartials / 64; ++k)
      if (first + lane + 64 * k < last) t += p[k];
    for (int off = 32; off > 0; off >>= 1) t += __shfl_xor(t, off);
    if (lane == 0) {
      nrm[v] = t > 0.0f ? sqrtf(t) : t;   // safe sqrt via where(l2sum > 0)
      if (blockIdx.x == 0) A.norms[v] = nrm[v];
    }
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < kAdamGroups; ++u) {
    const int64_t qq = q0 + u * st;
    if (qq < n4) {
      const int64_t i0 = qq * 4;
      const int var = adam_var_of(i0);
      const float denom = fmaxf(nrm[var], A.clipnorm);
      f32x4 o;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float mk = m[u][k], vk = vs[u][k];
        o[k] = adam_elem(g[u][k], A.scale, A.clipnorm, denom, A.alpha, A.beta1, A.beta2, A.eps, mk, vk, w[u][k]);
        m[u][k] = mk;
        vs[u][k] = vk;
      }
      *reinterpret_cast<f32x4*>(A.w + i0) = o;
      *reinterpret_cast<f32x4*>(A.m + i0) = m[u];
      *reinterpret_cast<f32x4*>(A.v + i0) = vs[u];
      pack_group(A.pack, i0, var, o);
    } else if (qq == n4) {   // the tail (b4's last elements), element by element
      for (int64_t i = n4 * 4; i < A.count; ++i) {
        const int var = adam_var_of(i);
        const float denom = fmaxf(nrm[var], A.clipnorm);
        float mi = A.m[i], vi = A.v[i];
        const float wi = adam_elem(A.g[i], A.scale, A.clipnorm, denom, A.alpha, A.beta1, A.beta2, A.eps, mi, vi, A.w[i]);
        A.m[i] = mi;
        A.v[i] = vi;
        A.w[i] = wi;
        pack_one(A.pack, i, wi);
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// host side

static size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

void model_workspace(qlx_model* m, int B) {
  if (m->f32) { f32_workspace(m, B); return; }
  if (B <= m->ws_batch) return;
  model_dense_join(m, m->stream);
  QLX_HIP(hipStreamSynchronize(m->stream));
  if (m->ws) (void)hipFree(m->ws);
  m->ws = nullptr;
  ModelWs& w = m->w;
  size_t off = 0;
  auto take = [&](size_t bytes) { const size_t o = off; off = align_up(off + bytes, 256); return o; };
  const size_t o_frames = take((size_t)B * 4 * kFramePix);
  const size_t o_table = take((size_t)B * 4 * sizeof(void*));
  const size_t o_a1 = take((size_t)B * 12800 * 2), o_a2 = take((size_t)B * 5184 * 2), o_a3 = take((size_t)B * kA3Ld * 2);
  const size_t o_a4 = take((size_t)B * 512 * 2), o_q = take((size_t)B * 3 * 4);
  const size_t o_dz1 = take((size_t)B * 12800 * 2), o_dz2 = take((size_t)B * 5184 * 2), o_dz3 = take((size_t)B * 3136 * 2);
  const size_t o_dz4 = take((size_t)B * 512 * 2);
  const size_t o_gs = take((size_t)B * 4), o_hs = take((size_t)B * 4), o_y = take((size_t)B * 4);
  const size_t o_act = take((size_t)B), o_argmax = take((size_t)B), o_rew = take((size_t)B * 4), o_done = take((size_t)B);
  const size_t o_fc1slab = take((size_t)kFc1Split * B * 512 * 4);
  const size_t o_slab = take(kWgradSlabFloats * 4);
  const size_t o_bslab = take(kBiasSlabFloats * 4);
  const size_t o_loss = take(64);
  QLX_HIP(hipMalloc(&m->ws, off));
  char* base = (char*)m->ws;
  w.frames = (uint8_t*)(base + o_frames);
  w.table = (const uint8_t**)(base + o_table);
  w.a1 = (bf16*)(base + o_a1); w.a2 = (bf16*)(base + o_a2); w.a3 = (bf16*)(base + o_a3); w.a4 = (bf16*)(base + o_a4);
  w.q = (float*)(base + o_q);
  w.dz1 = (bf16*)(base + o_dz1); w.dz2 = (bf16*)(base + o_dz2); w.dz3 = (bf16*)(base + o_dz3); w.dz4 = (bf16*)(base + o_dz4);
  w.gs = (float*)(base + o_gs); w.hs = (float*)(base + o_hs); w.y = (float*)(base + o_y);
  w.act = (uint8_t*)(base + o_act); w.argmax = (uint8_t*)(base + o_argmax); w.rew = (float*)(base + o_rew);
  w.done = (uint8_t*)(base + o_done);
  w.fc1slab = (float*)(base + o_fc1slab);
  w.slab = (float*)(base + o_slab);
  w.bslab = (float*)(base + o_bslab);
  w.loss = (float*)(base + o_loss);
  hipLaunchKernelGGL(k_a3_pad, dim3((B * 8 + 255) / 256), dim3(256), 0, m->stream, w.a3, B);
  QLX_HIP(hipGetLastError());
  m->ws_batch = B;
}

static PackPtrs pack_ptrs(qlx_model* m) {
  PackPtrs P;
  P.wf0 = m->wf0; P.wf1 = m->wf1; P.wb1 = m->wb1; P.wf2 = m->wf2; P.wb2 = m->wb2; P.wb3 = m->wb3;
  return P;
}

void model_pack(qlx_model* m) {
  m->version += 1;
  if (m->f32) return;   // the fp32 path reads the master weights directly
  hipLaunchKernelGGL(k_pack_all, dim3(2048), dim3(256), 0, m->stream, m->d_params, (int64_t)kNumParams, pack_ptrs(m));
  QLX_HIP(hipGetLastError());
}

// one block per CU (LDS-limited), persistent over samples
static int trunk_grid(int B) { return std::max(1, std::min(B, 256)); }

template <class Kern>
static void set_lds_attr(Kern k, size_t bytes) {
  set_lds_limit((const void*)k, bytes);
}

// XCD-grouped tile order (xcd_tile): each XCD runs a contiguous range of the tile order, so the operand panels its tiles
// share are fetched into its own L2 once (for the split forward: about one k split per XCD)
// bgemm.h's host-checked requirements: every split's k range a multiple of 32, and K % 32 == 0 for a row-major operand
// (its buffer descriptor spans the whole tensor, so a ragged K would read the next row's data instead of zeros)
template <class C, class Epi>
static void bgemm_check(const BGemmProblem<Epi>& P) {
  QLX_CHECK(P.kps > 0 && P.kps % 32 == 0, QLX_E_STATE, "bgemm: k per split must be a multiple of 32");
  QLX_CHECK((C::AK && C::BKM) || P.K % 32 == 0, QLX_E_STATE, "bgemm: a row-major operand needs K % 32 == 0");
}

template <class C, class Epi>
static void launch_bgemm(const BGemmProblem<Epi>& P, hipStream_t s) {
  bgemm_check<C>(P);
  set_lds_attr(k_bgemm<C, Epi>, C::LDS);
  hipLaunchKernelGGL((k_bgemm<C, Epi>), dim3(xcd_grid(P.tiles())), dim3(C::T), C::LDS, s, P, 1);
}

void model_forward_trunk(qlx_model* m, const uint8_t* const* table, int B, hipStream_t s, bool store_acts) {
  if (m->f32) { f32_forward(m, table, B, s); return; }
  ModelWs& w = m->w;
  m->last_batch = B;
  const float* p = m->d_params;
  {  // conv1 -> conv2 -> conv3 fused per sample (trunk_kernels.h)
    // scope per role so each maps to one kernel instantiation (trunk_fwd = online pass with stored activations)
    // timed with dispatch-bound events (bench.py's roofline kernel: its average must match rocprofv3's)
    hipEvent_t ea = nullptr, eb = nullptr;
    if (m->prof)
      m->prof->ext(store_acts ? "trunk_fwd" : "trunk_fwd_nostore", 2.0 * B * (400.0 * 32 * 256 + 81.0 * 64 * 512 + 49.0 * 64 * 576),
                   &ea, &eb);
    set_lds_attr(k_trunk_fwd<true>, kTrunkFwdLds);
    set_lds_attr(k_trunk_fwd<false>, kTrunkFwdLds);
    auto kern = store_acts ? k_trunk_fwd<true> : k_trunk_fwd<false>;
    hipExtLaunchKernelGGL(kern, dim3(trunk_grid(B)), dim3(kTrunkThreads), kTrunkFwdLds, s, ea, eb, 0u, table, B, m->wf0, m->wf1,
                          m->wf2, p + var_offset(1), p + var_offset(3), p + var_offset(5), w.a1, w.a2, w.a3,
                          (unsigned long long*)nullptr);
  }
  {  // fc1: M = B, N = 512, K = 3136.  Small batches split K into kFc1Split fp32 slabs (reduced with bias +
     // ReLU in fixed order) to fill the chip; from 64 M tiles on (B >= 8192) one pass with the epilogue fused
    ProfScope ps(m->prof, "fc1_fwd", s, 2.0 * B * 512 * 3136);
    const BOp A{w.a3, kA3Ld, B}, W{m->wb3, 512, 512};
    if (B >= 64 * 128 || m->fc1_single) {
      launch_bgemm<CfgFc1FwdBig>(bproblem(A, W, B, 512, 3136, 1, CfgFc1FwdBig::BM, CfgFc1FwdBig::BN,
                                          Epi4BiasRelu{w.a4, p + var_offset(7), 512}), s);
      w.a4_splits = 0;
    } else {
      const auto P = bproblem(A, W, B, 512, 3136, kFc1Split, CfgFc1Fwd::BM, CfgFc1Fwd::BN, Epi4Slab{w.fc1slab, 512, (size_t)B * 512});
      QLX_CHECK(P.splits == kFc1Split, QLX_E_STATE, "fc1 split count");
      launch_bgemm<CfgFc1Fwd>(P, s);
      w.a4_splits = kFc1Split;   // bias + ReLU + the fixed-order sum happen in the fc2 head that follows
    }
  }
  QLX_HIP(hipGetLastError());
}

Fc2Args fc2_args(qlx_model* m, int B) {
  Fc2Args a{};
  a.a4 = m->w.a4;
  a.a4f = m->f32 ? m->w.fa4 : nullptr;
  a.w4 = m->d_params + var_offset(8);
  a.b4 = m->d_params + var_offset(9);
  a.B = B;
  a.q = m->w.q;
  a.slab = m->w.fc1slab;
  a.zstride = (size_t)B * 512;
  a.splits = m->w.a4_splits;
  a.b3 = m->d_params + var_offset(7);
  a.a4_out = m->w.a4;
  m->w.a4_splits = 0;
  return a;
}

// Huber loss (mean over the batch -> *loss_dev) and its raw, unclipped gradients into m->d_grads, after
// model_forward_trunk on the same batch; actions / y are device arrays [B]
void model_backward(qlx_model* m, const uint8_t* const* table, int B, const uint8_t* actions, const float* y, float* loss_dev,
                    hipStream_t s, const float* weights, float* td_abs, bool fuse_update) {
  model_backward_dense(m, B, actions, y, loss_dev, s, weights, td_abs);
  // fp32, no all-reduce: the dense variables' update can leave the learner stream here (qnet32.hip f32_dense_async)
  if (m->f32 && fuse_update && m->dense_overlap) f32_dense_async(m, s);
  model_backward_conv(m, table, B, s, fuse_update);
}

// the head and dense part of the backward: Huber (+ dz4), dW4 / db4 / loss, dW3 / db3 and dz3
void model_backward_dense(qlx_model* m, int B, const uint8_t* actions, const float* y, float* loss_dev, hipStream_t s,
                          const float* weights, float* td_abs) {
  if (m->f32) { f32_backward_dense(m, B, actions, y, loss_dev, s, weights, td_abs); return; }
  ModelWs& w = m->w;
  float* G = m->d_grads;
  {  // head: q, Huber, dz4 (one wave per sample)
    ProfScope ps(m->prof, "fc2_head", s);
    Fc2Args a = fc2_args(m, B);
    a.actions = actions;
    a.y = y;
    a.gsample = w.gs;
    a.hsample = w.hs;
    a.weights = weights;
    a.td_abs = td_abs;
    hipLaunchKernelGGL(k_fc2_train, dim3((B + 3) / 4), dim3(256), 0, s, a, w.dz4);
  }
  // fc1 in one launch of two independent GEMMs (both only read dz4 / a3), plus dW4 / db4 / loss:
  //   dW3 = a3^T dz4 and db3 (row 3136 = the all-ones row; db3 follows dW3 [3136][512] in the flat gradient)
  //   dz3 = (dz4 W3^T) * (a3 > 0)
  {
    ProfScope ps(m->prof, "fc1_bwd", s, 2.0 * 2.0 * B * 512 * 3136);
    const auto Pd = bproblem(BOp{w.dz4, 512, B}, BOp{m->wb3, 512, 3136}, B, 3136, 512, 1, 128, 128,
                             Epi4ReluMask{w.dz3, w.a3, 3136, kA3Ld});
    const Fc2WgradArgs F{w.a4, actions, w.gs, w.hs, B, G + var_offset(8), G + var_offset(9), loss_dev,
                         m->d_sqf + sq_first(8), m->d_sqf + sq_first(9)};
    auto launch = [&](const auto& Pw, auto kern) {
      QLX_CHECK(Pw.tiles() == kFc1WgradTiles, QLX_E_STATE, "fc1 wgrad tiling changed: update kSqSlots");
      bgemm_check<CfgFc1Wg>(Pw);
      bgemm_check<CfgFc1Dg>(Pd);
      fc1_bwd_map(m, Pw, Pd, kFc2WgradBlocks, s);
      constexpr size_t lds_req = CfgFc1Wg::LDS;
      static_assert(lds_req >= (kFc1BwdThreads / 64 + 1) * 24 * sizeof(float), "fc2 wgrad block scratch");
      set_lds_attr(kern, lds_req);
      hipLaunchKernelGGL(kern, dim3(m->fc1bwd_grid), dim3(kFc1BwdThreads), lds_req, s, Pw, Pd, F, (const int*)m->d_fc1bwd_map);
    };
    // dW3 rows 0..3135 and db3 as row 3136 (a3's ones column), written straight into the flat gradient (b3 follows W3)
    launch(bproblem(BOp{w.a3, kA3Ld, 3137}, BOp{w.dz4, 512, 512}, 3137, 512, B, 1, 128, 128,
                    Epi4StoreF32{G + var_offset(6), 512, m->d_sqf + sq_first(6)}, 3136),
           k_fc1_bwd<Epi4StoreF32, Epi4ReluMask>);
  }
  QLX_HIP(hipGetLastError());
}

// the conv part of the backward (after model_backward_dense on the same batch): dz3 -> dz2 -> dz1 and the
// three conv weight gradients into m->d_grads
void model_backward_conv(qlx_model* m, const uint8_t* const* table, int B, hipStream_t s, bool fuse_update, hipEvent_t dense_ready,
                         float dense_scale) {
  if (m->f32) { f32_backward_conv(m, table, B, s, fuse_update, dense_ready, dense_scale); return; }
  ModelWs& w = m->w;
  float* G = m->d_grads;
  // dz2 = convT(dz3, W2) * (a2 > 0); dz1 = convT(dz2, W1) * (a1 > 0), fused per sample (trunk_kernels.h)
  {
    ProfScope ps(m->prof, "trunk_bwd_data", s, 2.0 * B * (49.0 * 64 * 576 + 81.0 * 64 * 512));
    set_lds_attr(k_trunk_bwd_data<false>, kTrunkBwdLds);
    hipLaunchKernelGGL(k_trunk_bwd_data<false>, dim3(trunk_grid(B)), dim3(kTrunkThreads), kTrunkBwdLds, s, w.dz3, w.a2, w.a1, B,
                       m->wb2, m->wb1, w.dz2, w.dz1, nullptr);
  }
  // conv3 (3 tap groups of 3 taps) + conv2 (2 groups of 8 taps) weight gradients in one launch, then
  // conv1's; per-block fp32 partials of [dW | db] rows, reduced in fixed order by one grouped launch
  // straight into the flat gradient (each layer's b follows its W; conv1 goes s2d -> HWIO)
  using CW3 = ConvWgradCfg<9, 9, 64, 3, 1, 7, 7, 3, 3, 2, kWg3Samples>;
  using CW2 = ConvWgradCfg<20, 20, 32, 4, 2, 9, 9, 8, 2, 4, kWg2Samples>;
  static_assert(85 * CW3::ZS <= kSlabConv2 && kSlabConv2 + 128 * CW2::ZS <= kSlabConv1 &&
                    kSlabConv1 + 256 * (size_t)kConv1SlabStride <= kWgradSlabFloats,
                "slab regions overlap");
  // about 256 blocks per layer; a chunk is a whole number of LDS rounds (ns samples each)
  auto chunking = [&](int groups, int ns, int& per) {
    const int chunks = std::max(1, std::min(B, 256 / groups));
    per = ((B + chunks - 1) / chunks + ns - 1) / ns * ns;
    return (B + per - 1) / per;
  };
  int per3 = 0, per2 = 0;
  const int used3 = chunking(3, kWg3Samples, per3), used2 = chunking(2, kWg2Samples, per2);
  {
    ProfScope ps(m->prof, "conv23_wgrad", s, 2.0 * B * (49.0 * 576 * 64 + 81.0 * 512 * 64));
    constexpr size_t lds = std::max(CW3::LDS, CW2::LDS);
    auto kern = k_conv23_wgrad;
    set_lds_attr(kern, lds);
    hipLaunchKernelGGL(kern, dim3(wgrad_blocks(3, used3) + wgrad_blocks(2, used2)), dim3(kTrunkThreads), lds, s, w.a2, w.dz3, per3, used3,
                       w.slab + kSlabConv3, w.a1, w.dz2, per2, used2, w.slab + kSlabConv2, B);
  }
  const int grid1 = trunk_grid(B);
  {  // conv1: dW0 = im2col_s2d(x)^T dz1 per sample from the LDS-staged frames
    ProfScope ps(m->prof, "conv1_wgrad", s, 2.0 * B * 400 * 256 * 32);
    if (m->conv1_halves) {   // two channel-half blocks per sample chunk, two blocks per CU
      set_lds_attr(k_conv1_wgrad_h, kConv1WgradHLds);
      hipLaunchKernelGGL(k_conv1_wgrad_h, dim3(2 * grid1), dim3(kTrunkThreads), kConv1WgradHLds, s, table, w.dz1, B, grid1,
                         w.slab + kSlabConv1);
    } else {
      set_lds_attr(k_conv1_wgrad, kConv1WgradLds);
      hipLaunchKernelGGL(k_conv1_wgrad, dim3(grid1), dim3(kTrunkThreads), kConv1WgradLds, s, table, w.dz1, B,
                         w.slab + kSlabConv1);
    }
  }
  {
    ProfScope ps(m->prof, "wgrad_reduce", s);
    // slot ranges: each layer's weight blocks then its one bias block (sq_first(W) + blocks == sq_first(b))
    static_assert(CW3::ZS == 576 * 64 + 64 && CW2::ZS == 512 * 64 + 64 && kConv1SlabStride == 128 * 64 + 32, "slab blocks");
    SlabSeg segs[3] = {
        {w.slab + kSlabConv3, CW3::ZS, used3, CW3::ZS, G + var_offset(4), 0, m->d_sqf + sq_first(4)},
        {w.slab + kSlabConv2, CW2::ZS, used2, CW2::ZS, G + var_offset(2), 0, m->d_sqf + sq_first(2)},
        {w.slab + kSlabConv1, (size_t)kConv1SlabStride, grid1, (size_t)kConv1SlabStride, G, 1, m->d_sqf + sq_first(0)},
    };
    SlabSegs3 a;
    int blocks = 0;
    for (int i = 0; i < 3; ++i) {
      a.seg[i] = segs[i];
      a.first_block[i] = blocks;
      blocks += (int)((segs[i].count + 63) / 64);
    }
    a.first_block[3] = blocks;
    hipLaunchKernelGGL(k_slab_reduce3, dim3(blocks), dim3(256), 0, s, a);
  }
  QLX_HIP(hipGetLastError());
}


void model_norms(qlx_model* m, hipStream_t s, float scale) {
  if (m->f32) { f32_norms(m, s, scale); return; }
  m->norms_fused = scale == 1.0f;   // the gradients are exactly what model_backward produced
  if (m->norms_fused) return;
  ProfScope ps(m->prof, "norms", s);
  hipLaunchKernelGGL(k_sumsq, dim3(m->n_ranges), dim3(256), 0, s, m->d_grads, m->d_rbeg, m->d_rend, scale, m->d_partial);
  QLX_HIP(hipGetLastError());
}

void model_adam(qlx_model* m, hipStream_t s, float scale) {
  if (m->f32) { f32_adam(m, s, scale); return; }
  const int64_t t = m->iterations + 1;
  const float tf = (float)t;
  const float b1p = std::pow(m->beta1, tf), b2p = std::pow(m->beta2, tf);
  AdamArgs a;
  a.w = m->d_params; a.m = m->d_m; a.v = m->d_v; a.g = m->d_grads; a.norms = m->d_norms;
  a.partial = m->norms_fused ? m->d_sqf : m->d_partial;
  a.var_first = m->norms_fused ? m->d_sqf_first : m->d_var_first;
  a.count = kNumParams; a.scale = scale;
  a.alpha = m->lr * std::sqrt(1.0f - b2p) / (1.0f - b1p);
  a.beta1 = m->beta1; a.beta2 = m->beta2; a.eps = m->eps; a.clipnorm = m->clipnorm;
  a.pack = pack_ptrs(m);
  ProfScope ps(m->prof, "adam", s, 32.0 * kNumParams);
  const int64_t groups = kNumParams / 4 + 1;   // float4 groups + the tail group
  hipLaunchKernelGGL(k_adam, dim3((unsigned)((groups + 256 * kAdamGroups - 1) / (256 * kAdamGroups))), dim3(256), 0, s, a);
  QLX_HIP(hipGetLastError());
  m->iterations = t;
}

void model_frame_table_from_host(qlx_model* m, const uint8_t* obs_host, int B) {
  model_workspace(m, B);
  uint8_t* d_obs = nullptr;
  const size_t bytes = (size_t)B * kFramePix * 4;
  QLX_HIP(hipMalloc(&d_obs, bytes));
  QLX_HIP(hipMemcpyAsync(d_obs, obs_host, bytes, hipMemcpyHostToDevice, m->stream));
  hipLaunchKernelGGL(k_pack_obs, dim3((B * kFramePix + 255) / 256), dim3(256), 0, m->stream, d_obs, B, m->w.frames);
  hipLaunchKernelGGL(k_frame_table, dim3((B * 4 + 255) / 256), dim3(256), 0, m->stream, m->w.frames, B, m->w.table);
  QLX_HIP(hipGetLastError());
  model_dense_join(m, m->stream);
  QLX_HIP(hipStreamSynchronize(m->stream));
  QLX_HIP(hipFree(d_obs));
}

static void glorot_host(std::vector<float>& params, uint64_t seed) {
  const int fan_in[5] = {8 * 8 * 4, 4 * 4 * 32, 3 * 3 * 64, 3136, 512};
  const int fan_out[5] = {8 * 8 * 32, 4 * 4 * 64, 3 * 3 * 64, 512, 3};
  params.assign(kNumParams, 0.0f);
  int64_t off = 0;
  for (int v = 0; v < kNumVars; ++v) {
    if (v % 2 == 0) {
      const int l = v / 2;
      const float limit = std::sqrt(6.0f / (float)(fan_in[l] + fan_out[l]));
      RngStream s(seed, (uint32_t)v, 0, P_INIT);
      for (int i = 0; i < kVarSize[v]; ++i) params[off + i] = uniform_f32(s, -limit, limit);
    }
    off += kVarSize[v];
  }
}

}  // namespace qlx

using namespace qlx;

extern "C" {

int32_t qlx_model_num_vars(void) { return kNumVars; }

int32_t qlx_model_hparams(float* out) {
  return guard([&] {
    QLX_CHECK(out, QLX_E_INVALID, "null out");
    const qlx_model m;   // the defaults every created model starts from (no device state is touched)
    out[0] = m.lr; out[1] = m.beta1; out[2] = m.beta2; out[3] = m.eps; out[4] = m.clipnorm;
  });
}
int64_t qlx_model_var_size(int32_t v) { return (v >= 0 && v < kNumVars) ? kVarSize[v] : -1; }

int32_t qlx_model_create(int32_t arch, uint64_t seed, int32_t device, qlx_model** out) {
  return guard([&] {
    QLX_CHECK((arch == QLX_ARCH_NATURE_DQN || arch == QLX_ARCH_NATURE_DQN_BF16) && out, QLX_E_INVALID, "unknown model arch");
    current_device_checked(device);
    auto* m = new qlx_model;
    m->f32 = arch == QLX_ARCH_NATURE_DQN;
    const char* ch = std::getenv("QLX_CONV1_HALVES");
    m->conv1_halves = !(ch && ch[0] == '0');
    const char* bg = std::getenv("QLX_F32_BG");
    m->f32_bg_rows = !(bg && bg[0] == '0');
    const char* sk = std::getenv("QLX_F32_C1_SKIP");
    m->f32_c1_skip = (sk && sk[0] == '0') ? 0 : 1;
    const char* dov = std::getenv("QLX_F32_DENSE_OVERLAP");
    m->dense_overlap = dov && dov[0] == '1';
    try {   // a failure part-way releases what was built
      m->device = device;
      QLX_HIP(hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking));
      const size_t pb = kNumParams * sizeof(float);
      QLX_HIP(hipMalloc(&m->d_params, pb));
      QLX_HIP(hipMalloc(&m->d_m, pb));
      QLX_HIP(hipMalloc(&m->d_v, pb));
      QLX_HIP(hipMalloc(&m->d_grads, pb));
      if (!m->f32) {   // bf16 MFMA operand copies
        QLX_HIP(hipMalloc(&m->wf0, 32 * 256 * 2));
        QLX_HIP(hipMalloc(&m->wf1, 64 * 512 * 2));
        QLX_HIP(hipMalloc(&m->wb1, 32 * 1024 * 2));
        QLX_HIP(hipMalloc(&m->wf2, 64 * 576 * 2));
        QLX_HIP(hipMalloc(&m->wb2, 64 * 576 * 2));
        QLX_HIP(hipMalloc(&m->wb3, 3136 * 512 * 2));
      }
      // norm ranges: chunks of <= 2048 elements (~830 blocks) that never cross a variable
      std::vector<int64_t> rb, re;
      std::vector<int> vf(kNumVars + 1, 0);
      int64_t off = 0;
      for (int v = 0; v < kNumVars; ++v) {
        vf[v] = (int)rb.size();
        for (int64_t i = 0; i < kVarSize[v]; i += 2048) {
          rb.push_back(off + i);
          re.push_back(off + std::min<int64_t>(kVarSize[v], i + 2048));
        }
        off += kVarSize[v];
      }
      vf[kNumVars] = (int)rb.size();
      for (int v = 0; v < kNumVars; ++v)
        QLX_CHECK(vf[v + 1] - vf[v] <= kAdamMaxPartials && kSqSlots[v] <= kAdamMaxPartials, QLX_E_STATE, "k_adam partial bound");
      m->n_ranges = (int)rb.size();
      QLX_HIP(hipMalloc(&m->d_rbeg, rb.size() * 8));
      QLX_HIP(hipMalloc(&m->d_rend, re.size() * 8));
      QLX_HIP(hipMalloc(&m->d_partial, rb.size() * 4));
      QLX_HIP(hipMalloc(&m->d_var_first, vf.size() * 4));
      QLX_HIP(hipMalloc(&m->d_norms, 64));
      std::vector<int> sf(kNumVars + 1);
      for (int v = 0; v <= kNumVars; ++v) sf[v] = v < kNumVars ? sq_first(v) : sq_first(kNumVars - 1) + kSqSlots[kNumVars - 1];
      QLX_HIP(hipMalloc(&m->d_sqf, sf[kNumVars] * 4));
      QLX_HIP(hipMalloc(&m->d_sqf_first, sf.size() * 4));
      QLX_HIP(hipMemcpy(m->d_sqf_first, sf.data(), sf.size() * 4, hipMemcpyHostToDevice));
      QLX_HIP(hipMemset(m->d_sqf, 0, sf[kNumVars] * 4));
      QLX_HIP(hipMemcpy(m->d_rbeg, rb.data(), rb.size() * 8, hipMemcpyHostToDevice));
      QLX_HIP(hipMemcpy(m->d_rend, re.data(), re.size() * 8, hipMemcpyHostToDevice));
      QLX_HIP(hipMemcpy(m->d_var_first, vf.data(), vf.size() * 4, hipMemcpyHostToDevice));
      std::vector<float> params;
      glorot_host(params, seed);
      QLX_HIP(hipMemcpy(m->d_params, params.data(), pb, hipMemcpyHostToDevice));
      QLX_HIP(hipMemset(m->d_m, 0, pb));
      QLX_HIP(hipMemset(m->d_v, 0, pb));
      QLX_HIP(hipMemset(m->d_grads, 0, pb));
      model_pack(m);
      model_dense_join(m, m->stream);
      QLX_HIP(hipStreamSynchronize(m->stream));
    } catch (...) {
      qlx_model_destroy(m);
      throw;
    }
    *out = m;
  });
}

int32_t qlx_model_destroy(qlx_model* m) {
  return guard([&] {
    if (!m) return;
    (void)hipSetDevice(m->device);
    (void)hipStreamSynchronize(m->stream);
    if (m->f32_aux) {
      (void)hipStreamSynchronize(m->f32_aux);
      (void)hipStreamDestroy(m->f32_aux);
      (void)hipEventDestroy(m->ev_dense_ready);
      (void)hipEventDestroy(m->ev_dense_done);
    }
    void* ptrs[] = {m->d_params, m->d_m, m->d_v, m->d_grads, m->wf0, m->wf1, m->wb1, m->wf2, m->wb2, m->wb3,
                    m->d_rbeg, m->d_rend, m->d_partial, m->d_var_first, m->d_norms, m->d_sqf, m->d_sqf_first, m->ws, m->d_fc1bwd_map,
                    m->w.fgrad};
    for (void* p : ptrs) (void)hipFree(p);
    if (m->own_stream) (void)hipStreamDestroy(m->stream);
    delete m;
  });
}

int32_t qlx_model_get_var(qlx_model* m, int32_t var, int32_t which, float* out) {
  return guard([&] {
    QLX_CHECK(m && out && var >= 0 && var < kNumVars && which >= 0 && which <= 2, QLX_E_INVALID, "bad argument");
    QLX_HIP(hipSetDevice(m->device));
    model_dense_join(m, m->stream);
    QLX_HIP(hipStreamSynchronize(m->stream));
    const float* src = (which == 0 ? m->d_params : which == 1 ? m->d_m : m->d_v) + var_offset(var);
    QLX_HIP(hipMemcpy(out, src, kVarSize[var] * sizeof(float), hipMemcpyDeviceToHost));
  });
}

int32_t qlx_model_set_var(qlx_model* m, int32_t var, int32_t which, const float* in) {
  return guard([&] {
    QLX_CHECK(m && in && var >= 0 && var < kNumVars && which >= 0 && which <= 2, QLX_E_INVALID, "bad argument");
    QLX_HIP(hipSetDevice(m->device));
    model_dense_join(m, m->stream);
    QLX_HIP(hipStreamSynchronize(m->stream));
    float* dst = (which == 0 ? m->d_params : which == 1 ? m->d_m : m->d_v) + var_offset(var);
    QLX_HIP(hipMemcpy(dst, in, kVarSize[var] * sizeof(float), hipMemcpyHostToDevice));
    if (which == 0) {
      model_pack(m);
      QLX_HIP(hipStreamSynchronize(m->stream));
    }
  });
}

int64_t qlx_model_iterations(qlx_model* m) { return m ? m->iterations : -1; }

int32_t qlx_model_copy_weights(qlx_model* dst, const qlx_model* src) {
  return guard([&] {
    QLX_CHECK(dst && src, QLX_E_INVALID, "null model");
    QLX_HIP(hipSetDevice(dst->device));
    model_dense_join(const_cast<qlx_model*>(src), src->stream);   // src's weights complete, dst's not still being written
    model_dense_join(dst, dst->stream);
    QLX_HIP(hipStreamSynchronize(src->stream));
    QLX_HIP(hipMemcpyAsync(dst->d_params, src->d_params, kNumParams * sizeof(float), hipMemcpyDeviceToDevice, dst->stream));
    model_pack(dst);
    QLX_HIP(hipStreamSynchronize(dst->stream));
  });
}

int32_t qlx_model_predict(qlx_model* m, const uint8_t* obs, uint32_t n, float* q_out, uint8_t* actions) {
  return guard([&] {
    QLX_CHECK(m && obs && n > 0, QLX_E_INVALID, "bad argument");
    QLX_HIP(hipSetDevice(m->device));
    model_frame_table_from_host(m, obs, (int)n);
    model_forward_trunk(m, m->w.table, (int)n, m->stream);
    Fc2Args a = fc2_args(m, (int)n);
    a.argmax = m->w.argmax;
    launch_fc2(1, a, (int)n, m->stream);
    if (q_out) QLX_HIP(hipMemcpyAsync(q_out, m->w.q, n * 3 * sizeof(float), hipMemcpyDeviceToHost, m->stream));
    if (actions) QLX_HIP(hipMemcpyAsync(actions, m->w.argmax, n, hipMemcpyDeviceToHost, m->stream));
    model_dense_join(m, m->stream);
    QLX_HIP(hipStreamSynchronize(m->stream));
  });
}

int32_t qlx_model_batch_max_q(qlx_model* m, const uint8_t* obs, uint32_t n, float* out) {
  return guard([&] {
    QLX_CHECK(m && obs && out && n > 0, QLX_E_INVALID, "bad argument");
    QLX_HIP(hipSetDevice(m->device));
    model_frame_table_from_host(m, obs, (int)n);
    model_forward_trunk(m, m->w.table, (int)n, m->stream);
    // y = 0 + max * 1 with done = 0: the bare reduce_max of the reference signature
    QLX_HIP(hipMemsetAsync(m->w.rew, 0, n * 4, m->stream));
    QLX_HIP(hipMemsetAsync(m->w.done, 0, n, m->stream));
    Fc2Args a = fc2_args(m, (int)n);
    a.rewards = m->w.rew; a.dones = m->w.done; a.gamma = 1.0f; a.y_out = m->w.y;
    launch_fc2(2, a, (int)n, m->stream);
    QLX_HIP(hipMemcpyAsync(out, m->w.y, n * sizeof(float), hipMemcpyDeviceToHost, m->stream));
    model_dense_join(m, m->stream);
    QLX_HIP(hipStreamSynchronize(m->stream));
  });
}

int32_t qlx_model_train(qlx_model* m, const uint8_t* obs, const uint8_t* actions, const float* y, uint32_t B,
                        float* loss_out, float* grads_out, float* norms_out) {
  return guard([&] {
    QLX_CHECK(m && obs && actions && y && B > 0, QLX_E_INVALID, "bad argument");
    for (uint32_t b = 0; b < B; ++b) QLX_CHECK(actions[b] < kActions, QLX_E_INVALID, "action out of range");
    QLX_HIP(hipSetDevice(m->device));
    model_frame_table_from_host(m, obs, (int)B);
    hipStream_t s = m->stream;
    QLX_HIP(hipMemcpyAsync(m->w.act, actions, B, hipMemcpyHostToDevice, s));
    QLX_HIP(hipMemcpyAsync(m->w.y, y, B * 4, hipMemcpyHostToDevice, s));
    model_forward_trunk(m, m->w.table, (int)B, s);
    model_backward(m, m->w.table, (int)B, m->w.act, m->w.y, m->w.loss, s, nullptr, nullptr, true);
    if (grads_out) QLX_HIP(hipMemcpyAsync(grads_out, m->d_grads, kNumParams * 4, hipMemcpyDeviceToHost, s));
    model_norms(m, s, 1.0f);
    model_adam(m, s, 1.0f);
    model_dense_join(m, s);   // the dense norms / weights of an update on the aux stream
    if (norms_out) QLX_HIP(hipMemcpyAsync(norms_out, m->d_norms, kNumVars * 4, hipMemcpyDeviceToHost, s));
    if (loss_out) QLX_HIP(hipMemcpyAsync(loss_out, m->w.loss, 4, hipMemcpyDeviceToHost, s));
    QLX_HIP(hipStreamSynchronize(s));
  });
}

// The update tail alone on a given gradient (test hook of the data-parallel tail, whose all-reduced gradient is scaled by
// 1 / world): clip_by_norm of (grads x scale) per variable + legacy Adam, exactly as learner_update runs them after an
// all-reduce (model_norms, then model_adam at that scale).  fp32: the same two launches as a rank's DP tail; bf16: the
// explicit sum-of-squares pass (the backward's fused partials do not belong to this gradient) and the Adam launch.
int32_t qlx_model_apply_gradient(qlx_model* m, const float* grads, float scale, float* norms_out) {
  return guard([&] {
    QLX_CHECK(m && grads, QLX_E_INVALID, "null argument");
    QLX_CHECK(std::isfinite(scale) && scale > 0.0f, QLX_E_INVALID, "scale must be finite and > 0");
    QLX_HIP(hipSetDevice(m->device));
    hipStream_t s = m->stream;
    model_dense_join(m, s);
    model_workspace(m, std::max(m->ws_batch, 1));   // (the norm partial buffers)
    QLX_HIP(hipMemcpyAsync(m->d_grads, grads, kNumParams * 4, hipMemcpyHostToDevice, s));
    if (m->f32) {
      m->f32_update_scheduled = false;
      model_norms(m, s, scale);
    } else {
      m->norms_fused = false;
      hipLaunchKernelGGL(k_sumsq, dim3(m->n_ranges), dim3(256), 0, s, m->d_grads, m->d_rbeg, m->d_rend, scale, m->d_partial);
      QLX_HIP(hipGetLastError());
    }
    model_adam(m, s, scale);
    if (norms_out) QLX_HIP(hipMemcpyAsync(norms_out, m->d_norms, kNumVars * 4, hipMemcpyDeviceToHost, s));
    QLX_HIP(hipStreamSynchronize(s));
  });
}

int32_t qlx_model_last_activation(qlx_model* m, int32_t layer, float* out) {
  return guard([&] {
    QLX_CHECK(m && out && layer >= 1 && layer <= 4 && m->ws_batch > 0, QLX_E_INVALID, "bad argument");
    QLX_HIP(hipSetDevice(m->device));
    if (m->f32) {   // a1..a3 of the last forward chunk (the whole batch up to kF32FwdChunk samples), a4 of all
      QLX_CHECK(layer == 4 || m->last_batch <= m->w.fchunk, QLX_E_STATE, "activations of a chunked forward");
      model_dense_join(m, m->stream);
      QLX_HIP(hipStreamSynchronize(m->stream));
      const size_t per[5] = {0, 12800, 5184, 3136, 512};
      const float* src = layer == 1 ? m->w.fa1 : layer == 2 ? m->w.fa2 : layer == 3 ? m->w.fa3 : m->w.fa4;
      QLX_HIP(hipMemcpy(out, src, per[layer] * (size_t)m->last_batch * 4, hipMemcpyDeviceToHost));
      return;
    }
    if (layer == 4 && m->w.a4_splits > 0) {   // forward without a head yet: finish a4 from the fc1 partials
      const int B = m->last_batch;
      hipLaunchKernelGGL(k_slab_reduce_bias_relu, dim3(std::min(2048, (B * 512 + 255) / 256)), dim3(256), 0, m->stream,
                         m->w.fc1slab, (size_t)B * 512, m->w.a4_splits, B, 512, m->d_params + var_offset(7), m->w.a4);
      QLX_HIP(hipGetLastError());
      m->w.a4_splits = 0;
    }
    model_dense_join(m, m->stream);
    QLX_HIP(hipStreamSynchronize(m->stream));
    const size_t per[5] = {0, 12800, 5184, 3136, 512};
    const bf16* src = layer == 1 ? m->w.a1 : layer == 2 ? m->w.a2 : layer == 3 ? m->w.a3 : m->w.a4;
    const size_t count = per[layer] * (size_t)m->last_batch;
    std::vector<uint16_t> tmp(count);
    if (layer == 3)   // rows kA3Ld apart
      QLX_HIP(hipMemcpy2D(tmp.data(), 3136 * 2, src, (size_t)kA3Ld * 2, 3136 * 2, (size_t)m->last_batch, hipMemcpyDeviceToHost));
    else
      QLX_HIP(hipMemcpy(tmp.data(), src, count * 2, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < count; ++i) {
      const uint32_t b = (uint32_t)tmp[i] << 16;
      std::memcpy(&out[i], &b, 4);
    }
  });
}

int32_t qlx_model_write_checkpoint(qlx_model* m, const char* path) {
  return guard([&] {
    QLX_CHECK(m && path, QLX_E_INVALID, "bad argument");
    model_dense_join(m, m->stream);
    QLX_HIP(hipStreamSynchronize(m->stream));
    std::vector<float> buf(kNumParams * 3);
    QLX_HIP(hipMemcpy(buf.data(), m->d_params, kNumParams * 4, hipMemcpyDeviceToHost));
    QLX_HIP(hipMemcpy(buf.data() + kNumParams, m->d_m, kNumParams * 4, hipMemcpyDeviceToHost));
    QLX_HIP(hipMemcpy(buf.data() + 2 * kNumParams, m->d_v, kNumParams * 4, hipMemcpyDeviceToHost));
    FILE* f = std::fopen(path, "wb");
    QLX_CHECK(f, QLX_E_IO, std::string("cannot open ") + path);
    const char magic[8] = {'Q', 'L', 'X', 'C', 'K', 'P', 'T', '1'};
    const int64_t hdr[2] = {kNumParams, m->iterations};
    bool ok = std::fwrite(magic, 1, 8, f) == 8 && std::fwrite(hdr, 8, 2, f) == 2 &&
              std::fwrite(buf.data(), 4, buf.size(), f) == buf.size();
    ok = (std::fclose(f) == 0) && ok;
    QLX_CHECK(ok, QLX_E_IO, "checkpoint write failed");
  });
}

int32_t qlx_model_load_tf(qlx_model* m, const char* prefix) {
  return guard([&] {
    QLX_CHECK(m && prefix, QLX_E_INVALID, "null argument");
    std::vector<float> w, mm, vv;
    int64_t it = 0;
    load_keras_bundle(prefix, 5, kVarSize, w, mm, vv, &it);
    QLX_HIP(hipSetDevice(m->device));
    model_dense_join(m, m->stream);
    QLX_HIP(hipStreamSynchronize(m->stream));
    QLX_HIP(hipMemcpy(m->d_params, w.data(), kNumParams * 4, hipMemcpyHostToDevice));
    QLX_HIP(hipMemcpy(m->d_m, mm.data(), kNumParams * 4, hipMemcpyHostToDevice));
    QLX_HIP(hipMemcpy(m->d_v, vv.data(), kNumParams * 4, hipMemcpyHostToDevice));
    m->iterations = it;
    model_pack(m);
    model_dense_join(m, m->stream);
    QLX_HIP(hipStreamSynchronize(m->stream));
  });
}

int32_t qlx_model_read_checkpoint(qlx_model* m, const char* path) {
  return guard([&] {
    QLX_CHECK(m && path, QLX_E_INVALID, "bad argument");
    FILE* f = std::fopen(path, "rb");
    QLX_CHECK(f, QLX_E_IO, std::string("cannot open ") + path);
    char magic[8];
    int64_t hdr[2];
    std::vector<float> buf(kNumParams * 3);
    bool ok = std::fread(magic, 1, 8, f) == 8 && std::memcmp(magic, "QLXCKPT1", 8) == 0 && std::fread(hdr, 8, 2, f) == 2 &&
              hdr[0] == kNumParams && std::fread(buf.data(), 4, buf.size(), f) == buf.size();
    std::fclose(f);
    QLX_CHECK(ok, QLX_E_IO, "not a qlx checkpoint");
    QLX_HIP(hipSetDevice(m->device));
    model_dense_join(m, m->stream);
    QLX_HIP(hipStreamSynchronize(m->stream));
    QLX_HIP(hipMemcpy(m->d_params, buf.data(), kNumParams * 4, hipMemcpyHostToDevice));
    QLX_HIP(hipMemcpy(m->d_m, buf.data() + kNumParams, kNumParams * 4, hipMemcpyHostToDevice));
    QLX_HIP(hipMemcpy(m->d_v, buf.data() + 2 * kNumParams, kNumParams * 4, hipMemcpyHostToDevice));
    m->iterations = hdr[1];
    model_pack(m);
    model_dense_join(m, m->stream);
    QLX_HIP(hipStreamSynchronize(m->stream));
  });
}

int32_t qlx_model_sync(qlx_model* m) {
  return guard([&] {
    QLX_CHECK(m, QLX_E_INVALID, "null model");
    model_dense_join(m, m->stream);
    QLX_HIP(hipStreamSynchronize(m->stream));
  });
}

}  // extern "C"
