// fp32 DeepQLearningModel path (the reference's arithmetic): Nature-DQN forward / Huber / backward /
// clip_by_norm / Adam on v_mfma_f32_16x16x4_f32, bit-exact against oracle/qnet32_ref.cpp.
//
// Reference (restated): create_ql_model_breakout_84x84x4_3_32.py:20-33 (float32 Keras graph), :36-55 (predict_action,
// batch_predict_max_future_reward), :63-82 (train_model; intended q_a = Q(s)[a] of
// create_ql_model_ballgame_3x3x4_5_512.py:71-78), legacy Keras Adam(lr 2.5e-4, clipnorm 1.0) = tf.clip_by_norm per
// variable + ResourceApplyAdam, Huber(delta = 1) mean over the batch.  Orders of every reduction: DESIGN.md §6.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <map>
#include <tuple>
#include <vector>

#include "objects.h"
#include "profiler.h"
#include "qnet.h"
#include "qnet32_kernels.h"

namespace qlx {

using namespace q32;

static int64_t voff(int v) {
  int64_t o = 0;
  for (int i = 0; i < v; ++i) o += kVarSize[i];
  return o;
}

// ---------------------------------------------------------------------------------------------------------------
// dense 512 -> 3 head: q[b][n] = (fmaf chain over k ascending of a4[b][k] W4[k][n]) + b4[n], as the MFMA product
// W4^T a4^T (one wave per 16 samples: A = W4^T rows n < 3, B = a4 columns; each output is the k-ordered chain), the
// three q of a sample in one lane.
//   MODE 0: q;  1: q + argmax (predict_action);  2: Bellman target y = r + max_a q * gamma (or q at the online net's
//   argmax, double DQN), y = r if done;  3: training head (Huber value h, dloss/dq_a g, |e|) and, with dz4_out, the
//   dense-3 backward dz4[b][k] = (a4 > 0) ? W4[k][a_b] * g_b : 0 (dq is g_b at a_b and 0 elsewhere, so the fmaf chain
//   over n of W4[k][n] dq[b][n] is the single rounded product)
// Block = 16 samples; wave w chains the k quarter [128 w, 128 w + 128) on v_mfma_f32_16x16x4_f32 (A = W4^T rows n < 3,
// B = a4 columns), q = (((C0 + C1) + C2) + C3) + b4: four 32-step chains side by side instead of one 128-step chain.
// The block's 16 a4 rows and W4 are staged in LDS with coalesced 16-byte loads (one memory round), the MFMA operands and
// the dz4 epilogue read them from there.  Row pitch 514 floats: a fragment read's 32-lane group (16 rows x 2 k) hits 32
// distinct banks (ds_read_b32: 32 banks, (address / 4) mod 32); rows are 8-byte aligned, so stores / epilogue reads are b64.
constexpr int kHeadPitch = 514;
template <int MODE, int HS = 16>   // HS samples per block (<= 16: rows past HS are MFMA padding)
__global__ __launch_bounds__(256) void k_head32(Fc2Args A) {
  __shared__ f32x4 part[4][16];
  __shared__ float gsh[16];
  __shared__ int ash[16];
  __shared__ __attribute__((aligned(16))) float xs[16 * kHeadPitch];
  __shared__ __attribute__((aligned(16))) float w4s[512 * 3];
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int s0 = blockIdx.x * HS;
  const int j = lane & 15, g = lane >> 4, n = lane & 15;
  const int b = s0 + j;
  const bool valid = j < HS && b < A.B;
  // the per-sample operands of the head's tail, loaded with the stage (one memory round instead of a second one after the
  // MFMA chain): MODE 3 action, target and IS weight; MODE 2 reward, done and the double-DQN selector's q
  const bool tail = wave == 0 && g == 0 && valid;
  const int bt = tail ? b : 0;
  int t_act = 0;
  float t_y = 0.0f, t_w = 1.0f, t_r = 0.0f, t_qs[3] = {0.0f, 0.0f, 0.0f};
  bool t_done = false;
  if (tail) {
    if (MODE == 3) {
      t_act = A.actions[bt];
      t_y = A.y[bt];
      if (A.weights) t_w = A.weights[bt];
    } else if (MODE == 2) {
      t_r = A.rewards[bt];
      t_done = A.dones[bt] != 0;
      if (A.q_select)
        for (int r = 0; r < 3; ++r) t_qs[r] = A.q_select[bt * 3 + r];
    }
  }
  {   // stage: 16 rows x 128 float4 of a4 (8 per thread; rows past B read row s0) and W4's 384 float4
    f32x4 xr[8], wr[2];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int f = threadIdx.x + 256 * r, jj = f >> 7, k4 = f & 127;
      xr[r] = ld4(A.a4f + (size_t)(jj < HS && s0 + jj < A.B ? s0 + jj : s0) * 512 + 4 * k4);
    }
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int f = threadIdx.x + 256 * r;
      if (f < 384) wr[r] = ld4(A.w4 + 4 * f);
    }
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int f = threadIdx.x + 256 * r, jj = f >> 7, k4 = f & 127;
      f32x2* d = reinterpret_cast<f32x2*>(xs + jj * kHeadPitch + 4 * k4);
      d[0] = f32x2{xr[r][0], xr[r][1]};
      d[1] = f32x2{xr[r][2], xr[r][3]};
    }
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int f = threadIdx.x + 256 * r;
      if (f < 384) *reinterpret_cast<f32x4*>(w4s + 4 * f) = wr[r];
    }
  }
  __syncthreads();
  const float* x = xs + j * kHeadPitch + 128 * wave + g;        // a4[b][128 w + 4 t + g]
  const float* wp = w4s + (128 * wave + g) * 3 + (n < 3 ? n : 0);   // W4[128 w + 4 t + g][n]
  float wv[32], xv[32];
#pragma unroll
  for (int t = 0; t < 32; ++t) wv[t] = wp[t * 12];
#pragma unroll
  for (int t = 0; t < 32; ++t) xv[t] = x[4 * t];
  f32x4 acc = zero4();
#pragma unroll
  for (int t = 0; t < 32; ++t) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(n < 3 ? wv[t] : 0.0f, xv[t], acc, 0, 0, 0);
  if (g == 0) part[wave][j] = acc;   // lane (j, 0): rows n = 0 .. 3 of sample j
  __syncthreads();
  if (wave == 0 && g == 0 && valid) {
    const f32x4 c0 = part[0][j], c1 = part[1][j], c2 = part[2][j], c3 = part[3][j];
    float qv[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) qv[r] = __fadd_rn(__fadd_rn(__fadd_rn(__fadd_rn(c0[r], c1[r]), c2[r]), c3[r]), A.b4[r]);
    const float q0 = qv[0], q1 = qv[1], q2 = qv[2];
    if (A.q) { A.q[b * 3 + 0] = q0; A.q[b * 3 + 1] = q1; A.q[b * 3 + 2] = q2; }
    if (MODE == 1) {   // tf.argmax: first maximal index
      int best = 0;
      float bv = q0;
      if (q1 > bv) { best = 1; bv = q1; }
      if (q2 > bv) best = 2;
      A.argmax[b] = (uint8_t)best;
    } else if (MODE == 2) {
      float mx;
      if (A.q_select) {
        int best = 0;
        float bv = t_qs[0];
        if (t_qs[1] > bv) { best = 1; bv = t_qs[1]; }
        if (t_qs[2] > bv) best = 2;
        mx = best == 0 ? q0 : (best == 1 ? q1 : q2);
      } else {
        mx = fmaxf(fmaxf(q0, q1), q2);
      }
      const float r = t_r;
      // add_arrays(reward, array_mul(max_future, gamma)) (self_driving_tf_q_learner.rs:189-199,298-315): two roundings
      A.y_out[b] = t_done ? r : __fadd_rn(r, __fmul_rn(mx, A.gamma));
    } else if (MODE == 3) {
      const int a = t_act;
      const float qa = a == 0 ? q0 : (a == 1 ? q1 : q2);
      const float e = __fsub_rn(qa, t_y);
      const float ae = fabsf(e);
      const float wgt = t_w;   // prioritized replay: the IS weight scales h and dloss/dq
      const float ge = ae <= 1.0f ? e : (e > 0.0f ? 1.0f : -1.0f);
      const float gb = __fmul_rn(wgt, ge) / (float)A.B;
      A.gsample[b] = gb;
      A.hsample[b] = __fmul_rn(wgt, ae <= 1.0f ? __fmul_rn(__fmul_rn(0.5f, e), e) : __fsub_rn(ae, 0.5f));
      if (A.td_abs) A.td_abs[b] = ae;
      gsh[j] = gb;
      ash[j] = a;
    }
  }
  if (MODE == 3 && A.dz4_out) {   // the block's 16 x 512 dz4 as float4s, 8 per thread (a4 and W4 from LDS)
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int f = threadIdx.x + 256 * r, jj = f >> 7, k = 4 * (f & 127), bb = s0 + jj;
      if (jj < HS && bb < A.B) {
        const f32x2* xp = reinterpret_cast<const f32x2*>(xs + jj * kHeadPitch + k);
        const f32x2 x01 = xp[0], x23 = xp[1];
        const float xa[4] = {x01[0], x01[1], x23[0], x23[1]};
        const int a = ash[jj];
        const float gb = gsh[jj];
        f32x4 d;
#pragma unroll
        for (int e = 0; e < 4; ++e) d[e] = xa[e] > 0.0f ? __fmul_rn(w4s[(k + e) * 3 + a], gb) : 0.0f;
        *reinterpret_cast<f32x4*>(A.dz4_out + (size_t)bb * 512 + k) = d;
      }
    }
  }
}

// clip_by_norm sums of squares: segment j of variable v = elements [j S, min(n_v, (j + 1) S)), S = kNormSeg = 2048;
// thread t chains t = fmaf(x, x, t) over its elements j S + 4 t .. + 3, then j S + 1024 + 4 t .. + 3 (x = g * scale);
// wave xor butterfly (32, 16, .., 1); then ((w0 + w1) + w2) + w3 -> partial j.  Norm_v from its partials in k_update32.
// (Measured and reverted: the last block to finish - a device-scope counter - reducing the partials to the ten norms, so
// Adam loads ten values: Adam 16.3 -> 12.5 us, but the per-block release fence took the norm launch 6.2 -> 24.6 us.)
constexpr int kNormSeg = 2048;
constexpr int kNormSegMax = 832;   // partials per variable (13 per lane; W3 has 784)
struct NormArgs {
  const float* g;
  float scale;
  float* partial;
  int seg_first[kNumVars + 1];
  int64_t off[kNumVars + 1];
};
// thread tl (0 .. 255) of segment j of variable v (elements off[v] ..): its fmaf chain over its eight elements, then its
// wave's xor butterfly (every lane ends with the wave sum); segments past the variable's end chain zeros.
// The loads are split from the chain so a caller can put every segment's loads in flight before the first add: variables
// whose length is a multiple of 4 (all but b4) read through a buffer descriptor spanning the variable, elements past its
// end reading as zeros - no per-lane branch around the loads (round 5: the branchy form serialised the five segment
// rounds of a conv update block).
struct NormLd {
  f32x4 x[2];
};
__device__ __forceinline__ NormLd norm32_load(const float* gall, const int64_t* off, int v, int j, int tl, bool live) {
  const int64_t n = off[v + 1] - off[v];
  const int64_t b = (int64_t)j * kNormSeg;
  const float* g = gall + off[v];   // variable offsets are multiples of 4 floats (16-byte loads)
  NormLd L;
  if (n % 4 == 0) {   // wave-uniform
    const __amdgpu_buffer_rsrc_t rs = buf_rsrc(g, live ? (uint32_t)(n * 4) : 0u);
#pragma unroll
    for (int h = 0; h < 2; ++h) L.x[h] = buf_ld4(rs, (uint32_t)((b + 1024 * h + 4 * tl) * 4), 0);
    return L;
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int64_t i = b + 1024 * h + 4 * tl;
#pragma unroll
    for (int k = 0; k < 4; ++k) L.x[h][k] = live && i + k < n ? g[i + k] : 0.0f;   // zeros leave the chain unchanged
  }
  return L;
}
__device__ __forceinline__ float norm32_chain(const NormLd& L, float scale) {
  float t = 0.0f;
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float y = __fmul_rn(L.x[h][k], scale);
      t = fmaf(y, y, t);
    }
  for (int o = 32; o > 0; o >>= 1) t = __fadd_rn(t, __shfl_xor(t, o));
  return t;
}
__device__ __forceinline__ float norm32_lane(const float* gall, const int64_t* off, float scale, int v, int j, int tl) {
  return norm32_chain(norm32_load(gall, off, v, j, tl, true), scale);
}

// Conv weight gradients from the sample-chunk partials, two levels: the chunks in groups of kWGroup (group q = chunks
// [16 q, 16 q + 16)), S_q = chain over its chunks in order, dW = chain over q of S_q (each chain t = 0; t = t + x).
// Segment 0 conv3 [577][64], 1 conv2 [513][64], 2 conv1 [257][32], rows in HWIO order, the last row of each the bias.
// Block = 16 waves = 16 / W slices of 64 consecutive outputs, W waves per slice (W = wv[L], the power of two >= the
// segment's group count, at most 16; 256-byte rows per load): wave g of a slice chains groups g, g + W, .. (16 partial
// loads in flight each); the group sums meet in LDS and the slice's wave 0 chains them in q order.  (One slice per block
// left 12 of 16 waves idle at 64 chunks - conv2 / conv3 at B = 1024 - and held the CUs' wave slots.)
constexpr int kWGroup = 16;
constexpr int kWGroupsMax = 256;   // chunks <= 4,096 (conv1 at the largest fp32 batch, 8,192, in chunks of 2)
struct WRed {
  const float* slab[3];
  int nz[3];
  int count[3];   // (M + 1) * OC; segments 0 and 1 are multiples of 64
  int oc[3];
  int wv[3];      // waves per 64-output slice
  int nb[3];      // blocks of the segment
  float* gw[3];   // W gradient
  float* gb[3];   // b gradient
  // segments 0, 1 (conv3, conv2: compacted weight gradients; null: none): each chunk's partial gets u[m] S[z][n] first
  // (fmaf; u[m] = the layer's constant input row at channel m % C - conv2: relu(b0), C = 32; conv3: c2, C = 64 - and 1
  // for the bias row): the chunk's background rows (PConvWgrad CMP)
  const float* sbg[2];
  const float* ubg[2];
};
__host__ __device__ inline int wred_waves(int nz) {
  const int ng = (nz + kWGroup - 1) / kWGroup;
  int w = 1;
  while (w < ng && w < 16) w *= 2;
  return w;
}
// Blocks [nred, ..) of the launch (update schedule 2, qnet.h): clip-norm segment partials of segments seg0 .. seg0 + nseg
// - the dense variables', final since the fc1 backward - four 256-thread groups per block, one segment's
// arithmetic each (norm32_lane, then ((w0 + w1) + w2) + w3).
__global__ __launch_bounds__(1024) void k_wreduce32(WRed R, NormArgs N, int nred, int seg0, int nseg) {
  __shared__ float gs[kWGroupsMax * 64];
  if ((int)blockIdx.x >= nred) {
    const int grp = threadIdx.x >> 8, tl = threadIdx.x & 255;
    const int sg = seg0 + 4 * ((int)blockIdx.x - nred) + grp;
    const bool live = sg < seg0 + nseg;
    int v = 0;
    while (v < kNumVars - 1 && sg >= N.seg_first[v + 1]) ++v;
    const float t = live ? norm32_lane(N.g, N.off, N.scale, v, sg - N.seg_first[v], tl) : 0.0f;
    if ((tl & 63) == 0) gs[grp * 4 + (tl >> 6)] = t;
    __syncthreads();
    if (tl == 0 && live) N.partial[sg] = __fadd_rn(__fadd_rn(__fadd_rn(gs[grp * 4], gs[grp * 4 + 1]), gs[grp * 4 + 2]), gs[grp * 4 + 3]);
    return;
  }
  int b = blockIdx.x, L = 0;
  while (L < 3 && b >= R.nb[L]) { b -= R.nb[L]; ++L; }
  if (L >= 3) return;   // block-uniform
  const int W = R.wv[L], o = threadIdx.x & 63, wave = threadIdx.x >> 6, sub = wave / W, g0 = wave - sub * W;
  const int e = (b * (16 / W) + sub) * 64;
  const bool live = e + o < R.count[L];
  const size_t stride = (size_t)R.count[L];
  const int nz = R.nz[L], ng = (nz + kWGroup - 1) / kWGroup;
  const float* p = R.slab[L] + (live ? e + o : 0);
  float* gsub = gs + sub * ng * 64;   // (16 / W) * ng <= kWGroupsMax slices of 64
  const float* sbg = L < 2 ? R.sbg[L] : nullptr;   // (block-uniform)
  const bool bg = sbg != nullptr;
  const int oc = R.oc[L], me = (e + o) / oc, ne = (e + o) - me * oc;
  const int Mr = R.count[L] / oc - 1, uc = L == 0 ? 64 : 32;
  const float um = bg && live ? (me < Mr ? R.ubg[L][me % uc] : 1.0f) : 0.0f;
  for (int q = g0; q < ng; q += W) {
    float v[kWGroup];
#pragma unroll
    for (int j = 0; j < kWGroup; ++j) v[j] = q * kWGroup + j < nz ? p[(size_t)(q * kWGroup + j) * stride] : 0.0f;
    if (bg) {
#pragma unroll
      for (int j = 0; j < kWGroup; ++j)
        if (q * kWGroup + j < nz) v[j] = fmaf(um, sbg[(size_t)(q * kWGroup + j) * 64 + ne], v[j]);
    }
    float t = 0.0f;
#pragma unroll
    for (int j = 0; j < kWGroup; ++j) t = __fadd_rn(t, v[j]);   // + 0 past the last chunk leaves t unchanged
    gsub[q * 64 + o] = t;
  }
  __syncthreads();
  if (g0 != 0 || !live) return;
  float t = 0.0f;
  for (int q = 0; q < ng; ++q) t = __fadd_rn(t, gsub[q * 64 + o]);
  const int m = me, n = ne;
  const int M = R.count[L] / oc - 1;
  if (m == M) R.gb[L][n] = t;
  else R.gw[L][(size_t)m * oc + n] = t;
}

struct Adam32Args {
  float* w;
  float* m;
  float* v;
  const float* g;
  const float* partial;
  int seg_first[kNumVars + 1];
  int64_t off[kNumVars + 1];
  float* norms;
  float scale, alpha, beta1, beta2, eps, clipnorm;
};

// tf.clip_by_norm + ResourceApplyAdam per element, explicit roundings in the oracle's order
__device__ __forceinline__ float adam32_elem(float g, float scale, float clipnorm, float denom, float alpha, float beta1,
                                             float beta2, float eps, float& m, float& v, float w) {
  const float gc = __fmul_rn(__fmul_rn(g, scale), clipnorm) / denom;
  m = __fadd_rn(m, __fmul_rn(__fsub_rn(gc, m), 1.0f - beta1));
  v = __fadd_rn(v, __fmul_rn(__fsub_rn(__fmul_rn(gc, gc), v), 1.0f - beta2));
  return __fsub_rn(w, __fmul_rn(m, alpha) / __fadd_rn(sqrtf(v), eps));
}

// the variable of flat element i (branch-free: the number of variable starts at or below i, minus one)
__device__ __forceinline__ int var_of(const Adam32Args& A, int64_t i) {
  int v = 0;
#pragma unroll
  for (int k = 1; k < kNumVars; ++k) v += i >= A.off[k] ? 1 : 0;
  return v;
}

// norm_v for v = V0 .. 9 into nrm[v] (wave 0; lane chain over the partials lane, lane + 64, ... of v - zeros past the
// end - then the xor butterfly).  Every partial is loaded at once (13 per lane for W3, one per lane for each smaller
// variable: one memory round), through buffer descriptors spanning each variable's partials (past the end reads 0, no
// per-lane branch - the branchy form put a vmcnt(0) after several of these loads).  write: also store them to A.norms.
struct NormPart {
  float x[kNormSegMax / 64], y[kNumVars];
};
template <int V0>
__device__ __forceinline__ void norms_load(const Adam32Args& A, int lane, NormPart& P) {
  const int f6 = A.seg_first[6], c6 = A.seg_first[7] - f6;
  const __amdgpu_buffer_rsrc_t r6 = buf_rsrc(A.partial + f6, (uint32_t)c6 * 4u);
#pragma unroll
  for (int i = 0; i < kNormSegMax / 64; ++i) P.x[i] = buf_ld1(r6, (uint32_t)(lane + 64 * i) * 4u, 0);
#pragma unroll
  for (int vv = V0; vv < kNumVars; ++vv) {
    const int f = A.seg_first[vv], c = A.seg_first[vv + 1] - f;
    P.y[vv] = vv != 6 ? buf_ld1(buf_rsrc(A.partial + f, (uint32_t)c * 4u), (uint32_t)lane * 4u, 0) : 0.0f;   // <= 64 partials
  }
}
template <int V0>
__device__ __forceinline__ void norms_sum(const Adam32Args& A, int lane, const NormPart& P, float* nrm, bool write) {
#pragma unroll
  for (int vv = V0; vv < kNumVars; ++vv) {
    float t = 0.0f;
    if (vv == 6) {
#pragma unroll
      for (int i = 0; i < kNormSegMax / 64; ++i) t = __fadd_rn(t, P.x[i]);
    } else {
      t = __fadd_rn(t, P.y[vv]);
    }
    for (int o = 32; o > 0; o >>= 1) t = __fadd_rn(t, __shfl_xor(t, o));
    if (lane == 0) {
      nrm[vv] = t > 0.0f ? sqrtf(t) : t;   // safe sqrt via where(l2sum > 0)
      if (write) A.norms[vv] = nrm[vv];
    }
  }
}

// The dense variables' blocks of k_update32: clip_by_norm + Adam of W3, b3, W4, b4 (95 % of the update's Adam bytes)
// from their norm partials.  Explicit roundings in the oracle's order (adam32_elem).
struct AdamDense {
  static constexpr size_t LDS = 64;
  Adam32Args A;
  int nblocks;
  __host__ __device__ int blocks() const { return nblocks; }
  __device__ void run(int t, float* lds) const {
    float* nrm = lds;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t o6 = A.off[6], count = A.off[kNumVars], n4 = (count - o6) / 4;   // o6 is a multiple of 4
    const int64_t st = (int64_t)nblocks * blockDim.x, q0 = (int64_t)t * blockDim.x + threadIdx.x;
    const bool two = 2 * st > n4;   // (wave-uniform)
    const int64_t qq[2] = {q0, q0 + st};
    f32x4 g[2], w[2], m[2], v[2];
    NormPart P;
    if (wave == 0) norms_load<6>(A, lane, P);   // the norm partials first, then the element loads: one memory round for both
    if (two) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int64_t i0 = o6 + (qq[u] < n4 ? qq[u] : 0) * 4;
        g[u] = ld4(A.g + i0);
        w[u] = ld4(A.w + i0);
        m[u] = ld4(A.m + i0);
        v[u] = ld4(A.v + i0);
      }
    }
    if (wave == 0) norms_sum<6>(A, lane, P, nrm, t == 0);
    lds_barrier();   // (LDS only: the element loads stay in flight)
    if (two) {   // at most two float4 groups per thread (k_update32's grid): all eight loads in one round
      // (measured: 16.3 -> 14.8 us per update against one group per thread on twice the blocks)
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (qq[u] >= n4) continue;
        const int64_t i0 = o6 + qq[u] * 4;
        const float denom = fmaxf(nrm[var_of(A, i0)], A.clipnorm);
        f32x4 o;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          float mk = m[u][k], vk = v[u][k];
          o[k] = adam32_elem(g[u][k], A.scale, A.clipnorm, denom, A.alpha, A.beta1, A.beta2, A.eps, mk, vk, w[u][k]);
          m[u][k] = mk;
          v[u][k] = vk;
        }
        *reinterpret_cast<f32x4*>(A.w + i0) = o;
        *reinterpret_cast<f32x4*>(A.m + i0) = m[u];
        *reinterpret_cast<f32x4*>(A.v + i0) = v[u];
      }
      if (q0 == n4 || q0 + st == n4)   // the tail group, element by element
        for (int64_t i = o6 + n4 * 4; i < count; ++i) {
          const float denom = fmaxf(nrm[var_of(A, i)], A.clipnorm);
          float mi = A.m[i], vi = A.v[i];
          A.w[i] = adam32_elem(A.g[i], A.scale, A.clipnorm, denom, A.alpha, A.beta1, A.beta2, A.eps, mi, vi, A.w[i]);
          A.m[i] = mi;
          A.v[i] = vi;
        }
      return;
    }
    for (int64_t q = q0; q <= n4; q += st) {
      const int64_t i0 = o6 + q * 4;
      if (q < n4) {
        const float denom = fmaxf(nrm[var_of(A, i0)], A.clipnorm);
        const f32x4 g = ld4(A.g + i0), w = ld4(A.w + i0);
        f32x4 m = ld4(A.m + i0), v = ld4(A.v + i0), o;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          float mk = m[k], vk = v[k];
          o[k] = adam32_elem(g[k], A.scale, A.clipnorm, denom, A.alpha, A.beta1, A.beta2, A.eps, mk, vk, w[k]);
          m[k] = mk;
          v[k] = vk;
        }
        *reinterpret_cast<f32x4*>(A.w + i0) = o;
        *reinterpret_cast<f32x4*>(A.m + i0) = m;
        *reinterpret_cast<f32x4*>(A.v + i0) = v;
      } else {
        for (int64_t i = i0; i < count; ++i) {
          const float denom = fmaxf(nrm[var_of(A, i)], A.clipnorm);
          float mi = A.m[i], vi = A.v[i];
          A.w[i] = adam32_elem(A.g[i], A.scale, A.clipnorm, denom, A.alpha, A.beta1, A.beta2, A.eps, mi, vi, A.w[i]);
          A.m[i] = mi;
          A.v[i] = vi;
        }
      }
    }
  }
};

// clip_by_norm + Adam of the six conv variables (W0 .. b2, 78K elements) in one launch of independent 1024-thread blocks:
// block = (variable v, chunk c of 4,096 elements).  Each block finishes v's norm itself - every gradient element of v
// loaded at once (four 256-thread groups, group q taking segments q, q + 4, .., each with one segment's
// arithmetic), then the partials and the final chain in LDS - and updates its chunk (one float4 per thread).  The
// re-read of v per chunk (<= 147 KB, from L2) buys a launch with one memory round per phase.
constexpr int kConvAdamChunk = 4096;
constexpr int kConvSegsPerGroup = 5;   // segments per 256-thread group: W2 has 18 = 4 x 4 + 2
__device__ __forceinline__ void conv_adam_block(const Adam32Args& A, const NormArgs& N, int blk) {
  __shared__ float wsum[kConvSegsPerGroup][4][4];
  __shared__ float part[64];
  __shared__ float nrm;
  // block -> (variable, chunk): chunks of the six variables in order
  int v = 0, c = blk;
  for (;;) {
    const int nc = (int)((A.off[v + 1] - A.off[v] + kConvAdamChunk - 1) / kConvAdamChunk);
    if (c < nc || v == 5) break;
    c -= nc;
    ++v;
  }
  const int grp = threadIdx.x >> 8, tl = threadIdx.x & 255, lane = threadIdx.x & 63;
  const int nseg = N.seg_first[v + 1] - N.seg_first[v];
  // this thread's float4 of the chunk, loaded in the same memory round as the norm's gradient reads
  const int64_t o = A.off[v], n = A.off[v + 1] - o;   // conv variables are multiples of 4 long
  const int64_t e = (int64_t)c * kConvAdamChunk + 4 * threadIdx.x, i0 = o + e;
  f32x4 g = zero4(), w = zero4(), m = zero4(), vv = zero4();
  if (e < n) {
    g = ld4(A.g + i0);
    w = ld4(A.w + i0);
    m = ld4(A.m + i0);
    vv = ld4(A.v + i0);
  }
  // every segment's loads in flight at once, then the chains (segments past the variable: zeros, t = 0)
  NormLd ld[kConvSegsPerGroup];
#pragma unroll
  for (int r = 0; r < kConvSegsPerGroup; ++r) ld[r] = norm32_load(N.g, N.off, v, grp + 4 * r, tl, grp + 4 * r < nseg);
  float t[kConvSegsPerGroup];
#pragma unroll
  for (int r = 0; r < kConvSegsPerGroup; ++r) t[r] = grp + 4 * r < nseg ? norm32_chain(ld[r], N.scale) : 0.0f;
#pragma unroll
  for (int r = 0; r < kConvSegsPerGroup; ++r)
    if ((tl & 63) == 0) wsum[r][grp][tl >> 6] = t[r];
  __syncthreads();
  if (tl == 0) {
#pragma unroll
    for (int r = 0; r < kConvSegsPerGroup; ++r) {
      const int j = grp + 4 * r;
      if (j < nseg) part[j] = __fadd_rn(__fadd_rn(__fadd_rn(wsum[r][grp][0], wsum[r][grp][1]), wsum[r][grp][2]), wsum[r][grp][3]);
    }
  }
  __syncthreads();
  if (threadIdx.x < 64) {   // <= 64 partials: each lane's chain is 0 + its partial
    float s = __fadd_rn(0.0f, lane < nseg ? part[lane] : 0.0f);
    for (int o = 32; o > 0; o >>= 1) s = __fadd_rn(s, __shfl_xor(s, o));
    if (lane == 0) {
      nrm = s > 0.0f ? sqrtf(s) : s;
      if (c == 0) A.norms[v] = nrm;
    }
  }
  __syncthreads();
  const float denom = fmaxf(nrm, A.clipnorm);
  if (e < n) {
    f32x4 out;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float mk = m[k], vk = vv[k];
      out[k] = adam32_elem(g[k], A.scale, A.clipnorm, denom, A.alpha, A.beta1, A.beta2, A.eps, mk, vk, w[k]);
      m[k] = mk;
      vv[k] = vk;
    }
    *reinterpret_cast<f32x4*>(A.w + i0) = out;
    *reinterpret_cast<f32x4*>(A.m + i0) = m;
    *reinterpret_cast<f32x4*>(A.v + i0) = vv;
  }
}

// The scheduled update (qnet.h f32_update_scheduled): clip_by_norm + Adam of every variable in one launch after the
// weight-gradient reduction -
// blocks [0, nconv) the conv variables (conv_adam_block: norm from the gradient itself), the rest the dense variables
// (their segment partials came from the reduction launch; AdamDense arithmetic).  No block depends on another.
__global__ __launch_bounds__(1024) void k_update32(Adam32Args A, NormArgs N, int nconv, int ndense) {
  __shared__ float nrm[kNumVars];
  if ((int)blockIdx.x < nconv) conv_adam_block(A, N, blockIdx.x);
  else AdamDense{A, ndense}.run((int)blockIdx.x - nconv, nrm);
}

static int conv_adam_blocks() {
  int n = 0;
  for (int v = 0; v < 6; ++v) n += (kVarSize[v] + kConvAdamChunk - 1) / kConvAdamChunk;
  return n;
}

// ---------------------------------------------------------------------------------------------------------------
// host side

static size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

#ifndef QLX_PB_OFF
#define QLX_PB_OFF 0   // (timing only: the conv2 backward without conv1's bias partials - the conv1 bias is then wrong)
#endif
constexpr int kSC1 = QLX_F32_WGRAD_CHUNK_CONV1, kSC2 = QLX_F32_WGRAD_CHUNK_CONV2, kSC3 = QLX_F32_WGRAD_CHUNK_CONV3;
// weight-gradient chunk tiles 64 x 64 on 1 x 4 waves (each wave 64 rows x 16 channels): conv3 / conv2 pairs 73.0 -> 72.3 /
// 102.2 -> 101.2 us in place against 2 x 2 (4 x 1: no change; gpurun_out/w14)
// conv3's offset table after the images (3 blocks per CU: pair 72.1 us; in the images' pads, 4 per CU: 76.1 us, held to 3
// by a 44 KB LDS request: 73.1 us - gpurun_out/w22, w31); conv2's in the pads (4 blocks per CU: pair 99.6 -> 96.8 us)
using PConv3Wgrad = PConvWgrad<9, 9, 64, 3, 1, 7, 7, 64, kSC3, 64, 64, 1, 4, 16, false, true>;   // (compacted)
using PConv3WgradD = PConvWgrad<9, 9, 64, 3, 1, 7, 7, 64, kSC3, 64, 64, 1, 4, 16, false>;         // (every row: QLX_F32_BG=0)
static_assert(kSC3 == 16, "conv3 weight-gradient chunks are the fc1 backward's 16-row fragments (pbg)");
using PConv2Wgrad = PConvWgrad<20, 20, 32, 4, 2, 9, 9, 64, kSC2, 64, 64, 1, 4, 16, true, true>;   // (compacted)
using PConv2WgradD = PConvWgrad<20, 20, 32, 4, 2, 9, 9, 64, kSC2, 64, 64, 1, 4>;                  // (every row: QLX_F32_BG=0)
static_assert(kSC2 == 16, "conv2 weight-gradient chunks are the conv3 backward's 16-row fragments (pbg)");

static int segs_of(int v) { return (kVarSize[v] + kNormSeg - 1) / kNormSeg; }
static_assert((1605632 + kNormSeg - 1) / kNormSeg <= kNormSegMax, "norm partials per variable");
static_assert((36864 + kNormSeg - 1) / kNormSeg <= 4 * kConvSegsPerGroup && (32768 + kNormSeg - 1) / kNormSeg <= 4 * kConvSegsPerGroup,
              "conv variable segments per conv_adam_block");
static_assert((512 * 3 + kNormSeg - 1) / kNormSeg <= 64 && (32768 + kNormSeg - 1) / kNormSeg <= 64 &&
              (36864 + kNormSeg - 1) / kNormSeg <= 64 && (8192 + kNormSeg - 1) / kNormSeg <= 64, "<= 64 partials but W3");

static int num_cus();

// conv1 forward blocks for n samples: two per CU, but never more than kC1MaxIt samples per block (a block keeps its samples'
// background flags in LDS until it writes its lists) - so a part with few CUs (a CPX partition) runs more blocks
constexpr int kC1MaxIt = 64;
static int c1_blocks(int n) { return std::max(std::min(n, 2 * num_cus()), (n + kC1MaxIt - 1) / kC1MaxIt); }
// the training-batch forward (n <= 2,048: not a chunk pass) runs one sample per block (k_conv1_fwd32 ONE)
#ifndef QLX_C1_ONE
#define QLX_C1_ONE 1
#endif
#ifndef QLX_C2_FWD_KS
#define QLX_C2_FWD_KS 2   // training-batch conv2 / conv3 list forwards: chains in wave groups (2) or in turn (1)
#endif
#ifndef QLX_C3_FWD_KS
#define QLX_C3_FWD_KS 2
#endif
constexpr int kC2FwdKs = QLX_C2_FWD_KS <= kConvFwdChains ? QLX_C2_FWD_KS : 1;
constexpr int kC3FwdKs = QLX_C3_FWD_KS <= kConvFwdChains ? QLX_C3_FWD_KS : 1;
static bool c1_one(int n) {
  static const bool all = [] { const char* e = std::getenv("QLX_C1_ONE_ALL"); return e && e[0] == '1'; }();   // (A/B)
  return QLX_C1_ONE && (n <= 2048 || all);
}
static int c1_grid(int n) { return c1_one(n) ? n : c1_blocks(n); }

void f32_workspace(qlx_model* m, int B) {
  if (B <= m->ws_batch) return;
  QLX_HIP(hipStreamSynchronize(m->stream));
  if (m->ws) (void)hipFree(m->ws);
  m->ws = nullptr;
  ModelWs& w = m->w;
  const int C = std::min(B, kF32FwdChunk);   // conv activations are held per forward chunk
  size_t off = 0;
  auto take = [&](size_t bytes) { const size_t o = off; off = align_up(off + bytes, 256); return o; };
  const size_t o_frames = take((size_t)B * 4 * kFramePix);
  const size_t o_table = take((size_t)B * 4 * sizeof(void*));
  const size_t o_a1 = take((size_t)C * 12800 * 4), o_a2 = take((size_t)C * 5184 * 4), o_a3 = take((size_t)C * 3136 * 4);
  const size_t o_a4 = take((size_t)B * 512 * 4), o_q = take((size_t)B * 3 * 4);
  const size_t o_gs = take((size_t)B * 4), o_hs = take((size_t)B * 4), o_y = take((size_t)B * 4);
  const size_t o_act = take((size_t)B), o_argmax = take((size_t)B), o_rew = take((size_t)B * 4), o_done = take((size_t)B);
  int nseg = 0;
  for (int v = 0; v < kNumVars; ++v) nseg += segs_of(v);
  const size_t o_part = take((size_t)nseg * 4);
  const size_t o_loss = take(64);
  // row lists: kListSlots regions of ceil(G / kListSlots) blocks x ceil(n / G) samples each (G = c1_blocks(n) for a chunk of
  // n <= C samples): kListSlots x that <= (G + kListSlots)(n / G + 1) = n + G + kListSlots n / G + kListSlots, with
  // G >= min(n, 2 CUs) and G <= max(2 CUs, C / kC1MaxIt + 1) (one sample per block, c1_one: G = n, n + kListSlots)
  const int frl_cap = C + kListSlots * (C / std::max(1, std::min(C, 2 * num_cus())) + 1) +
                      std::max(2 * num_cus(), C / kC1MaxIt + 1) + kListSlots;
  static_assert(2048 + kListSlots <= 2048 + kListSlots * 2, "c1_one list capacity");
  const size_t o_rl2 = take((size_t)frl_cap * 81 * 4), o_rl3 = take((size_t)frl_cap * 49 * 4);
  const size_t o_rcnt = take(2 * 2 * kListSlots * kCntStride * 8), o_bgc = take(160 * 4), o_steps = take((size_t)C * 4 * 4);
  const int need_ld = (C + 63) / 64 * 64;   // (the conv2 backward-data tiles read 64-row blocks of it)
  const size_t o_need = take((size_t)100 * need_ld);
  const size_t o_rows2 = take((size_t)C * 4 * 4), o_bg2 = take((size_t)81 * need_ld);
  const size_t o_rows3 = take((size_t)C * 4 * 4), o_bg3 = take((size_t)49 * need_ld);
  QLX_HIP(hipMalloc(&m->ws, off));
  char* base = (char*)m->ws;
  w.frames = (uint8_t*)(base + o_frames);
  w.table = (const uint8_t**)(base + o_table);
  w.fa1 = (float*)(base + o_a1); w.fa2 = (float*)(base + o_a2); w.fa3 = (float*)(base + o_a3); w.fa4 = (float*)(base + o_a4);
  w.q = (float*)(base + o_q);
  w.gs = (float*)(base + o_gs); w.hs = (float*)(base + o_hs); w.y = (float*)(base + o_y);
  w.act = (uint8_t*)(base + o_act); w.argmax = (uint8_t*)(base + o_argmax); w.rew = (float*)(base + o_rew);
  w.done = (uint8_t*)(base + o_done);
  w.fpart = (float*)(base + o_part);
  w.loss = (float*)(base + o_loss);
  w.frl2 = (int*)(base + o_rl2); w.frl3 = (int*)(base + o_rl3);
  w.frcnt = (unsigned long long*)(base + o_rcnt);
  w.fbgc = (float*)(base + o_bgc);
  w.fsteps = (uint32_t*)(base + o_steps);
  w.fneed = (uint8_t*)(base + o_need);
  w.fneed_ld = need_ld;
  w.frows2 = (uint32_t*)(base + o_rows2);
  w.fbg2 = (uint8_t*)(base + o_bg2);
  w.frows3 = (uint32_t*)(base + o_rows3);
  w.fbg3 = (uint8_t*)(base + o_bg3);
  QLX_HIP(hipMemset(w.frcnt, 0, 2 * 2 * kListSlots * kCntStride * 8));
  w.frl_cap = frl_cap;
  w.fparity = 0;
  w.fchunk = C;
  m->ws_batch = B;
}

// gradient workspace (dz buffers, weight-gradient slabs) for training batches up to B (<= the forward chunk)
static void f32_grad_workspace(qlx_model* m, int B) {
  ModelWs& w = m->w;
  if (B <= w.fgrad_batch) return;
  QLX_HIP(hipStreamSynchronize(m->stream));
  if (w.fgrad) (void)hipFree(w.fgrad);
  w.fgrad = nullptr;
  size_t off = 0;
  auto take = [&](size_t bytes) { const size_t o = off; off = align_up(off + bytes, 256); return o; };
  const size_t o_dz1 = take((size_t)B * 12800 * 4), o_dz2 = take((size_t)B * 5184 * 4), o_dz3 = take((size_t)B * 3136 * 4);
  const size_t o_dz4 = take((size_t)B * 512 * 4);
  const size_t o_s1 = take((size_t)((B + kSC1 - 1) / kSC1) * 257 * 32 * 4);
  const size_t o_s2 = take((size_t)((B + kSC2 - 1) / kSC2) * 513 * 64 * 4);
  const size_t o_s3 = take((size_t)((B + kSC3 - 1) / kSC3) * 577 * 64 * 4);
  const size_t o_pb = take((size_t)((B + 15) / 16) * 400 * 32 * 4);
  const size_t o_pbg = take((size_t)((B + 15) / 16) * 81 * 64 * 4), o_bgs = take((size_t)((B + 15) / 16) * 64 * 4);
  const size_t o_pbg3 = take((size_t)((B + 15) / 16) * 49 * 64 * 4), o_bgs3 = take((size_t)((B + 15) / 16) * 64 * 4);
  void* p = nullptr;
  QLX_HIP(hipMalloc(&p, off));
  w.fgrad = p;
  char* base = (char*)p;
  w.fdz1 = (float*)(base + o_dz1); w.fdz2 = (float*)(base + o_dz2); w.fdz3 = (float*)(base + o_dz3);
  w.fdz4 = (float*)(base + o_dz4);
  w.fslab1 = (float*)(base + o_s1); w.fslab2 = (float*)(base + o_s2); w.fslab3 = (float*)(base + o_s3);
  w.fpb1 = (float*)(base + o_pb);
  w.fpbg2 = (float*)(base + o_pbg);
  w.fs2 = (float*)(base + o_bgs);
  w.fpbg3 = (float*)(base + o_pbg3);
  w.fs3 = (float*)(base + o_bgs3);
  w.fgrad_batch = B;
}

// Every fp32 launch is timed (when the learner profiles) by start / stop events bound to its own dispatch
// (hipExtLaunchKernelGGL), so a scope's average is the kernel's duration as a kernel trace reports it.
template <class P>
static void launch(qlx_model* m, const P& p, const char* scope, double work, hipStream_t s) {
  hipEvent_t ea = nullptr, eb = nullptr;
  if (m->prof) m->prof->ext(scope, work, &ea, &eb);
  hipExtLaunchKernelGGL(k_gemm32<P>, dim3(p.g.blocks()), dim3(threads_of<P>()), gemm_lds_bytes<P>(), s, ea, eb, 0u, p);
  QLX_HIP(hipGetLastError());
  debug_sync(s, scope);
}

template <class P1, class P2, class S, class T = NoSide>
static void launch_pair(qlx_model* m, const P1& p1, const P2& p2, const S& side, const char* scope, double work, hipStream_t s,
                        const T& tail = T{}) {
  const size_t lds = std::max({gemm_lds_bytes<P1>(), gemm_lds_bytes<P2>(), S::LDS, T::LDS});
  hipEvent_t ea = nullptr, eb = nullptr;
  if (m->prof) m->prof->ext(scope, work, &ea, &eb);
  hipExtLaunchKernelGGL((k_gemm32_pair<P1, P2, S, T>), dim3(side.blocks() + p1.g.blocks() + p2.g.blocks() + tail.blocks()), dim3(256),
                        lds, s, ea, eb, 0u, p1, p2, side, tail);
  QLX_HIP(hipGetLastError());
  debug_sync(s, scope);
}

// CUs of the device (QLX_NUM_CUS overrides it: tests of the grid-shape logic of a part with fewer CUs)
static int num_cus() {
  static int n = 0;
  if (!n) {
    const char* e = std::getenv("QLX_NUM_CUS");
    if (e && atoi(e) > 0) {
      n = atoi(e);
    } else {
      int dev = 0;
      QLX_HIP(hipGetDevice(&dev));
      QLX_HIP(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev));
    }
  }
  return n;
}

static Grid grid(int M, int BM, int N, int BN, int nz) { return Grid{(M + BM - 1) / BM, (N + BN - 1) / BN, nz}; }

// conv1 forward / weight gradient: MFMA steps whose frame operands are all 0 are not issued (exact, see k_conv1_fwd32);
// a model created under QLX_F32_C1_SKIP=0 issues every step (qlx_model::f32_c1_skip)
static int c1_skip(const qlx_model* m) { return m->f32_c1_skip; }

// training-batch conv2 / conv3 forward over M rows on a balanced grid (PConv2FwdR / PConv3FwdR): `whole` 64 x 64 tiles,
// a multiple of the CU count, plus the remaining rows as 16 x 64 tiles; 0 when the shape has no such split (fewer whole
// tiles than CUs, or more than half a tile per CU left over) and the plain grid runs.  At B = 1024 (784 / 1296 whole
// tiles: 16 left over after 3 / 5 per CU) in place at C3: conv3 forward 42.4 -> 38.4 us, conv2 forward 56.2 -> 53.3 us
// against the plain 64 x 32 grid.
static int balanced_whole_tiles(int M) {
  const int ncu = num_cus(), t = M / 64, whole = t - t % ncu;
  if (whole < ncu || M - whole * 64 > 32 * ncu) return 0;
  return whole;
}

// conv2 / conv3 forward over the non-background rows (PConvFwdL) with the background rows written by the side blocks
template <class P, class S>
static void launch_list(qlx_model* m, const P& p, const S& side, const char* scope, double work, hipStream_t s) {
  hipEvent_t ea = nullptr, eb = nullptr;
  if (m->prof) m->prof->ext(scope, work, &ea, &eb);
  const size_t lds = std::max(gemm_lds_bytes<P>(), S::LDS);
  hipExtLaunchKernelGGL((k_gemm32_side<P, S>), dim3(side.blocks() + p.g.blocks()), dim3(threads_of<P>()), lds, s, ea, eb, 0u, p, side);
  QLX_HIP(hipGetLastError());
  debug_sync(s, scope);
}

// background rows (see C1Lists in qnet32_kernels.h): on by default; a model created under QLX_F32_BG=0 computes every
// conv2 / conv3 row (qlx_model::f32_bg_rows)
static bool bg_rows(const qlx_model* m) { return m->f32_bg_rows; }

// the conv1 step masks of the training forward (written with its row lists) select the dz1 rows the conv2 backward
// stores and the conv1 weight gradient fetches; without zero-step skipping every row is multiplied, so every row
#ifndef QLX_DZ1_SKIP
#define QLX_DZ1_SKIP 1   // 0: the conv2 backward stores every dz1 row (the weight gradient still fetches the set steps' only)
#endif
static bool c1_sparse_dz(const qlx_model* m) { return bg_rows(m) && c1_skip(m); }
template <class PW, class PR, class PF>
static void conv_fwd(qlx_model* m, int M, const float* in, const float* wt, const float* bias, float* out, const char* scope,
                     double work, hipStream_t s, const PF& plain) {
  const int whole = balanced_whole_tiles(M);
  if (!whole) {
    launch(m, plain, scope, work, s);
    return;
  }
  const PW pw{Grid{whole, 1, 1}, in, wt, bias, out, M};
  const PR pr{{Grid{(M - whole * 64 + 15) / 16, 1, 1}, in, wt, bias, out, M}, whole * 4};
  launch_pair(m, pw, pr, NoSide{}, scope, work, s);
}

// forward over B samples in chunks of the workspace's forward chunk: a1..a3 hold the last chunk (the whole batch when
// B <= chunk, as training needs), a4 all B samples
void f32_forward(qlx_model* m, const uint8_t* const* table, int B, hipStream_t s) {
  ModelWs& w = m->w;
  QLX_CHECK(m->ws_batch >= B, QLX_E_STATE, "f32 forward: workspace too small");
  m->last_batch = B;
  const float* p = m->d_params;
  for (int c0 = 0; c0 < B; c0 += w.fchunk) {
    const int n = std::min(w.fchunk, B - c0);
    // tiles by batch: at chunk-size batches (target pass, acting) 64 x 64 tiles run best (~65 % of the fp32 peak), at
    // training-size batches the narrower tiles that put more blocks on the chip (scripts/ubench32.hip sweep); the two
    // shapes are separate kernels and separate profiler scopes (suffix _big)
    const bool big = n > 2048;
    // background rows: conv1 lists them, conv2 / conv3 run the rest (the list counters alternate between forwards)
    const bool lists = bg_rows(m);
    unsigned long long* cnt = w.frcnt + 2 * kListSlots * kCntStride * w.fparity;
    const bool one = c1_one(n);
    const int G = c1_grid(n);                                          // conv1 blocks
    const int per_slot = ((G + kListSlots - 1) / kListSlots) * ((n + G - 1) / G);   // samples of a list region, at most
    const int cap2 = per_slot * 81, cap3 = per_slot * 49;
    QLX_CHECK((size_t)kListSlots * cap2 <= w.frl_cap * 81, QLX_E_STATE, "row lists too small");
    const C1Lists L{lists ? w.frl2 : nullptr, w.frl3, cap2, cap3, cnt, w.frcnt + 2 * kListSlots * kCntStride * (w.fparity ^ 1),
                    w.fbgc, w.fsteps, w.fneed, w.fneed_ld, w.frows2, w.fbg2, w.frows3, w.fbg3};
    if (lists) w.fparity ^= 1;
    {
      const char* sc = big ? "f32_conv1_fwd_big" : "f32_conv1_fwd";
      hipEvent_t ea = nullptr, eb = nullptr;
      if (m->prof) m->prof->ext(sc, 2.0 * n * 400 * 32 * 256, &ea, &eb);
      auto kern = big ? k_conv1_fwd32<1> : one ? k_conv1_fwd32<0, true> : k_conv1_fwd32<0>;
      QLX_CHECK((n + G - 1) / G <= (one ? 1 : kC1MaxIt), QLX_E_STATE, "conv1 forward: too many samples per block");
      const size_t frames = (one ? 1 : 2) * kC1Frames;
      const size_t lds = frames + 3 * kC1RmDw * 4 + (size_t)((n + G - 1) / G) * 6 * 8 + 8;   // frames, row masks, flags, claim
      set_lds_limit((const void*)kern, frames + 3 * kC1RmDw * 4 + (size_t)(one ? 1 : kC1MaxIt) * 6 * 8 + 8);
      hipExtLaunchKernelGGL(kern, dim3(G), dim3(256), lds, s, ea, eb, 0u, table + (size_t)c0 * 4, n,
                            p + voff(0), p + voff(1), w.fa1, c1_skip(m), L);
      QLX_HIP(hipGetLastError());
      debug_sync(s, sc);
    }
    if (lists) {
      // conv2: the non-background rows, the constant rows c2 and c3 in its first block (ConstRows); conv3: the non-background
      // rows (background conv2 taps read from c2), side blocks writing c2 / c3 to the background rows of a2 / a3
      const int nw = std::min(256, std::max(16, n / 16));   // background-row blocks per job
      float* c2 = w.fbgc + 32;
      float* c3 = w.fbgc + 96;
      const BgRows2 s23{{nw, w.frl2, cnt, cap2, c2, w.fa2}, {nw, w.frl3, cnt + kCntStride, cap3, c3, w.fa3}};
      auto lgrid = [&](int cap, int BM, int BN) { return Grid{1 + kListSlots * ((cap + BM - 1) / BM), 64 / BN, 1}; };
      auto run = [&](auto t2, auto t3, const char* sc2, const char* sc3) {
        using P2 = decltype(t2);
        using P3 = decltype(t3);
        // the constant rows' chains in the conv2 launch's blocks: the same K split form as its list tiles (block size)
        using PC2 = PConv2FwdL<16, 64, 1, 4, P2::KSPLIT>;
        using PC3 = PConv3FwdL<16, 64, 1, 4, P2::KSPLIT>;
        const ConstRows<PC2, PC3> cr{PC2{Grid{1, 1, 1}, w.fa1, p + voff(2), p + voff(3), w.fa2, w.frl2, cap2, cnt, w.fbgc, c2},
                                     PC3{Grid{1, 1, 1}, w.fa2, p + voff(4), p + voff(5), w.fa3, w.frl3, cap3, cnt + kCntStride, c2, c3}};
        // (the list tiles start at row tile 1; row tile 0, the constant row, is ConstRows' work: its blocks return)
        P2 p2{lgrid(cap2, P2::BM, P2::BN), w.fa1, p + voff(2), p + voff(3), w.fa2, w.frl2, cap2, cnt, w.fbgc, nullptr};
        p2.pre_batched = big;
        launch_list(m, p2, cr, sc2, 2.0 * n * 81 * 64 * 512, s);
        launch_list(m, P3{lgrid(cap3, P3::BM, P3::BN), w.fa2, p + voff(4), p + voff(5), w.fa3, w.frl3, cap3, cnt + kCntStride, c2, nullptr},
                    s23, sc3, 2.0 * n * 49 * 64 * 576, s);
      };
      if (big) {
        // (64 x 32 list tiles here: conv2 / conv3 145 / 185 us against 139 / 181 us, gpurun_out/w10)
        run(PConv2FwdL<64, 64, 2, 2>{}, PConv3FwdL<64, 64, 2, 2>{}, "f32_conv2_fwd_big", "f32_conv3_fwd_big");
        model_dense_join(m, s);   // W3 / b3 of a dense update in flight on the aux stream
        launch(m, PFc1FwdB{grid(n, PFc1FwdB::BM, 512, PFc1FwdB::BN, 1), w.fa3, p + voff(6), p + voff(7), w.fa4 + (size_t)c0 * 512, n}, "f32_fc1_fwd_big",
               2.0 * n * 3136 * 512, s);
      } else {
        // (on the stream core, in place: conv2 64 x 64 24.3 us against 27.9 us for 64 x 32 and 28.7 for 32 x 64; conv3 32 x 64
        // 27.6 us against 28.5 / 29.8 for 64 x 32 / 64 x 64 - gpurun_out/w10)
        // round 6: the two k chains (§6) in two wave groups per block (KSPLIT): twice the waves for the same tiles
        run(PConv2FwdL<64, 64, 2, 2, kC2FwdKs>{}, PConv3FwdL<32, 64, 2, 2, kC3FwdKs>{}, "f32_conv2_fwd", "f32_conv3_fwd");
        model_dense_join(m, s);
        launch(m, PFc1FwdS{grid(n, PFc1FwdS::BM, 512, PFc1FwdS::BN, 1), w.fa3, p + voff(6), p + voff(7), w.fa4 + (size_t)c0 * 512, n}, "f32_fc1_fwd",
               2.0 * n * 3136 * 512, s);
      }
    } else if (big) {
      // (plain grids: 40.5 / 24.5 whole tiles per CU at 8,192 samples; the balanced split measured 373 -> 385 us on conv2)
      launch(m, PConv2Fwd{grid(n * 81, 64, 64, 64, 1), w.fa1, p + voff(2), p + voff(3), w.fa2, n * 81}, "f32_conv2_fwd_big",
             2.0 * n * 81 * 64 * 512, s);
      launch(m, PConv3Fwd{grid(n * 49, 64, 64, 64, 1), w.fa2, p + voff(4), p + voff(5), w.fa3, n * 49}, "f32_conv3_fwd_big",
             2.0 * n * 49 * 64 * 576, s);
      model_dense_join(m, s);
      launch(m, PFc1FwdB{grid(n, PFc1FwdB::BM, 512, PFc1FwdB::BN, 1), w.fa3, p + voff(6), p + voff(7), w.fa4 + (size_t)c0 * 512, n}, "f32_fc1_fwd_big",
             2.0 * n * 3136 * 512, s);
    } else {
      conv_fwd<PConv2Fwd, PConv2FwdR>(m, n * 81, w.fa1, p + voff(2), p + voff(3), w.fa2, "f32_conv2_fwd", 2.0 * n * 81 * 64 * 512, s,
                                      PConv2FwdS{grid(n * 81, 64, 64, 32, 1), w.fa1, p + voff(2), p + voff(3), w.fa2, n * 81});
      conv_fwd<PConv3Fwd, PConv3FwdR>(m, n * 49, w.fa2, p + voff(4), p + voff(5), w.fa3, "f32_conv3_fwd", 2.0 * n * 49 * 64 * 576, s,
                                      PConv3FwdS{grid(n * 49, 64, 64, 32, 1), w.fa2, p + voff(4), p + voff(5), w.fa3, n * 49});
      model_dense_join(m, s);
      launch(m, PFc1FwdS{grid(n, PFc1FwdS::BM, 512, PFc1FwdS::BN, 1), w.fa3, p + voff(6), p + voff(7), w.fa4 + (size_t)c0 * 512, n}, "f32_fc1_fwd",
             2.0 * n * 3136 * 512, s);
    }
  }
}

void f32_head(int mode, const Fc2Args& a, int B, hipStream_t s) {
  // the training head on 4 samples per block (MFMA rows 4..15 padding): 256 blocks at B = 1024 instead of 64, 8.7 -> 7.9 us
  // (8 per block: 8.1 us; gpurun_out/w32); the chunk-size heads keep 16
  constexpr int kHs3 = 4;
  const dim3 g((B + 15) / 16), blk(256);   // 16 samples per block
  switch (mode) {
    case 0: hipLaunchKernelGGL(k_head32<0>, g, blk, 0, s, a); break;
    case 1: hipLaunchKernelGGL(k_head32<1>, g, blk, 0, s, a); break;
    case 2: hipLaunchKernelGGL(k_head32<2>, g, blk, 0, s, a); break;
    default: hipLaunchKernelGGL((k_head32<3, kHs3>), dim3((B + kHs3 - 1) / kHs3), blk, 0, s, a); break;
  }
  QLX_HIP(hipGetLastError());
  debug_sync(s, "k_head32");
}

void f32_backward_dense(qlx_model* m, int B, const uint8_t* actions, const float* y, float* loss_dev, hipStream_t s,
                        const float* weights, float* td_abs) {
  QLX_CHECK(B <= m->w.fchunk && B == m->last_batch, QLX_E_STATE, "f32 backward: batch must follow its forward");
  f32_grad_workspace(m, B);
  ModelWs& w = m->w;
  float* G = m->d_grads;
  const float* p = m->d_params;
  {
    ProfScope ps(m->prof, "f32_head", s);
    Fc2Args a = fc2_args(m, B);
    a.actions = actions;
    a.y = y;
    a.gsample = w.gs;
    a.hsample = w.hs;
    a.weights = weights;
    a.td_abs = td_abs;
    a.dz4_out = w.fdz4;
    f32_head(3, a, B, s);
  }
  {  // dW3 + db3 and dz3 tiles in one grid, dW4 / db4 / loss as its leading blocks
    PFc1WgradS Pw{grid(3136, PFc1WgradS::BM, 512, PFc1WgradS::BN, 1), w.fa3, w.fdz4, G + voff(6), G + voff(7), B};
    PFc1DgradS Pd{grid(B, PFc1DgradS::BM, 3136, PFc1DgradS::BN, 1), w.fdz4, p + voff(6), w.fa3, w.fdz3, B};
    if (bg_rows(m)) {   // conv3's background-row dz3 sums (the compacted conv3 weight gradient)
      Pd.pbg = w.fpbg3;
      Pd.bg = w.fbg3;
      Pd.bg_ld = w.fneed_ld;
    }
    SideFc2 S{w.fa4, actions, w.gs, w.hs, B, G + voff(8), G + voff(9), loss_dev};
    launch_pair(m, Pw, Pd, S, "f32_fc1_bwd", 2.0 * 2.0 * B * 512 * 3136, s);   // (3 blocks per CU: 72.8 vs 61.8 us, w23)
  }
}

static void seg_tables(int* seg_first, int64_t* off) {
  int sf = 0;
  int64_t o = 0;
  for (int v = 0; v < kNumVars; ++v) {
    seg_first[v] = sf;
    off[v] = o;
    sf += segs_of(v);
    o += kVarSize[v];
  }
  seg_first[kNumVars] = sf;
  off[kNumVars] = o;
}

static NormArgs norm_args(qlx_model* m, float scale) {
  NormArgs A;
  A.g = m->d_grads;
  A.scale = scale;
  A.partial = m->w.fpart;
  seg_tables(A.seg_first, A.off);
  return A;
}

// Adam arguments of the update about to run (iterations + 1)
static Adam32Args adam_args(qlx_model* m, float scale) {
  const float tf = (float)(m->iterations + 1);
  const float b1p = std::pow(m->beta1, tf), b2p = std::pow(m->beta2, tf);
  Adam32Args a;
  a.w = m->d_params; a.m = m->d_m; a.v = m->d_v; a.g = m->d_grads; a.partial = m->w.fpart; a.norms = m->d_norms;
  seg_tables(a.seg_first, a.off);
  a.scale = scale;
  a.alpha = m->lr * std::sqrt(1.0f - b2p) / (1.0f - b1p);
  a.beta1 = m->beta1; a.beta2 = m->beta2; a.eps = m->eps; a.clipnorm = m->clipnorm;
  return a;
}

void f32_backward_conv(qlx_model* m, const uint8_t* const* table, int B, hipStream_t s, bool fuse_update, hipEvent_t dense_ready,
                       float dense_scale) {
  ModelWs& w = m->w;
  m->f32_update_scheduled = fuse_update;
  QLX_CHECK(!(fuse_update && dense_ready), QLX_E_STATE, "dense partials: the scheduled update or the data-parallel form");
  const NormArgs N = norm_args(m, dense_ready ? dense_scale : 1.0f);
  const float* p = m->d_params;
  float* G = m->d_grads;
  const int z3 = (B + kSC3 - 1) / kSC3, z2 = (B + kSC2 - 1) / kSC2, z1 = (B + kSC1 - 1) / kSC1;
  // algorithmic FLOPs (backward-data + weight gradient of the layer; the pixel-major dgrad tiles multiply only the
  // valid taps, so MFMA work = algorithmic work)
  // pixel-major backward data, one pixel per tile.  On the operand-stream core (no per-slab address arithmetic) the
  // one-pixel conv3 tiles beat the balanced pixel groups (chained sub-tiles: scripts/ubench32.hip bwd, B = 1024: pair 84.4
  // vs 93.4 us; on the ldA / ldB core the groups had won, 97.1 vs 105.6 us); conv2 groups were slower on both cores
  {  // conv3: dz2 pixel tiles + weight-gradient chunk tiles
    PConv3Wgrad Pw{grid(576, 64, 64, 64, z3), w.fa2, w.fdz3, w.fslab3, B, w.frows3};
    PConv3WgradD Pw_dense{grid(576, 64, 64, 64, z3), w.fa2, w.fdz3, w.fslab3, B};
    // 64 x 64 pixel tiles on the stream core: pair 73.2 vs 75.0 us in place for 32 x 64 (gpurun_out/w3)
    using PD3 = PConv3DgradPx<64, 64, 2, 2>;
    PD3 Pd{Grid{(B + PD3::BM - 1) / PD3::BM, 1, 81}, w.fdz3, p + voff(4), w.fa2, w.fdz2, B};
    if (bg_rows(m)) {   // conv2's background-row dz2 sums (the compacted conv2 weight gradient)
      Pd.pbg = w.fpbg2;
      Pd.bg2 = w.fbg2;
      Pd.bg2_ld = w.fneed_ld;
    }
    
    if (bg_rows(m)) launch_pair(m, Pw, Pd, SideBgSum<49>{w.fpbg3, w.fs3, z3}, "f32_conv3_bwd", 2.0 * 2.0 * B * 49 * 64 * 576, s);
    else launch_pair(m, Pw_dense, Pd, NoSide{}, "f32_conv3_bwd", 2.0 * 2.0 * B * 49 * 64 * 576, s);
  }
  {  // conv2: dz1 pixel tiles (all 4 parity classes) + weight-gradient chunk tiles
    // the weight gradient over the non-background rows (their background share through SideBgSum and k_wreduce32), or
    // over every row on the dense-frame path
    PConv2Wgrad Pw{grid(512, 64, 64, 64, z2), w.fa1, w.fdz2, w.fslab2, B, w.frows2};
    PConv2WgradD Pw_dense{grid(512, 64, 64, 64, z2), w.fa1, w.fdz2, w.fslab2, B};
    PConv2DgradPx<64, 64, 2, 2> Pd{Grid{(B + 63) / 64, 2, 100}, w.fdz2, p + voff(2), w.fa1, w.fdz1, B, QLX_PB_OFF ? nullptr : w.fpb1};
    if (QLX_DZ1_SKIP && c1_sparse_dz(m)) {   // dz1 rows of clear conv1 steps are neither stored here nor fetched by the conv1 weight gradient
      Pd.need = w.fneed;
      Pd.need_ld = w.fneed_ld;
    }

    if (bg_rows(m)) launch_pair(m, Pw, Pd, SideBgSum<81>{w.fpbg2, w.fs2, z2}, "f32_conv2_bwd", 2.0 * 2.0 * B * 81 * 64 * 512, s);
    else launch_pair(m, Pw_dense, Pd, NoSide{}, "f32_conv2_bwd", 2.0 * 2.0 * B * 81 * 64 * 512, s);
  }
  {
    constexpr size_t lds = kC1WgradLds;   // 79,488 B
    hipEvent_t ea = nullptr, eb = nullptr;
    if (m->prof) m->prof->ext("f32_conv1_wgrad", 2.0 * B * 400 * 256 * 32, &ea, &eb);
    set_lds_limit((const void*)k_conv1_wgrad32, lds);
    // the forward's step masks (when it built row lists) select the dz1 rows to fetch; without skipping, every row
    const uint32_t* steps = c1_sparse_dz(m) ? w.fsteps : nullptr;
    hipExtLaunchKernelGGL(k_conv1_wgrad32, dim3(c1_wgrad_blocks(z1)), dim3(kC1WgradThreads), lds, s, ea, eb, 0u, table, w.fdz1, B, z1,
                          w.fslab1, c1_skip(m), steps, (const float*)w.fpb1);
    QLX_HIP(hipGetLastError());
    debug_sync(s, "k_conv1_wgrad32");
  }
  {
    ProfScope ps(m->prof, "f32_wgrad_reduce", s);
    WRed R;
    R.slab[0] = w.fslab3; R.nz[0] = z3; R.count[0] = 577 * 64; R.oc[0] = 64; R.gw[0] = G + voff(4); R.gb[0] = G + voff(5);
    R.slab[1] = w.fslab2; R.nz[1] = z2; R.count[1] = 513 * 64; R.oc[1] = 64; R.gw[1] = G + voff(2); R.gb[1] = G + voff(3);
    R.slab[2] = w.fslab1; R.nz[2] = z1; R.count[2] = 257 * 32; R.oc[2] = 32; R.gw[2] = G + voff(0); R.gb[2] = G + voff(1);
    R.sbg[0] = bg_rows(m) ? w.fs3 : nullptr;
    R.ubg[0] = w.fbgc + 32;   // c2, written by the training forward's conv2 launch (ConstRows)
    R.sbg[1] = bg_rows(m) ? w.fs2 : nullptr;
    R.ubg[1] = w.fbgc;        // relu(0 + b0), written by the training forward's conv1
    QLX_CHECK(std::max({z1, z2, z3}) <= kWGroup * kWGroupsMax, QLX_E_INVALID, "too many weight-gradient chunks");
    int nred = 0;
    for (int L = 0; L < 3; ++L) {
      R.wv[L] = wred_waves(R.nz[L]);
      const int per = 64 * (16 / R.wv[L]);
      R.nb[L] = (R.count[L] + per - 1) / per;
      nred += R.nb[L];
    }
    // the scheduled update: + the dense variables' clip-norm segment partials (4 per block); data parallel (dense_ready):
    // the same blocks over the reduced dense gradient x dense_scale, once its all-reduce has landed (long before the conv
    // backward ends) - the launch waits for it, so the update tail is the plain path's two launches (+ the conv all-reduce)
    const bool dp_dense = dense_ready != nullptr;
    if (dp_dense) QLX_HIP(hipStreamWaitEvent(s, dense_ready, 0));
    const int dseg = (m->f32_update_scheduled && !m->f32_dense_async) || dp_dense ? N.seg_first[kNumVars] - N.seg_first[6] : 0;
    hipLaunchKernelGGL(k_wreduce32, dim3(nred + (dseg + 3) / 4), dim3(1024), 0, s, R, N, nred, N.seg_first[6], dseg);
    QLX_HIP(hipGetLastError());
    debug_sync(s, "k_wreduce32");
    if (dp_dense) {
      m->f32_dense_partials = true;
      m->f32_partials_scale = dense_scale;
    }
  }
}

// Data parallel (an all-reduce sits between the backward and the update, so the reduction launch could not take the dense
// partials): the dense variables' clip-norm segment partials of the reduced gradient x scale, as k_wreduce32's extra
// blocks compute them at world 1 (the same blocks, no chunk sums).  Only the dense gradient is read, so a caller may run it
// as soon as the dense bucket is reduced (learner.hip: on the communicator stream, beside the conv backward).
void f32_norms(qlx_model* m, hipStream_t s, float scale) {
  if (m->f32_update_scheduled) return;   // the backward scheduled them (f32_backward_conv)
  if (m->f32_dense_partials && m->f32_partials_scale == scale) return;   // the data-parallel reduction launch computed them
  ProfScope ps(m->prof, "f32_norms", s, 4.0 * (kNumParams - kVarOffsetDense));
  const NormArgs N = norm_args(m, scale);
  const int dseg = N.seg_first[kNumVars] - N.seg_first[6];
  const WRed R{};   // no chunk-sum blocks (nred = 0)
  hipLaunchKernelGGL(k_wreduce32, dim3((dseg + 3) / 4), dim3(1024), 0, s, R, N, 0, N.seg_first[6], dseg);
  QLX_HIP(hipGetLastError());
  debug_sync(s, "k_wreduce32 (dense norm partials)");
  m->f32_dense_partials = true;
  m->f32_partials_scale = scale;
}

// clip_by_norm + Adam of every variable in one launch (k_update32): the conv blocks finish their variable's norm from the
// (scaled) gradient, the dense blocks from the partials of the reduction launch (world 1) or of f32_norms (data parallel).
// One tail for both, so a rank's update is the single-GPU update of its reduced gradient (bit-identical at world 1).
constexpr int kDenseAdamBlocks = (int)((kNumParams - kVarOffsetDense) / 4 / 2048 + 1);   // 2 float4 groups per thread

void f32_adam(qlx_model* m, hipStream_t s, float scale) {
  const int64_t t = m->iterations + 1;
  const Adam32Args a = adam_args(m, scale);
  QLX_CHECK(m->f32_update_scheduled ? scale == 1.0f : (m->f32_dense_partials && scale == m->f32_partials_scale), QLX_E_STATE,
            "fp32 update without the dense norm partials of this gradient scale (model_norms first)");
  const bool dense_here = !m->f32_dense_async;   // else the dense blocks run on f32_aux (f32_dense_async)
  ProfScope ps(m->prof, "f32_adam", s, dense_here ? 28.0 * kNumParams : 28.0 * kVarOffsetDense);
  const int nconv = conv_adam_blocks(), ndense = kDenseAdamBlocks;
  hipLaunchKernelGGL(k_update32, dim3(nconv + (dense_here ? ndense : 0)), dim3(1024), 0, s, a, norm_args(m, scale), nconv, ndense);
  QLX_HIP(hipGetLastError());
  debug_sync(s, "k_update32");
  m->f32_update_scheduled = false;
  m->f32_dense_partials = false;
  m->f32_dense_async = false;
  m->iterations = t;
}

// The dense variables (W3, b3, W4, b4: 95 % of the update's Adam bytes) are final after the fc1 backward and are next read
// by the next forward's fc1: their clip-norm segment partials (k_wreduce32's dense blocks) and clip_by_norm + Adam
// (k_update32's dense blocks) run on a second stream from there, beside the conv backward, the conv update and the next
// forward's convs.  Same kernels and arithmetic as the one-stream tail, so the results are bit-identical.
void f32_dense_async(qlx_model* m, hipStream_t s) {
  if (!m->f32_aux) {
    QLX_HIP(hipStreamCreateWithFlags(&m->f32_aux, hipStreamNonBlocking));
    QLX_HIP(hipEventCreateWithFlags(&m->ev_dense_ready, hipEventDisableTiming));
    QLX_HIP(hipEventCreateWithFlags(&m->ev_dense_done, hipEventDisableTiming));
  }
  hipStream_t a = m->f32_aux;
  QLX_HIP(hipEventRecord(m->ev_dense_ready, s));
  QLX_HIP(hipStreamWaitEvent(a, m->ev_dense_ready, 0));
  ProfScope ps(m->prof, "f32_dense_update", a, 28.0 * (kNumParams - kVarOffsetDense));
  const NormArgs N = norm_args(m, 1.0f);
  const int dseg = N.seg_first[kNumVars] - N.seg_first[6];
  const WRed R{};
  hipLaunchKernelGGL(k_wreduce32, dim3((dseg + 3) / 4), dim3(1024), 0, a, R, N, 0, N.seg_first[6], dseg);
  hipLaunchKernelGGL(k_update32, dim3(kDenseAdamBlocks), dim3(1024), 0, a, adam_args(m, 1.0f), N, 0, kDenseAdamBlocks);
  QLX_HIP(hipGetLastError());
  QLX_HIP(hipEventRecord(m->ev_dense_done, a));
  debug_sync(a, "dense update (aux stream)");
  m->f32_dense_async = true;
  m->dense_pending = true;
}

void model_dense_join(qlx_model* m, hipStream_t s) {
  if (!m->dense_pending) return;
  QLX_HIP(hipStreamWaitEvent(s, m->ev_dense_done, 0));
  m->dense_pending = false;
}


// ---- frame sparsity of a batch (diagnostic, bench.py): how much of the fp32 conv work the exact skips leave out ----
// Per sample, in the kernels' own units (the same predicates, re-evaluated from the frames): conv1 forward (tile, kq)
// steps whose 64 frame dwords are all 0 (k_conv1_fwd32: 25 tiles x 16 per sample), conv1 weight-gradient (wave, rs)
// steps likewise (k_conv1_wgrad32: 4 x 100), conv2 / conv3 background rows (c1_flags: 81 / 49).  Counts into cnt[4].
__global__ __launch_bounds__(256) void k_frame_sparsity(const uint8_t* const* table, int n, unsigned long long* cnt) {
  __shared__ uint32_t fr[4][84][21];   // row layout: pixels (x, 4 d .. 4 d + 3) at fr[slot][x][d]
  __shared__ uint32_t bm[4][21];       // per block row bx: bit by = the 4 x 4 pixel block (bx, by) of any frame non-zero
  __shared__ int tot[4];
  int mine[4] = {0, 0, 0, 0};
  for (int b = blockIdx.x; b < n; b += gridDim.x) {
    __syncthreads();
    if (threadIdx.x < 21) bm[0][threadIdx.x] = 0u;
    __syncthreads();
    for (int q = threadIdx.x; q < kC1Chunks; q += blockDim.x) {   // s2d chunk (slot, bx, by): rows 4 bx + xl, dword by
      const int slot = q / 441, pos = q - slot * 441, bx = pos / 21, by = pos - bx * 21;
      const uint8_t* f = table[(size_t)b * 4 + slot];
      uint4 v = uint4{0u, 0u, 0u, 0u};
      if (f) v = *reinterpret_cast<const uint4*>(f + (size_t)pos * 16);
      fr[slot][4 * bx][by] = v.x;
      fr[slot][4 * bx + 1][by] = v.y;
      fr[slot][4 * bx + 2][by] = v.z;
      fr[slot][4 * bx + 3][by] = v.w;
      if ((v.x | v.y | v.z | v.w) != 0u) atomicOr(&bm[0][bx], 1u << by);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 400; i += blockDim.x) {
      {  // forward step (tile t, kq): lanes (g = slot, l = patch position), dword (4 oh + kh, ow + hw)
        const int t = i >> 4, kq = i & 15, kh = kq >> 1, hw = kq & 1;
        uint32_t o = 0u;
        for (int g = 0; g < 4; ++g)
          for (int l = 0; l < 16; ++l) {
            const int oh = 4 * (t / 5) + (l >> 2), ow = 4 * (t % 5) + (l & 3);
            o |= fr[g][4 * oh + kh][ow + hw];
          }
        mine[0] += o == 0u;
      }
      {  // weight-gradient step (wave w, rs): lanes (g, l15), position r = 4 rs + g, slot l15 & 3, kh = 2 w + l15 / 8
        const int w = i / 100, rs = i - 100 * w;
        uint32_t o = 0u;
        for (int g = 0; g < 4; ++g)
          for (int l = 0; l < 16; ++l) {
            const int r = 4 * rs + g, oh = r / 20, ow = r - 20 * oh, kh = 2 * w + (l >> 3), h = (l >> 2) & 1;
            o |= fr[l & 3][4 * oh + kh][ow + h];
          }
        mine[1] += o == 0u;
      }
    }
    for (int p = threadIdx.x; p < 81 + 49; p += blockDim.x) {   // background rows from the 4 x 4 block marks
      const bool c2 = p < 81;
      const int pp = c2 ? p : p - 81, R = c2 ? 9 : 7, i = pp / R, j = pp - R * i, span = c2 ? 5 : 9;
      uint32_t mm = 0u;
      for (int r = 0; r < span; ++r) mm |= bm[0][2 * i + r];
      const bool bg = ((mm >> (2 * j)) & ((1u << span) - 1u)) == 0u;
      mine[c2 ? 2 : 3] += bg;
    }
  }
  if (threadIdx.x < 4) tot[threadIdx.x] = 0;
  __syncthreads();
  for (int k = 0; k < 4; ++k) atomicAdd(&tot[k], mine[k]);
  __syncthreads();
  if (threadIdx.x < 4) atomicAdd(cnt + threadIdx.x, (unsigned long long)tot[threadIdx.x]);
}

void frame_sparsity(const uint8_t* const* table, int n, unsigned long long* d_cnt, unsigned long long* h_cnt, double* out,
                    hipStream_t s) {
  for (int k = 0; k < 4; ++k) out[k] = std::nan("");
  if (n <= 0) return;
  // counters and read-back buffer allocated once by the caller; memset, kernel, copy into the pinned buffer and the
  // drain all on s (round 5's stream-ordered allocation + asynchronous copy into pageable memory returned zeros now and
  // then for the second of two back-to-back calls: scripts/readback_probe.hip)
  QLX_HIP(hipMemsetAsync(d_cnt, 0, 4 * sizeof(unsigned long long), s));
  hipLaunchKernelGGL(k_frame_sparsity, dim3(std::min(n, 4 * num_cus())), dim3(256), 0, s, table, n, d_cnt);
  QLX_HIP(hipGetLastError());
  QLX_HIP(hipMemcpyAsync(h_cnt, d_cnt, 4 * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
  QLX_HIP(hipStreamSynchronize(s));
  const double per[4] = {400.0, 400.0, 81.0, 49.0};
  for (int k = 0; k < 4; ++k) out[k] = (double)h_cnt[k] / (per[k] * n);
}

}  // namespace qlx
