// ORACLE — TEST INFRASTRUCTURE ONLY (see rng_ref.h / qnet_ref.h headers).
//
// fp32 restatement of the reference Q-network and its train step with every reduction a single fmaf chain in the
// order the build defines.  The reference graph is float32 Keras
// (create_ql_model_breakout_84x84x4_3_32.py:20-33,37-61; tf.float32 TensorSpecs) run by TF 2.12, whose reduction
// order is internal to its CPU kernels and pinned by no reference test: the order is therefore part of
// this build's definition of the arithmetic, stated here once and followed by the GPU kernels
// (q-learning_amd/csrc/qnet32_kernels.h).  tests/test_oracle_qnet32_pin.py pins this restatement against float64 torch
// autograd of the Keras graph (activations, Q, loss, all ten gradients, norms, w / m / v after two Adam steps; B 4..256)
// and against the double-accumulating restatement qnet_ref.cpp at B = 1024.
//   conv1 .. conv3  z = sum over (kh, kw, c) of in[S oh+kh][S ow+kw][c] W[kh][kw][c][oc]          (HWIO order)
//                   conv2 / conv3 (round 6): z = C0 + C1, Ch = chain over the half h of the flattened (kh, kw, c)
//   dense 3136->512 z = C0 + C1, Ch = chain over k in [1568 h, 1568 h + 1568) ascending (Flatten order h, w, c; round 6 -
//                   before: one chain over all k)
//   dense 512->3    z = ((C0 + C1) + C2) + C3, Cw = chain over k in [128 w, 128 w + 128) ascending
//   every sum: acc = 0; acc = fmaf(x, w, acc) in that order; then + bias, ReLU (v > 0 ? v : 0)
//   Huber head      e = q_a - y, h = w (|e| <= 1 ? (0.5 e) e : |e| - 0.5), g = (w clip(e, -1, 1)) / B,
//                   loss = (sum over b ascending of h) / B
//   dense-3 bwd     dz4[b][k] = a4 > 0 ? W4[k][a_b] g_b : 0; dW4[k][n] = chain over b of a4[b][k] dq[b][n]
//   dense-512 bwd   dW3[k][n] = chain over b of a3[b][k] dz4[b][n]; dz3 = a3 > 0 ? chain over n : 0
//   conv dgrad      dz_in[b][ih][iw][c] = a_in > 0 ? chain over the valid taps (kh, kw, oc) lexicographic : 0
//   conv wgrad      per sample chunk z of SC_l samples: P_z = chain over (b, oh, ow) ascending; chunks in groups of 16:
//                   S_q = chain over z in [16 q, 16 q + 16), dW = chain over q of S_q
//                   bias: P_z = ((C0 + C1) + C2) + C3, Cq = chain over the chunk-local rows r = q mod 4 ascending
//   dense-512 db3   ((C0 + C1) + C2) + C3, Cq = chain over b = q mod 4 ascending
//   clip_by_norm    per variable: segments of 2048 elements; lane l < 256 chains fmaf(g, g, t) over the segment's
//                   elements 4 l .. 4 l + 3, 1024 + 4 l .. + 3; 4 x 64-lane xor butterflies (32 .. 1); ((w0 + w1) + w2)
//                   + w3 -> partial j; 64 lane chains over the partials j = lane mod 64 ascending, one xor butterfly
//   Adam            legacy ResourceApplyAdam with explicit roundings (qnet_ref.cpp)
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include <omp.h>

#include "qnet_ref.h"

namespace orc {

// chunk sizes of the conv weight-gradient partials (include/qlx.h QLX_F32_WGRAD_CHUNK_CONV*; tests check equality)
constexpr int kSC1 = 2, kSC2 = 16, kSC3 = 16;   // (round 6: conv1 4 -> 2)
constexpr int kNormSeg = 2048;

static inline float fma32(float a, float b, float c) { return std::fmaf(a, b, c); }
static inline float relu(float v) { return v > 0.0f ? v : 0.0f; }

// conv1 forward from the u8 tensor view [B][84][84][4]
static void conv1_fwd(const uint8_t* x, int B, const float* W, const float* bias, float* out) {
#pragma omp parallel for schedule(static)
  for (int b = 0; b < B; ++b)
    for (int oh = 0; oh < 20; ++oh)
      for (int ow = 0; ow < 20; ++ow) {
        float acc[32];
        for (int oc = 0; oc < 32; ++oc) acc[oc] = 0.0f;
        for (int kh = 0; kh < 8; ++kh)
          for (int kw = 0; kw < 8; ++kw)
            for (int c = 0; c < 4; ++c) {
              const float v = (float)x[(((size_t)b * 84 + oh * 4 + kh) * 84 + ow * 4 + kw) * 4 + c];
              if (v == 0.0f) continue;   // fmaf(0, w, acc) == acc (acc is never -0)
              const float* wr = W + ((kh * 8 + kw) * 4 + c) * 32;
              for (int oc = 0; oc < 32; ++oc) acc[oc] = fma32(v, wr[oc], acc[oc]);
            }
        float* o = out + (((size_t)b * 20 + oh) * 20 + ow) * 32;
        for (int oc = 0; oc < 32; ++oc) o[oc] = relu(acc[oc] + bias[oc]);
      }
}

struct Cfg { int H, W, C, K, S, OH, OW, OC; };
static const Cfg kC2 = {20, 20, 32, 4, 2, 9, 9, 64}, kC3 = {9, 9, 64, 3, 1, 7, 7, 64};

// conv2 / conv3 forward: z = C0 + C1, Ch = chain over the half h of k = (kh, kw, c) (flattened HWIO order; round 6)
constexpr int kConvFwdChains = 1;   // (qnet32_kernels.h kConvFwdChains; 2 = two chains over the k halves, measured slower)
static void conv_fwd(const Cfg& c, const float* in, int B, const float* W, const float* bias, float* out) {
  const int K = c.K * c.K * c.C, half = K / kConvFwdChains;
#pragma omp parallel for schedule(static)
  for (int b = 0; b < B; ++b)
    for (int oh = 0; oh < c.OH; ++oh)
      for (int ow = 0; ow < c.OW; ++ow) {
        float acc[64], first[64];
        for (int oc = 0; oc < c.OC; ++oc) acc[oc] = 0.0f;
        for (int kh = 0; kh < c.K; ++kh)
          for (int kw = 0; kw < c.K; ++kw) {
            const float* src = in + (((size_t)b * c.H + oh * c.S + kh) * c.W + ow * c.S + kw) * c.C;
            for (int ch = 0; ch < c.C; ++ch) {
              if (kConvFwdChains == 2 && (kh * c.K + kw) * c.C + ch == half) {   // the second chain starts here
                for (int oc = 0; oc < c.OC; ++oc) {
                  first[oc] = acc[oc];
                  acc[oc] = 0.0f;
                }
              }
              const float v = src[ch];
              if (v == 0.0f) continue;
              const float* wr = W + ((size_t)(kh * c.K + kw) * c.C + ch) * c.OC;
              for (int oc = 0; oc < c.OC; ++oc) acc[oc] = fma32(v, wr[oc], acc[oc]);
            }
          }
        if (kConvFwdChains == 2)
          for (int oc = 0; oc < c.OC; ++oc) acc[oc] = first[oc] + acc[oc];
        float* o = out + (((size_t)b * c.OH + oh) * c.OW + ow) * c.OC;
        for (int oc = 0; oc < c.OC; ++oc) o[oc] = relu(acc[oc] + bias[oc]);
      }
}

// y[b][n] = act(((C0 + C1) + ..) + bias[n]), Ch = chain over k in [h K / chains, (h + 1) K / chains) of x[b][k] W[k][n]
static void dense_fwd(const float* x, int B, int K, int N, const float* W, const float* bias, bool relu_out, float* y,
                      int chains) {
#pragma omp parallel for schedule(static)
  for (int b = 0; b < B; ++b) {
    std::vector<float> tot(N, 0.0f), acc(N);
    for (int h = 0; h < chains; ++h) {
      std::fill(acc.begin(), acc.end(), 0.0f);
      for (int k = h * K / chains; k < (h + 1) * K / chains; ++k) {
        const float v = x[(size_t)b * K + k];
        if (v == 0.0f) continue;
        const float* wr = W + (size_t)k * N;
        for (int n = 0; n < N; ++n) acc[n] = fma32(v, wr[n], acc[n]);
      }
      for (int n = 0; n < N; ++n) tot[n] = h == 0 ? acc[n] : tot[n] + acc[n];
    }
    for (int n = 0; n < N; ++n) {
      const float t = tot[n] + bias[n];
      y[(size_t)b * N + n] = relu_out ? relu(t) : t;
    }
  }
}
constexpr int kFc1Chains = 2;   // (qnet32_kernels.h kFc1Chains)

// dense 512 -> 3 head: q[b][n] = (((C0 + C1) + C2) + C3) + b4[n], Cw = fmaf chain over k in [128 w, 128 w + 128)
static void head_fwd(const float* x, int B, const float* W, const float* bias, float* y) {
#pragma omp parallel for schedule(static)
  for (int b = 0; b < B; ++b)
    for (int n = 0; n < kActions; ++n) {
      float c[4];
      for (int w = 0; w < 4; ++w) {
        float acc = 0.0f;
        for (int k = 128 * w; k < 128 * w + 128; ++k) acc = fma32(x[(size_t)b * 512 + k], W[(size_t)k * kActions + n], acc);
        c[w] = acc;
      }
      y[(size_t)b * kActions + n] = ((((c[0] + c[1]) + c[2]) + c[3]) + bias[n]);
    }
}

void qnet32_forward(const QNet& q, const uint8_t* x8, int B, Acts& a) {
  a.a1.assign((size_t)B * 20 * 20 * 32, 0.0f);
  a.a2.assign((size_t)B * 9 * 9 * 64, 0.0f);
  a.a3.assign((size_t)B * 7 * 7 * 64, 0.0f);
  a.a4.assign((size_t)B * 512, 0.0f);
  a.q.assign((size_t)B * kActions, 0.0f);
  conv1_fwd(x8, B, q.w[0].data(), q.w[1].data(), a.a1.data());
  conv_fwd(kC2, a.a1.data(), B, q.w[2].data(), q.w[3].data(), a.a2.data());
  conv_fwd(kC3, a.a2.data(), B, q.w[4].data(), q.w[5].data(), a.a3.data());
  dense_fwd(a.a3.data(), B, 3136, 512, q.w[6].data(), q.w[7].data(), true, a.a4.data(), kFc1Chains);
  head_fwd(a.a4.data(), B, q.w[8].data(), q.w[9].data(), a.q.data());
}

// conv weight gradient of one layer, chunked: dW [K*K*C][OC] and db [OC] from input `in` (fp32 NHWC, or the u8
// tensor view when in8 != null: conv1) and the ReLU-masked output gradient dz [B][OH][OW][OC]
static void conv_wgrad(const Cfg& c, const float* in, const uint8_t* in8, const float* dz, int B, int SC, float* dW, float* db,
                       const float* pb = nullptr) {
  const int KK = c.K * c.K * c.C, nz = (B + SC - 1) / SC;
  std::vector<float> part((size_t)nz * (KK + 1) * c.OC, 0.0f);
  std::vector<float> Pq((size_t)nz * 4 * c.OC, 0.0f);   // bias: chains C0..C3 per chunk
#pragma omp parallel for schedule(dynamic)
  for (int z = 0; z < nz; ++z) {
    float* P = part.data() + (size_t)z * (KK + 1) * c.OC;
    for (int b = z * SC; b < std::min(B, (z + 1) * SC); ++b)
      for (int oh = 0; oh < c.OH; ++oh)
        for (int ow = 0; ow < c.OW; ++ow) {
          const float* d = dz + (((size_t)b * c.OH + oh) * c.OW + ow) * c.OC;
          bool any = false;
          for (int oc = 0; oc < c.OC; ++oc) {
            // four interleaved chains over the chunk-local row index r mod 4 (combined below)
            float* Cq = Pq.data() + ((size_t)z * 4 + ((b - z * SC) * c.OH * c.OW + oh * c.OW + ow) % 4) * c.OC;
            Cq[oc] = Cq[oc] + d[oc];
            any |= d[oc] != 0.0f;
          }
          if (!any) continue;   // fmaf(x, 0, acc) == acc
          for (int kh = 0; kh < c.K; ++kh)
            for (int kw = 0; kw < c.K; ++kw)
              for (int ch = 0; ch < c.C; ++ch) {
                const int ih = oh * c.S + kh, iw = ow * c.S + kw;
                const float v = in8 ? (float)in8[(((size_t)b * c.H + ih) * c.W + iw) * c.C + ch]
                                    : in[(((size_t)b * c.H + ih) * c.W + iw) * c.C + ch];
                if (v == 0.0f) continue;
                float* pr = P + ((size_t)(kh * c.K + kw) * c.C + ch) * c.OC;
                for (int oc = 0; oc < c.OC; ++oc) pr[oc] = fma32(v, d[oc], pr[oc]);
              }
        }
  }
  // chunk partials in groups of 16: S_q = chain over the group's chunks, dW = chain over q of S_q
  auto combine = [&](size_t i) {
    float t = 0.0f;
    for (int q = 0; q * 16 < nz; ++q) {
      float sq = 0.0f;
      for (int z = 16 * q; z < std::min(nz, 16 * q + 16); ++z) sq = sq + part[(size_t)z * (KK + 1) * c.OC + i];
      t = t + sq;
    }
    return t;
  };
  for (int i = 0; i < KK * c.OC; ++i) dW[i] = combine(i);
  if (!pb) {
    for (int z = 0; z < nz; ++z)   // bias partial of chunk z = ((C0 + C1) + C2) + C3
      for (int oc = 0; oc < c.OC; ++oc) {
        const float* C = Pq.data() + (size_t)z * 4 * c.OC;
        part[((size_t)z * (KK + 1) + KK) * c.OC + oc] = ((C[oc] + C[c.OC + oc]) + C[2 * c.OC + oc]) + C[3 * c.OC + oc];
      }
  } else {
    // conv1 (round 6): rows i = g16 * (OH OW) + position of the backward's partials pb, R per chunk; chunk z's bias partial
    // = chain over jb = 0..15 of (chain over i = z R + jb + 16 k, k ascending, of pb[i][oc]) (k_conv1_wgrad32)
    const int NR = (B + 15) / 16 * c.OH * c.OW, R = (NR + nz - 1) / nz;
    for (int z = 0; z < nz; ++z)
      for (int oc = 0; oc < c.OC; ++oc) {
        const int i0 = z * R, i1 = std::min(NR, i0 + R);
        float sb = 0.0f;
        for (int jb = 0; jb < 16; ++jb) {
          float t = 0.0f;
          for (int i = i0 + jb; i < i1; i += 16) t = t + pb[(size_t)i * c.OC + oc];
          sb = sb + t;
        }
        part[((size_t)z * (KK + 1) + KK) * c.OC + oc] = sb;
      }
  }
  for (int oc = 0; oc < c.OC; ++oc) db[oc] = combine((size_t)KK * c.OC + oc);
}

// conv2 weight gradient, compacted (round 6, PConvWgrad CMP): per 16-sample chunk the chain runs over the chunk's
// non-background rows (b, oh, ow) ascending (bg[b][p]: the forward's classification - all frame pixels of the position's
// 20 x 20 receptive field 0), the bias chains Cq over the compacted row index mod 4; a background row's im2col row is
// u[m] = relu(b0[m % 32]) (m < 512), so the chunk's background share is u[m] S[oc], added per chunk before the two-level
// combine: part[z][m][oc] = fmaf(u[m], S_z[oc], chain) (u = 1 for the bias row).  S_z = ((T0 + T1) + T2) + T3, Tq = chain
// over p in [21 q, min(81, 21 q + 21)) of Pbg[z][p][oc] = (Q0 + Q1) + (Q2 + Q3), Qg = ((e0 + e1) + e2) + e3 over samples
// 16 z + 4 g .. + 3 of e = bg ? dz : 0 (0 past B) - the conv3 backward-data epilogue's sums (PConv3DgradPx::pbg, SideBgSum).
// (conv3 likewise: rows (b, oh, ow) of the 7 x 7 grid, u = the constant conv2 output row c2 at channel m % 64, S from
// the fc1 backward-data epilogue's sums over the 49 positions, Q = 13)
static void conv_wgrad_cmp(const Cfg& c, const float* in, const float* dz, int B, const uint8_t* bg, const float* uc, float* dW,
                           float* db) {
  constexpr int SC = 16;
  const int KK = c.K * c.K * c.C, P = c.OH * c.OW, nz = (B + SC - 1) / SC;   // (P <= 81)
  std::vector<float> part((size_t)nz * (KK + 1) * c.OC, 0.0f);
#pragma omp parallel for schedule(dynamic)
  for (int z = 0; z < nz; ++z) {
    float* Pz = part.data() + (size_t)z * (KK + 1) * c.OC;
    std::vector<float> Cq((size_t)4 * c.OC, 0.0f);
    int kc = 0;   // compacted row index
    for (int b = z * SC; b < std::min(B, (z + 1) * SC); ++b)
      for (int p = 0; p < P; ++p) {
        if (bg[(size_t)b * P + p]) continue;
        const int oh = p / c.OW, ow = p - oh * c.OW;
        const float* d = dz + ((size_t)b * P + p) * c.OC;
        for (int oc = 0; oc < c.OC; ++oc) Cq[(size_t)(kc % 4) * c.OC + oc] = Cq[(size_t)(kc % 4) * c.OC + oc] + d[oc];
        ++kc;
        for (int kh = 0; kh < c.K; ++kh)
          for (int kw = 0; kw < c.K; ++kw)
            for (int ch = 0; ch < c.C; ++ch) {
              const float v = in[(((size_t)b * c.H + oh * c.S + kh) * c.W + ow * c.S + kw) * c.C + ch];
              if (v == 0.0f) continue;   // fmaf(0, d, acc) == acc
              float* pr = Pz + ((size_t)(kh * c.K + kw) * c.C + ch) * c.OC;
              for (int oc = 0; oc < c.OC; ++oc) pr[oc] = fma32(v, d[oc], pr[oc]);
            }
      }
    for (int oc = 0; oc < c.OC; ++oc)
      Pz[(size_t)KK * c.OC + oc] = ((Cq[oc] + Cq[c.OC + oc]) + Cq[2 * c.OC + oc]) + Cq[3 * c.OC + oc];
    // the chunk's background rows: Pbg, S_z, then u[m] S_z[oc] into every row of the partial
    std::vector<float> pbg((size_t)P * c.OC);
    for (int p = 0; p < P; ++p)
      for (int oc = 0; oc < c.OC; ++oc) {
        float Q[4];
        for (int gq = 0; gq < 4; ++gq) {
          float e[4];
          for (int k = 0; k < 4; ++k) {
            const int b = SC * z + 4 * gq + k;
            e[k] = b < B && bg[(size_t)b * P + p] ? dz[((size_t)b * P + p) * c.OC + oc] : 0.0f;
          }
          Q[gq] = ((e[0] + e[1]) + e[2]) + e[3];
        }
        pbg[(size_t)p * c.OC + oc] = (Q[0] + Q[1]) + (Q[2] + Q[3]);
      }
    for (int oc = 0; oc < c.OC; ++oc) {
      float T[4];
      const int Q = (P + 3) / 4;
      for (int q = 0; q < 4; ++q) {
        float t = 0.0f;
        for (int p = Q * q; p < std::min(P, Q * q + Q); ++p) t = t + pbg[(size_t)p * c.OC + oc];
        T[q] = t;
      }
      const float S = ((T[0] + T[1]) + T[2]) + T[3];
      for (int m = 0; m <= KK; ++m) {
        const float u = m < KK ? uc[m % c.C] : 1.0f;
        Pz[(size_t)m * c.OC + oc] = fma32(u, S, Pz[(size_t)m * c.OC + oc]);
      }
    }
  }
  auto combine = [&](size_t i) {   // as conv_wgrad
    float t = 0.0f;
    for (int q = 0; q * 16 < nz; ++q) {
      float sq = 0.0f;
      for (int z = 16 * q; z < std::min(nz, 16 * q + 16); ++z) sq = sq + part[(size_t)z * (KK + 1) * c.OC + i];
      t = t + sq;
    }
    return t;
  };
  for (int i = 0; i < KK * c.OC; ++i) dW[i] = combine(i);
  for (int oc = 0; oc < c.OC; ++oc) db[oc] = combine((size_t)KK * c.OC + oc);
}

static bool g_dense = false;
void qnet32_set_dense(bool dense) { g_dense = dense; }

// background rows of each sample (c1_flags): position (i, j) of the n x n grid (conv2: 9, field 20; conv3: 7, field 36)
// whose frame pixels [8 i, 8 i + field) x [8 j, 8 j + field), all four channels, are 0
static std::vector<uint8_t> background(const uint8_t* x8, int B, int n, int field) {
  std::vector<uint8_t> bg((size_t)B * n * n);
  for (int b = 0; b < B; ++b)
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) {
        bool any = false;
        for (int y = 8 * i; y < 8 * i + field && !any; ++y)
          for (int x = 8 * j; x < 8 * j + field && !any; ++x)
            for (int ch = 0; ch < 4; ++ch) any |= x8[(((size_t)b * 84 + y) * 84 + x) * 4 + ch] != 0;
        bg[((size_t)b * n + i) * n + j] = any ? 0 : 1;
      }
  return bg;
}

// conv backward-data: din[b][ih][iw][c] = mask(a_in) * chain over the valid (kh, kw, oc) of dz[..][oc] W[kh][kw][c][oc]
static void conv_dgrad(const Cfg& c, const float* dz, int B, const float* W, const float* a_in, float* din) {
  // W transposed to [kh][kw][oc][c] so the per-c chains run along contiguous memory
  std::vector<float> WT((size_t)c.K * c.K * c.OC * c.C);
  for (int t = 0; t < c.K * c.K; ++t)
    for (int ch = 0; ch < c.C; ++ch)
      for (int oc = 0; oc < c.OC; ++oc) WT[((size_t)t * c.OC + oc) * c.C + ch] = W[((size_t)t * c.C + ch) * c.OC + oc];
#pragma omp parallel for schedule(static)
  for (int b = 0; b < B; ++b)
    for (int ih = 0; ih < c.H; ++ih)
      for (int iw = 0; iw < c.W; ++iw) {
        float acc[64];
        for (int ch = 0; ch < c.C; ++ch) acc[ch] = 0.0f;
        for (int kh = 0; kh < c.K; ++kh) {
          const int th = ih - kh;
          if (th < 0 || th % c.S != 0 || th / c.S >= c.OH) continue;
          for (int kw = 0; kw < c.K; ++kw) {
            const int tw = iw - kw;
            if (tw < 0 || tw % c.S != 0 || tw / c.S >= c.OW) continue;
            const float* d = dz + (((size_t)b * c.OH + th / c.S) * c.OW + tw / c.S) * c.OC;
            for (int oc = 0; oc < c.OC; ++oc) {
              const float v = d[oc];
              if (v == 0.0f) continue;
              const float* wr = WT.data() + ((size_t)(kh * c.K + kw) * c.OC + oc) * c.C;
              for (int ch = 0; ch < c.C; ++ch) acc[ch] = fma32(v, wr[ch], acc[ch]);
            }
          }
        }
        const size_t o = (((size_t)b * c.H + ih) * c.W + iw) * c.C;
        for (int ch = 0; ch < c.C; ++ch) din[o + ch] = a_in[o + ch] > 0.0f ? acc[ch] : 0.0f;
      }
}

float qnet32_loss_backward(const QNet& q, const uint8_t* x8, const uint8_t* actions, const float* y, int B, const Acts& a,
                           Grads& g, const float* weights, float* td_abs) {
  for (int v = 0; v < kNumVars; ++v) g.g[v].assign(kVarSize[v], 0.0f);
  // Huber head
  std::vector<float> gs(B), hs(B);
  float lsum = 0.0f;
  for (int b = 0; b < B; ++b) {
    const float qa = a.q[(size_t)b * kActions + actions[b]];
    const float e = qa - y[b];
    const float ae = std::fabs(e);
    const float w = weights ? weights[b] : 1.0f;
    const float ge = ae <= 1.0f ? e : (e > 0.0f ? 1.0f : -1.0f);
    gs[b] = (w * ge) / (float)B;
    hs[b] = w * (ae <= 1.0f ? 0.5f * e * e : ae - 0.5f);
    lsum = lsum + hs[b];
    if (td_abs) td_abs[b] = ae;
  }
  const float loss = lsum / (float)B;
  // dense 512 -> 3
  const float* W4 = q.w[8].data();
  std::vector<float> dz4((size_t)B * 512);
  for (int b = 0; b < B; ++b)
    for (int k = 0; k < 512; ++k) {
      const float av = a.a4[(size_t)b * 512 + k];
      dz4[(size_t)b * 512 + k] = av > 0.0f ? W4[k * 3 + actions[b]] * gs[b] : 0.0f;
    }
  for (int k = 0; k < 512; ++k) {
    float s[3] = {0.0f, 0.0f, 0.0f};
    for (int b = 0; b < B; ++b)
      for (int n = 0; n < 3; ++n) s[n] = fma32(a.a4[(size_t)b * 512 + k], actions[b] == n ? gs[b] : 0.0f, s[n]);
    for (int n = 0; n < 3; ++n) g.g[8][k * 3 + n] = s[n];
  }
  for (int n = 0; n < 3; ++n) {
    float s = 0.0f;
    for (int b = 0; b < B; ++b) s = s + (actions[b] == n ? gs[b] : 0.0f);
    g.g[9][n] = s;
  }
  // dense 3136 -> 512
  float* dW3 = g.g[6].data();
#pragma omp parallel for schedule(static)
  for (int k = 0; k < 3136; ++k) {
    float* row = dW3 + (size_t)k * 512;
    for (int b = 0; b < B; ++b) {
      const float v = a.a3[(size_t)b * 3136 + k];
      if (v == 0.0f) continue;
      const float* d = dz4.data() + (size_t)b * 512;
      for (int n = 0; n < 512; ++n) row[n] = fma32(v, d[n], row[n]);
    }
  }
  for (int n = 0; n < 512; ++n) {   // db3: four chains over b mod 4, ((C0 + C1) + C2) + C3
    float C[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    for (int b = 0; b < B; ++b) C[b % 4] = C[b % 4] + dz4[(size_t)b * 512 + n];
    g.g[7][n] = ((C[0] + C[1]) + C[2]) + C[3];
  }
  std::vector<float> W3T((size_t)512 * 3136);
  for (int k = 0; k < 3136; ++k)
    for (int n = 0; n < 512; ++n) W3T[(size_t)n * 3136 + k] = q.w[6][(size_t)k * 512 + n];
  std::vector<float> dz3((size_t)B * 3136);
#pragma omp parallel for schedule(static)
  for (int b = 0; b < B; ++b) {
    std::vector<float> acc(3136, 0.0f);
    for (int n = 0; n < 512; ++n) {
      const float v = dz4[(size_t)b * 512 + n];
      if (v == 0.0f) continue;
      const float* wr = W3T.data() + (size_t)n * 3136;
      for (int k = 0; k < 3136; ++k) acc[k] = fma32(v, wr[k], acc[k]);
    }
    for (int k = 0; k < 3136; ++k) dz3[(size_t)b * 3136 + k] = a.a3[(size_t)b * 3136 + k] > 0.0f ? acc[k] : 0.0f;
  }
  // conv3, conv2, conv1
  std::vector<float> dz2((size_t)B * 81 * 64), dz1((size_t)B * 400 * 32);
  static_assert(kSC3 == 16, "conv3 weight gradient: 16-sample chunks");
  const std::vector<uint8_t> bg2 = background(x8, B, 9, 20), bg3 = background(x8, B, 7, 36);
  if (g_dense) {
    conv_wgrad(kC3, a.a2.data(), nullptr, dz3.data(), B, kSC3, g.g[4].data(), g.g[5].data());
  } else {
    // u = c2: a2 at a conv2 background position (every such position holds it; none - no conv3 background row either)
    std::vector<float> c2(64, 0.0f);
    for (size_t r = 0; r < bg2.size(); ++r)
      if (bg2[r]) {
        std::memcpy(c2.data(), a.a2.data() + r * 64, 64 * 4);
        break;
      }
    conv_wgrad_cmp(kC3, a.a2.data(), dz3.data(), B, bg3.data(), c2.data(), g.g[4].data(), g.g[5].data());
  }
  conv_dgrad(kC3, dz3.data(), B, q.w[4].data(), a.a2.data(), dz2.data());
  static_assert(kSC2 == 16, "conv2 weight gradient: 16-sample chunks");
  if (g_dense) {
    conv_wgrad(kC2, a.a1.data(), nullptr, dz2.data(), B, kSC2, g.g[2].data(), g.g[3].data());
  } else {
    std::vector<float> u1(32);   // relu(0 + b0)
    for (int ch = 0; ch < 32; ++ch) u1[ch] = q.w[1][ch] > 0.0f ? q.w[1][ch] : 0.0f;
    conv_wgrad_cmp(kC2, a.a1.data(), dz2.data(), B, bg2.data(), u1.data(), g.g[2].data(), g.g[3].data());
  }
  conv_dgrad(kC2, dz2.data(), B, q.w[2].data(), a.a1.data(), dz1.data());
  const Cfg c1 = {84, 84, 4, 8, 4, 20, 20, 32};
  // conv1's bias partials as the conv2 backward-data epilogue forms them (PConv2DgradPx::pb): per 16-sample group and
  // position, (Q0 + Q1) + (Q2 + Q3) with Qg = ((d0 + d1) + d2) + d3 over samples 16 g16 + 4 g .. + 3 (0 past B)
  std::vector<float> pb1((size_t)(B + 15) / 16 * 400 * 32);
  for (int g16 = 0; g16 < (B + 15) / 16; ++g16)
    for (int r = 0; r < 400; ++r)
      for (int oc = 0; oc < 32; ++oc) {
        float Q[4];
        for (int gq = 0; gq < 4; ++gq) {
          float d[4];
          for (int e = 0; e < 4; ++e) {
            const int b = 16 * g16 + 4 * gq + e;
            d[e] = b < B ? dz1[((size_t)b * 400 + r) * 32 + oc] : 0.0f;
          }
          Q[gq] = ((d[0] + d[1]) + d[2]) + d[3];
        }
        pb1[((size_t)g16 * 400 + r) * 32 + oc] = (Q[0] + Q[1]) + (Q[2] + Q[3]);
      }
  conv_wgrad(c1, nullptr, x8, dz1.data(), B, kSC1, g.g[0].data(), g.g[1].data(), pb1.data());
  return loss;
}

// 64-lane xor butterfly (32 .. 1) of v[0..63]: every lane ends with the same value
static float butterfly64(const float* in) {
  float v[64];
  std::memcpy(v, in, sizeof(v));
  for (int off = 32; off > 0; off >>= 1) {
    float nv[64];
    for (int l = 0; l < 64; ++l) nv[l] = v[l] + v[l ^ off];
    std::memcpy(v, nv, sizeof(v));
  }
  return v[0];
}

// per-variable sums of squares in the build's order (header)
static float sumsq32(const float* g, int64_t n) {
  std::vector<float> part;
  for (int64_t b = 0; b < n; b += kNormSeg) {
    float t[256];
    for (int l = 0; l < 256; ++l) {
      float s = 0.0f;
      for (int h = 0; h < 2; ++h)
        for (int k = 0; k < 4; ++k) {
          const int64_t i = b + 1024 * h + 4 * l + k;
          if (i < n) s = fma32(g[i], g[i], s);
        }
      t[l] = s;
    }
    float w[4];
    for (int wv = 0; wv < 4; ++wv) w[wv] = butterfly64(t + 64 * wv);
    part.push_back(((w[0] + w[1]) + w[2]) + w[3]);
  }
  float c[64];
  for (int l = 0; l < 64; ++l) {
    float s = 0.0f;
    for (size_t j = l; j < part.size(); j += 64) s = s + part[j];
    c[l] = s;
  }
  return butterfly64(c);
}

void qnet32_apply_adam(QNet& q, const Grads& g, float* norms_out) {
  const float t = (float)(q.iterations + 1);
  const float b1p = std::pow(q.beta1, t), b2p = std::pow(q.beta2, t);
  const float alpha = q.lr * std::sqrt(1.0f - b2p) / (1.0f - b1p);
  for (int v = 0; v < kNumVars; ++v) {
    const float l2sum = sumsq32(g.g[v].data(), kVarSize[v]);
    const float l2norm = l2sum > 0.0f ? std::sqrt(l2sum) : l2sum;
    if (norms_out) norms_out[v] = l2norm;
    const float denom = std::max(l2norm, q.clipnorm);
    float* w = q.w[v].data();
    float* m = q.m[v].data();
    float* vv = q.v[v].data();
    for (int i = 0; i < kVarSize[v]; ++i) {
      const float gc = (g.g[v][i] * q.clipnorm) / denom;
      m[i] += (gc - m[i]) * (1.0f - q.beta1);
      vv[i] += (gc * gc - vv[i]) * (1.0f - q.beta2);
      w[i] -= (m[i] * alpha) / (std::sqrt(vv[i]) + q.eps);
    }
  }
  q.iterations += 1;
}

}  // namespace orc
