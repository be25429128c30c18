// ORACLE — TEST INFRASTRUCTURE ONLY (see rng_ref.h / qnet_ref.h headers).
#include "qnet_ref.h"

#include <algorithm>
#include <cmath>
#include <cstring>

#include <omp.h>

#include "rng_ref.h"

namespace orc {

const int kVarSize[kNumVars] = {8 * 8 * 4 * 32, 32, 4 * 4 * 32 * 64, 64, 3 * 3 * 64 * 64, 64, 3136 * 512, 512, 512 * 3, 3};

struct ConvCfg { int H, W, C, K, S, OC, OH, OW; };
static const ConvCfg kConv[3] = {
    {84, 84, 4, 8, 4, 32, 20, 20},
    {20, 20, 32, 4, 2, 64, 9, 9},
    {9, 9, 64, 3, 1, 64, 7, 7},
};

void qnet_init_glorot(QNet& q, uint64_t seed) {
  // keras GlorotUniform: limit = sqrt(6 / (fan_in + fan_out)); biases zeros
  const int fan_in[5] = {8 * 8 * 4, 4 * 4 * 32, 3 * 3 * 64, 3136, 512};
  const int fan_out[5] = {8 * 8 * 32, 4 * 4 * 64, 3 * 3 * 64, 512, 3};
  for (int v = 0; v < kNumVars; ++v) {
    q.w[v].assign(kVarSize[v], 0.0f);
    q.m[v].assign(kVarSize[v], 0.0f);
    q.v[v].assign(kVarSize[v], 0.0f);
    if (v % 2 == 0) {
      const int l = v / 2;
      const float limit = std::sqrt(6.0f / (float)(fan_in[l] + fan_out[l]));
      Stream s(seed, (uint32_t)v, 0, P_INIT);
      for (int i = 0; i < kVarSize[v]; ++i) q.w[v][i] = gen_range_f32(s, -limit, limit);
    }
  }
  q.iterations = 0;
}

void qnet_copy_weights(QNet& dst, const QNet& src) {
  for (int v = 0; v < kNumVars; ++v) dst.w[v] = src.w[v];
}

// out[b][oh][ow][oc] = relu(bias + sum_{kh,kw,c} in[b][oh*S+kh][ow*S+kw][c] * W[kh][kw][c][oc])
static void conv_fwd(const ConvCfg& c, const float* in, int B, const float* W, const float* bias, float* out) {
  const int KK = c.K * c.K * c.C;
#pragma omp parallel for schedule(static)
  for (int b = 0; b < B; ++b) {
    std::vector<float> patch(KK);
    std::vector<double> acc(c.OC);
    for (int oh = 0; oh < c.OH; ++oh)
      for (int ow = 0; ow < c.OW; ++ow) {
        int k = 0;
        for (int kh = 0; kh < c.K; ++kh)
          for (int kw = 0; kw < c.K; ++kw) {
            const float* src = in + (((size_t)b * c.H + oh * c.S + kh) * c.W + ow * c.S + kw) * c.C;
            for (int ch = 0; ch < c.C; ++ch) patch[k++] = src[ch];
          }
        for (int oc = 0; oc < c.OC; ++oc) acc[oc] = 0.0;
        for (int kk = 0; kk < KK; ++kk) {
          const double p = patch[kk];
          if (p == 0.0) continue;
          const float* wr = W + (size_t)kk * c.OC;
          for (int oc = 0; oc < c.OC; ++oc) acc[oc] += p * (double)wr[oc];
        }
        float* o = out + (((size_t)b * c.OH + oh) * c.OW + ow) * c.OC;
        for (int oc = 0; oc < c.OC; ++oc) {
          const float v = (float)acc[oc] + bias[oc];
          o[oc] = v > 0.0f ? v : 0.0f;
        }
      }
  }
}

// y[b][n] = act(bias[n] + sum_k x[b][k] W[k][n])
static void dense_fwd(const float* x, int B, int K, int N, const float* W, const float* bias, bool relu, float* y) {
#pragma omp parallel for schedule(static)
  for (int b = 0; b < B; ++b) {
    std::vector<double> acc(N, 0.0);
    for (int k = 0; k < K; ++k) {
      const double xv = x[(size_t)b * K + k];
      if (xv == 0.0) continue;
      const float* wr = W + (size_t)k * N;
      for (int n = 0; n < N; ++n) acc[n] += xv * (double)wr[n];
    }
    for (int n = 0; n < N; ++n) {
      const float v = (float)acc[n] + bias[n];
      y[(size_t)b * N + n] = relu ? (v > 0.0f ? v : 0.0f) : v;
    }
  }
}

void qnet_forward(const QNet& q, const uint8_t* x8, int B, Acts& a) {
  std::vector<float> x((size_t)B * 84 * 84 * 4);
  for (size_t i = 0; i < x.size(); ++i) x[i] = (float)x8[i];
  a.a1.assign((size_t)B * 20 * 20 * 32, 0.0f);
  a.a2.assign((size_t)B * 9 * 9 * 64, 0.0f);
  a.a3.assign((size_t)B * 7 * 7 * 64, 0.0f);
  a.a4.assign((size_t)B * 512, 0.0f);
  a.q.assign((size_t)B * kActions, 0.0f);
  conv_fwd(kConv[0], x.data(), B, q.w[0].data(), q.w[1].data(), a.a1.data());
  conv_fwd(kConv[1], a.a1.data(), B, q.w[2].data(), q.w[3].data(), a.a2.data());
  conv_fwd(kConv[2], a.a2.data(), B, q.w[4].data(), q.w[5].data(), a.a3.data());
  dense_fwd(a.a3.data(), B, 3136, 512, q.w[6].data(), q.w[7].data(), true, a.a4.data());
  dense_fwd(a.a4.data(), B, 512, kActions, q.w[8].data(), q.w[9].data(), false, a.q.data());
}

// Backward of conv with ReLU output `out` (dOut given wrt post-ReLU output).
// dW[kh][kw][c][oc] += in * dz ; db[oc] += dz ; dIn (optional) += W * dz.   dz = dOut * (out > 0)
static void conv_bwd(const ConvCfg& c, const float* in, const float* out, const float* dout, int B, const float* W,
                     double* dW, double* db, float* din) {
  const int KK = c.K * c.K * c.C;
  const int nthr = omp_get_max_threads();
  std::vector<std::vector<double>> parts_w(nthr), parts_b(nthr);
#pragma omp parallel num_threads(nthr)
  {
    std::vector<double>& ldW = parts_w[omp_get_thread_num()];
    std::vector<double>& ldb = parts_b[omp_get_thread_num()];
    ldW.assign((size_t)KK * c.OC, 0.0);
    ldb.assign(c.OC, 0.0);
    std::vector<double> dz(c.OC);
    std::vector<double> dinacc;
#pragma omp for schedule(static)
    for (int b = 0; b < B; ++b) {
      if (din) dinacc.assign((size_t)c.H * c.W * c.C, 0.0);
      for (int oh = 0; oh < c.OH; ++oh)
        for (int ow = 0; ow < c.OW; ++ow) {
          const size_t o = (((size_t)b * c.OH + oh) * c.OW + ow) * c.OC;
          bool any = false;
          for (int oc = 0; oc < c.OC; ++oc) {
            dz[oc] = out[o + oc] > 0.0f ? (double)dout[o + oc] : 0.0;
            any |= dz[oc] != 0.0;
            ldb[oc] += dz[oc];
          }
          if (!any) continue;
          int kk = 0;
          for (int kh = 0; kh < c.K; ++kh)
            for (int kw = 0; kw < c.K; ++kw) {
              const size_t ib = ((size_t)(oh * c.S + kh) * c.W + ow * c.S + kw) * c.C;
              for (int ch = 0; ch < c.C; ++ch, ++kk) {
                const double xv = in[(size_t)b * c.H * c.W * c.C + ib + ch];
                double* dwr = ldW.data() + (size_t)kk * c.OC;
                const float* wr = W + (size_t)kk * c.OC;
                if (xv != 0.0)
                  for (int oc = 0; oc < c.OC; ++oc) dwr[oc] += xv * dz[oc];
                if (din) {
                  double s = 0.0;
                  for (int oc = 0; oc < c.OC; ++oc) s += (double)wr[oc] * dz[oc];
                  dinacc[ib + ch] += s;
                }
              }
            }
        }
      if (din)
        for (size_t i = 0; i < dinacc.size(); ++i) din[(size_t)b * c.H * c.W * c.C + i] = (float)dinacc[i];
    }
  }
  // deterministic reduction order (thread index)
  for (int t = 0; t < nthr; ++t) {
    if (parts_w[t].empty()) continue;
    for (size_t i = 0; i < parts_w[t].size(); ++i) dW[i] += parts_w[t][i];
    for (int oc = 0; oc < c.OC; ++oc) db[oc] += parts_b[t][oc];
  }
}

float qnet_loss_backward(const QNet& q, const uint8_t* x8, const uint8_t* actions, const float* y, int B,
                         const Acts& a, Grads& g, const float* weights, float* td_abs) {
  for (int v = 0; v < kNumVars; ++v) g.g[v].assign(kVarSize[v], 0.0f);
  // Huber(delta=1), error = y_pred - y_true, mean over batch (keras SUM_OVER_BATCH_SIZE)
  std::vector<float> dq((size_t)B * kActions, 0.0f);
  double loss_sum = 0.0;
  for (int b = 0; b < B; ++b) {
    const float qa = a.q[(size_t)b * kActions + actions[b]];
    const float e = qa - y[b];
    const float ae = std::fabs(e);
    const float w = weights ? weights[b] : 1.0f;   // prioritized replay importance-sampling weight
    const float h = ae <= 1.0f ? 0.5f * e * e : ae - 0.5f;
    loss_sum += w * h;
    const float ge = ae <= 1.0f ? e : (e > 0.0f ? 1.0f : -1.0f);
    dq[(size_t)b * kActions + actions[b]] = (w * ge) / (float)B;
    if (td_abs) td_abs[b] = ae;
  }
  const float loss = (float)(loss_sum / (double)B);

  // fc2 (linear): dW4[k][n] = sum_b a4[b][k] dq[b][n]; db4; da4 = dq W4^T masked by relu(a4)
  std::vector<double> dW4((size_t)512 * kActions, 0.0), db4(kActions, 0.0);
  std::vector<float> da4((size_t)B * 512, 0.0f);
  for (int b = 0; b < B; ++b) {
    for (int n = 0; n < kActions; ++n) db4[n] += dq[(size_t)b * kActions + n];
    for (int k = 0; k < 512; ++k) {
      const float av = a.a4[(size_t)b * 512 + k];
      double s = 0.0;
      for (int n = 0; n < kActions; ++n) {
        const double d = dq[(size_t)b * kActions + n];
        dW4[(size_t)k * kActions + n] += (double)av * d;
        s += (double)q.w[8][(size_t)k * kActions + n] * d;
      }
      da4[(size_t)b * 512 + k] = av > 0.0f ? (float)s : 0.0f;
    }
  }
  // fc1 (relu; da4 already masked): dW3[k][n] = sum_b a3[b][k] da4[b][n]; da3 = da4 W3^T
  std::vector<double> dW3((size_t)3136 * 512, 0.0), db3(512, 0.0);
  std::vector<float> da3((size_t)B * 3136, 0.0f);
#pragma omp parallel for schedule(static)
  for (int k = 0; k < 3136; ++k) {
    double* row = dW3.data() + (size_t)k * 512;
    for (int b = 0; b < B; ++b) {
      const double xv = a.a3[(size_t)b * 3136 + k];
      if (xv == 0.0) continue;
      const float* d = da4.data() + (size_t)b * 512;
      for (int n = 0; n < 512; ++n) row[n] += xv * (double)d[n];
    }
  }
  for (int b = 0; b < B; ++b)
    for (int n = 0; n < 512; ++n) db3[n] += da4[(size_t)b * 512 + n];
#pragma omp parallel for schedule(static)
  for (int b = 0; b < B; ++b)
    for (int k = 0; k < 3136; ++k) {
      const float* wr = q.w[6].data() + (size_t)k * 512;
      const float* d = da4.data() + (size_t)b * 512;
      double s = 0.0;
      for (int n = 0; n < 512; ++n) s += (double)wr[n] * (double)d[n];
      da3[(size_t)b * 3136 + k] = (float)s;
    }
  // convs (conv_bwd applies the relu mask of its own output)
  std::vector<double> dW2(kVarSize[4], 0.0), db2(64, 0.0), dW1(kVarSize[2], 0.0), db1(64, 0.0), dW0(kVarSize[0], 0.0),
      db0(32, 0.0);
  std::vector<float> da2((size_t)B * 9 * 9 * 64, 0.0f), da1((size_t)B * 20 * 20 * 32, 0.0f);
  conv_bwd(kConv[2], a.a2.data(), a.a3.data(), da3.data(), B, q.w[4].data(), dW2.data(), db2.data(), da2.data());
  conv_bwd(kConv[1], a.a1.data(), a.a2.data(), da2.data(), B, q.w[2].data(), dW1.data(), db1.data(), da1.data());
  std::vector<float> x((size_t)B * 84 * 84 * 4);
  for (size_t i = 0; i < x.size(); ++i) x[i] = (float)x8[i];
  conv_bwd(kConv[0], x.data(), a.a1.data(), da1.data(), B, q.w[0].data(), dW0.data(), db0.data(), nullptr);

  auto put = [&](int v, const std::vector<double>& src) {
    for (int i = 0; i < kVarSize[v]; ++i) g.g[v][i] = (float)src[i];
  };
  put(0, dW0); put(1, db0); put(2, dW1); put(3, db1); put(4, dW2); put(5, db2);
  put(6, dW3); put(7, db3); put(8, dW4); put(9, db4);
  return loss;
}

void qnet_apply_adam(QNet& q, const Grads& g, float* norms_out) {
  // legacy keras Adam._resource_apply_dense -> ResourceApplyAdam, t = iterations + 1
  const float t = (float)(q.iterations + 1);
  const float b1p = std::pow(q.beta1, t), b2p = std::pow(q.beta2, t);
  const float alpha = q.lr * std::sqrt(1.0f - b2p) / (1.0f - b1p);
  for (int v = 0; v < kNumVars; ++v) {
    // tf.clip_by_norm(g, clipnorm): g * clipnorm / max(l2norm, clipnorm)
    double ss = 0.0;
    for (float x : g.g[v]) ss += (double)x * (double)x;
    const float l2sum = (float)ss;
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

int argmax_first(const float* q, int n) {
  int best = 0;
  for (int i = 1; i < n; ++i) if (q[i] > q[best]) best = i;
  return best;
}

}  // namespace orc
