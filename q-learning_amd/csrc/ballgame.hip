// BallGame on MI355X: the reference's second Environment / DeepQLearningModel pair,
// batched on the GPU behind the same C ABI conventions as Breakout.
//
// Reference (restated):
//   BallGameTestEnvironment   src/ql/src/test/ballgame_test_environment.rs:12-262 (random_initial_state
//                             :100-123, step :69-86, do_move :155-190, actions :240-249, goal mean 9.5 :88)
//   state tensor              src/ql-with-tensorflow/src/test/ballgame_test_env_addons.rs:7-50 (one-hot [x][y][4])
//   Q-model                   src/ql-with-tensorflow/python_model/create_ql_model_ballgame_3x3x4_5_512.py:24-40,
//                             :71-85 (Conv2D 32 2x2 'same' relu, Conv2D 32 1x1 relu, Dense 512 relu, Dense 5;
//                             MSE of q_a = sum(Q(s) * one_hot(a)); Adam(2.5e-4, clipnorm 1))
//   learner                   self_driving_tf_q_learner.rs:141-233, vectorised as the Breakout learner
// The net is 0.33 MFLOP per sample: fp32 SIMT kernels (LDS-tiled GEMM for the dense layers), every reduction in
// a fixed order.  Tolerances against the fp32 oracle are stated in tests/test_gpu_ballgame.py.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "objects.h"
#include "per.h"
#include "stats.h"

namespace qlx {
namespace bg {

constexpr int kObs = 36;        // [3][3][4] u8 one-hot
constexpr int kA = 5;
constexpr int kMaxSteps = 16;   // MAX_STEPS (:12)
enum : uint8_t { EMPTY = 0, GOAL = 1, BALL = 2, OBST = 3 };
constexpr int kVars = 8;
constexpr int kVarSize[kVars] = {2 * 2 * 4 * 32, 32, 32 * 32, 32, 288 * 512, 512, 512 * 5, 5};
constexpr int64_t var_off(int v) { return v == 0 ? 0 : var_off(v - 1) + kVarSize[v - 1]; }
constexpr int64_t kParams = var_off(kVars);
static_assert(kParams == 152133, "BallGame parameter count");

// ---------------- environment ----------------

__device__ void random_initial_state(qlx_ballgame_state& st, RngStream& s) {   // :100-123
  const uint8_t gx = (uint8_t)uniform_usize_single(s, 3);
  const uint8_t bx = (uint8_t)uniform_usize_single(s, 3);
  uint8_t ox, oy;
  for (;;) {
    ox = (uint8_t)uniform_usize_single(s, 3);
    oy = (uint8_t)uniform_usize_single(s, 3);
    if (!(ox == gx && oy == 0) && !(ox == bx && oy == 2) && !(ox == 1 && oy == 1)) break;
  }
  for (int i = 0; i < 9; ++i) st.field[i] = EMPTY;
  st.field[gx * 3 + 0] = GOAL;
  st.field[bx * 3 + 2] = BALL;
  st.field[1 * 3 + 1] = OBST;
  st.field[ox * 3 + oy] = OBST;
  st.ball_x = bx;
  st.ball_y = 2;
  st.pad = 0;
  st.steps = 0;
}

// new (bump = 0, reset_count 0) or Environment::reset (bump = 1) of every env or where mask[e] != 0
__global__ void k_env_init(qlx_ballgame_state* st, uint32_t* ep_steps, uint32_t n, uint64_t seed, uint32_t id_offset,
                           const uint8_t* mask, int bump) {
  const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n || (mask && !mask[e])) return;
  const uint32_t rc = bump ? st[e].reset_count + 1 : 0;
  RngStream s(seed, id_offset + e, rc, P_BALLGAME);
  qlx_ballgame_state v;
  random_initial_state(v, s);
  v.reset_count = rc;
  st[e] = v;
  ep_steps[e] = 0;
}

// Environment::step (:69-86) with do_move (:155-190)
__device__ void env_step(qlx_ballgame_state& st, uint8_t action, float* reward, uint8_t* done) {
  st.steps += 1;
  const int x = st.ball_x, y = st.ball_y;
  auto valid = [&](int tx, int ty) {
    const uint8_t v = st.field[tx * 3 + ty];
    return v == EMPTY || v == GOAL;
  };
  int tx = -1, ty = -1;
  switch (action) {
    case 0: if (x > 0 && valid(x - 1, y)) { tx = x - 1; ty = y; } break;   // West
    case 1: if (y > 0 && valid(x, y - 1)) { tx = x; ty = y - 1; } break;   // North
    case 2: if (x < 2 && valid(x + 1, y)) { tx = x + 1; ty = y; } break;   // East
    case 3: if (y < 2 && valid(x, y + 1)) { tx = x; ty = y + 1; } break;   // South
    default: tx = x; ty = y; break;                                        // Nothing
  }
  const bool legal = tx >= 0;
  bool reached = false;
  if (legal) {
    reached = st.field[tx * 3 + ty] == GOAL;
    st.field[x * 3 + y] = EMPTY;
    st.field[tx * 3 + ty] = BALL;
    st.ball_x = (uint8_t)tx;
    st.ball_y = (uint8_t)ty;
  }
  if (legal && reached) { *reward = 10.0f; *done = 1; }
  else if (st.steps >= (uint32_t)kMaxSteps) { *reward = -10.0f; *done = 1; }
  else if (legal) { *reward = -0.02f; *done = 0; }
  else { *reward = -1.0f; *done = 0; }
}

__global__ void k_env_step(qlx_ballgame_state* st, uint32_t* ep_steps, uint32_t n, const uint8_t* actions, float* rewards,
                           uint8_t* dones, uint32_t* bad) {
  const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const uint8_t a = actions[e];
  if (a >= kA) { atomicOr(bad, 1u); return; }   // Action::try_from_numeric error
  qlx_ballgame_state v = st[e];
  env_step(v, a, &rewards[e], &dones[e]);
  st[e] = v;
  ep_steps[e] += 1;
}

__device__ __forceinline__ void obs_of(const qlx_ballgame_state& st, uint8_t* out) {   // one-hot [x][y][4]
  for (int p = 0; p < 9; ++p)
    for (int c = 0; c < 4; ++c) out[p * 4 + c] = st.field[p] == c ? 1 : 0;
}

__global__ void k_env_obs(const qlx_ballgame_state* st, uint32_t n, uint8_t* obs) {
  const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e < n) obs_of(st[e], obs + (size_t)e * kObs);
}

// ---------------- Q-model kernels (fp32) ----------------

// conv1 (2x2 'same': taps past the edge read TF's trailing zero padding) + conv2 (1x1), one block per sample,
// thread t = position * 32 + channel.  a1 / a2 [B][9][32] (post-ReLU).
__global__ __launch_bounds__(288) void k_conv_fwd(const uint8_t* obs, int B, const float* prm, float* a1, float* a2) {
  __shared__ float x[kObs];
  __shared__ float s1[288];
  const int b = blockIdx.x, t = threadIdx.x, p = t >> 5, o = t & 31, i = p / 3, j = p - i * 3;
  if (b >= B) return;
  if (t < kObs) x[t] = (float)obs[(size_t)b * kObs + t];
  __syncthreads();
  const float* k0 = prm + var_off(0);
  float s = 0.0f;
  for (int di = 0; di < 2; ++di)
    for (int dj = 0; dj < 2; ++dj)
      if (i + di < 3 && j + dj < 3)
        for (int c = 0; c < 4; ++c) s += x[((i + di) * 3 + j + dj) * 4 + c] * k0[((di * 2 + dj) * 4 + c) * 32 + o];
  const float v1 = fmaxf(s + prm[var_off(1) + o], 0.0f);
  s1[t] = v1;
  a1[(size_t)b * 288 + t] = v1;
  __syncthreads();
  const float* k1 = prm + var_off(2);
  float s2 = 0.0f;
  for (int c = 0; c < 32; ++c) s2 += s1[p * 32 + c] * k1[c * 32 + o];
  a2[(size_t)b * 288 + t] = fmaxf(s2 + prm[var_off(3) + o], 0.0f);
}

// C[M][N] = op(A)[M][K] op(B)[K][N] in fp32, 64 x 64 tiles, 256 threads x 4 x 4 outputs, k through LDS in
// steps of 16 (fixed order per output).  A(m, k) = TA ? A[k lda + m] : A[m lda + k];  B(k, n) = TB ?
// B[n ldb + k] : B[k ldb + n].  EPI 0: store; 1: + bias[n], ReLU; 2: * (mask[m ldc + n] > 0).
template <bool TA, bool TB, int EPI>
__global__ __launch_bounds__(256) void k_gemm_f32(int M, int N, int K, const float* __restrict__ A, int lda,
                                                  const float* __restrict__ Bm, int ldb, float* __restrict__ C, int ldc,
                                                  const float* __restrict__ aux) {
  __shared__ float sa[16][64 + 1];
  __shared__ float sb[16][64 + 1];
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  const int m0 = blockIdx.x * 64, n0 = blockIdx.y * 64;
  float acc[4][4] = {};
  for (int k0 = 0; k0 < K; k0 += 16) {
    for (int i = tid; i < 16 * 64; i += 256) {
      const int kk = i >> 6, mm = i & 63;
      const int m = m0 + mm, k = k0 + kk;
      sa[kk][mm] = (m < M && k < K) ? (TA ? A[(size_t)k * lda + m] : A[(size_t)m * lda + k]) : 0.0f;
      const int n = n0 + mm;
      sb[kk][mm] = (n < N && k < K) ? (TB ? Bm[(size_t)n * ldb + k] : Bm[(size_t)k * ldb + n]) : 0.0f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
      float av[4], bv[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) { av[r] = sa[kk][ty * 4 + r]; bv[r] = sb[kk][tx * 4 + r]; }
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[r][c] += av[r] * bv[c];
    }
    __syncthreads();
  }
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int m = m0 + ty * 4 + r, n = n0 + tx * 4 + c;
      if (m >= M || n >= N) continue;
      float v = acc[r][c];
      if (EPI == 1) v = fmaxf(v + aux[n], 0.0f);
      if (EPI == 2) v = aux[(size_t)m * ldc + n] > 0.0f ? v : 0.0f;
      C[(size_t)m * ldc + n] = v;
    }
}

template <bool TA, bool TB, int EPI>
static void gemm(hipStream_t s, int M, int N, int K, const float* A, int lda, const float* Bm, int ldb, float* C, int ldc,
                 const float* aux = nullptr) {
  hipLaunchKernelGGL((k_gemm_f32<TA, TB, EPI>), dim3((M + 63) / 64, (N + 63) / 64), dim3(256), 0, s, M, N, K, A, lda, Bm, ldb, C,
                     ldc, aux);
  QLX_HIP(hipGetLastError());
}

struct HeadArgs {
  const float* a3;         // [B][512]
  const float* prm;
  int B;
  float* q;                // [B][5] (may be null)
  uint8_t* argmax;         // mode 1
  const float* rewards;    // mode 2
  const uint8_t* dones;
  float gamma;
  float* y_out;
  const float* q_select;   // mode 2, double DQN: [B][5] online Q(s'); y uses q[first argmax] instead of max q
  const uint8_t* actions;  // mode 3 (train)
  const float* y;
  float* dq;               // [B][5]
  float* hs;               // [B] squared errors
  float* dz3;              // [B][512]
  const float* weights;    // mode 3 (optional): per-sample loss weights (prioritized-replay IS weights)
  float* td_abs;           // mode 3 (optional): |q_a - y| out
};

// dense 512 -> 5, one wave per sample.  MODE 0: q; 1: argmax (predict_action); 2: y = r + gamma max q (or r if
// done); 3: MSE train head: e = q_a - y, dq = 2 e / B at a, dz3 = dq_a W3[:, a] * (a3 > 0).
template <int MODE>
__global__ __launch_bounds__(256) void k_head(HeadArgs H) {
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (b >= H.B) return;
  const float* w = H.prm + var_off(6);
  const float* a = H.a3 + (size_t)b * 512;
  float s[kA] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
  for (int n = lane; n < 512; n += 64) {
    const float x = a[n];
#pragma unroll
    for (int k = 0; k < kA; ++k) s[k] += x * w[n * kA + k];
  }
#pragma unroll
  for (int k = 0; k < kA; ++k)
    for (int off = 32; off > 0; off >>= 1) s[k] += __shfl_xor(s[k], off);
  float q[kA];
#pragma unroll
  for (int k = 0; k < kA; ++k) q[k] = s[k] + H.prm[var_off(7) + k];
  if (lane == 0 && H.q)
    for (int k = 0; k < kA; ++k) H.q[(size_t)b * kA + k] = q[k];
  if (MODE == 1 && lane == 0) {
    int best = 0;
    for (int k = 1; k < kA; ++k) if (q[k] > q[best]) best = k;
    H.argmax[b] = (uint8_t)best;
  }
  if (MODE == 2 && lane == 0) {
    float mx = q[0];
    if (H.q_select) {   // double DQN
      const float* qs = H.q_select + (size_t)b * kA;
      int best = 0;
      for (int k = 1; k < kA; ++k) if (qs[k] > qs[best]) best = k;
      mx = q[best];
    } else {
      for (int k = 1; k < kA; ++k) mx = fmaxf(mx, q[k]);
    }
    H.y_out[b] = H.dones[b] ? H.rewards[b] : __fadd_rn(H.rewards[b], __fmul_rn(mx, H.gamma));
  }
  if (MODE == 3) {
    const int act = H.actions[b];
    const float e = q[act] - H.y[b];
    const float wt = H.weights ? H.weights[b] : 1.0f;
    const float g = 2.0f * (wt * e) / (float)H.B;
    if (lane == 0) {
      H.hs[b] = wt * (e * e);
      if (H.td_abs) H.td_abs[b] = fabsf(e);
      for (int k = 0; k < kA; ++k) H.dq[(size_t)b * kA + k] = k == act ? g : 0.0f;
    }
    for (int n = lane; n < 512; n += 64) H.dz3[(size_t)b * 512 + n] = a[n] > 0.0f ? g * w[n * kA + act] : 0.0f;
  }
}

// out[j] = sum_r A[r][j] (rows x cols, row stride lda); column j of block blockIdx.x * 64 + (t & 63), 4 row
// phases combined in order.  scale multiplies the result (loss = sum / B).
__global__ __launch_bounds__(256) void k_colsum(const float* A, int rows, int cols, int lda, float scale, float* out) {
  __shared__ float part[4][64];
  const int t = threadIdx.x, j = blockIdx.x * 64 + (t & 63), ph = t >> 6;
  float s = 0.0f;
  if (j < cols)
    for (int r = ph; r < rows; r += 4) s += A[(size_t)r * lda + j];
  part[ph][t & 63] = s;
  __syncthreads();
  if (t < 64 && j < cols) out[j] = (((part[0][t] + part[1][t]) + part[2][t]) + part[3][t]) * scale;
}

static void colsum(hipStream_t s, const float* A, int rows, int cols, int lda, float* out, float scale = 1.0f) {
  hipLaunchKernelGGL(k_colsum, dim3((cols + 63) / 64), dim3(256), 0, s, A, rows, cols, lda, scale, out);
  QLX_HIP(hipGetLastError());
}

// dK0[(di*2+dj)*4 + c][o] = sum_(b,i,j) x[b][i+di][j+dj][c] dz1[b][i*3+j][o] over in-range taps; block = one
// (di, dj, c) row, thread = (o, row phase r of 8), phases combined in order
__global__ __launch_bounds__(256) void k_conv1_wgrad(const uint8_t* obs, const float* dz1, int B, float* g0) {
  __shared__ float part[8][32];
  const int kr = blockIdx.x, tap = kr >> 2, c = kr & 3, di = tap >> 1, dj = tap & 1;
  const int t = threadIdx.x, o = t & 31, ph = t >> 5;
  float s = 0.0f;
  for (int q = ph; q < B * 9; q += 8) {
    const int b = q / 9, p = q - b * 9, i = p / 3, j = p - i * 3;
    if (i + di < 3 && j + dj < 3) s += (float)obs[(size_t)b * kObs + ((i + di) * 3 + j + dj) * 4 + c] * dz1[(size_t)q * 32 + o];
  }
  part[ph][o] = s;
  __syncthreads();
  if (t < 32) {
    float v = 0.0f;
    for (int r = 0; r < 8; ++r) v += part[r][t];
    g0[kr * 32 + t] = v;
  }
}

// per-variable L2 norms (one block per variable, fixed-order tree) and legacy Adam with clip_by_norm
__global__ __launch_bounds__(256) void k_norms(const float* g, float* norms) {
  __shared__ float red[256];
  const int v = blockIdx.x;
  const float* gv = g + var_off(v);
  float s = 0.0f;
  for (int i = threadIdx.x; i < kVarSize[v]; i += 256) s += gv[i] * gv[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) norms[v] = red[0] > 0.0f ? sqrtf(red[0]) : red[0];
}

__global__ __launch_bounds__(256) void k_adam(float* w, float* m, float* vv, const float* g, const float* norms, float alpha,
                                              float beta1, float beta2, float eps, float clipnorm) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < kParams; i += (int64_t)gridDim.x * blockDim.x) {
    int var = 0;
    while (var + 1 < kVars && i >= var_off(var + 1)) ++var;
    const float gc = (g[i] * clipnorm) / fmaxf(norms[var], clipnorm);
    float mi = m[i], vi = vv[i], wi = w[i];
    mi += (gc - mi) * (1.0f - beta1);
    vi += (gc * gc - vi) * (1.0f - beta2);
    wi -= (mi * alpha) / (sqrtf(vi) + eps);
    m[i] = mi;
    vv[i] = vi;
    w[i] = wi;
  }
}

}  // namespace bg
}  // namespace qlx

using namespace qlx;

// ---------------- objects ----------------

struct qlx_bg_env {
  int device = 0;
  uint32_t n = 0;
  uint64_t seed = 0;
  uint32_t id_offset = 0;
  hipStream_t stream = nullptr;
  bool own_stream = true;
  qlx_ballgame_state* d_state = nullptr;
  uint32_t* d_ep_steps = nullptr;
  uint32_t* d_bad = nullptr;
  uint8_t* d_tmp_u8 = nullptr;
  uint8_t* d_tmp_u8b = nullptr;
  float* d_tmp_f32 = nullptr;
};

struct BgWs {
  uint8_t* obs = nullptr;   // [B][36]
  float *a1 = nullptr, *a2 = nullptr, *a3 = nullptr, *q = nullptr, *dq = nullptr, *hs = nullptr;
  float *dz3 = nullptr, *dz2 = nullptr, *dz1 = nullptr, *y = nullptr, *rew = nullptr, *loss = nullptr;
  uint8_t *act = nullptr, *argmax = nullptr, *done = nullptr;
};

struct qlx_bg_model {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = true;
  float *d_params = nullptr, *d_m = nullptr, *d_v = nullptr, *d_grads = nullptr, *d_norms = nullptr;
  int64_t iterations = 0;
  float lr = 0.00025f, beta1 = 0.9f, beta2 = 0.999f, eps = 1e-7f, clipnorm = 1.0f;
  void* ws = nullptr;
  int ws_batch = 0;
  BgWs w;
};

namespace qlx {
namespace bg {

static void model_workspace(qlx_bg_model* m, int B) {
  if (B <= m->ws_batch) return;
  QLX_HIP(hipStreamSynchronize(m->stream));
  if (m->ws) (void)hipFree(m->ws);
  m->ws = nullptr;
  size_t off = 0;
  auto take = [&](size_t bytes) { const size_t o = off; off = (off + bytes + 255) / 256 * 256; return o; };
  const size_t o_obs = take((size_t)B * kObs), o_a1 = take((size_t)B * 288 * 4), o_a2 = take((size_t)B * 288 * 4);
  const size_t o_a3 = take((size_t)B * 512 * 4), o_q = take((size_t)B * kA * 4), o_dq = take((size_t)B * kA * 4);
  const size_t o_hs = take((size_t)B * 4), o_dz3 = take((size_t)B * 512 * 4), o_dz2 = take((size_t)B * 288 * 4);
  const size_t o_dz1 = take((size_t)B * 288 * 4), o_y = take((size_t)B * 4), o_rew = take((size_t)B * 4), o_loss = take(64);
  const size_t o_act = take((size_t)B), o_am = take((size_t)B), o_done = take((size_t)B);
  QLX_HIP(hipMalloc(&m->ws, off));
  char* base = (char*)m->ws;
  BgWs& w = m->w;
  w.obs = (uint8_t*)(base + o_obs);
  w.a1 = (float*)(base + o_a1); w.a2 = (float*)(base + o_a2); w.a3 = (float*)(base + o_a3);
  w.q = (float*)(base + o_q); w.dq = (float*)(base + o_dq); w.hs = (float*)(base + o_hs);
  w.dz3 = (float*)(base + o_dz3); w.dz2 = (float*)(base + o_dz2); w.dz1 = (float*)(base + o_dz1);
  w.y = (float*)(base + o_y); w.rew = (float*)(base + o_rew); w.loss = (float*)(base + o_loss);
  w.act = (uint8_t*)(base + o_act); w.argmax = (uint8_t*)(base + o_am); w.done = (uint8_t*)(base + o_done);
  m->ws_batch = B;
}

// conv1 + conv2 + dense 512 (activations a1, a2, a3 in the workspace)
static void forward(qlx_bg_model* m, const uint8_t* d_obs, int B, hipStream_t s) {
  BgWs& w = m->w;
  hipLaunchKernelGGL(k_conv_fwd, dim3(B), dim3(288), 0, s, d_obs, B, m->d_params, w.a1, w.a2);
  QLX_HIP(hipGetLastError());
  gemm<false, false, 1>(s, B, 512, 288, w.a2, 288, m->d_params + var_off(4), 512, w.a3, 512, m->d_params + var_off(5));
}

static HeadArgs head_args(qlx_bg_model* m, int B) {
  HeadArgs h{};
  h.a3 = m->w.a3;
  h.prm = m->d_params;
  h.B = B;
  h.q = m->w.q;
  return h;
}

template <int MODE>
static void head(const HeadArgs& h, hipStream_t s) {
  hipLaunchKernelGGL(k_head<MODE>, dim3((h.B + 3) / 4), dim3(256), 0, s, h);
  QLX_HIP(hipGetLastError());
}

// MSE head + backward after forward() on the same batch: loss -> *loss_dev, raw gradients -> m->d_grads
static void backward(qlx_bg_model* m, const uint8_t* d_obs, int B, const uint8_t* d_act, const float* d_y, float* loss_dev,
                     hipStream_t s, const float* weights = nullptr, float* td_abs = nullptr) {
  BgWs& w = m->w;
  float* G = m->d_grads;
  const float* P = m->d_params;
  HeadArgs h = head_args(m, B);
  h.actions = d_act;
  h.y = d_y;
  h.dq = w.dq;
  h.hs = w.hs;
  h.dz3 = w.dz3;
  h.weights = weights;
  h.td_abs = td_abs;
  head<3>(h, s);
  colsum(s, w.hs, B, 1, 1, loss_dev, 1.0f / (float)B);                          // MSE mean
  gemm<true, false, 0>(s, 512, kA, B, w.a3, 512, w.dq, kA, G + var_off(6), kA);  // dW3 = a3^T dq
  colsum(s, w.dq, B, kA, kA, G + var_off(7));                                   // db3
  gemm<true, false, 0>(s, 288, 512, B, w.a2, 288, w.dz3, 512, G + var_off(4), 512);   // dW2 = flat(a2)^T dz3
  colsum(s, w.dz3, B, 512, 512, G + var_off(5));                                      // db2
  gemm<false, true, 2>(s, B, 288, 512, w.dz3, 512, P + var_off(4), 512, w.dz2, 288, w.a2);   // dz2 = dz3 W2^T * (a2 > 0)
  gemm<true, false, 0>(s, 32, 32, B * 9, w.a1, 32, w.dz2, 32, G + var_off(2), 32);         // dK1 = a1^T dz2
  colsum(s, w.dz2, B * 9, 32, 32, G + var_off(3));                                        // db1
  gemm<false, true, 2>(s, B * 9, 32, 32, w.dz2, 32, P + var_off(2), 32, w.dz1, 32, w.a1);  // dz1 = dz2 K1^T * (a1 > 0)
  hipLaunchKernelGGL(k_conv1_wgrad, dim3(16), dim3(256), 0, s, d_obs, w.dz1, B, G + var_off(0));
  QLX_HIP(hipGetLastError());
  colsum(s, w.dz1, B * 9, 32, 32, G + var_off(1));                                        // db0
}

static void apply_adam(qlx_bg_model* m, hipStream_t s) {
  hipLaunchKernelGGL(k_norms, dim3(kVars), dim3(256), 0, s, m->d_grads, m->d_norms);
  const int64_t t = m->iterations + 1;
  const float b1p = std::pow(m->beta1, (float)t), b2p = std::pow(m->beta2, (float)t);
  const float alpha = m->lr * std::sqrt(1.0f - b2p) / (1.0f - b1p);
  hipLaunchKernelGGL(k_adam, dim3(256), dim3(256), 0, s, m->d_params, m->d_m, m->d_v, m->d_grads, m->d_norms, alpha, m->beta1,
                     m->beta2, m->eps, m->clipnorm);
  QLX_HIP(hipGetLastError());
  m->iterations = t;
}

static void glorot_host(std::vector<float>& params, uint64_t seed) {   // keras GlorotUniform / zeros
  const int fan_in[4] = {2 * 2 * 4, 32, 288, 512};
  const int fan_out[4] = {2 * 2 * 32, 32, 512, 5};
  params.assign(kParams, 0.0f);
  for (int v = 0; v < kVars; v += 2) {
    const float limit = std::sqrt(6.0f / (float)(fan_in[v / 2] + fan_out[v / 2]));
    RngStream s(seed, (uint32_t)v, 1, P_INIT);
    for (int i = 0; i < kVarSize[v]; ++i) params[var_off(v) + i] = uniform_f32(s, -limit, limit);
  }
}

// obs staged from the host ([n][3][3][4] u8)
static const uint8_t* stage_obs(qlx_bg_model* m, const uint8_t* obs_host, int n) {
  model_workspace(m, n);
  QLX_HIP(hipMemcpyAsync(m->w.obs, obs_host, (size_t)n * kObs, hipMemcpyHostToDevice, m->stream));
  return m->w.obs;
}

}  // namespace bg
}  // namespace qlx

// ---------------- learner ----------------

struct qlx_bg_learner {
  qlx_params p{};
  int device = 0;
  hipStream_t stream = nullptr;
  qlx_bg_env* env = nullptr;
  qlx_bg_model* online = nullptr;
  qlx_bg_model* target = nullptr;
  uint32_t N = 0, B = 0, max_updates = 0;
  uint64_t cap = 0, total = 0;
  // replay columns (replay_buffer.rs: one FIFO position for all)
  qlx_ballgame_state *d_rs = nullptr, *d_rsn = nullptr;
  uint8_t *d_ra = nullptr, *d_rd = nullptr;
  float* d_rr = nullptr;
  // per vector step
  uint8_t *d_obs = nullptr, *d_actions = nullptr, *d_dones = nullptr, *d_reset = nullptr;
  float *d_rewards = nullptr, *d_q = nullptr;
  double* d_eps = nullptr;
  uint64_t eps_len = 0;
  float *d_ep_reward = nullptr, *d_hist = nullptr;
  Book* d_book = nullptr;
  uint64_t* d_idx = nullptr;
  uint8_t *d_xs = nullptr, *d_xn = nullptr, *d_bact = nullptr, *d_bdone = nullptr;
  float *d_brew = nullptr, *d_targets = nullptr, *d_losses = nullptr;
  float* d_qsel = nullptr;   // double DQN: online Q(s') of the step's batches [U*B][5]
  bool ddqn = false, per = false;
  qlx::PerState prio;
  uint64_t step_count = 0, vec_steps = 0, update_count = 0;
  uint32_t last_updates = 0;
};

namespace qlx {
namespace bg {

// s, s', a, r, done of each env's step into the FIFO at total + e (ReplayBuffer::add)
__global__ void k_step_push(qlx_ballgame_state* st, uint32_t* ep_steps, uint32_t n, const uint8_t* actions, float* rewards,
                            uint8_t* dones, qlx_ballgame_state* rs, qlx_ballgame_state* rsn, uint8_t* ra, float* rr, uint8_t* rd,
                            uint64_t total, uint64_t cap) {
  const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  qlx_ballgame_state v = st[e];
  const uint64_t t = (total + e) % cap;
  rs[t] = v;
  env_step(v, actions[e], &rewards[e], &dones[e]);
  st[e] = v;
  ep_steps[e] += 1;
  rsn[t] = v;
  ra[t] = actions[e];
  rr[t] = rewards[e];
  rd[t] = dones[e];
}

// ReplayBuffer::get_many for logical indices (0 = oldest) -> one-hot s / s' and metadata
__global__ void k_gather(const qlx_ballgame_state* rs, const qlx_ballgame_state* rsn, const uint8_t* ra, const float* rr,
                         const uint8_t* rd, uint64_t total, uint64_t len, uint64_t cap, const uint64_t* idx, uint32_t n,
                         uint8_t* xs, uint8_t* xn, uint8_t* act, float* rew, uint8_t* done) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t t = (total - len + idx[i]) % cap;
  obs_of(rs[t], xs + (size_t)i * kObs);
  obs_of(rsn[t], xn + (size_t)i * kObs);
  act[i] = ra[t];
  rew[i] = rr[t];
  done[i] = rd[t];
}

static void learner_vector_step(qlx_bg_learner* L) {
  hipStream_t s = L->stream;
  const uint32_t N = L->N, B = L->B;
  const uint64_t step_before = L->step_count;
  qlx_bg_env* env = L->env;
  if (step_before + N >= L->p.epsilon_pure_random_steps) {   // acting forward with the weights at the step start
    hipLaunchKernelGGL(k_env_obs, dim3((N + 255) / 256), dim3(256), 0, s, env->d_state, N, L->d_obs);
    forward(L->online, L->d_obs, (int)N, s);
    HeadArgs h = head_args(L->online, (int)N);
    h.q = L->d_q;
    head<0>(h, s);
  }
  launch_select_actions(s, N, kA, step_before, L->p.epsilon_pure_random_steps, L->d_eps, L->eps_len, L->p.epsilon_min,
                        L->p.learner_seed, env->id_offset, (uint32_t)L->vec_steps, L->d_q, L->d_actions);
  L->step_count += N;
  hipLaunchKernelGGL(k_step_push, dim3((N + 255) / 256), dim3(256), 0, s, env->d_state, env->d_ep_steps, N, L->d_actions,
                     L->d_rewards, L->d_dones, L->d_rs, L->d_rsn, L->d_ra, L->d_rr, L->d_rd, L->total, L->cap);
  if (L->per) per_launch_push(s, L->prio.leaves(), L->cap, L->total, N, L->prio.d_max);
  L->total += N;
  launch_episode_book(s, N, L->d_rewards, L->d_dones, env->d_ep_steps, L->p.max_steps_per_episode, L->d_ep_reward, L->d_hist,
                      (uint32_t)L->p.episode_reward_history_buffer_len, L->d_book, L->d_reset);
  hipLaunchKernelGGL(k_env_init, dim3((N + 255) / 256), dim3(256), 0, s, env->d_state, env->d_ep_steps, N, env->seed,
                     env->id_offset, L->d_reset, 1);
  const uint64_t ua = L->p.update_after_actions;
  const uint64_t triggers = L->step_count / ua - step_before / ua;
  const uint64_t len = std::min(L->total, L->cap);
  L->last_updates = 0;
  if (len > B && triggers > 0) {
    const uint32_t U = (uint32_t)triggers;
    QLX_CHECK(U <= L->max_updates, QLX_E_STATE, "too many updates per vector step");
    const uint64_t start = (L->total - len) % L->cap;
    if (L->per) {
      per_launch_build(s, L->prio.d_tree, L->prio.L);
      per_launch_sample(s, L->prio.d_tree, L->prio.L, L->p.learner_seed, (uint32_t)L->update_count, U, L->p.rank, len,
                        L->p.per_beta, B, L->cap, start, L->d_idx, L->prio.d_w);
    } else {
      launch_sample_distinct(s, L->p.learner_seed, (uint32_t)L->update_count, U, L->p.rank, len, B, L->d_idx);
    }
    const uint32_t n = U * B;
    hipLaunchKernelGGL(k_gather, dim3((n + 255) / 256), dim3(256), 0, s, L->d_rs, L->d_rsn, L->d_ra, L->d_rr, L->d_rd, L->total, len,
                       L->cap, L->d_idx, n, L->d_xs, L->d_xn, L->d_bact, L->d_brew, L->d_bdone);
    // targets of all U updates from the fixed target weights (a sync happens only between vector steps); double
    // DQN picks a* with the online weights as they stand before this step's updates
    if (L->ddqn) {
      forward(L->online, L->d_xn, (int)n, s);
      HeadArgs o = head_args(L->online, (int)n);
      o.q = L->d_qsel;
      head<0>(o, s);
    }
    forward(L->target, L->d_xn, (int)n, s);
    HeadArgs t = head_args(L->target, (int)n);
    t.q_select = L->ddqn ? L->d_qsel : nullptr;
    t.rewards = L->d_brew;
    t.dones = L->d_bdone;
    t.gamma = L->p.gamma;
    t.y_out = L->d_targets;
    head<2>(t, s);
    for (uint32_t u = 0; u < U; ++u) {
      const uint8_t* xs = L->d_xs + (size_t)u * B * kObs;
      forward(L->online, xs, (int)B, s);
      backward(L->online, xs, (int)B, L->d_bact + (size_t)u * B, L->d_targets + (size_t)u * B, L->d_losses + u, s,
               L->per ? L->prio.d_w + (size_t)u * B : nullptr, L->per ? L->prio.d_td + (size_t)u * B : nullptr);
      apply_adam(L->online, s);
      L->update_count += 1;
    }
    if (L->per)
      per_launch_update(s, L->d_idx, L->prio.d_td, n, L->cap, start, L->p.per_alpha, L->p.per_eps, L->prio.d_owner,
                        L->prio.leaves(), L->prio.d_max);
    L->last_updates = U;
  }
  const uint64_t ts = L->p.target_sync_steps;
  if (ts > 0 && L->step_count / ts != step_before / ts)
    QLX_HIP(hipMemcpyAsync(L->target->d_params, L->online->d_params, kParams * 4, hipMemcpyDeviceToDevice, s));
  L->vec_steps += 1;
  QLX_HIP(hipGetLastError());
}

}  // namespace bg
}  // namespace qlx

using namespace qlx::bg;

extern "C" {

// ---------------- environment ----------------

int32_t qlx_bg_env_create(uint32_t n_envs, uint64_t seed, int32_t device, qlx_bg_env** out) {
  return guard([&] {
    QLX_CHECK(n_envs > 0 && out, QLX_E_INVALID, "n_envs must be > 0");
    current_device_checked(device);
    auto* e = new qlx_bg_env;
    try {   // a failure part-way releases what was built
      e->device = device;
      e->n = n_envs;
      e->seed = seed;
      QLX_HIP(hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking));
      QLX_HIP(hipMalloc(&e->d_state, (size_t)n_envs * sizeof(qlx_ballgame_state)));
      QLX_HIP(hipMalloc(&e->d_ep_steps, (size_t)n_envs * 4));
      QLX_HIP(hipMalloc(&e->d_bad, 4));
      QLX_HIP(hipMalloc(&e->d_tmp_u8, n_envs));
      QLX_HIP(hipMalloc(&e->d_tmp_u8b, n_envs));
      QLX_HIP(hipMalloc(&e->d_tmp_f32, (size_t)n_envs * 4));
      QLX_HIP(hipMemsetAsync(e->d_bad, 0, 4, e->stream));
      hipLaunchKernelGGL(k_env_init, dim3((n_envs + 255) / 256), dim3(256), 0, e->stream, e->d_state, e->d_ep_steps, n_envs, seed,
                         0u, (const uint8_t*)nullptr, 0);
      QLX_HIP(hipGetLastError());
      QLX_HIP(hipStreamSynchronize(e->stream));
    } catch (...) {
      qlx_bg_env_destroy(e);
      throw;
    }
    *out = e;
  });
}

int32_t qlx_bg_env_destroy(qlx_bg_env* e) {
  return guard([&] {
    if (!e) return;
    (void)hipSetDevice(e->device);
    (void)hipStreamSynchronize(e->stream);
    void* ptrs[] = {e->d_state, e->d_ep_steps, e->d_bad, e->d_tmp_u8, e->d_tmp_u8b, e->d_tmp_f32};
    for (void* p : ptrs) (void)hipFree(p);
    if (e->own_stream) (void)hipStreamDestroy(e->stream);
    delete e;
  });
}

int32_t qlx_bg_env_reset(qlx_bg_env* e, const uint8_t* mask) {
  return guard([&] {
    QLX_CHECK(e, QLX_E_INVALID, "null env");
    QLX_HIP(hipSetDevice(e->device));
    const uint8_t* dm = nullptr;
    if (mask) {
      QLX_HIP(hipMemcpyAsync(e->d_tmp_u8, mask, e->n, hipMemcpyHostToDevice, e->stream));
      dm = e->d_tmp_u8;
    }
    hipLaunchKernelGGL(k_env_init, dim3((e->n + 255) / 256), dim3(256), 0, e->stream, e->d_state, e->d_ep_steps, e->n, e->seed,
                       e->id_offset, dm, 1);
    QLX_HIP(hipGetLastError());
    QLX_HIP(hipStreamSynchronize(e->stream));
  });
}

int32_t qlx_bg_env_step(qlx_bg_env* e, const uint8_t* actions, float* rewards, uint8_t* dones) {
  return guard([&] {
    QLX_CHECK(e && actions && rewards && dones, QLX_E_INVALID, "null argument");
    QLX_HIP(hipSetDevice(e->device));
    QLX_HIP(hipMemcpyAsync(e->d_tmp_u8, actions, e->n, hipMemcpyHostToDevice, e->stream));
    hipLaunchKernelGGL(k_env_step, dim3((e->n + 255) / 256), dim3(256), 0, e->stream, e->d_state, e->d_ep_steps, e->n,
                       e->d_tmp_u8, e->d_tmp_f32, e->d_tmp_u8b, e->d_bad);
    QLX_HIP(hipGetLastError());
    uint32_t bad = 0;
    QLX_HIP(hipMemcpyAsync(&bad, e->d_bad, 4, hipMemcpyDeviceToHost, e->stream));
    QLX_HIP(hipMemcpyAsync(rewards, e->d_tmp_f32, (size_t)e->n * 4, hipMemcpyDeviceToHost, e->stream));
    QLX_HIP(hipMemcpyAsync(dones, e->d_tmp_u8b, e->n, hipMemcpyDeviceToHost, e->stream));
    QLX_HIP(hipStreamSynchronize(e->stream));
    if (bad) {
      QLX_HIP(hipMemsetAsync(e->d_bad, 0, 4, e->stream));
      QLX_HIP(hipStreamSynchronize(e->stream));
      throw Error{QLX_E_INVALID, "action out of range (ACTION_SPACE = 5)"};
    }
  });
}

int32_t qlx_bg_env_obs(qlx_bg_env* e, uint8_t* out) {
  return guard([&] {
    QLX_CHECK(e && out, QLX_E_INVALID, "null argument");
    QLX_HIP(hipSetDevice(e->device));
    uint8_t* d = nullptr;
    QLX_HIP(hipMalloc(&d, (size_t)e->n * kObs));
    hipLaunchKernelGGL(k_env_obs, dim3((e->n + 255) / 256), dim3(256), 0, e->stream, e->d_state, e->n, d);
    QLX_HIP(hipMemcpyAsync(out, d, (size_t)e->n * kObs, hipMemcpyDeviceToHost, e->stream));
    QLX_HIP(hipStreamSynchronize(e->stream));
    QLX_HIP(hipFree(d));
  });
}

int32_t qlx_bg_env_states(qlx_bg_env* e, qlx_ballgame_state* out) {
  return guard([&] {
    QLX_CHECK(e && out, QLX_E_INVALID, "null argument");
    QLX_HIP(hipSetDevice(e->device));
    QLX_HIP(hipMemcpyAsync(out, e->d_state, (size_t)e->n * sizeof(qlx_ballgame_state), hipMemcpyDeviceToHost, e->stream));
    QLX_HIP(hipStreamSynchronize(e->stream));
  });
}

int32_t qlx_bg_env_set_states(qlx_bg_env* e, const qlx_ballgame_state* in) {
  return guard([&] {
    QLX_CHECK(e && in, QLX_E_INVALID, "null argument");
    QLX_HIP(hipSetDevice(e->device));
    QLX_HIP(hipMemcpyAsync(e->d_state, in, (size_t)e->n * sizeof(qlx_ballgame_state), hipMemcpyHostToDevice, e->stream));
    QLX_HIP(hipMemsetAsync(e->d_ep_steps, 0, (size_t)e->n * 4, e->stream));
    QLX_HIP(hipStreamSynchronize(e->stream));
  });
}

// ---------------- model ----------------

int32_t qlx_bg_model_hparams(float* out) {
  return guard([&] {
    QLX_CHECK(out, QLX_E_INVALID, "null out");
    const qlx_bg_model m;   // the defaults every created model starts from (no device state is touched)
    out[0] = m.lr; out[1] = m.beta1; out[2] = m.beta2; out[3] = m.eps; out[4] = m.clipnorm;
  });
}

int32_t qlx_bg_model_create(uint64_t seed, int32_t device, qlx_bg_model** out) {
  return guard([&] {
    QLX_CHECK(out, QLX_E_INVALID, "null argument");
    current_device_checked(device);
    auto* m = new qlx_bg_model;
    try {   // a failure part-way releases what was built
      m->device = device;
      QLX_HIP(hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking));
      const size_t pb = kParams * 4;
      QLX_HIP(hipMalloc(&m->d_params, pb));
      QLX_HIP(hipMalloc(&m->d_m, pb));
      QLX_HIP(hipMalloc(&m->d_v, pb));
      QLX_HIP(hipMalloc(&m->d_grads, pb));
      QLX_HIP(hipMalloc(&m->d_norms, kVars * 4));
      std::vector<float> params;
      glorot_host(params, seed);
      QLX_HIP(hipMemcpy(m->d_params, params.data(), pb, hipMemcpyHostToDevice));
      QLX_HIP(hipMemset(m->d_m, 0, pb));
      QLX_HIP(hipMemset(m->d_v, 0, pb));
      QLX_HIP(hipMemset(m->d_grads, 0, pb));
    } catch (...) {
      qlx_bg_model_destroy(m);
      throw;
    }
    *out = m;
  });
}

int32_t qlx_bg_model_destroy(qlx_bg_model* m) {
  return guard([&] {
    if (!m) return;
    (void)hipSetDevice(m->device);
    (void)hipStreamSynchronize(m->stream);
    void* ptrs[] = {m->d_params, m->d_m, m->d_v, m->d_grads, m->d_norms, m->ws};
    for (void* p : ptrs) (void)hipFree(p);
    if (m->own_stream) (void)hipStreamDestroy(m->stream);
    delete m;
  });
}

int64_t qlx_bg_model_var_size(int32_t v) { return (v >= 0 && v < kVars) ? kVarSize[v] : -1; }

int32_t qlx_bg_model_get_var(qlx_bg_model* m, int32_t var, int32_t which, float* out) {
  return guard([&] {
    QLX_CHECK(m && out && var >= 0 && var < kVars && which >= 0 && which <= 2, QLX_E_INVALID, "bad argument");
    QLX_HIP(hipSetDevice(m->device));
    QLX_HIP(hipStreamSynchronize(m->stream));
    const float* src = (which == 0 ? m->d_params : which == 1 ? m->d_m : m->d_v) + var_off(var);
    QLX_HIP(hipMemcpy(out, src, kVarSize[var] * 4, hipMemcpyDeviceToHost));
  });
}

int32_t qlx_bg_model_set_var(qlx_bg_model* m, int32_t var, int32_t which, const float* in) {
  return guard([&] {
    QLX_CHECK(m && in && var >= 0 && var < kVars && which >= 0 && which <= 2, QLX_E_INVALID, "bad argument");
    QLX_HIP(hipSetDevice(m->device));
    QLX_HIP(hipStreamSynchronize(m->stream));
    float* dst = (which == 0 ? m->d_params : which == 1 ? m->d_m : m->d_v) + var_off(var);
    QLX_HIP(hipMemcpy(dst, in, kVarSize[var] * 4, hipMemcpyHostToDevice));
  });
}

int64_t qlx_bg_model_iterations(qlx_bg_model* m) { return m ? m->iterations : -1; }

int32_t qlx_bg_model_load_tf(qlx_bg_model* m, const char* prefix) {
  return guard([&] {
    QLX_CHECK(m && prefix, QLX_E_INVALID, "null argument");
    std::vector<float> w, mm, vv;
    int64_t it = 0;
    load_keras_bundle(prefix, 4, kVarSize, w, mm, vv, &it);
    QLX_HIP(hipSetDevice(m->device));
    QLX_HIP(hipStreamSynchronize(m->stream));
    QLX_HIP(hipMemcpy(m->d_params, w.data(), kParams * 4, hipMemcpyHostToDevice));
    QLX_HIP(hipMemcpy(m->d_m, mm.data(), kParams * 4, hipMemcpyHostToDevice));
    QLX_HIP(hipMemcpy(m->d_v, vv.data(), kParams * 4, hipMemcpyHostToDevice));
    m->iterations = it;
  });
}

int32_t qlx_bg_model_predict(qlx_bg_model* m, const uint8_t* obs, uint32_t n, float* q_out, uint8_t* actions) {
  return guard([&] {
    QLX_CHECK(m && obs && n > 0, QLX_E_INVALID, "bad argument");
    QLX_HIP(hipSetDevice(m->device));
    const uint8_t* d = stage_obs(m, obs, (int)n);
    forward(m, d, (int)n, m->stream);
    HeadArgs h = head_args(m, (int)n);
    h.argmax = m->w.argmax;
    head<1>(h, m->stream);
    if (q_out) QLX_HIP(hipMemcpyAsync(q_out, m->w.q, (size_t)n * kA * 4, hipMemcpyDeviceToHost, m->stream));
    if (actions) QLX_HIP(hipMemcpyAsync(actions, m->w.argmax, n, hipMemcpyDeviceToHost, m->stream));
    QLX_HIP(hipStreamSynchronize(m->stream));
  });
}

int32_t qlx_bg_model_batch_max_q(qlx_bg_model* m, const uint8_t* obs, uint32_t n, float* out) {
  return guard([&] {
    QLX_CHECK(m && obs && out && n > 0, QLX_E_INVALID, "bad argument");
    QLX_HIP(hipSetDevice(m->device));
    const uint8_t* d = stage_obs(m, obs, (int)n);
    forward(m, d, (int)n, m->stream);
    QLX_HIP(hipMemsetAsync(m->w.rew, 0, (size_t)n * 4, m->stream));
    QLX_HIP(hipMemsetAsync(m->w.done, 0, n, m->stream));
    HeadArgs h = head_args(m, (int)n);
    h.rewards = m->w.rew;
    h.dones = m->w.done;
    h.gamma = 1.0f;
    h.y_out = m->w.y;
    head<2>(h, m->stream);
    QLX_HIP(hipMemcpyAsync(out, m->w.y, (size_t)n * 4, hipMemcpyDeviceToHost, m->stream));
    QLX_HIP(hipStreamSynchronize(m->stream));
  });
}

int32_t qlx_bg_model_train(qlx_bg_model* m, const uint8_t* obs, const uint8_t* actions, const float* y, uint32_t B,
                           float* loss_out, float* grads_out, float* norms_out) {
  return guard([&] {
    QLX_CHECK(m && obs && actions && y && B > 0, QLX_E_INVALID, "bad argument");
    for (uint32_t b = 0; b < B; ++b) QLX_CHECK(actions[b] < kA, QLX_E_INVALID, "action out of range");
    QLX_HIP(hipSetDevice(m->device));
    hipStream_t s = m->stream;
    const uint8_t* d = stage_obs(m, obs, (int)B);
    QLX_HIP(hipMemcpyAsync(m->w.act, actions, B, hipMemcpyHostToDevice, s));
    QLX_HIP(hipMemcpyAsync(m->w.y, y, (size_t)B * 4, hipMemcpyHostToDevice, s));
    forward(m, d, (int)B, s);
    backward(m, d, (int)B, m->w.act, m->w.y, m->w.loss, s);
    if (grads_out) QLX_HIP(hipMemcpyAsync(grads_out, m->d_grads, kParams * 4, hipMemcpyDeviceToHost, s));
    apply_adam(m, s);
    if (norms_out) QLX_HIP(hipMemcpyAsync(norms_out, m->d_norms, kVars * 4, hipMemcpyDeviceToHost, s));
    if (loss_out) QLX_HIP(hipMemcpyAsync(loss_out, m->w.loss, 4, hipMemcpyDeviceToHost, s));
    QLX_HIP(hipStreamSynchronize(s));
  });
}

// ---------------- learner ----------------

int32_t qlx_bg_learner_create(const qlx_params* p, int32_t device, qlx_bg_learner** out) {
  return guard([&] {
    QLX_CHECK(p && out, QLX_E_INVALID, "null argument");
    QLX_CHECK(p->n_envs > 0 && p->batch_size > 0 && p->batch_size <= 4096, QLX_E_INVALID, "bad n_envs / batch_size");
    QLX_CHECK(p->update_after_actions > 0 && p->history_buffer_len >= p->batch_size, QLX_E_INVALID, "bad parameters");
    QLX_CHECK(p->episode_reward_history_buffer_len > 0, QLX_E_INVALID, "episode_reward_history_buffer_len must be > 0");
    QLX_CHECK((p->flags & ~(QLX_LEARNER_DOUBLE_DQN | QLX_LEARNER_PER)) == 0, QLX_E_INVALID, "unknown learner flags");
    QLX_CHECK(!(p->flags & QLX_LEARNER_PER) || (p->per_alpha >= 0.0f && p->per_beta >= 0.0f && p->per_eps > 0.0f),
              QLX_E_INVALID, "prioritized replay needs alpha >= 0, beta >= 0, eps > 0");
    current_device_checked(device);
    auto* L = new qlx_bg_learner;
    try {   // a failure part-way releases what was built
      L->ddqn = (p->flags & QLX_LEARNER_DOUBLE_DQN) != 0;
      L->per = (p->flags & QLX_LEARNER_PER) != 0;
      L->p = *p;
      L->device = device;
      L->N = p->n_envs;
      L->B = p->batch_size;
      L->cap = p->history_buffer_len;
      QLX_HIP(hipStreamCreateWithFlags(&L->stream, hipStreamNonBlocking));
      int32_t st = qlx_bg_env_create(L->N, p->env_seed, device, &L->env);
      QLX_CHECK(st == QLX_OK, st, qlx_last_error());
      st = qlx_bg_model_create(p->init_seed, device, &L->online);
      QLX_CHECK(st == QLX_OK, st, qlx_last_error());
      st = qlx_bg_model_create(p->init_seed, device, &L->target);   // same initial weights (:107-108)
      QLX_CHECK(st == QLX_OK, st, qlx_last_error());
      L->env->stream = L->stream; L->env->own_stream = false;
      L->online->stream = L->stream; L->online->own_stream = false;
      L->target->stream = L->stream; L->target->own_stream = false;
      if (p->rank != 0) {   // data-parallel ranks own env ids rank * N + e
        L->env->id_offset = p->rank * L->N;
        hipLaunchKernelGGL(k_env_init, dim3((L->N + 255) / 256), dim3(256), 0, L->stream, L->env->d_state, L->env->d_ep_steps, L->N,
                           L->env->seed, L->env->id_offset, (const uint8_t*)nullptr, 0);
      }
      const std::vector<double> eps = epsilon_table(*p);
      L->eps_len = eps.size();
      QLX_HIP(hipMalloc(&L->d_eps, eps.size() * 8));
      QLX_HIP(hipMemcpy(L->d_eps, eps.data(), eps.size() * 8, hipMemcpyHostToDevice));
      const uint32_t N = L->N, B = L->B;
      L->max_updates = (uint32_t)(N / p->update_after_actions + 2);
      const size_t UB = (size_t)L->max_updates * B;
      QLX_HIP(hipMalloc(&L->d_rs, L->cap * sizeof(qlx_ballgame_state)));
      QLX_HIP(hipMalloc(&L->d_rsn, L->cap * sizeof(qlx_ballgame_state)));
      QLX_HIP(hipMalloc(&L->d_ra, L->cap));
      QLX_HIP(hipMalloc(&L->d_rd, L->cap));
      QLX_HIP(hipMalloc(&L->d_rr, L->cap * 4));
      QLX_HIP(hipMalloc(&L->d_obs, (size_t)N * kObs));
      QLX_HIP(hipMalloc(&L->d_actions, N));
      QLX_HIP(hipMalloc(&L->d_dones, N));
      QLX_HIP(hipMalloc(&L->d_reset, N));
      QLX_HIP(hipMalloc(&L->d_rewards, (size_t)N * 4));
      QLX_HIP(hipMalloc(&L->d_q, (size_t)N * kA * 4));
      QLX_HIP(hipMalloc(&L->d_ep_reward, (size_t)N * 4));
      QLX_HIP(hipMalloc(&L->d_hist, p->episode_reward_history_buffer_len * 4));
      QLX_HIP(hipMalloc(&L->d_book, sizeof(Book)));
      QLX_HIP(hipMalloc(&L->d_idx, UB * 8));
      QLX_HIP(hipMalloc(&L->d_xs, UB * kObs));
      QLX_HIP(hipMalloc(&L->d_xn, UB * kObs));
      QLX_HIP(hipMalloc(&L->d_bact, UB));
      QLX_HIP(hipMalloc(&L->d_bdone, UB));
      QLX_HIP(hipMalloc(&L->d_brew, UB * 4));
      QLX_HIP(hipMalloc(&L->d_targets, UB * 4));
      QLX_HIP(hipMalloc(&L->d_losses, L->max_updates * 4));
      QLX_HIP(hipMemsetAsync(L->d_ep_reward, 0, (size_t)N * 4, L->stream));
      QLX_HIP(hipMemsetAsync(L->d_book, 0, sizeof(Book), L->stream));
      QLX_HIP(hipMemsetAsync(L->d_q, 0, (size_t)N * kA * 4, L->stream));
      model_workspace(L->online, (int)std::max(N, B));
      model_workspace(L->target, (int)UB);
      if (L->ddqn) {
        model_workspace(L->online, (int)UB);
        QLX_HIP(hipMalloc(&L->d_qsel, UB * kA * 4));
      }
      if (L->per) L->prio.init(L->cap, UB);
      QLX_HIP(hipStreamSynchronize(L->stream));
    } catch (...) {
      qlx_bg_learner_destroy(L);
      throw;
    }
    *out = L;
  });
}

int32_t qlx_bg_learner_destroy(qlx_bg_learner* L) {
  return guard([&] {
    if (!L) return;
    (void)hipSetDevice(L->device);
    (void)hipStreamSynchronize(L->stream);
    qlx_bg_env_destroy(L->env);
    qlx_bg_model_destroy(L->online);
    qlx_bg_model_destroy(L->target);
    void* ptrs[] = {L->d_rs, L->d_rsn, L->d_ra, L->d_rd, L->d_rr, L->d_obs, L->d_actions, L->d_dones, L->d_reset, L->d_rewards,
                    L->d_q, L->d_eps, L->d_ep_reward, L->d_hist, L->d_book, L->d_idx, L->d_xs, L->d_xn, L->d_bact, L->d_bdone,
                    L->d_brew, L->d_targets, L->d_losses, L->d_qsel};
    for (void* p : ptrs) (void)hipFree(p);
    L->prio.release();
    (void)hipStreamDestroy(L->stream);
    delete L;
  });
}

int32_t qlx_bg_learner_run(qlx_bg_learner* L, uint64_t n) {
  return guard([&] {
    QLX_CHECK(L, QLX_E_INVALID, "null learner");
    QLX_HIP(hipSetDevice(L->device));
    for (uint64_t i = 0; i < n; ++i) learner_vector_step(L);
  });
}

int32_t qlx_bg_learner_sync(qlx_bg_learner* L) {
  return guard([&] {
    QLX_CHECK(L, QLX_E_INVALID, "null learner");
    QLX_HIP(hipStreamSynchronize(L->stream));
  });
}

int32_t qlx_bg_learner_stats_get(qlx_bg_learner* L, qlx_learner_stats* out) {
  return guard([&] {
    QLX_CHECK(L && out, QLX_E_INVALID, "null argument");
    QLX_HIP(hipStreamSynchronize(L->stream));
    Book b;
    QLX_HIP(hipMemcpy(&b, L->d_book, sizeof(Book), hipMemcpyDeviceToHost));
    std::vector<float> ring(L->p.episode_reward_history_buffer_len);
    QLX_HIP(hipMemcpy(ring.data(), L->d_hist, ring.size() * 4, hipMemcpyDeviceToHost));
    out->step_count = L->step_count;
    out->vec_steps = L->vec_steps;
    out->update_count = L->update_count;
    out->episode_count = b.episode_count;
    out->replay_len = std::min(L->total, L->cap);
    double e = L->p.epsilon_min;
    if (L->step_count < L->eps_len) QLX_HIP(hipMemcpy(&e, L->d_eps + L->step_count, 8, hipMemcpyDeviceToHost));
    out->epsilon = e;
    float running = 0.0f;
    uint64_t solved = 0;
    learner_book_stats(b, ring.data(), (uint32_t)ring.size(), 9.5f, L->p.lowest_episode_reward_goal_threshold_pct, &running, &solved);
    out->running_reward = running;
    out->solved = solved;
    float loss = 0.0f;
    if (L->last_updates) QLX_HIP(hipMemcpy(&loss, L->d_losses + L->last_updates - 1, 4, hipMemcpyDeviceToHost));
    out->last_loss = loss;
  });
}

static std::vector<float> bg_episode_rewards(qlx_bg_learner* L) {
  QLX_HIP(hipStreamSynchronize(L->stream));
  Book b;
  QLX_HIP(hipMemcpy(&b, L->d_book, sizeof(Book), hipMemcpyDeviceToHost));
  std::vector<float> ring(L->p.episode_reward_history_buffer_len), out(b.hist_len);
  QLX_HIP(hipMemcpy(ring.data(), L->d_hist, ring.size() * 4, hipMemcpyDeviceToHost));
  for (uint32_t i = 0; i < b.hist_len; ++i) out[i] = ring[(b.hist_head + i) % ring.size()];
  return out;
}

int32_t qlx_bg_learner_action_counts(qlx_bg_learner* L, uint64_t* counts) {
  return guard([&] {
    QLX_CHECK(L && counts, QLX_E_INVALID, "null argument");
    std::vector<uint64_t> c;
    action_counts(L->stream, L->d_ra, std::min(L->total, L->cap), bg::kA, c);
    std::copy(c.begin(), c.end(), counts);
  });
}

int32_t qlx_bg_learner_episode_rewards(qlx_bg_learner* L, float* out, uint64_t cap, uint64_t* n) {
  return guard([&] {
    QLX_CHECK(L, QLX_E_INVALID, "null learner");
    const std::vector<float> r = bg_episode_rewards(L);
    if (n) *n = r.size();
    if (out) std::copy(r.begin(), r.begin() + std::min<uint64_t>(cap, r.size()), out);
  });
}

int32_t qlx_bg_learner_update_log(qlx_bg_learner* L, char* buf, size_t cap, size_t* len) {
  return guard([&] {
    QLX_CHECK(L, QLX_E_INVALID, "null learner");
    // BallGameAction Display (ballgame_test_environment.rs:222-234) by numeric value West 0 .. Nothing 4
    static const char* const kNames[bg::kA] = {"\xE2\x86\x90", "\xE2\x86\x91", "\xE2\x86\x92", "\xE2\x86\x93", "o"};
    qlx_learner_stats st;
    int32_t rc = qlx_bg_learner_stats_get(L, &st);
    QLX_CHECK(rc == QLX_OK, rc, qlx_last_error());
    LogInputs in{st.episode_count, st.step_count, L->p.gamma, st.epsilon, 9.5f, L->p.lowest_episode_reward_goal_threshold_pct,
                 bg_episode_rewards(L), {}, kNames};
    action_counts(L->stream, L->d_ra, std::min(L->total, L->cap), bg::kA, in.counts);
    copy_text(learning_log(in), buf, cap, len);
  });
}

int32_t qlx_bg_learner_priorities(qlx_bg_learner* L, float* is_weights, float* leaves, float* per_max) {
  return guard([&] {
    QLX_CHECK(L && L->per, QLX_E_STATE, "learner was created without QLX_LEARNER_PER");
    QLX_HIP(hipStreamSynchronize(L->stream));
    const uint32_t U = L->last_updates;
    if (U && is_weights) QLX_HIP(hipMemcpy(is_weights, L->prio.d_w, (size_t)U * L->B * 4, hipMemcpyDeviceToHost));
    if (leaves) QLX_HIP(hipMemcpy(leaves, L->prio.leaves(), L->prio.cap * 4, hipMemcpyDeviceToHost));
    if (per_max) QLX_HIP(hipMemcpy(per_max, L->prio.d_max, 4, hipMemcpyDeviceToHost));
  });
}

int32_t qlx_bg_learner_last(qlx_bg_learner* L, uint8_t* actions, float* rewards, uint8_t* dones, float* losses,
                            uint64_t* indices, float* targets, uint32_t* n_updates) {
  return guard([&] {
    QLX_CHECK(L, QLX_E_INVALID, "null learner");
    QLX_HIP(hipStreamSynchronize(L->stream));
    const uint32_t U = L->last_updates;
    if (actions) QLX_HIP(hipMemcpy(actions, L->d_actions, L->N, hipMemcpyDeviceToHost));
    if (rewards) QLX_HIP(hipMemcpy(rewards, L->d_rewards, (size_t)L->N * 4, hipMemcpyDeviceToHost));
    if (dones) QLX_HIP(hipMemcpy(dones, L->d_dones, L->N, hipMemcpyDeviceToHost));
    if (U && losses) QLX_HIP(hipMemcpy(losses, L->d_losses, (size_t)U * 4, hipMemcpyDeviceToHost));
    if (U && indices) QLX_HIP(hipMemcpy(indices, L->d_idx, (size_t)U * L->B * 8, hipMemcpyDeviceToHost));
    if (U && targets) QLX_HIP(hipMemcpy(targets, L->d_targets, (size_t)U * L->B * 4, hipMemcpyDeviceToHost));
    if (n_updates) *n_updates = U;
  });
}

qlx_bg_env* qlx_bg_learner_env(qlx_bg_learner* L) { return L ? L->env : nullptr; }
qlx_bg_model* qlx_bg_learner_model(qlx_bg_learner* L, int32_t which) { return L ? (which == 0 ? L->online : L->target) : nullptr; }

}  // extern "C"
