// Kernel micro-benchmark harness (development tool, not part of the product): builds the Q-net kernels
// from source, times individual launches and experimental variants with HIP events on one stream.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I q-learning_amd/csrc scripts/ubench.hip -o scripts/ubench
//   ./scripts/ubench
#include "../q-learning_amd/csrc/common.cpp"
#include "../q-learning_amd/csrc/qnet.hip"
#include "../q-learning_amd/csrc/tf_bundle.cpp"

#include <cstdio>
#include <functional>
#include <random>

using namespace qlx;
using namespace qlx::qn;

template <bool AK, bool BK, int S, int OCC, bool REMAP, class Epi, int DBG = 0>
__global__ __launch_bounds__(256, OCC) void k_gemm_v(GemmProblem<Epi> P) {
  const int t = REMAP ? xcd_tile(blockIdx.x, gridDim.x) : blockIdx.x;
  if (t < P.tiles()) gemm_tile<AK, BK, S, Epi, DBG>(P, t);
}
template <bool AK1, bool BK1, class E1, bool AK2, bool BK2, class E2, int S, int OCC, bool REMAP>
__global__ __launch_bounds__(256, OCC) void k_gemm_pair_v(GemmProblem<E1> P1, GemmProblem<E2> P2) {
  const int t = REMAP ? xcd_tile(blockIdx.x, gridDim.x) : blockIdx.x;
  if (t < P1.tiles()) gemm_tile<AK1, BK1, S>(P1, t);
  else if (t < P1.tiles() + P2.tiles()) gemm_tile<AK2, BK2, S>(P2, t - P1.tiles());
}

// the pre-vectorisation Adam (scalar per element) for comparison
__global__ __launch_bounds__(256) void k_adam_scalar(AdamArgs A) {
  __shared__ int64_t offs[kNumVars + 1];
  __shared__ float nrm[kNumVars];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (threadIdx.x == 0) {
    int64_t o = 0;
    for (int i = 0; i < kNumVars; ++i) { offs[i] = o; o += kVarSize[i]; }
    offs[kNumVars] = o;
  }
  for (int v = wave; v < kNumVars; v += 4) {
    float t = 0.0f;
    for (int r = A.var_first[v] + lane; r < A.var_first[v + 1]; r += 64) t += A.partial[r];
    for (int off = 32; off > 0; off >>= 1) t += __shfl_xor(t, off);
    if (lane == 0) nrm[v] = t > 0.0f ? sqrtf(t) : t;
  }
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < A.count; i += (int64_t)gridDim.x * blockDim.x) {
    int var = 0;
    while (i >= offs[var + 1]) ++var;
    const float denom = fmaxf(nrm[var], A.clipnorm);
    const float gc = (A.g[i] * A.scale * A.clipnorm) / denom;
    float m = A.m[i], v = A.v[i], w = A.w[i];
    m += (gc - m) * (1.0f - A.beta1);
    v += (gc * gc - v) * (1.0f - A.beta2);
    w -= (m * A.alpha) / (sqrtf(v) + A.eps);
    A.m[i] = m;
    A.v[i] = v;
    A.w[i] = w;
    pack_one(A.pack, i, w);
  }
}

// 4 independent elements per thread per grid-stride step (more loads in flight per wave)
__global__ __launch_bounds__(256) void k_adam_ilp4(AdamArgs A) {
  __shared__ int64_t offs[kNumVars + 1];
  __shared__ float nrm[kNumVars];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (threadIdx.x == 0) {
    int64_t o = 0;
    for (int i = 0; i < kNumVars; ++i) { offs[i] = o; o += kVarSize[i]; }
    offs[kNumVars] = o;
  }
  for (int v = wave; v < kNumVars; v += 4) {
    float t = 0.0f;
    for (int r = A.var_first[v] + lane; r < A.var_first[v + 1]; r += 64) t += A.partial[r];
    for (int off = 32; off > 0; off >>= 1) t += __shfl_xor(t, off);
    if (lane == 0) nrm[v] = t > 0.0f ? sqrtf(t) : t;
  }
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i0 < A.count; i0 += 4 * stride) {
    float g[4], m[4], v[4], w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t i = i0 + k * stride;
      if (i < A.count) { g[k] = A.g[i]; m[k] = A.m[i]; v[k] = A.v[i]; w[k] = A.w[i]; }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t i = i0 + k * stride;
      if (i < A.count) {
        int var = 0;
        while (i >= offs[var + 1]) ++var;
        const float denom = fmaxf(nrm[var], A.clipnorm);
        const float nw = adam_elem(g[k], A.scale, A.clipnorm, denom, A.alpha, A.beta1, A.beta2, A.eps, m[k], v[k], w[k]);
        A.m[i] = m[k];
        A.v[i] = v[k];
        A.w[i] = nw;
        pack_one(A.pack, i, nw);
      }
    }
  }
}

static hipStream_t g_s;
static double time_us(const std::function<void()>& f, int iters = 50) {
  for (int i = 0; i < 5; ++i) f();
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  (void)hipEventRecord(a, g_s);
  for (int i = 0; i < iters; ++i) f();
  (void)hipEventRecord(b, g_s);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  (void)hipGetLastError();
  return ms * 1000.0 / iters;
}

static void fill_bf16(bf16* d, size_t n, float scale, uint32_t seed) {
  std::vector<__bf16> h(n);
  std::mt19937 r(seed);
  std::uniform_real_distribution<float> u(-scale, scale);
  for (auto& x : h) x = (__bf16)u(r);
  QLX_HIP(hipMemcpy(d, h.data(), n * 2, hipMemcpyHostToDevice));
}
static void fill_f32(float* d, size_t n, float scale, uint32_t seed) {
  std::vector<float> h(n);
  std::mt19937 r(seed);
  std::uniform_real_distribution<float> u(-scale, scale);
  for (auto& x : h) x = u(r);
  QLX_HIP(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice));
}

int main(int argc, char** argv) {
  qlx_model* m = nullptr;
  if (qlx_model_create(QLX_ARCH_NATURE_DQN, 2, 0, &m) != 0) { printf("create failed: %s\n", qlx_last_error()); return 1; }
  g_s = m->stream;
  const int BT = 8192;
  model_workspace(m, BT);
  ModelWs& w = m->w;
  fill_bf16(w.a3, (size_t)BT * 3136, 1.0f, 1);
  fill_bf16(w.dz4, (size_t)BT * 512, 0.01f, 2);
  fill_f32(m->d_grads, kNumParams, 0.01f, 3);
  QLX_HIP(hipStreamSynchronize(g_s));
  float* G = m->d_grads;
  const float* p = m->d_params;
  auto report = [](const char* name, double us, double work, const char* unit) {
    printf("%-48s %9.2f us  %8.1f %s\n", name, us, work / us / 1e6, unit);
  };
  // ---- Adam
  model_norms(m, g_s, 1.0f);
  report("k_sumsq", time_us([&] { model_norms(m, g_s, 1.0f); }), 4.0 * kNumParams * 1e-3 * 1e3, "GB/s");
  AdamArgs a;
  {
    const int64_t t = 1;
    const float b1p = std::pow(m->beta1, (float)t), b2p = std::pow(m->beta2, (float)t);
    a.w = m->d_params; a.m = m->d_m; a.v = m->d_v; a.g = m->d_grads; a.norms = m->d_norms;
    a.partial = m->d_partial; a.var_first = m->d_var_first;
    a.count = kNumParams; a.scale = 1.0f;
    a.alpha = m->lr * std::sqrt(1.0f - b2p) / (1.0f - b1p);
    a.beta1 = m->beta1; a.beta2 = m->beta2; a.eps = m->eps; a.clipnorm = m->clipnorm;
    a.pack = pack_ptrs(m);
  }
  const double adam_bytes = 30.0 * kNumParams;   // 4 reads + 3 writes fp32 + the bf16 copy
  const bool only_gemm = argc > 1 && std::string(argv[1]) == "gemm";
  const bool only_adam = argc > 1 && std::string(argv[1]) == "adam";
  for (int grid : {256, 512, 1024, 2048, 4096}) {
    if (only_gemm) break;
    char nm[64];
    snprintf(nm, sizeof nm, "k_adam grid %d", grid);
    report(nm, time_us([&] { hipLaunchKernelGGL(k_adam, dim3(grid), dim3(256), 0, g_s, a); }), adam_bytes, "GB/s");
    snprintf(nm, sizeof nm, "k_adam_ilp4 grid %d", grid);
    report(nm, time_us([&] { hipLaunchKernelGGL(k_adam_ilp4, dim3(grid), dim3(256), 0, g_s, a); }), adam_bytes, "GB/s");
  }
  if (only_adam) {
    qlx_model_destroy(m);
    return 0;
  }
  // ---- per-sample conv kernels: time vs batch (intercept = per-launch ramp, slope = per-sample cost)
  if (argc > 1 && std::string(argv[1]) == "trunk") {
    set_lds_attr(k_trunk_fwd<true>, kTrunkFwdLds);
    set_lds_attr(k_trunk_fwd<false>, kTrunkFwdLds);
    set_lds_attr(k_trunk_bwd_data<false>, kTrunkBwdLds);
    set_lds_attr(k_trunk_bwd_data<true>, kTrunkBwdLds);
    set_lds_attr(k_conv1_wgrad, kConv1WgradLds);
    // frames: random u8 s2d frames for BT samples
    {
      std::vector<uint8_t> h((size_t)BT * 4 * kFramePix);
      std::mt19937 r(5);
      for (auto& x : h) x = (uint8_t)(r() & 255);
      QLX_HIP(hipMemcpy(w.frames, h.data(), h.size(), hipMemcpyHostToDevice));
      hipLaunchKernelGGL(k_frame_table, dim3((BT * 4 + 255) / 256), dim3(256), 0, g_s, w.frames, BT, w.table);
    }
    fill_bf16(w.dz3, (size_t)BT * 3136, 0.01f, 6);
    {   // per-phase cycles of the forward (wave 0 of each block), B = 8192 (32 samples per block)
      unsigned long long* dt = nullptr;
      QLX_HIP(hipMalloc(&dt, 256 * 4 * 8));
      set_lds_attr(k_trunk_fwd<false, true>, kTrunkFwdLds);
      set_lds_attr(k_trunk_fwd<true, true>, kTrunkFwdLds);
      set_lds_attr(k_trunk_fwd<false, true>, kTrunkFwdLds);
      set_lds_attr(k_trunk_fwd<true, true>, kTrunkFwdLds);
      for (int st = 0; st < 2; ++st) {
        auto k = st ? k_trunk_fwd<true, true> : k_trunk_fwd<false, true>;
        hipLaunchKernelGGL(k, dim3(256), dim3(kTrunkThreads), kTrunkFwdLds, g_s, w.table, BT, m->wf0, m->wf1, m->wf2, p + var_offset(1),
                           p + var_offset(3), p + var_offset(5), w.a1, w.a2, w.a3, dt);
        std::vector<unsigned long long> h(256 * 4);
        QLX_HIP(hipMemcpy(h.data(), dt, h.size() * 8, hipMemcpyDeviceToHost));
        double acc[4] = {0, 0, 0, 0};
        for (int b = 0; b < 256; ++b)
          for (int i = 0; i < 4; ++i) acc[i] += (double)h[b * 4 + i] / 256.0 / 32.0;
        QLX_HIP(hipDeviceSynchronize());
        printf("trunk_fwd<%s> cycles per sample: stage %.0f conv1 %.0f conv2 %.0f conv3 %.0f total %.0f\n", st ? "store" : "nostore",
               acc[0], acc[1], acc[2], acc[3], acc[0] + acc[1] + acc[2] + acc[3]);
      }
    }
    {
      unsigned long long* dt = nullptr;
      QLX_HIP(hipMalloc(&dt, 256 * 4 * 8));
      QLX_HIP(hipMemset(dt, 0, 256 * 4 * 8));
      hipLaunchKernelGGL(k_trunk_bwd_data<true>, dim3(256), dim3(kTrunkThreads), kTrunkBwdLds, g_s, w.dz3, w.a2, w.a1, BT, m->wb2,
                         m->wb1, w.dz2, w.dz1, dt);
      QLX_HIP(hipDeviceSynchronize());
      std::vector<unsigned long long> h(256 * 4);
      QLX_HIP(hipMemcpy(h.data(), dt, h.size() * 8, hipMemcpyDeviceToHost));
      double acc[4] = {0, 0, 0, 0};
      for (int b = 0; b < 256; ++b)
        for (int i = 0; i < 4; ++i) acc[i] += (double)h[b * 4 + i] / 256.0 / 32.0;
      printf("trunk_bwd_data cycles per sample: stage+dz1out %.0f dz2 %.0f dz2out+dz1 %.0f total %.0f\n", acc[0], acc[1], acc[2],
             acc[0] + acc[1] + acc[2]);
    }
    for (int B : {256, 512, 1024, 2048, 4096, 8192}) {
      const double fwd_fl = 2.0 * B * (400.0 * 32 * 256 + 81.0 * 64 * 512 + 49.0 * 64 * 576);
      const int grid = std::min(B, 256);
      char nm[96];
      snprintf(nm, sizeof nm, "trunk_fwd<store> B=%d", B);
      report(nm, time_us([&] {
        hipLaunchKernelGGL(k_trunk_fwd<true>, dim3(grid), dim3(kTrunkThreads), kTrunkFwdLds, g_s, w.table, B, m->wf0, m->wf1, m->wf2,
                           p + var_offset(1), p + var_offset(3), p + var_offset(5), w.a1, w.a2, w.a3, nullptr);
      }), fwd_fl, "TF/s");
      snprintf(nm, sizeof nm, "trunk_fwd<nostore> B=%d", B);
      report(nm, time_us([&] {
        hipLaunchKernelGGL(k_trunk_fwd<false>, dim3(grid), dim3(kTrunkThreads), kTrunkFwdLds, g_s, w.table, B, m->wf0, m->wf1, m->wf2,
                           p + var_offset(1), p + var_offset(3), p + var_offset(5), w.a1, w.a2, w.a3, nullptr);
      }), fwd_fl, "TF/s");
      snprintf(nm, sizeof nm, "trunk_bwd_data B=%d", B);
      report(nm, time_us([&] {
        hipLaunchKernelGGL(k_trunk_bwd_data<false>, dim3(grid), dim3(kTrunkThreads), kTrunkBwdLds, g_s, w.dz3, w.a2, w.a1, B, m->wb2,
                           m->wb1, w.dz2, w.dz1, nullptr);
      }), 2.0 * B * (49.0 * 64 * 576 + 81.0 * 64 * 512), "TF/s");
      snprintf(nm, sizeof nm, "conv1_wgrad B=%d", B);
      report(nm, time_us([&] {
        hipLaunchKernelGGL(k_conv1_wgrad, dim3(grid), dim3(kTrunkThreads), kConv1WgradLds, g_s, w.table, w.dz1, B, w.slab + kSlabConv1);
      }), 2.0 * B * 400 * 256 * 32, "TF/s");
    }
    qlx_model_destroy(m);
    return 0;
  }
  // ---- fc1 GEMMs: variants (register stages S, occupancy, XCD remap)
#define VARIANTS(X) X(2, 2, false, 0) X(2, 2, true, 0) X(2, 2, true, 1) X(2, 2, true, 2) X(3, 2, true, 0) X(3, 2, true, 1) X(2, 1, true, 0) X(3, 1, true, 0) X(3, 1, true, 1)
  for (int B : {1024, 8192}) {
    const double fl = 2.0 * B * 512 * 3136;
    char nm[128];
    for (int nf = 0; nf < 2; ++nf) {
      const auto Pw = gemm_problem(false, w.a3, 3136, w.dz4, 512, 3137, 512, B, 1, Epi4StoreF32{G + var_offset(6), 512, nullptr}, 3136, nf == 1);
      const auto Pd = gemm_problem(true, w.dz4, 512, m->wb3, 512, B, 3136, 512, 1, Epi4ReluMask{w.dz3, w.a3, 3136});
#define RUNW(S, O, R, D)                                                                                                     \
  {                                                                                                                       \
    auto k = k_gemm_v<true, true, S, O, R, Epi4StoreF32, D>;                                                                 \
    set_lds_attr(k, GemmCfg::LDS);                                                                                        \
    const int g = R ? xcd_grid(Pw.tiles()) : Pw.tiles();                                                                  \
    snprintf(nm, sizeof nm, "wgrad B=%d nf=%d S=%d occ=%d remap=%d dbg=%d", B, nf, S, O, (int)R, D);                                \
    report(nm, time_us([&] { hipLaunchKernelGGL(k, dim3(g), dim3(256), GemmCfg::LDS, g_s, Pw); }), fl, "TF/s");          \
  }
      VARIANTS(RUNW)
      if (nf == 0) {
#define RUND(S, O, R, D)                                                                                                     \
  {                                                                                                                       \
    auto k = k_gemm_v<false, false, S, O, R, Epi4ReluMask, D>;                                                               \
    set_lds_attr(k, GemmCfg::LDS);                                                                                        \
    const int g = R ? xcd_grid(Pd.tiles()) : Pd.tiles();                                                                  \
    snprintf(nm, sizeof nm, "dgrad B=%d S=%d occ=%d remap=%d dbg=%d", B, S, O, (int)R, D);                                          \
    report(nm, time_us([&] { hipLaunchKernelGGL(k, dim3(g), dim3(256), GemmCfg::LDS, g_s, Pd); }), fl, "TF/s");          \
  }
        VARIANTS(RUND)
      }
#define RUNP(S, O, R, D)                                                                                                     \
  {                                                                                                                       \
    auto k = k_gemm_pair_v<true, true, Epi4StoreF32, false, false, Epi4ReluMask, S, O, R>;                                \
    set_lds_attr(k, GemmCfg::LDS);                                                                                        \
    const int g = R ? xcd_grid(Pw.tiles() + Pd.tiles()) : Pw.tiles() + Pd.tiles();                                        \
    snprintf(nm, sizeof nm, "pair B=%d nf=%d S=%d occ=%d remap=%d", B, nf, S, O, (int)R);                                 \
    report(nm, time_us([&] { hipLaunchKernelGGL(k, dim3(g), dim3(256), GemmCfg::LDS, g_s, Pw, Pd); }), 2 * fl, "TF/s");  \
  }
    }
    if (B == 1024) {   // fc1 backward pair: dW3 as one K pass (16 k-steps per tile) vs split-K 2 into a slab (8 + 8)
      float* slab2 = nullptr;
      QLX_HIP(hipMalloc(&slab2, (size_t)2 * 3137 * 512 * 4));
      const auto Pd = gemm_problem(true, w.dz4, 512, m->wb3, 512, B, 3136, 512, 1, Epi4ReluMask{w.dz3, w.a3, 3136});
      const auto Pw1 = gemm_problem(false, w.a3, 3136, w.dz4, 512, 3137, 512, B, 1, Epi4StoreF32{G + var_offset(6), 512, nullptr}, 3136);
      const auto Pw2 = gemm_problem(false, w.a3, 3136, w.dz4, 512, 3137, 512, B, 2, Epi4Slab{slab2, 512, (size_t)3137 * 512}, 3136);
      auto k1 = k_gemm_pair_v<true, true, Epi4StoreF32, false, false, Epi4ReluMask, 2, 2, false>;
      auto k2 = k_gemm_pair_v<true, true, Epi4Slab, false, false, Epi4ReluMask, 2, 2, false>;
      set_lds_attr(k1, GemmCfg::LDS);
      set_lds_attr(k2, GemmCfg::LDS);
      report("pair dW3 split=1 (dW3 tiles first)", time_us([&] { hipLaunchKernelGGL(k1, dim3(Pw1.tiles() + Pd.tiles()), dim3(256), GemmCfg::LDS, g_s, Pw1, Pd); }), 2 * fl, "TF/s");
      report("pair dW3 split=2 (dW3 tiles first)", time_us([&] { hipLaunchKernelGGL(k2, dim3(Pw2.tiles() + Pd.tiles()), dim3(256), GemmCfg::LDS, g_s, Pw2, Pd); }), 2 * fl, "TF/s");
      QLX_HIP(hipFree(slab2));
    }
    for (int splits : {1, 7}) {
      if (B == 8192 && splits == 7) continue;
      if (B == 1024 && splits == 1) continue;
      const auto Pf = gemm_problem(true, w.a3, 3136, m->wb3, 512, B, 512, 3136, splits, Epi4Slab{w.fc1slab, 512, (size_t)B * 512});
#define RUNF(S, O, R, D)                                                                                                     \
  {                                                                                                                       \
    auto k = k_gemm_v<false, true, S, O, R, Epi4Slab, D>;                                                                    \
    set_lds_attr(k, GemmCfg::LDS);                                                                                        \
    const int g = R ? xcd_grid(Pf.tiles()) : Pf.tiles();                                                                  \
    snprintf(nm, sizeof nm, "fwd B=%d split=%d S=%d occ=%d remap=%d dbg=%d", B, splits, S, O, (int)R, D);                           \
    report(nm, time_us([&] { hipLaunchKernelGGL(k, dim3(g), dim3(256), GemmCfg::LDS, g_s, Pf); }), fl, "TF/s");          \
  }
      VARIANTS(RUNF)
    }
  }
  qlx_model_destroy(m);
  return 0;
}
