// Micro-benchmark + correctness check of the bf16 GEMM core (q-learning_amd/csrc/bgemm.h) on the fc1 shapes of the bf16
// path: forward at the training batch (B = 1024, split-K 7 into fp32 slabs) and at a chunk batch (8,192, bias + ReLU
// epilogue), backward data (dz4 W3^T with the ReLU mask of a3) and the weight gradient (a3^T dz4 with the ones row:
// dW3 + db3, fp32, with the clip-norm tile partials).  Every output is compared against a naive fp32 GPU GEMM of the same
// bf16 operands (different summation order: relative tolerance 2e-3 of the output's max |value|).  Rates against the
// 2.5 PFLOP/s dense bf16 MFMA peak.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I q-learning_amd/csrc -I include scripts/ubench_bgemm.hip -o scripts/ubench_bgemm
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "bgemm.h"

using namespace qlx::qn;

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

// reference: C[m][n] = sum_k A(m,k) B(n,k) in fp32 (one thread per output)
__global__ void k_ref(const bf16* A, int lda, bool ak, const bf16* B, int ldb, bool bk, int M, int N, int K, float* C) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)M * N) return;
  const int m = (int)(i / N), n = (int)(i % N);
  float s = 0.0f;
  for (int k = 0; k < K; ++k) {
    const float a = (float)(ak ? A[(size_t)k * lda + m] : A[(size_t)m * lda + k]);
    const float b = (float)(bk ? B[(size_t)k * ldb + n] : B[(size_t)n * ldb + k]);
    s += a * b;
  }
  C[i] = s;
}

// reference conv weight gradient: dW[(kh KS + kw) C + c][n] = sum_b,oh,ow in[b][oh S + kh][ow S + kw][c] dz[b][oh][ow][n]
__global__ void k_ref_conv(const bf16* in, const bf16* dz, int B, int IH, int IW, int C, int KS, int S, int OH, int OW, float* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x, M = KS * KS * C;
  if (i >= M * 64) return;
  const int m = i / 64, n = i % 64, tap = m / C, c = m % C, kh = tap / KS, kw = tap % KS;
  float s = 0.0f;
  for (int b = 0; b < B; ++b)
    for (int oh = 0; oh < OH; ++oh)
      for (int ow = 0; ow < OW; ++ow)
        s += (float)in[(((size_t)b * IH + oh * S + kh) * IW + ow * S + kw) * C + c] * (float)dz[(((size_t)b * OH + oh) * OW + ow) * 64 + n];
  out[i] = s;
}

__global__ void k_fill(bf16* p, int64_t n, uint32_t seed, float lo, float hi, float zero_frac) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
    const float u = (float)(h >> 8) * (1.0f / 16777216.0f);
    uint32_t h2 = h * 747796405u + 2891336453u;
    const float z = (float)(h2 >> 8) * (1.0f / 16777216.0f);
    p[i] = (bf16)(z < zero_frac ? 0.0f : lo + (hi - lo) * u);
  }
}

// a3 with pitch ld: columns >= 3136 are 1 at 3136, 0 after
__global__ void k_ones_col(bf16* a3, int B, int ld) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  for (int c = 3136; c < ld; ++c) a3[(size_t)b * ld + c] = (bf16)(c == 3136 ? 1.0f : 0.0f);
}

static double check(const std::vector<float>& got, const std::vector<float>& ref, const char* what, double tol) {
  double mx = 0.0, err = 0.0;
  for (size_t i = 0; i < ref.size(); ++i) mx = std::max(mx, (double)std::fabs(ref[i]));
  size_t worst = 0;
  for (size_t i = 0; i < ref.size(); ++i) {
    const double e = std::fabs((double)got[i] - (double)ref[i]);
    if (!(e <= err)) { err = e; worst = i; }
  }
  const double rel = err / std::max(mx, 1e-30);
  std::printf("  %-28s max|ref| %.4g  max err %.3g (rel %.2e at %zu: got %.6g ref %.6g) %s\n", what, mx, err, rel, worst,
              got[worst], ref[worst], rel <= tol ? "OK" : "FAIL");
  if (!(rel <= tol)) std::exit(2);
  return rel;
}

// per-launch time with the caches emptied first: a hipMemsetAsync of `flush` bytes before every launch (128 MB: the L2s, the
// operands then come from the Infinity Cache as they do in place after their producers; 1 GB: the Infinity Cache too)
static char* g_flush = nullptr;
template <class F>
static float time_cold_us(F f, size_t flush, int iters = 20) {
  if (!g_flush) CK(hipMalloc(&g_flush, (size_t)1 << 30));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float tot = 0.0f;
  for (int i = 0; i < iters; ++i) {
    CK(hipMemsetAsync(g_flush, i & 0xff, flush));
    CK(hipEventRecord(a));
    f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0.0f;
    CK(hipEventElapsedTime(&ms, a, b));
    if (i > 1) tot += ms;
  }
  return tot * 1e3f / (iters - 2);
}

template <class F>
static float time_us(F f, int iters = 50) {
  for (int i = 0; i < 5; ++i) f();
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a));
  for (int i = 0; i < iters; ++i) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0.0f;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1e3f / iters;
}

template <class Epi>
static BGemmProblem<Epi> problem(BOp A, BOp B, int M, int N, int K, int splits, int bm, int bn, Epi e, int ones_m = -1) {
  const int kps = ((K + splits - 1) / splits + 31) / 32 * 32;
  return BGemmProblem<Epi>{A, B, M, N, K, kps, ones_m, (M + bm - 1) / bm, (N + bn - 1) / bn, (K + kps - 1) / kps, 0, e};
}

template <class C, class Epi>
static void launch(const BGemmProblem<Epi>& P, int remap) {
  const void* k = (const void*)k_bgemm<C, Epi>;
  CK(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)C::LDS));
  const int g = remap ? xcd_grid(P.tiles()) : P.tiles();
  hipLaunchKernelGGL((k_bgemm<C, Epi>), dim3(g), dim3(C::T), C::LDS, 0, P, remap);
  CK(hipGetLastError());
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? std::atoi(argv[1]) : 1024, BIG = 8192, LD3 = 3144;
  bf16 *a3, *a3big, *w3, *dz4;
  CK(hipMalloc(&a3, (size_t)B * LD3 * 2));
  CK(hipMalloc(&a3big, (size_t)BIG * LD3 * 2));
  CK(hipMalloc(&w3, (size_t)3136 * 512 * 2));
  CK(hipMalloc(&dz4, (size_t)B * 512 * 2));
  k_fill<<<1024, 256>>>(a3, (int64_t)B * LD3, 1, 0.0f, 4.0f, 0.5f);
  k_fill<<<1024, 256>>>(a3big, (int64_t)BIG * LD3, 2, 0.0f, 4.0f, 0.5f);
  k_fill<<<1024, 256>>>(w3, (int64_t)3136 * 512, 3, -0.04f, 0.04f, 0.0f);
  k_fill<<<1024, 256>>>(dz4, (int64_t)B * 512, 4, -1e-3f, 1e-3f, 0.3f);
  k_ones_col<<<(B + 255) / 256, 256>>>(a3, B, LD3);
  k_ones_col<<<(BIG + 255) / 256, 256>>>(a3big, BIG, LD3);
  float *ref, *slab, *g3, *sq;
  bf16 *a4, *dz3;
  CK(hipMalloc(&ref, (size_t)BIG * 3136 * 4));
  CK(hipMalloc(&slab, (size_t)8 * BIG * 512 * 4));
  CK(hipMalloc(&g3, (size_t)3137 * 512 * 4));
  CK(hipMalloc(&sq, 4096 * 4));
  CK(hipMalloc(&a4, (size_t)BIG * 512 * 2));
  CK(hipMalloc(&dz3, (size_t)B * 3136 * 2));
  std::vector<float> bias(512, 0.0f);
  float* d_bias;
  CK(hipMalloc(&d_bias, 512 * 4));
  CK(hipMemcpy(d_bias, bias.data(), 512 * 4, hipMemcpyHostToDevice));
  CK(hipDeviceSynchronize());
  auto get_f = [](const float* d, size_t n) { std::vector<float> h(n); CK(hipMemcpy(h.data(), d, n * 4, hipMemcpyDeviceToHost)); return h; };
  auto get_b = [](const bf16* d, size_t n) {
    std::vector<bf16> h(n);
    CK(hipMemcpy(h.data(), d, n * 2, hipMemcpyDeviceToHost));
    std::vector<float> f(n);
    for (size_t i = 0; i < n; ++i) f[i] = (float)h[i];
    return f;
  };
  std::vector<float> fwd_ref, big_ref, dg_ref, wg_ref;
  auto reference = [&](const bf16* A, int lda, bool ak, const bf16* Bm, int ldb, bool bk, int M, int N, int K) {
    hipLaunchKernelGGL(k_ref, dim3((unsigned)(((int64_t)M * N + 255) / 256)), dim3(256), 0, 0, A, lda, ak, Bm, ldb, bk, M, N, K, ref);
    CK(hipDeviceSynchronize());
    return get_f(ref, (size_t)M * N);
  };
  const double peak = 2500.0;
  const double fl = 2.0 * B * 512 * 3136;
  std::printf("bf16 GEMM core, B = %d (times: 50 back-to-back launches, warm caches)\n", B);
  auto fwd = [&](auto cfg, int splits, const char* name) {
    using C = decltype(cfg);
    auto P = problem(BOp{a3, LD3, B}, BOp{w3, 512, 512}, B, 512, 3136, splits, C::BM, C::BN, Epi4Slab{slab, 512, (size_t)B * 512});
    launch<C>(P, 1);
    CK(hipDeviceSynchronize());
    auto sl = get_f(slab, (size_t)P.splits * B * 512);
    std::vector<float> got((size_t)B * 512, 0.0f);
    for (int z = 0; z < P.splits; ++z)
      for (size_t i = 0; i < got.size(); ++i) got[i] += sl[(size_t)z * B * 512 + i];
    check(got, fwd_ref, name, 2e-3);
    const float us = time_us([&] { launch<C>(P, 1); });
    const float l2 = time_cold_us([&] { launch<C>(P, 1); }, (size_t)128 << 20), cold = time_cold_us([&] { launch<C>(P, 1); }, (size_t)1 << 30);
    std::printf("    %.2f us  %.1f TF  %.3f of peak (%d blocks, LDS %zu); L2 flushed %.2f us, all caches flushed %.2f us\n", us,
                fl / us * 1e-6, fl / us * 1e-6 / peak, P.tiles(), C::LDS, l2, cold);
  };
  auto fwd_big = [&](auto cfg, const char* name) {
    using C = decltype(cfg);
    auto P = problem(BOp{a3big, LD3, BIG}, BOp{w3, 512, 512}, BIG, 512, 3136, 1, C::BM, C::BN, Epi4BiasRelu{a4, d_bias, 512});
    launch<C>(P, 1);
    CK(hipDeviceSynchronize());
    check(get_b(a4, (size_t)BIG * 512), big_ref, name, 4.0e-3);   // bf16 outputs: one bf16 ulp of rounding-boundary moves
    const float us = time_us([&] { launch<C>(P, 1); }, 20);
    const double f = 2.0 * BIG * 512 * 3136;
    std::printf("    %.2f us  %.1f TF  %.3f of peak (%d blocks)\n", us, f / us * 1e-6, f / us * 1e-6 / peak, P.tiles());
  };
  auto dgrad = [&](auto cfg, const char* name) {
    using C = decltype(cfg);
    auto Q = problem(BOp{dz4, 512, B}, BOp{w3, 512, 3136}, B, 3136, 512, 1, C::BM, C::BN, Epi4Slab{slab, 3136, 0});
    launch<C>(Q, 0);
    CK(hipDeviceSynchronize());
    check(get_f(slab, (size_t)B * 3136), dg_ref, name, 2e-3);
    const float us = time_us([&] { launch<C>(Q, 0); });
    const float l2 = time_cold_us([&] { launch<C>(Q, 0); }, (size_t)128 << 20);
    std::printf("    %.2f us  %.1f TF  %.3f of peak (%d blocks); L2 flushed %.2f us\n", us, fl / us * 1e-6, fl / us * 1e-6 / peak, Q.tiles(), l2);
  };
  auto wgrad = [&](auto cfg, const char* name) {
    using C = decltype(cfg);
    auto P = problem(BOp{a3, LD3, 3137}, BOp{dz4, 512, 512}, 3137, 512, B, 1, C::BM, C::BN, Epi4StoreF32{g3, 512, sq}, 3136);
    launch<C>(P, 0);
    CK(hipDeviceSynchronize());
    check(get_f(g3, (size_t)3137 * 512), wg_ref, name, 2e-3);
    const float us = time_us([&] { launch<C>(P, 0); });
    const float l2 = time_cold_us([&] { launch<C>(P, 0); }, (size_t)128 << 20);
    std::printf("    %.2f us  %.1f TF  %.3f of peak (%d blocks); L2 flushed %.2f us\n", us, fl / us * 1e-6, fl / us * 1e-6 / peak, P.tiles(), l2);
  };
  fwd_ref = reference(a3, LD3, false, w3, 512, true, B, 512, 3136);
  big_ref = reference(a3big, LD3, false, w3, 512, true, BIG, 512, 3136);
  for (auto& v : big_ref) v = (float)(bf16)(v > 0.0f ? v : 0.0f);
  dg_ref = reference(dz4, 512, false, w3, 512, false, B, 3136, 512);
  wg_ref = reference(a3, LD3, true, dz4, 512, true, 3137, 512, B);
  auto fwd_dbg = [&](auto cfg, int splits, const char* name) {   // timing only (results not checked)
    using C = decltype(cfg);
    auto P = problem(BOp{a3, LD3, B}, BOp{w3, 512, 512}, B, 512, 3136, splits, C::BM, C::BN, Epi4Slab{slab, 512, (size_t)B * 512});
    const float us = time_us([&] { launch<C>(P, 1); });
    std::printf("  %-28s %.2f us\n", name, us);
  };
  auto big_dbg = [&](auto cfg, const char* name) {
    using C = decltype(cfg);
    auto P = problem(BOp{a3big, LD3, BIG}, BOp{w3, 512, 512}, BIG, 512, 3136, 1, C::BM, C::BN, Epi4BiasRelu{a4, d_bias, 512});
    const float us = time_us([&] { launch<C>(P, 1); }, 20);
    std::printf("  %-28s %.2f us\n", name, us);
  };
  if (argc > 2 && std::string(argv[2]) == "pmc") {   // the two kernels of the PMC passes (scripts/pmc_ubench.sh)
    fwd(BGemmCfg<128, 128, 2, 2, false, true, 4>{}, 7, "fwd 128x128 S4 split7");
    fwd_big(BGemmCfg<128, 128, 2, 2, false, true, 4>{}, "fwd8192 128x128 S4");
    return 0;
  }
  {  // conv weight gradients on the gathered (im2col) operand: conv3 (a2 x dz3) and conv2 (a1 x dz2)
    bf16 *a1, *a2, *dz2, *dz3;
    CK(hipMalloc(&a1, (size_t)B * 12800 * 2));
    CK(hipMalloc(&a2, (size_t)B * 5184 * 2));
    CK(hipMalloc(&dz2, (size_t)B * 5184 * 2));
    CK(hipMalloc(&dz3, (size_t)B * 3136 * 2));
    k_fill<<<1024, 256>>>(a1, (int64_t)B * 12800, 5, 0.0f, 2.0f, 0.5f);
    k_fill<<<1024, 256>>>(a2, (int64_t)B * 5184, 6, 0.0f, 2.0f, 0.5f);
    k_fill<<<1024, 256>>>(dz2, (int64_t)B * 5184, 7, -1e-3f, 1e-3f, 0.5f);
    k_fill<<<1024, 256>>>(dz3, (int64_t)B * 3136, 8, -1e-3f, 1e-3f, 0.3f);
    CK(hipDeviceSynchronize());
    auto conv = [&](auto cfg, const bf16* in, int inel, const bf16* dz, int P_, int M, int SC, int IH, int IW, int C_, int KS, int S_, int OH,
                    int OW, const char* name) {
      using C = decltype(cfg);
      const int K = B * P_, kps = SC * P_;
      BGemmProblem<Epi4Slab> Pr{BOp{in, inel, M}, BOp{dz, 64, 64}, M, 64, K, kps, -1, (M + C::BM - 1) / C::BM, 1,
                                (K + kps - 1) / kps, 0, Epi4Slab{slab, 64, (size_t)M * 64}};
      launch<C>(Pr, 0);
      CK(hipDeviceSynchronize());
      auto sl = get_f(slab, (size_t)Pr.splits * M * 64);
      std::vector<float> got((size_t)M * 64, 0.0f);
      for (int z = 0; z < Pr.splits; ++z)
        for (size_t i = 0; i < got.size(); ++i) got[i] += sl[(size_t)z * M * 64 + i];
      hipLaunchKernelGGL(k_ref_conv, dim3((M * 64 + 255) / 256), dim3(256), 0, 0, in, dz, B, IH, IW, C_, KS, S_, OH, OW, ref);
      CK(hipDeviceSynchronize());
      check(got, get_f(ref, (size_t)M * 64), name, 2e-3);
      const float us = time_us([&] { launch<C>(Pr, 0); });
      const float l2 = time_cold_us([&] { launch<C>(Pr, 0); }, (size_t)128 << 20);
      const double f = 2.0 * K * M * 64;
      std::printf("    %.2f us  %.1f TF  %.3f of peak (%d blocks, %d chunks); L2 flushed %.2f us\n", us, f / us * 1e-6,
                  f / us * 1e-6 / peak, Pr.tiles(), Pr.splits, l2);
    };
    using G3 = ConvGather<9, 9, 64, 3, 1, 7, 7>;
    using G2 = ConvGather<20, 20, 32, 4, 2, 9, 9>;
    conv(BGemmCfg<128, 64, 2, 2, true, true, 4, 0, G3>{}, a2, B * 5184, dz3, 49, 576, 20, 9, 9, 64, 3, 1, 7, 7, "conv3 wgrad SC20 S4");
    conv(BGemmCfg<128, 64, 2, 2, true, true, 6, 0, G3>{}, a2, B * 5184, dz3, 49, 576, 20, 9, 9, 64, 3, 1, 7, 7, "conv3 wgrad SC20 S6");
    conv(BGemmCfg<128, 64, 2, 2, true, true, 4, 0, G3>{}, a2, B * 5184, dz3, 49, 576, 40, 9, 9, 64, 3, 1, 7, 7, "conv3 wgrad SC40 S4");
    conv(BGemmCfg<128, 64, 2, 2, true, true, 4, 0, G2>{}, a1, B * 12800, dz2, 81, 512, 16, 20, 20, 32, 4, 2, 9, 9, "conv2 wgrad SC16 S4");
    conv(BGemmCfg<128, 64, 2, 2, true, true, 6, 0, G2>{}, a1, B * 12800, dz2, 81, 512, 16, 20, 20, 32, 4, 2, 9, 9, "conv2 wgrad SC16 S6");
    conv(BGemmCfg<128, 64, 2, 2, true, true, 4, 0, G2>{}, a1, B * 12800, dz2, 81, 512, 32, 20, 20, 32, 4, 2, 9, 9, "conv2 wgrad SC32 S4");
  }
  fwd(BGemmCfg<128, 64, 2, 2, false, true, 4>{}, 4, "fwd 128x64 S4 split4");
  fwd(BGemmCfg<128, 64, 2, 2, false, true, 6>{}, 4, "fwd 128x64 S6 split4");
  fwd(BGemmCfg<128, 64, 2, 2, false, true, 8>{}, 4, "fwd 128x64 S8 split4");
  fwd(BGemmCfg<128, 128, 2, 2, false, true, 4>{}, 7, "fwd 128x128 S4 split7");
  fwd(BGemmCfg<128, 128, 2, 2, false, true, 8>{}, 7, "fwd 128x128 S8 split7");
  fwd(BGemmCfg<128, 128, 2, 4, false, true, 6>{}, 7, "fwd 128x128 8w S6 split7");
  fwd(BGemmCfg<64, 64, 2, 2, false, true, 8>{}, 2, "fwd 64x64 S8 split2");
  dgrad(BGemmCfg<128, 128, 2, 4, false, false, 4>{}, "dgrad 128x128 8w S4");
  dgrad(BGemmCfg<128, 128, 2, 4, false, false, 6>{}, "dgrad 128x128 8w S6");
  dgrad(BGemmCfg<128, 64, 2, 2, false, false, 6>{}, "dgrad 128x64 S6");
  wgrad(BGemmCfg<128, 128, 2, 4, true, true, 4>{}, "wgrad 128x128 8w S4");
  wgrad(BGemmCfg<128, 128, 2, 4, true, true, 8>{}, "wgrad 128x128 8w S8");
  wgrad(BGemmCfg<128, 64, 2, 2, true, true, 8>{}, "wgrad 128x64 S8");
  std::printf("ok\n");
  return 0;
}
