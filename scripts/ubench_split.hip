// Split-bf16 MFMA GEMM micro-benchmark (development tool, not part of the product): is a bf16-split core a route to
// fp32-class Q-net arithmetic faster than v_mfma_f32_16x16x4_f32?  x = x0 + x1 (+ x2), each part bf16 (x0 = rn(x),
// x1 = rn(x - x0), x2 = rn(x - x0 - x1)); products accumulated in fp32 on v_mfma_f32_16x16x32_bf16:
//   x3: a0 b0 + a0 b1 + a1 b0                    (~16-bit operands: relative error ~2^-17 per product)
//   x6: x3 + a0 b2 + a1 b1 + a2 b0               (~24-bit operands: fp32-class)
// against the shipped fp32 core (gemm_body on v_mfma_f32_16x16x4_f32) on the fc1 forward shape (1024 x 512 x 3136) and a
// conv2-forward-sized GEMM (82,944 x 64 x 512, plain row-major A: the implicit-GEMM gather is left out on both sides).
// Error: max |C - C_f64| / max |C_f64| over 4,096 sampled outputs, activations ReLU-like (half zeros, [0, 4)), weights
// Glorot-like (+-0.04).  Operands are pre-split in HBM (a producer epilogue would write the parts).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I q-learning_amd/csrc scripts/ubench_split.hip -o scripts/ubench_split
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "qnet32_kernels.h"

using namespace qlx;
using namespace qlx::q32;

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e = (x);                                                                        \
    if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); }   \
  } while (0)

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16;

static u16 bf16_rn(float x) {   // round to nearest even
  uint32_t u;
  std::memcpy(&u, &x, 4);
  const uint32_t r = u + 0x7FFFu + ((u >> 16) & 1u);
  return (u16)(r >> 16);
}
static float bf16_f(u16 h) {
  const uint32_t u = (uint32_t)h << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

// C [M][N] = A [M][K] Bt[N][K]^T from NPART bf16 planes each; block BM x BN, 4 waves (2 x 2), wave tile (BM/2) x (BN/2)
// of 16 x 16 fragments; one 32-deep k step per LDS slab, double-buffered, the next slab's planes in registers.
template <int BM, int BN, int NPART, int NPROD, int KS = 1>
__global__ __launch_bounds__(256) void k_split(const u16* const* Ap, const u16* const* Bp, float* C, int M, int N, int K) {
  constexpr int PITCH = 32 * KS + 8;   // bf16 per LDS row (KS 32-deep k steps + 16 B: fragment reads spread over the banks)
  constexpr int TM = BM / 32, TN = BN / 32;
  constexpr int AC = BM * 4 * KS, BC = BN * 4 * KS;   // 16-byte chunks per plane per slab
  constexpr int NA = (AC + 255) / 256, NB = (BC + 255) / 256;
  constexpr int AF = BM * PITCH, BF = BN * PITCH;   // bf16 per plane image
  extern __shared__ __attribute__((aligned(16))) u16 sm[];
  u16* As = sm;                                  // [2][NPART][AF]
  u16* Bs = sm + 2 * NPART * AF;                 // [2][NPART][BF]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wm = wave & 1, wn = wave >> 1;
  const int tiles_n = N / BN, lb = xcd_logical(blockIdx.x, gridDim.x), tm = lb / tiles_n, tn = lb % tiles_n;
  const int row0 = tm * BM, col0 = tn * BN, ns = K / (32 * KS);
  uint4 ra[NPART][NA], rb[NPART][NB];
  auto load = [&](int s) {
#pragma unroll
    for (int p = 0; p < NPART; ++p) {
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int c = tid + 256 * i, r = c / (4 * KS), q = c % (4 * KS);
        if (AC % 256 == 0 || c < AC) ra[p][i] = *reinterpret_cast<const uint4*>(Ap[p] + (size_t)(row0 + r) * K + s * 32 * KS + q * 8);
      }
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int c = tid + 256 * i, r = c / (4 * KS), q = c % (4 * KS);
        if (BC % 256 == 0 || c < BC) rb[p][i] = *reinterpret_cast<const uint4*>(Bp[p] + (size_t)(col0 + r) * K + s * 32 * KS + q * 8);
      }
    }
  };
  auto store = [&](int s) {
#pragma unroll
    for (int p = 0; p < NPART; ++p) {
      u16* a = As + ((s & 1) * NPART + p) * AF;
      u16* b = Bs + ((s & 1) * NPART + p) * BF;
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int c = tid + 256 * i, r = c / (4 * KS), q = c % (4 * KS);
        if (AC % 256 == 0 || c < AC) *reinterpret_cast<uint4*>(a + r * PITCH + q * 8) = ra[p][i];
      }
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int c = tid + 256 * i, r = c / (4 * KS), q = c % (4 * KS);
        if (BC % 256 == 0 || c < BC) *reinterpret_cast<uint4*>(b + r * PITCH + q * 8) = rb[p][i];
      }
    }
  };
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = zero4();
  // product list: (part of A, part of B), small terms first
  constexpr int PA[6] = {1, 0, 2, 1, 0, 0}, PB[6] = {0, 1, 0, 1, 2, 0};
  constexpr int PA3[3] = {1, 0, 0}, PB3[3] = {0, 1, 0};
  auto compute = [&](int s) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
    const u16* a = As + (s & 1) * NPART * AF + 32 * ks;
    const u16* b = Bs + (s & 1) * NPART * BF + 32 * ks;
    bf16x8 af[NPART][TM], bfr[NPART][TN];
#pragma unroll
    for (int p = 0; p < NPART; ++p) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
        af[p][i] = *reinterpret_cast<const bf16x8*>(a + p * AF + ((wm * TM + i) * 16 + (lane & 15)) * PITCH + (lane >> 4) * 8);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bfr[p][j] = *reinterpret_cast<const bf16x8*>(b + p * BF + ((wn * TN + j) * 16 + (lane & 15)) * PITCH + (lane >> 4) * 8);
    }
#pragma unroll
    for (int t = 0; t < NPROD; ++t) {
      const int pa = NPROD == 6 ? PA[t] : PA3[t], pb = NPROD == 6 ? PB[t] : PB3[t];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[pa][i], bfr[pb][j], acc[i][j], 0, 0, 0);
    }
    }
  };
  load(0);
  store(0);
  if (ns > 1) load(1);
  lds_barrier();
  for (int s = 0; s < ns; ++s) {
    compute(s);
    if (s + 1 < ns) store(s + 1);
    if (s + 2 < ns) load(s + 2);
    lds_barrier();
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int r = row0 + (wm * TM + i) * 16 + (lane >> 4) * 4, c = col0 + (wn * TN + j) * 16 + (lane & 15);
#pragma unroll
      for (int e = 0; e < 4; ++e) C[(size_t)(r + e) * N + c] = acc[i][j][e];
    }
}

// fp32 reference core: the product's gemm_body on v_mfma_f32_16x16x4_f32, A row-major [M][K], B row-major [K][N]
template <int BM_, int BN_, int WM_, int WN_>
struct PGenF {
  static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_;
  static constexpr bool A_KMAJ = false, B_KMAJ = true, BIAS = false;
  Grid g;
  const float* A;
  const float* Bm;
  float* C;
  int M, N, K;
  __host__ __device__ void decode(int lb, int& tm, int& tn, int& z) const { g.decode(lb, tm, tn, z); }
  __host__ __device__ int nslabs(int) const { return K / BK; }
  __device__ f32x4 ldA(int, int s, int row, int k) const { return ld4(A + (size_t)row * K + s * BK + k); }
  __device__ f32x4 ldB(int, int s, int col, int k) const { return ld4(Bm + (size_t)(s * BK + k) * N + col); }
  __device__ void epi(int, int row, int col, f32x4 v) const {
#pragma unroll
    for (int r = 0; r < 4; ++r) C[(size_t)(row + r) * N + col] = v[r];
  }
};

template <class F>
static double time_us(F f, int reps = 21) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  std::vector<float> t;
  for (int i = 0; i < reps; ++i) {
    CK(hipEventRecord(a, 0));
    f();
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    t.push_back(ms * 1e3f);
  }
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

template <class T>
static T* dput(const std::vector<T>& h) {
  T* d = nullptr;
  CK(hipMalloc(&d, h.size() * sizeof(T)));
  CK(hipMemcpy(d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
  return d;
}

struct Shape { const char* name; int M, N, K; };

template <int BM, int BN>
static void run_shape(const Shape& sh) {
  const int M = sh.M, N = sh.N, K = sh.K;
  std::mt19937 g(7);
  std::uniform_real_distribution<float> ua(0.0f, 4.0f), uw(-0.04f, 0.04f), coin(0.0f, 1.0f);
  std::vector<float> A((size_t)M * K), Bk((size_t)K * N);   // A row-major, B [K][N]
  for (auto& x : A) x = coin(g) < 0.5f ? 0.0f : ua(g);
  for (auto& x : Bk) x = uw(g);
  // split planes: A [M][K], Bt [N][K]
  std::vector<u16> ap[3], bp[3];
  for (int p = 0; p < 3; ++p) { ap[p].resize((size_t)M * K); bp[p].resize((size_t)N * K); }
  for (size_t i = 0; i < A.size(); ++i) {
    float r = A[i];
    for (int p = 0; p < 3; ++p) { ap[p][i] = bf16_rn(r); r = r - bf16_f(ap[p][i]); }
  }
  for (int k = 0; k < K; ++k)
    for (int n = 0; n < N; ++n) {
      float r = Bk[(size_t)k * N + n];
      for (int p = 0; p < 3; ++p) { bp[p][(size_t)n * K + k] = bf16_rn(r); r = r - bf16_f(bp[p][(size_t)n * K + k]); }
    }
  float* dA = dput(A);
  float* dB = dput(Bk);
  float* dC = nullptr;
  CK(hipMalloc(&dC, (size_t)M * N * 4));
  const u16* hap[3];
  const u16* hbp[3];
  for (int p = 0; p < 3; ++p) { hap[p] = dput(ap[p]); hbp[p] = dput(bp[p]); }
  const u16** dAp = nullptr;
  const u16** dBp = nullptr;
  CK(hipMalloc(&dAp, sizeof(hap)));
  CK(hipMalloc(&dBp, sizeof(hbp)));
  CK(hipMemcpy(dAp, hap, sizeof(hap), hipMemcpyHostToDevice));
  CK(hipMemcpy(dBp, hbp, sizeof(hbp), hipMemcpyHostToDevice));
  // sampled reference outputs (f64)
  std::vector<int> si(4096), sj(4096);
  std::vector<double> ref(4096);
  double rmax = 0.0;
  for (int t = 0; t < 4096; ++t) {
    si[t] = (int)(g() % M);
    sj[t] = (int)(g() % N);
    double s = 0.0;
    for (int k = 0; k < K; ++k) s += (double)A[(size_t)si[t] * K + k] * (double)Bk[(size_t)k * N + sj[t]];
    ref[t] = s;
    rmax = std::max(rmax, std::fabs(s));
  }
  std::vector<float> hC((size_t)M * N);
  auto err = [&]() {
    CK(hipMemcpy(hC.data(), dC, hC.size() * 4, hipMemcpyDeviceToHost));
    double e = 0.0;
    for (int t = 0; t < 4096; ++t) e = std::max(e, std::fabs((double)hC[(size_t)si[t] * N + sj[t]] - ref[t]));
    return e / rmax;
  };
  const double flop = 2.0 * M * N * K;
  double t32 = 0.0;
  {
    using P = PGenF<64, 64, 2, 2>;
    P p{Grid{M / 64, N / 64, 1}, dA, dB, dC, M, N, K};
    CK(hipFuncSetAttribute((const void*)k_gemm32<P>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)gemm_lds_bytes<P>()));
    t32 = time_us([&] { hipLaunchKernelGGL(k_gemm32<P>, dim3(p.g.blocks()), dim3(256), gemm_lds_bytes<P>(), 0, p); });
    printf("%-8s %6dx%4dx%4d fp32 MFMA 16x16x4 t64x64     %8.2f us  %7.1f TF  x%.2f  max rel err %.2e\n", sh.name, M, N, K, t32,
           flop / t32 / 1e6, 1.0, err());
  }
  auto split = [&](auto kern, int npart, int ks, const char* tag) {
    const size_t lds = (size_t)2 * npart * (BM + BN) * (32 * ks + 8) * 2;
    CK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    const int G = (M / BM) * (N / BN);
    const double us = time_us([&] { hipLaunchKernelGGL(kern, dim3(G), dim3(256), lds, 0, dAp, dBp, dC, M, N, K); });
    printf("%-8s %6dx%4dx%4d %-10s t%dx%d ks%d  %8.2f us  %7.1f TF  x%.2f  max rel err %.2e\n", sh.name, M, N, K, tag, BM, BN, ks,
           us, flop / us / 1e6, t32 / us, err());
  };
  split(k_split<BM, BN, 2, 3>, 2, 1, "bf16x3");
  split(k_split<BM, BN, 2, 3, 2>, 2, 2, "bf16x3");
  split(k_split<BM, BN, 2, 3, 4>, 2, 4, "bf16x3");
  split(k_split<BM, BN, 3, 6>, 3, 1, "bf16x6");
  split(k_split<BM, BN, 3, 6, 2>, 3, 2, "bf16x6");
  CK(hipFree(dA)); CK(hipFree(dB)); CK(hipFree(dC));
  for (int p = 0; p < 3; ++p) { CK(hipFree((void*)hap[p])); CK(hipFree((void*)hbp[p])); }
  CK(hipFree(dAp)); CK(hipFree(dBp));
}

int main() {
  // K = 3072 (a multiple of the 128-deep slabs) for the fc1 shapes
  run_shape<64, 64>(Shape{"fc1", 1024, 512, 3072});
  run_shape<128, 64>(Shape{"fc1", 1024, 512, 3072});
  run_shape<128, 128>(Shape{"fc1x8", 8192, 512, 3072});
  run_shape<128, 64>(Shape{"conv2", 82944, 64, 512});
  run_shape<64, 64>(Shape{"conv2", 82944, 64, 512});
  return 0;
}
