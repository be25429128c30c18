// fp32 GEMM-core micro-benchmark (development tool, not part of the product): times the qnet32 layer policies at the
// learner's batch sizes and a generic GEMM policy at several tile shapes, each launch alone on one stream (HIP events,
// median of repeats).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I include -I q-learning_amd/csrc scripts/ubench32.hip \
//         -o scripts/ubench32 && ./scripts/ubench32
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

#include "qnet32_kernels.h"

using namespace qlx;
using namespace qlx::q32;

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e = (x);                                                                        \
    if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); }   \
  } while (0)

typedef float f32x16 __attribute__((ext_vector_type(16)));
// experimental core: v_mfma_f32_32x32x2_f32, wave tile TM x TN of 32 x 32 (A pitch PA, B k-major pitch rows + 32 mod 64)
template <int BM, int BN, int WM, int WN, int PA>
__global__ __launch_bounds__(256) void k_gen32x32(const float* A, const float* Bm, float* C, int M, int N, int K) {
  constexpr int TM = BM / (WM * 32), TN = BN / (WN * 32), T = 256;
  constexpr int PB = BN + (((32 - BN % 64) % 64) + 64) % 64;
  constexpr int AF = BM * PA, BF = BK * PB;
  constexpr int NA = BM * BK / 4 / T, NB = BN * BK / 4 / T;
  extern __shared__ float lds[];
  float* As[2] = {lds, lds + AF};
  float* Bs[2] = {lds + 2 * AF, lds + 2 * AF + BF};
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wm = wave % WM, wn = wave / WM;
  const int tiles_n = N / BN, lb = xcd_logical(blockIdx.x, gridDim.x), tm = lb / tiles_n, tn = lb % tiles_n;
  const int row0 = tm * BM, col0 = tn * BN, ns = K / BK;
  f32x4 ra[2][NA], rb[2][NB];
  auto load = [&](int s, f32x4(&a)[NA], f32x4(&b)[NB]) {
#pragma unroll
    for (int i = 0; i < NA; ++i) { const int idx = tid + i * T, r = idx >> 3, k = (idx & 7) * 4; a[i] = ld4(A + (size_t)(row0 + r) * K + s * BK + k); }
#pragma unroll
    for (int i = 0; i < NB; ++i) { const int idx = tid + i * T, k = idx / (BN / 4), c = (idx % (BN / 4)) * 4; b[i] = ld4(Bm + (size_t)(s * BK + k) * N + col0 + c); }
  };
  auto store = [&](int s, const f32x4(&a)[NA], const f32x4(&b)[NB]) {
#pragma unroll
    for (int i = 0; i < NA; ++i) { const int idx = tid + i * T, r = idx >> 3, k = (idx & 7) * 4; *reinterpret_cast<f32x4*>(As[s & 1] + r * PA + k) = a[i]; }
#pragma unroll
    for (int i = 0; i < NB; ++i) { const int idx = tid + i * T, k = idx / (BN / 4), c = (idx % (BN / 4)) * 4; *reinterpret_cast<f32x4*>(Bs[s & 1] + k * PB + c) = b[i]; }
  };
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;
  auto compute = [&](int s) {
    const float* a = As[s & 1];
    const float* b = Bs[s & 1];
#pragma unroll
    for (int kk = 0; kk < BK / 2; ++kk) {
      float af[TM], bf[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = a[((wm * TM + i) * 32 + (lane & 31)) * PA + 2 * kk + (lane >> 5)];
#pragma unroll
      for (int j = 0; j < TN; ++j) bf[j] = b[(2 * kk + (lane >> 5)) * PB + (wn * TN + j) * 32 + (lane & 31)];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
  };
  load(0, ra[1], rb[1]);
  store(0, ra[1], rb[1]);
  if (ns > 1) load(1, ra[0], rb[0]);
  lds_barrier();
  for (int s = 0; s < ns; s += 2) {
    if (s + 2 < ns) load(s + 2, ra[1], rb[1]);
    compute(s);
    if (s + 1 < ns) store(s + 1, ra[0], rb[0]);
    lds_barrier();
    if (s + 1 >= ns) break;
    if (s + 3 < ns) load(s + 3, ra[0], rb[0]);
    compute(s + 1);
    if (s + 2 < ns) store(s + 2, ra[1], rb[1]);
    lds_barrier();
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = row0 + (wm * TM + i) * 32 + 8 * (e >> 2) + 4 * (lane >> 5) + (e & 3), col = col0 + (wn * TN + j) * 32 + (lane & 31);
        C[(size_t)row * N + col] = acc[i][j][e];
      }
}

// experimental core 2: v_mfma_f32_32x32x2_f32 with an MFMA-fragment-major LDS image: operand row r holds its slab's 32 k as
// [h = k % 2][j = k / 2] (+4 pad, pitch 36), so a lane's 16 values for the slab are contiguous: 4 ds_read_b128 per
// fragment per slab, all issued at the slab's start, then 16 MFMAs back to back.  A row-major [M][K] (float4 along k ->
// two 8-byte stores), B row-major [K][N] (a thread loads 4 k x 4 n and writes each n's 4 k as two 8-byte stores).
template <int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(256) void k_gen32p(const float* A, const float* Bm, float* C, int M, int N, int K) {
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  constexpr int TM = BM / (WM * 32), TN = BN / (WN * 32), T = 256, P = 36;
  constexpr int AF = BM * P, BF = BN * P;
  constexpr int NA = BM * BK / 4 / T;               // float4 of A per thread
  constexpr int NBT = (BK / 4) * (BN / 4);          // B threads (each 4 k x 4 n)
  static_assert(NA >= 1 && NBT <= T, "tile");
  extern __shared__ float lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wm = wave % WM, wn = wave / WM;
  const int tiles_n = N / BN, lb = xcd_logical(blockIdx.x, gridDim.x), tm = lb / tiles_n, tn = lb % tiles_n;
  const int row0 = tm * BM, col0 = tn * BN, ns = K / BK;
  f32x4 ra[NA], rb[4];
  auto load = [&](int s) {
#pragma unroll
    for (int i = 0; i < NA; ++i) { const int idx = tid + i * T, r = idx >> 3, k = (idx & 7) * 4; ra[i] = ld4(A + (size_t)(row0 + r) * K + s * BK + k); }
    if (tid < NBT) {
      const int q = tid / (BN / 4), c = (tid % (BN / 4)) * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e) rb[e] = ld4(Bm + (size_t)(s * BK + 4 * q + e) * N + col0 + c);
    }
  };
  auto store = [&](int s) {
    float* a = lds + (s & 1) * AF;
    float* b = lds + 2 * AF + (s & 1) * BF;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int idx = tid + i * T, r = idx >> 3, q = idx & 7;
      *reinterpret_cast<f32x2*>(a + r * P + 2 * q) = f32x2{ra[i][0], ra[i][2]};
      *reinterpret_cast<f32x2*>(a + r * P + 16 + 2 * q) = f32x2{ra[i][1], ra[i][3]};
    }
    if (tid < NBT) {
      const int q = tid / (BN / 4), c = (tid % (BN / 4)) * 4;
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        *reinterpret_cast<f32x2*>(b + (c + n) * P + 2 * q) = f32x2{rb[0][n], rb[2][n]};
        *reinterpret_cast<f32x2*>(b + (c + n) * P + 16 + 2 * q) = f32x2{rb[1][n], rb[3][n]};
      }
    }
  };
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;
  const int lr = lane & 31, lh = (lane >> 5) * 16;
  auto compute = [&](int s) {
    const float* a = lds + (s & 1) * AF;
    const float* b = lds + 2 * AF + (s & 1) * BF;
    f32x4 af[TM][4], bf[TN][4];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) af[i][q] = *reinterpret_cast<const f32x4*>(a + ((wm * TM + i) * 32 + lr) * P + lh + 4 * q);
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) bf[j][q] = *reinterpret_cast<const f32x4*>(b + ((wn * TN + j) * 32 + lr) * P + lh + 4 * q);
#pragma unroll
    for (int kk = 0; kk < 16; ++kk)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i][kk >> 2][kk & 3], bf[j][kk >> 2][kk & 3], acc[i][j], 0, 0, 0);
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
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = row0 + (wm * TM + i) * 32 + 8 * (e >> 2) + 4 * (lane >> 5) + (e & 3), col = col0 + (wn * TN + j) * 32 + (lane & 31);
        C[(size_t)row * N + col] = acc[i][j][e];
      }
}

template <int BM, int BN, int WM, int WN>
static void gen32p(int M, int N, int K, const float* A, const float* B, float* C) {
  const size_t lds = 2 * (size_t)(BM + BN) * 36 * 4;
  auto kern = k_gen32p<BM, BN, WM, WN>;
  CK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  const int G = (M / BM) * (N / BN);
  const double us = time_us([&] { hipLaunchKernelGGL(kern, dim3(G), dim3(256), lds, 0, A, B, C, M, N, K); });
  const double f = 2.0 * M * N * K;
  printf("gen32p %dx%dx%d t%dx%d w%dx%d        blocks %6d lds %6zu  %9.2f us  %7.2f TF  %5.1f %%\n", M, N, K, BM, BN, WM, WN, G,
         lds, us, f / us / 1e6, f / us / 1e6 / 157.3 * 100);
}

template <int BM, int BN, int WM, int WN, int PA>
static void gen32(int M, int N, int K, const float* A, const float* B, float* C) {
  constexpr int PB = BN + (((32 - BN % 64) % 64) + 64) % 64;
  const size_t lds = 2 * (size_t)(BM * PA + BK * PB) * 4;
  auto kern = k_gen32x32<BM, BN, WM, WN, PA>;
  CK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  const int G = (M / BM) * (N / BN);
  const double us = time_us([&] { hipLaunchKernelGGL(kern, dim3(G), dim3(256), lds, 0, A, B, C, M, N, K); });
  const double f = 2.0 * M * N * K;
  printf("gen32x32 %dx%dx%d t%dx%d w%dx%d pa%d     blocks %6d lds %6zu  %9.2f us  %7.2f TF  %5.1f %%\n", M, N, K, BM, BN, WM, WN, PA, G,
         lds, us, f / us / 1e6, f / us / 1e6 / 157.3 * 100);
}

// C [M][N] = A [M][K] B [K][N], both row-major
template <int BM_, int BN_, int WM_, int WN_>
struct PGen {
  static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_;
  static constexpr bool A_KMAJ = false, B_KMAJ = true, BIAS = false;
  Grid g;
  const float* A;
  const float* Bm;
  float* C;
  int M, N, K;
  __host__ __device__ void decode(int lb, int& tm, int& tn, int& z) const { g.decode(lb, tm, tn, z); }
  __host__ __device__ int nslabs(int) const { return K / BK; }
  __device__ f32x4 ldA(int, int s, int row, int k) const { return row < M ? ld4(A + (size_t)row * K + s * BK + k) : zero4(); }
  __device__ f32x4 ldB(int, int s, int col, int k) const { return ld4(Bm + (size_t)(s * BK + k) * N + col); }
  __device__ void epi(int, int row, int col, f32x4 v) const {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (row + r < M) C[(size_t)(row + r) * N + col] = v[r];
  }
};

static float* dbuf(size_t n, uint32_t seed) {
  std::vector<float> h(n);
  std::mt19937 g(seed);
  std::uniform_real_distribution<float> u(-1.0f, 1.0f);
  for (auto& x : h) x = u(g);
  float* d = nullptr;
  CK(hipMalloc(&d, n * 4));
  CK(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice));
  return d;
}

template <class F>
static double time_us(F f, int reps = 15) {
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

static Grid grid(int M, int BM, int N, int BN, int nz) { return Grid{(M + BM - 1) / BM, (N + BN - 1) / BN, nz}; }

// row-tile-fastest block order (consecutive blocks share a column tile: an XCD's blocks keep one slice of B in its L2)
template <class Base>
struct RowFast : Base {
  __host__ __device__ void decode(int lb, int& tm, int& tn, int& z) const {
    tm = lb % this->g.tiles_m;
    const int q = lb / this->g.tiles_m;
    tn = q % this->g.tiles_n;
    z = q / this->g.tiles_n;
  }
};

// K-split wave groups on any policy (gemm_body KSPLIT)
template <class Base, int K>
struct KSplit : Base {
  static constexpr int KSPLIT = K;
};

template <class P>
static void run1(const char* name, const P& p, double flop) {
  CK(hipFuncSetAttribute((const void*)k_gemm32<P>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)gemm_lds_bytes<P>()));
  const double us = time_us([&] { hipLaunchKernelGGL(k_gemm32<P>, dim3(p.g.blocks()), dim3(threads_of<P>()), gemm_lds_bytes<P>(), 0, p); });
  printf("%-34s blocks %6d lds %6zu  %9.2f us  %7.2f TF  %5.1f %%\n", name, p.g.blocks(), gemm_lds_bytes<P>(), us,
         flop / us / 1e6, flop / us / 1e6 / 157.3 * 100);
}

template <class P1, class P2>
static void run2(const char* name, const P1& p1, const P2& p2, double flop) {
  const size_t lds = std::max(gemm_lds_bytes<P1>(), gemm_lds_bytes<P2>());
  const double us = time_us([&] {
    hipLaunchKernelGGL((k_gemm32_pair<P1, P2, NoSide, NoSide>), dim3(p1.g.blocks() + p2.g.blocks()), dim3(256), lds, 0, p1, p2, NoSide{},
                       NoSide{});
  });
  printf("%-34s blocks %6d lds %6zu  %9.2f us  %7.2f TF  %5.1f %%\n", name, p1.g.blocks() + p2.g.blocks(), lds, us,
         flop / us / 1e6, flop / us / 1e6 / 157.3 * 100);
}

template <int BM, int BN, int WM, int WN>
static void gen(int M, int N, int K, const float* A, const float* B, float* C) {
  PGen<BM, BN, WM, WN> p{grid(M, BM, N, BN, 1), A, B, C, M, N, K};
  char name[96];
  snprintf(name, sizeof name, "gen %dx%dx%d t%dx%d w%dx%d", M, N, K, BM, BN, WM, WN);
  run1(name, p, 2.0 * M * N * K);
}

// c1probe: the conv1 forward's a1 store pattern alone (lane (g, c) of wave (ct, rp) stores its 13 tiles x 4 rows per
// sample, as k_conv1_fwd32 does) and its frame fetch + LDS staging alone, B samples over G blocks
__global__ __launch_bounds__(256, 2) void k_probe_a1_stores(int B, float* a1, float v) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, ct = wave & 1, rp = wave >> 1;
  const int col = ct * 16 + (lane & 15), g = lane >> 4, nt = rp == 0 ? 13 : 12;
  for (int b = blockIdx.x; b < B; b += gridDim.x) {
#pragma unroll
    for (int j = 0; j < 13; ++j)
      if (j < nt) {
        const int t = rp + 2 * j, r0 = (4 * (t / 5) + g) * 20 + 4 * (t % 5);
#pragma unroll
        for (int i = 0; i < 4; ++i) a1[((size_t)b * 400 + r0 + i) * 32 + col] = v + i;
      }
  }
}
__global__ __launch_bounds__(256, 2) void k_probe_a1_stores_row(int B, float* a1, float v) {   // the same bytes, row-contiguous
  for (int b = blockIdx.x; b < B; b += gridDim.x) {
    f32x4* d = reinterpret_cast<f32x4*>(a1 + (size_t)b * 12800);
    for (int q = threadIdx.x; q < 3200; q += 256) d[q] = f32x4{v, v, v, v};
  }
}
__global__ __launch_bounds__(256, 2) void k_probe_frames(const uint8_t* const* table, int B, float* out) {
  extern __shared__ __attribute__((aligned(16))) uint32_t c1w[];
  int b = blockIdx.x;
  if (b >= B) return;
  uint4 pf[7];
  c1_prefetch(c1_ptrs(table, b), pf);
  C1Ptrs nxt = c1_ptrs(table, b + (int)gridDim.x < B ? b + (int)gridDim.x : b);
  c1_stage(c1w, pf);
  __syncthreads();
  uint32_t acc = 0;
  for (int it = 0; b < B; b += gridDim.x, ++it) {
    const uint32_t* fr = c1w + (it & 1) * (4 * kC1SlotDw);
    const int nb = b + gridDim.x;
    if (nb < B) {
      c1_prefetch(nxt, pf);
      nxt = c1_ptrs(table, nb + (int)gridDim.x < B ? nb + (int)gridDim.x : nb);
    }
    acc += fr[threadIdx.x];
    if (nb < B) c1_stage(c1w + ((it + 1) & 1) * (4 * kC1SlotDw), pf);
    __syncthreads();
  }
  if (acc == 0x12345678u) out[threadIdx.x] = 1.0f;
}

int main(int argc, char** argv) {
  const bool only_c1 = argc > 1 && std::string(argv[1]) == "conv1";   // just the two conv1 kernels
  const int Bs[2] = {1024, 8192};
  // layer buffers sized for the larger batch
  const int Bmax = 8192;
  float* w = dbuf(1685667, 1);
  float* a1 = dbuf((size_t)Bmax * 12800, 2);
  float* a2 = dbuf((size_t)Bmax * 5184, 3);
  float* a3 = dbuf((size_t)Bmax * 3136, 4);
  float* a4 = dbuf((size_t)Bmax * 512, 5);
  float* dz1 = dbuf((size_t)Bmax * 12800, 6);
  float* dz2 = dbuf((size_t)Bmax * 5184, 7);
  float* dz3 = dbuf((size_t)Bmax * 3136, 8);
  float* dz4 = dbuf((size_t)Bmax * 512, 9);
  float* slab = dbuf((size_t)2048 * 577 * 64, 10);
  float* gw = dbuf((size_t)3136 * 513, 11);
  // frames: one 7056-byte frame per (sample, slot)
  uint8_t* frames = nullptr;
  CK(hipMalloc(&frames, (size_t)Bmax * 4 * 7056));
  CK(hipMemset(frames, 7, (size_t)Bmax * 4 * 7056));
  std::vector<const uint8_t*> ht(Bmax * 4);
  for (int i = 0; i < Bmax * 4; ++i) ht[i] = frames + (size_t)i * 7056;
  const uint8_t** table = nullptr;
  CK(hipMalloc(&table, ht.size() * sizeof(void*)));
  CK(hipMemcpy(table, ht.data(), ht.size() * sizeof(void*), hipMemcpyHostToDevice));
  const float* W0 = w;
  const float* W1 = w + 8192 + 32;
  const float* W2 = W1 + 32768 + 64;
  const float* W3 = W2 + 36864 + 64;
  if (argc > 1 && std::string(argv[1]) == "split") {   // balanced grids: whole tiles per CU + the remainder as 16-row tiles
    const int B = 1024;
    const double f3 = 2.0 * B * 49 * 64 * 576, f2 = 2.0 * B * 81 * 64 * 512;
    using C3W = PConvFwd<9, 9, 64, 3, 1, 7, 7, 64>;
    using C3N = PConvFwd<9, 9, 64, 3, 1, 7, 7, 64, 64, 32, 2, 2>;
    using C3M = RowShift<PConvFwd<9, 9, 64, 3, 1, 7, 7, 64, 16, 64, 1, 4>>;
    using C3H = RowShift<PConvFwd<9, 9, 64, 3, 1, 7, 7, 64, 32, 64, 2, 2>>;
    using C2W = PConvFwd<20, 20, 32, 4, 2, 9, 9, 64>;
    using C2N = PConvFwd<20, 20, 32, 4, 2, 9, 9, 64, 64, 32, 2, 2>;
    using C2M = RowShift<PConvFwd<20, 20, 32, 4, 2, 9, 9, 64, 16, 64, 1, 4>>;
    const int M3 = B * 49, M2 = B * 81;
    for (int rep = 0; rep < 2; ++rep) {
      run1("conv3_fwd t64x32 (now)", C3N{grid(M3, 64, 64, 32, 1), a2, W2, W2, a3, M3}, f3);
      run1("conv3_fwd t64x64", C3W{grid(M3, 64, 64, 64, 1), a2, W2, W2, a3, M3}, f3);
      run2("conv3_fwd 768 t64x64 + 64 t16x64", C3W{Grid{768, 1, 1}, a2, W2, W2, a3, M3},
           C3M{{Grid{64, 1, 1}, a2, W2, W2, a3, M3}, 3072}, f3);
      run2("conv3_fwd 64 t16x64 + 768 t64x64", C3M{{Grid{64, 1, 1}, a2, W2, W2, a3, M3}, 3072},
           C3W{Grid{768, 1, 1}, a2, W2, W2, a3, M3}, f3);
      run2("conv3_fwd 768 t64x64 + 32 t32x64", C3W{Grid{768, 1, 1}, a2, W2, W2, a3, M3},
           C3H{{Grid{32, 1, 1}, a2, W2, W2, a3, M3}, 1536}, f3);
      run2("conv3_fwd 1536 t64x32 + 64 t16x64", C3N{Grid{768, 2, 1}, a2, W2, W2, a3, M3},
           C3M{{Grid{64, 1, 1}, a2, W2, W2, a3, M3}, 3072}, f3);
      run2("conv3_fwd 64 t16x64 + 1536 t64x32", C3M{{Grid{64, 1, 1}, a2, W2, W2, a3, M3}, 3072},
           C3N{Grid{768, 2, 1}, a2, W2, W2, a3, M3}, f3);
      run1("conv2_fwd t64x32 (now)", C2N{grid(M2, 64, 64, 32, 1), a1, W1, W1, a2, M2}, f2);
      run1("conv2_fwd t64x64", C2W{grid(M2, 64, 64, 64, 1), a1, W1, W1, a2, M2}, f2);
      run2("conv2_fwd 1280 t64x64 + 64 t16x64", C2W{Grid{1280, 1, 1}, a1, W1, W1, a2, M2},
           C2M{{Grid{64, 1, 1}, a1, W1, W1, a2, M2}, 5120}, f2);
      run2("conv2_fwd 64 t16x64 + 1280 t64x64", C2M{{Grid{64, 1, 1}, a1, W1, W1, a2, M2}, 5120},
           C2W{Grid{1280, 1, 1}, a1, W1, W1, a2, M2}, f2);
      run2("conv2_fwd 2560 t64x32 + 64 t16x64", C2N{Grid{1280, 2, 1}, a1, W1, W1, a2, M2},
           C2M{{Grid{64, 1, 1}, a1, W1, W1, a2, M2}, 5120}, f2);
      run2("conv2_fwd 64 t16x64 + 2560 t64x32", C2M{{Grid{64, 1, 1}, a1, W1, W1, a2, M2}, 5120},
           C2N{Grid{1280, 2, 1}, a1, W1, W1, a2, M2}, f2);
    }
    return 0;
  }
  if (argc > 1 && std::string(argv[1]) == "tail") {   // grid-tail check: the B = 1024 layer launches at batches around 1024
    for (int B : {896, 960, 992, 1002, 1008, 1016, 1024, 1040, 1088, 1152}) {
      char n[64];
      printf("--- B = %d\n", B);
      snprintf(n, sizeof n, "conv2_fwd t64x32 B%d", B);
      run1(n, PConvFwd<20, 20, 32, 4, 2, 9, 9, 64, 64, 32>{grid(B * 81, 64, 64, 32, 1), a1, W1, W1, a2, B * 81}, 2.0 * B * 81 * 64 * 512);
      snprintf(n, sizeof n, "conv3_fwd t64x32 B%d", B);
      run1(n, PConvFwd<9, 9, 64, 3, 1, 7, 7, 64, 64, 32>{grid(B * 49, 64, 64, 32, 1), a2, W2, W2, a3, B * 49}, 2.0 * B * 49 * 64 * 576);
      snprintf(n, sizeof n, "conv3_fwd t64x64 B%d", B);
      run1(n, PConvFwd<9, 9, 64, 3, 1, 7, 7, 64>{grid(B * 49, 64, 64, 64, 1), a2, W2, W2, a3, B * 49}, 2.0 * B * 49 * 64 * 576);
      snprintf(n, sizeof n, "fc1_fwd t32x32 B%d", B);
      run1(n, PFc1FwdT<32, 32, 2, 2>{grid(B, 32, 512, 32, 1), a3, W3, W3, a4, B}, 2.0 * B * 3136 * 512);
      snprintf(n, sizeof n, "conv3 pair pxg B%d", B);
      run2(n, PConvWgrad<9, 9, 64, 3, 1, 7, 7, 64, 16>{grid(576, 64, 64, 64, (B + 15) / 16), a2, dz3, slab, B},
           PConv3DgradPxG<32, 64, 2, 2>{{Grid{(B + 31) / 32, 1, 49}, dz3, W2, a2, dz2, B}}, 4.0 * B * 49 * 64 * 576);
      snprintf(n, sizeof n, "conv2 pair px B%d", B);
      run2(n, PConvWgrad<20, 20, 32, 4, 2, 9, 9, 64, 16>{grid(512, 64, 64, 64, (B + 15) / 16), a1, dz2, slab, B},
           PConv2DgradPx<64, 64, 2, 2>{Grid{(B + 63) / 64, 2, 100}, dz2, W1, a1, dz1, B}, 4.0 * B * 81 * 64 * 512);
    }
    return 0;
  }
  if (argc > 1 && std::string(argv[1]) == "bwd") {   // pixel-major backward data: one pixel per tile vs pixel groups
    for (int B : {1024, 8192}) {
      const double f3 = 2.0 * B * 49 * 64 * 576, f2 = 2.0 * B * 81 * 64 * 512;
      const int z3 = B / 16, z2 = B / 16;
      printf("--- B = %d\n", B);
      run1("conv3_dgrad px t32x64", PConv3DgradPx<32, 64, 2, 2>{Grid{(B + 31) / 32, 1, 81}, dz3, W2, a2, dz2, B}, f3);
      run1("conv3_dgrad pxg t32x64", PConv3DgradPxG<32, 64, 2, 2>{{Grid{(B + 31) / 32, 1, 49}, dz3, W2, a2, dz2, B}}, f3);
      run1("conv3_dgrad pxg t64x64", PConv3DgradPxG<64, 64, 2, 2>{{Grid{(B + 63) / 64, 1, 49}, dz3, W2, a2, dz2, B}}, f3);
      run1("conv3_dgrad pxg t32x32", PConv3DgradPxG<32, 32, 2, 2>{{Grid{(B + 31) / 32, 2, 49}, dz3, W2, a2, dz2, B}}, f3);
      run1("conv3_wgrad sc16", PConvWgrad<9, 9, 64, 3, 1, 7, 7, 64, 16>{grid(576, 64, 64, 64, z3), a2, dz3, slab, B}, f3);
      run2("conv3 pair px", PConvWgrad<9, 9, 64, 3, 1, 7, 7, 64, 16>{grid(576, 64, 64, 64, z3), a2, dz3, slab, B},
           PConv3DgradPx<32, 64, 2, 2>{Grid{(B + 31) / 32, 1, 81}, dz3, W2, a2, dz2, B}, 2 * f3);
      run2("conv3 pair pxg", PConvWgrad<9, 9, 64, 3, 1, 7, 7, 64, 16>{grid(576, 64, 64, 64, z3), a2, dz3, slab, B},
           PConv3DgradPxG<32, 64, 2, 2>{{Grid{(B + 31) / 32, 1, 49}, dz3, W2, a2, dz2, B}}, 2 * f3);
      run1("conv2_dgrad px t64x64", PConv2DgradPx<64, 64, 2, 2>{Grid{(B + 63) / 64, 2, 100}, dz2, W1, a1, dz1, B}, f2);
      run1("conv2_dgrad pxg t64x64", PConv2DgradPxG<64, 64, 2, 2>{{Grid{(B + 63) / 64, 2, 81}, dz2, W1, a1, dz1, B}}, f2);
      run1("conv2_dgrad pxg t32x64", PConv2DgradPxG<32, 64, 2, 2>{{Grid{(B + 31) / 32, 2, 81}, dz2, W1, a1, dz1, B}}, f2);
      run1("conv2_wgrad sc16", PConvWgrad<20, 20, 32, 4, 2, 9, 9, 64, 16>{grid(512, 64, 64, 64, z2), a1, dz2, slab, B}, f2);
      run2("conv2 pair px", PConvWgrad<20, 20, 32, 4, 2, 9, 9, 64, 16>{grid(512, 64, 64, 64, z2), a1, dz2, slab, B},
           PConv2DgradPx<64, 64, 2, 2>{Grid{(B + 63) / 64, 2, 100}, dz2, W1, a1, dz1, B}, 2 * f2);
      run2("conv2 pair pxg", PConvWgrad<20, 20, 32, 4, 2, 9, 9, 64, 16>{grid(512, 64, 64, 64, z2), a1, dz2, slab, B},
           PConv2DgradPxG<64, 64, 2, 2>{{Grid{(B + 63) / 64, 2, 81}, dz2, W1, a1, dz1, B}}, 2 * f2);
      if (B > 1024) break;
    }
    return 0;
  }
  if (argc > 1 && std::string(argv[1]) == "sweep") {   // backward-pair tile shapes on the operand-stream core, B = 1024
    const int B = 1024, z = B / 16;
    const double ff = 4.0 * B * 512 * 3136, f3 = 4.0 * B * 49 * 64 * 576, f2 = 4.0 * B * 81 * 64 * 512;
    using Wg3 = PConvWgrad<9, 9, 64, 3, 1, 7, 7, 64, 16>;
    using Wg2 = PConvWgrad<20, 20, 32, 4, 2, 9, 9, 64, 16>;
    for (int rep = 0; rep < 2; ++rep) {
      printf("--- rep %d\n", rep);
      run2("fc1 W64x64 D32x64 (shipped)", PFc1WgradT<64, 64, 2, 2>{grid(3136, 64, 512, 64, 1), a3, dz4, gw, gw, B},
           PFc1DgradT<32, 64, 2, 2>{grid(B, 32, 3136, 64, 1), dz4, W3, a3, dz3, B}, ff);
      run2("fc1 W64x64 D64x64", PFc1WgradT<64, 64, 2, 2>{grid(3136, 64, 512, 64, 1), a3, dz4, gw, gw, B},
           PFc1DgradT<64, 64, 2, 2>{grid(B, 64, 3136, 64, 1), dz4, W3, a3, dz3, B}, ff);
      run2("fc1 W64x64 D32x32", PFc1WgradT<64, 64, 2, 2>{grid(3136, 64, 512, 64, 1), a3, dz4, gw, gw, B},
           PFc1DgradT<32, 32, 2, 2>{grid(B, 32, 3136, 32, 1), dz4, W3, a3, dz3, B}, ff);
      run2("fc1 W64x64 D64x32", PFc1WgradT<64, 64, 2, 2>{grid(3136, 64, 512, 64, 1), a3, dz4, gw, gw, B},
           PFc1DgradT<64, 32, 2, 2>{grid(B, 64, 3136, 32, 1), dz4, W3, a3, dz3, B}, ff);
      run2("fc1 W64x32 D32x64", PFc1WgradT<64, 32, 2, 2>{grid(3136, 64, 512, 32, 1), a3, dz4, gw, gw, B},
           PFc1DgradT<32, 64, 2, 2>{grid(B, 32, 3136, 64, 1), dz4, W3, a3, dz3, B}, ff);
      run2("fc1 W128x64 D32x64", PFc1WgradT<128, 64, 2, 2>{grid(3136, 128, 512, 64, 1), a3, dz4, gw, gw, B},
           PFc1DgradT<32, 64, 2, 2>{grid(B, 32, 3136, 64, 1), dz4, W3, a3, dz3, B}, ff);
      run2("conv3 W64x64 Dpx32x64 (shipped)", Wg3{grid(576, 64, 64, 64, z), a2, dz3, slab, B},
           PConv3DgradPx<32, 64, 2, 2>{Grid{(B + 31) / 32, 1, 81}, dz3, W2, a2, dz2, B}, f3);
      run2("conv3 W64x64 Dpx64x64", Wg3{grid(576, 64, 64, 64, z), a2, dz3, slab, B},
           PConv3DgradPx<64, 64, 2, 2>{Grid{(B + 63) / 64, 1, 81}, dz3, W2, a2, dz2, B}, f3);
      run2("conv3 W64x64 Dpx32x32", Wg3{grid(576, 64, 64, 64, z), a2, dz3, slab, B},
           PConv3DgradPx<32, 32, 2, 2>{Grid{(B + 31) / 32, 2, 81}, dz3, W2, a2, dz2, B}, f3);
      run2("conv3 W64x64 Dpx16x64", Wg3{grid(576, 64, 64, 64, z), a2, dz3, slab, B},
           PConv3DgradPx<16, 64, 1, 4>{Grid{(B + 15) / 16, 1, 81}, dz3, W2, a2, dz2, B}, f3);
      run2("conv3 W64x32 Dpx32x64", Wg3{grid(576, 64, 64, 32, z), a2, dz3, slab, B},
           PConv3DgradPx<32, 64, 2, 2>{Grid{(B + 31) / 32, 1, 81}, dz3, W2, a2, dz2, B}, f3);
      run2("conv2 W64x64 Dpx64x64 (shipped)", Wg2{grid(512, 64, 64, 64, z), a1, dz2, slab, B},
           PConv2DgradPx<64, 64, 2, 2>{Grid{(B + 63) / 64, 2, 100}, dz2, W1, a1, dz1, B}, f2);
      run2("conv2 W64x64 Dpx32x64", Wg2{grid(512, 64, 64, 64, z), a1, dz2, slab, B},
           PConv2DgradPx<32, 64, 2, 2>{Grid{(B + 31) / 32, 2, 100}, dz2, W1, a1, dz1, B}, f2);
      run2("conv2 W64x64 Dpx64x128", Wg2{grid(512, 64, 64, 64, z), a1, dz2, slab, B},
           PConv2DgradPx<64, 128, 2, 2>{Grid{(B + 63) / 64, 1, 100}, dz2, W1, a1, dz1, B}, f2);
      run2("conv2 W64x64 Dpx64x32", Wg2{grid(512, 64, 64, 64, z), a1, dz2, slab, B},
           PConv2DgradPx<64, 32, 2, 2>{Grid{(B + 63) / 64, 4, 100}, dz2, W1, a1, dz1, B}, f2);
      run2("conv2 W64x64 Dpx128x64", Wg2{grid(512, 64, 64, 64, z), a1, dz2, slab, B},
           PConv2DgradPx<128, 64, 2, 2>{Grid{(B + 127) / 128, 2, 100}, dz2, W1, a1, dz1, B}, f2);
      run2("conv3 W64x64 Dpx128x64", Wg3{grid(576, 64, 64, 64, z), a2, dz3, slab, B},
           PConv3DgradPx<128, 64, 2, 2>{Grid{(B + 127) / 128, 1, 81}, dz3, W2, a2, dz2, B}, f3);
      run2("fc1 W64x64 D128x64", PFc1WgradT<64, 64, 2, 2>{grid(3136, 64, 512, 64, 1), a3, dz4, gw, gw, B},
           PFc1DgradT<128, 64, 2, 2>{grid(B, 128, 3136, 64, 1), dz4, W3, a3, dz3, B}, ff);
      run2("conv2 W64x32 Dpx64x64", Wg2{grid(512, 64, 64, 32, z), a1, dz2, slab, B},
           PConv2DgradPx<64, 64, 2, 2>{Grid{(B + 63) / 64, 2, 100}, dz2, W1, a1, dz1, B}, f2);
    }
    return 0;
  }
  if (argc > 1 && std::string(argv[1]) == "c1probe") {
    // what the conv1 kernels cost besides their MFMAs: live frames (nothing skippable) vs all-zero frames (a null table:
    // every step skippable) with the zero-step skip on / off, B = 1024
    const uint8_t** ztab = nullptr;
    CK(hipMalloc(&ztab, ht.size() * sizeof(void*)));
    CK(hipMemset(ztab, 0, ht.size() * sizeof(void*)));
    const int B = 1024, G = 512, nz = B / 4, lds = (int)kC1WgradLds;
    CK(hipFuncSetAttribute((const void*)k_conv1_fwd32<0>, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * kC1Frames));
    CK(hipFuncSetAttribute((const void*)k_conv1_wgrad32, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    for (int zero = 0; zero < 2; ++zero)
      for (int skip = 0; skip < 2; ++skip) {
        const uint8_t* const* t = zero ? ztab : table;
        const double uf = time_us([&] { hipLaunchKernelGGL(k_conv1_fwd32<0>, dim3(G), dim3(256), 2 * kC1Frames, 0, t, B, W0, W0 + 8192, a1, skip, C1Lists{}); });
        const double uw = time_us([&] { hipLaunchKernelGGL(k_conv1_wgrad32, dim3(c1_wgrad_blocks(nz)), dim3(kC1WgradThreads), lds, 0, t, dz1, B, nz, slab, skip, nullptr, dz1); });
        printf("conv1 B=%d frames %-5s skip %d: forward %8.2f us  weight gradient %8.2f us\n", B, zero ? "zero" : "live", skip, uf, uw);
      }
    for (int nb : {1024, 8192}) {
      const double us_st = time_us([&] { hipLaunchKernelGGL(k_probe_a1_stores, dim3(G), dim3(256), 0, 0, nb, a1, 1.0f); });
      const double us_row = time_us([&] { hipLaunchKernelGGL(k_probe_a1_stores_row, dim3(G), dim3(256), 0, 0, nb, a1, 1.0f); });
      CK(hipFuncSetAttribute((const void*)k_probe_frames, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * kC1Frames));
      const double us_fr = time_us([&] { hipLaunchKernelGGL(k_probe_frames, dim3(G), dim3(256), 2 * kC1Frames, 0, table, nb, a4); });
      const double us_frz = time_us([&] { hipLaunchKernelGGL(k_probe_frames, dim3(G), dim3(256), 2 * kC1Frames, 0, ztab, nb, a4); });
      printf("B=%d: a1 stores (conv1 pattern) %8.2f us (%.2f TB/s), row-contiguous %8.2f us; frame fetch + stage %8.2f us, zero table %8.2f us\n",
             nb, us_st, nb * 51200.0 / us_st / 1e6, us_row, us_fr, us_frz);
    }
    return 0;
  }
  for (int B : Bs) {
    printf("--- B = %d\n", B);
    {
      const int G = std::min(B, 512);
      CK(hipFuncSetAttribute((const void*)k_conv1_fwd32<0>, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * kC1Frames));
      const double us = time_us([&] { hipLaunchKernelGGL(k_conv1_fwd32<0>, dim3(G), dim3(256), 2 * kC1Frames, 0, table, B, W0, W0 + 8192, a1, 1, C1Lists{}); });
      const double f = 2.0 * B * 400 * 32 * 256;
      printf("%-34s blocks %6d lds %6d  %9.2f us  %7.2f TF  %5.1f %%\n", "conv1_fwd (k_conv1_fwd32)", G, 2 * kC1Frames, us, f / us / 1e6,
             f / us / 1e6 / 157.3 * 100);
    }
    if (!only_c1) {
    run1("conv2_fwd", PConvFwd<20, 20, 32, 4, 2, 9, 9, 64>{grid(B * 81, 64, 64, 64, 1), a1, W1, W1, a2, B * 81},
         2.0 * B * 81 * 64 * 512);
    run1("conv3_fwd", PConvFwd<9, 9, 64, 3, 1, 7, 7, 64>{grid(B * 49, 64, 64, 64, 1), a2, W2, W2, a3, B * 49},
         2.0 * B * 49 * 64 * 576);
    run1("fc1_fwd", PFc1Fwd{grid(B, PFc1Fwd::BM, 512, 64, 1), a3, W3, W3, a4, B}, 2.0 * B * 3136 * 512);
    if (B > 1024) continue;
    run1("fc1_wgrad", PFc1Wgrad{grid(3136, 64, 512, 64, 1), a3, dz4, gw, gw, B}, 2.0 * B * 3136 * 512);
    run1("fc1_dgrad", PFc1Dgrad{grid(B, 64, 3136, 64, 1), dz4, W3, a3, dz3, B}, 2.0 * B * 3136 * 512);
    run2("fc1_bwd pair", PFc1Wgrad{grid(3136, 64, 512, 64, 1), a3, dz4, gw, gw, B}, PFc1Dgrad{grid(B, 64, 3136, 64, 1), dz4, W3, a3, dz3, B},
         4.0 * B * 3136 * 512);
    {
      uint8_t* act = nullptr;
      CK(hipMalloc(&act, B));
      CK(hipMemset(act, 1, B));
      PFc1WgradS Pw{grid(3136, PFc1WgradS::BM, 512, PFc1WgradS::BN, 1), a3, dz4, gw, gw, B};
      PFc1DgradS Pd{grid(B, PFc1DgradS::BM, 3136, PFc1DgradS::BN, 1), dz4, W3, a3, dz3, B};
      SideFc2 S{a4, act, dz4, dz4 + 1024, B, gw, gw + 2000, gw + 3000};
      const size_t lds = std::max({gemm_lds_bytes<PFc1WgradS>(), gemm_lds_bytes<PFc1DgradS>(), SideFc2::LDS});
      double us = time_us([&] {
        hipLaunchKernelGGL((k_gemm32_pair<PFc1WgradS, PFc1DgradS, SideFc2, NoSide>), dim3(SideFc2::BLOCKS + Pw.g.blocks() + Pd.g.blocks()),
                           dim3(256), lds, 0, Pw, Pd, S, NoSide{});
      });
      printf("%-34s %9.2f us\n", "fc1_bwd pair + SideFc2", us);
      PFc1WgradS Pw0{Grid{0, 1, 1}, a3, dz4, gw, gw, B};
      PFc1DgradS Pd0{Grid{0, 1, 1}, dz4, W3, a3, dz3, B};
      us = time_us([&] {
        hipLaunchKernelGGL((k_gemm32_pair<PFc1WgradS, PFc1DgradS, SideFc2, NoSide>), dim3(SideFc2::BLOCKS), dim3(256), lds, 0, Pw0, Pd0, S,
                           NoSide{});
      });
      printf("%-34s %9.2f us\n", "SideFc2 alone", us);
    }
    run1("conv3_dgrad", PConv3Dgrad{grid(B * 81, 64, 64, 64, 1), dz3, W2, a2, dz2, B * 81}, 2.0 * B * 49 * 64 * 576);
    run1("conv3_wgrad", PConvWgrad<9, 9, 64, 3, 1, 7, 7, 64, 16>{grid(576, 64, 64, 64, B / 16), a2, dz3, slab, B},
         2.0 * B * 49 * 64 * 576);
    run1("conv2_dgrad", PConv2Dgrad{grid(B * 100, PConv2Dgrad::BM, 32, 32, 4), dz2, W1, a1, dz1, B * 100}, 2.0 * B * 81 * 64 * 512);
    run1("conv2_wgrad", PConvWgrad<20, 20, 32, 4, 2, 9, 9, 64, 16>{grid(512, 64, 64, 64, B / 16), a1, dz2, slab, B},
         2.0 * B * 81 * 64 * 512);
    }
    {
      const int nz = B / 4, lds = (int)kC1WgradLds;
      CK(hipFuncSetAttribute((const void*)k_conv1_wgrad32, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
      const double us = time_us([&] { hipLaunchKernelGGL(k_conv1_wgrad32, dim3(c1_wgrad_blocks(nz)), dim3(kC1WgradThreads), lds, 0, table, dz1, B, nz, slab, 1, nullptr, dz1); });
      const double f = 2.0 * B * 400 * 256 * 32;
      printf("%-34s blocks %6d lds %6d  %9.2f us  %7.2f TF  %5.1f %%\n", "conv1_wgrad (k_conv1_wgrad32)", 2 * nz, lds, us,
             f / us / 1e6, f / us / 1e6 / 157.3 * 100);
    }
  }
  if (only_c1 || (argc > 1 && std::string(argv[1]) == "layers")) return 0;   // "layers": just the per-layer list above
  printf("--- tile variants, B = 1024\n");
  {
    const int B = 1024;
#define V(NAME, P, ...) run1(NAME " " #P, P{__VA_ARGS__}, flop)
    double flop = 2.0 * B * 3136 * 512;
    run1("fc1_fwd t32x32 w2x2", PFc1FwdT<32, 32, 2, 2>{grid(B, 32, 512, 32, 1), a3, W3, W3, a4, B}, flop);
    run1("fc1_fwd t64x32 w2x2", PFc1FwdT<64, 32, 2, 2>{grid(B, 64, 512, 32, 1), a3, W3, W3, a4, B}, flop);
    run1("fc1_fwd t64x64 w2x2", PFc1FwdT<64, 64, 2, 2>{grid(B, 64, 512, 64, 1), a3, W3, W3, a4, B}, flop);
    run1("fc1_fwd t32x128 w2x2", PFc1FwdT<32, 128, 2, 2>{grid(B, 32, 512, 128, 1), a3, W3, W3, a4, B}, flop);
    run1("fc1_dgrad t64x32 w2x2", PFc1DgradT<64, 32, 2, 2>{grid(B, 64, 3136, 32, 1), dz4, W3, a3, dz3, B}, flop);
    run1("fc1_dgrad t32x64 w2x2", PFc1DgradT<32, 64, 2, 2>{grid(B, 32, 3136, 64, 1), dz4, W3, a3, dz3, B}, flop);
    run1("fc1_dgrad t128x64 w2x2", PFc1DgradT<128, 64, 2, 2>{grid(B, 128, 3136, 64, 1), dz4, W3, a3, dz3, B}, flop);
    run1("fc1_wgrad t64x32 w2x2", PFc1WgradT<64, 32, 2, 2>{grid(3136, 64, 512, 32, 1), a3, dz4, gw, gw, B}, flop);
    run1("fc1_wgrad t128x64 w2x2", PFc1WgradT<128, 64, 2, 2>{grid(3136, 128, 512, 64, 1), a3, dz4, gw, gw, B}, flop);
    run1("fc1_wgrad t64x128 w2x2", PFc1WgradT<64, 128, 2, 2>{grid(3136, 64, 512, 128, 1), a3, dz4, gw, gw, B}, flop);
    flop = 2.0 * B * 81 * 64 * 512;
    run1("conv2_fwd t64x32 w2x2", PConvFwd<20, 20, 32, 4, 2, 9, 9, 64, 64, 32, 2, 2>{grid(B * 81, 64, 64, 32, 1), a1, W1, W1, a2, B * 81}, flop);
    run1("conv2_fwd t32x64 w2x2", PConvFwd<20, 20, 32, 4, 2, 9, 9, 64, 32, 64, 2, 2>{grid(B * 81, 32, 64, 64, 1), a1, W1, W1, a2, B * 81}, flop);
    run1("conv2_fwd t128x64 w2x2", PConvFwd<20, 20, 32, 4, 2, 9, 9, 64, 128, 64, 2, 2>{grid(B * 81, 128, 64, 64, 1), a1, W1, W1, a2, B * 81}, flop);
    run1("conv2_fwd t128x64 w4x1", PConvFwd<20, 20, 32, 4, 2, 9, 9, 64, 128, 64, 4, 1>{grid(B * 81, 128, 64, 64, 1), a1, W1, W1, a2, B * 81}, flop);
    run1("conv2_dgrad t64x32 w2x2", PConv2DgradT<64, 32, 2, 2>{grid(B * 100, 64, 32, 32, 4), dz2, W1, a1, dz1, B * 100}, flop);
    run1("conv2_dgrad t64x32 w4x1", PConv2DgradT<64, 32, 4, 1>{grid(B * 100, 64, 32, 32, 4), dz2, W1, a1, dz1, B * 100}, flop);
    run1("conv2_dgrad t32x32 w2x2", PConv2DgradT<32, 32, 2, 2>{grid(B * 100, 32, 32, 32, 4), dz2, W1, a1, dz1, B * 100}, flop);
    run1("conv2_wgrad t64x32 w2x2", PConvWgrad<20, 20, 32, 4, 2, 9, 9, 64, 16, 64, 32, 2, 2>{grid(512, 64, 64, 32, B / 16), a1, dz2, slab, B}, flop);
    run1("conv2_wgrad t128x64 w2x2", PConvWgrad<20, 20, 32, 4, 2, 9, 9, 64, 16, 128, 64, 2, 2>{grid(512, 128, 64, 64, B / 16), a1, dz2, slab, B}, flop);
    flop = 2.0 * B * 49 * 64 * 576;
    run1("conv3_fwd t64x32 w2x2", PConvFwd<9, 9, 64, 3, 1, 7, 7, 64, 64, 32, 2, 2>{grid(B * 49, 64, 64, 32, 1), a2, W2, W2, a3, B * 49}, flop);
    run1("conv3_fwd t32x64 w2x2", PConvFwd<9, 9, 64, 3, 1, 7, 7, 64, 32, 64, 2, 2>{grid(B * 49, 32, 64, 64, 1), a2, W2, W2, a3, B * 49}, flop);
    run1("conv3_fwd t128x64 w2x2", PConvFwd<9, 9, 64, 3, 1, 7, 7, 64, 128, 64, 2, 2>{grid(B * 49, 128, 64, 64, 1), a2, W2, W2, a3, B * 49}, flop);
    run1("conv3_dgrad t64x32 w2x2", PConv3DgradT<64, 32, 2, 2>{grid(B * 81, 64, 64, 32, 1), dz3, W2, a2, dz2, B * 81}, flop);
    run1("conv3_dgrad t32x64 w2x2", PConv3DgradT<32, 64, 2, 2>{grid(B * 81, 32, 64, 64, 1), dz3, W2, a2, dz2, B * 81}, flop);
    run1("conv3_dgrad t128x64 w2x2", PConv3DgradT<128, 64, 2, 2>{grid(B * 81, 128, 64, 64, 1), dz3, W2, a2, dz2, B * 81}, flop);
    run1("conv3_wgrad t64x32 w2x2", PConvWgrad<9, 9, 64, 3, 1, 7, 7, 64, 16, 64, 32, 2, 2>{grid(576, 64, 64, 32, B / 16), a2, dz3, slab, B}, flop);
    printf("--- block order: column-tile fastest (shipped) vs row-tile fastest, B = 1024\n");
    {
      const int BB = 1024;
      const double f1 = 2.0 * BB * 3136 * 512, f2 = 2.0 * BB * 81 * 64 * 512;
      run1("fc1_fwd S colfast", PFc1FwdT<32, 32, 2, 2>{grid(BB, 32, 512, 32, 1), a3, W3, W3, a4, BB}, f1);
      run1("fc1_fwd S rowfast", RowFast<PFc1FwdT<32, 32, 2, 2>>{{grid(BB, 32, 512, 32, 1), a3, W3, W3, a4, BB}}, f1);
      run1("fc1_dgrad S colfast", PFc1DgradT<32, 64, 2, 2>{grid(BB, 32, 3136, 64, 1), dz4, W3, a3, dz3, BB}, f1);
      run1("fc1_dgrad S rowfast", RowFast<PFc1DgradT<32, 64, 2, 2>>{{grid(BB, 32, 3136, 64, 1), dz4, W3, a3, dz3, BB}}, f1);
      run1("fc1_wgrad S colfast", PFc1WgradT<64, 32, 2, 2>{grid(3136, 64, 512, 32, 1), a3, dz4, gw, gw, BB}, f1);
      run1("fc1_wgrad S rowfast", RowFast<PFc1WgradT<64, 32, 2, 2>>{{grid(3136, 64, 512, 32, 1), a3, dz4, gw, gw, BB}}, f1);
      run1("conv2_fwd S colfast", PConvFwd<20, 20, 32, 4, 2, 9, 9, 64, 64, 32, 2, 2>{grid(BB * 81, 64, 64, 32, 1), a1, W1, W1, a2, BB * 81}, f2);
      run1("conv2_fwd S rowfast", RowFast<PConvFwd<20, 20, 32, 4, 2, 9, 9, 64, 64, 32, 2, 2>>{{grid(BB * 81, 64, 64, 32, 1), a1, W1, W1, a2, BB * 81}}, f2);
    }
    printf("--- weight-gradient sample-chunk size, B = 1024\n");
    {
      const int BB = 1024;
      const double f3 = 2.0 * BB * 49 * 64 * 576, f2 = 2.0 * BB * 81 * 64 * 512;
      run1("conv3_wgrad sc16 t64x64", PConvWgrad<9, 9, 64, 3, 1, 7, 7, 64, 16>{grid(576, 64, 64, 64, BB / 16), a2, dz3, slab, BB}, f3);
      run1("conv3_wgrad sc8 t64x64", PConvWgrad<9, 9, 64, 3, 1, 7, 7, 64, 8>{grid(576, 64, 64, 64, BB / 8), a2, dz3, slab, BB}, f3);
      run1("conv3_wgrad sc4 t64x64", PConvWgrad<9, 9, 64, 3, 1, 7, 7, 64, 4>{grid(576, 64, 64, 64, BB / 4), a2, dz3, slab, BB}, f3);
      run1("conv3_wgrad sc32 t64x64", PConvWgrad<9, 9, 64, 3, 1, 7, 7, 64, 32>{grid(576, 64, 64, 64, BB / 32), a2, dz3, slab, BB}, f3);
      run1("conv2_wgrad sc16 t64x64", PConvWgrad<20, 20, 32, 4, 2, 9, 9, 64, 16>{grid(512, 64, 64, 64, BB / 16), a1, dz2, slab, BB}, f2);
      run1("conv2_wgrad sc8 t64x64", PConvWgrad<20, 20, 32, 4, 2, 9, 9, 64, 8>{grid(512, 64, 64, 64, BB / 8), a1, dz2, slab, BB}, f2);
      run1("conv2_wgrad sc4 t64x64", PConvWgrad<20, 20, 32, 4, 2, 9, 9, 64, 4>{grid(512, 64, 64, 64, BB / 4), a1, dz2, slab, BB}, f2);
      run1("conv2_wgrad sc32 t64x64", PConvWgrad<20, 20, 32, 4, 2, 9, 9, 64, 32>{grid(512, 64, 64, 64, BB / 32), a1, dz2, slab, BB}, f2);
      run1("conv2_wgrad sc8 t128x64", PConvWgrad<20, 20, 32, 4, 2, 9, 9, 64, 8, 128, 64, 2, 2>{grid(512, 128, 64, 64, BB / 8), a1, dz2, slab, BB}, f2);
      run1("conv3_wgrad sc8 t64x32", PConvWgrad<9, 9, 64, 3, 1, 7, 7, 64, 8, 64, 32, 2, 2>{grid(576, 64, 64, 32, BB / 8), a2, dz3, slab, BB}, f3);
    }
    printf("--- K-split wave groups, B = 1024 and 8192\n");
    for (int BB : {1024, 8192}) {
      const double f1 = 2.0 * BB * 3136 * 512, f2 = 2.0 * BB * 81 * 64 * 512, f3 = 2.0 * BB * 49 * 64 * 576;
      printf("B = %d\n", BB);
      run1("fc1_fwd t32x32 ks1", PFc1FwdT<32, 32, 2, 2>{grid(BB, 32, 512, 32, 1), a3, W3, W3, a4, BB}, f1);
      run1("fc1_fwd t32x32 ks2", KSplit<PFc1FwdT<32, 32, 2, 2>, 2>{{grid(BB, 32, 512, 32, 1), a3, W3, W3, a4, BB}}, f1);
      run1("fc1_fwd t64x32 ks2", KSplit<PFc1FwdT<64, 32, 2, 2>, 2>{{grid(BB, 64, 512, 32, 1), a3, W3, W3, a4, BB}}, f1);
      run1("fc1_fwd t32x64 ks2", KSplit<PFc1FwdT<32, 64, 2, 2>, 2>{{grid(BB, 32, 512, 64, 1), a3, W3, W3, a4, BB}}, f1);
      run1("fc1_fwd t64x64 ks2", KSplit<PFc1FwdT<64, 64, 2, 2>, 2>{{grid(BB, 64, 512, 64, 1), a3, W3, W3, a4, BB}}, f1);
      run1("fc1_fwd t32x32 ks4", KSplit<PFc1FwdT<32, 32, 2, 2>, 4>{{grid(BB, 32, 512, 32, 1), a3, W3, W3, a4, BB}}, f1);
      run1("fc1_fwd t64x64 ks4", KSplit<PFc1FwdT<64, 64, 2, 2>, 4>{{grid(BB, 64, 512, 64, 1), a3, W3, W3, a4, BB}}, f1);
      run1("conv2_fwd t64x32 ks1", PConvFwd<20, 20, 32, 4, 2, 9, 9, 64, 64, 32, 2, 2>{grid(BB * 81, 64, 64, 32, 1), a1, W1, W1, a2, BB * 81}, f2);
      run1("conv2_fwd t64x32 ks2", KSplit<PConvFwd<20, 20, 32, 4, 2, 9, 9, 64, 64, 32, 2, 2>, 2>{{grid(BB * 81, 64, 64, 32, 1), a1, W1, W1, a2, BB * 81}}, f2);
      run1("conv2_fwd t64x64 ks2", KSplit<PConvFwd<20, 20, 32, 4, 2, 9, 9, 64, 64, 64, 2, 2>, 2>{{grid(BB * 81, 64, 64, 64, 1), a1, W1, W1, a2, BB * 81}}, f2);
      run1("conv3_fwd t64x32 ks1", PConvFwd<9, 9, 64, 3, 1, 7, 7, 64, 64, 32, 2, 2>{grid(BB * 49, 64, 64, 32, 1), a2, W2, W2, a3, BB * 49}, f3);
      run1("conv3_fwd t64x32 ks2", KSplit<PConvFwd<9, 9, 64, 3, 1, 7, 7, 64, 64, 32, 2, 2>, 2>{{grid(BB * 49, 64, 64, 32, 1), a2, W2, W2, a3, BB * 49}}, f3);
      run1("conv3_fwd t64x64 ks2", KSplit<PConvFwd<9, 9, 64, 3, 1, 7, 7, 64, 64, 64, 2, 2>, 2>{{grid(BB * 49, 64, 64, 64, 1), a2, W2, W2, a3, BB * 49}}, f3);
      if (BB > 1024) continue;
      run1("fc1_dgrad t32x64 ks1", PFc1DgradT<32, 64, 2, 2>{grid(BB, 32, 3136, 64, 1), dz4, W3, a3, dz3, BB}, f1);
      run1("fc1_dgrad t32x64 ks2", KSplit<PFc1DgradT<32, 64, 2, 2>, 2>{{grid(BB, 32, 3136, 64, 1), dz4, W3, a3, dz3, BB}}, f1);
      run1("fc1_dgrad t64x64 ks2", KSplit<PFc1DgradT<64, 64, 2, 2>, 2>{{grid(BB, 64, 3136, 64, 1), dz4, W3, a3, dz3, BB}}, f1);
    }
    printf("--- pixel-major backward data\n");
    for (int BB : {1024, 8192}) {
      if (BB > Bmax) break;
      const double f3 = 2.0 * BB * 49 * 64 * 576, f2 = 2.0 * BB * 81 * 64 * 512;
      printf("B = %d\n", BB);
      run1("conv3_dgrad px t32x64 w2x2", PConv3DgradPx<32, 64, 2, 2>{grid(BB, 32, 64, 64, 81), dz3, W2, a2, dz2, BB}, f3);
      run1("conv3_dgrad px t64x64 w2x2", PConv3DgradPx<64, 64, 2, 2>{grid(BB, 64, 64, 64, 81), dz3, W2, a2, dz2, BB}, f3);
      run1("conv3_dgrad px t64x32 w2x2", PConv3DgradPx<64, 32, 2, 2>{grid(BB, 64, 64, 32, 81), dz3, W2, a2, dz2, BB}, f3);
      run1("conv3_dgrad px t128x64 w2x2", PConv3DgradPx<128, 64, 2, 2>{grid(BB, 128, 64, 64, 81), dz3, W2, a2, dz2, BB}, f3);
      run1("conv2_dgrad px t32x128 w2x2", PConv2DgradPx<32, 128, 2, 2>{grid(BB, 32, 128, 128, 100), dz2, W1, a1, dz1, BB}, f2);
      run1("conv2_dgrad px t64x64 w2x2", PConv2DgradPx<64, 64, 2, 2>{grid(BB, 64, 128, 64, 100), dz2, W1, a1, dz1, BB}, f2);
      run1("conv2_dgrad px t32x64 w2x2", PConv2DgradPx<32, 64, 2, 2>{grid(BB, 32, 128, 64, 100), dz2, W1, a1, dz1, BB}, f2);
      run1("conv2_dgrad px t64x128 w2x2", PConv2DgradPx<64, 128, 2, 2>{grid(BB, 64, 128, 128, 100), dz2, W1, a1, dz1, BB}, f2);
      run1("conv2_dgrad all t64x128 w2x2", PConv2DgradAll<64, 128, 2, 2>{grid(BB * 100, 64, 128, 128, 1), dz2, W1, a1, dz1, BB * 100}, f2);
      run1("conv2_dgrad all t64x64 w2x2", PConv2DgradAll<64, 64, 2, 2>{grid(BB * 100, 64, 128, 64, 1), dz2, W1, a1, dz1, BB * 100}, f2);
      run1("conv2_dgrad all t128x64 w2x2", PConv2DgradAll<128, 64, 2, 2>{grid(BB * 100, 128, 128, 64, 1), dz2, W1, a1, dz1, BB * 100}, f2);
      run1("conv2_dgrad (shipped S)", PConv2DgradS{grid(BB * 100, 64, 32, 32, 4), dz2, W1, a1, dz1, BB * 100}, f2);
      run1("conv3_dgrad (shipped S)", PConv3DgradS{grid(BB * 81, 32, 64, 64, 1), dz3, W2, a2, dz2, BB * 81}, f3);
    }
    printf("--- MF 32 (v_mfma_f32_32x32x2_f32) variants\n");
    for (int BB : {1024, 8192}) {
      double f2 = 2.0 * BB * 81 * 64 * 512, f3 = 2.0 * BB * 49 * 64 * 576, f1 = 2.0 * BB * 3136 * 512;
      printf("B = %d\n", BB);
      run1("conv2_fwd t64x64 w2x2 mf32", PConvFwd<20, 20, 32, 4, 2, 9, 9, 64, 64, 64, 2, 2, 32>{grid(BB * 81, 64, 64, 64, 1), a1, W1, W1, a2, BB * 81}, f2);
      run1("conv2_fwd t128x32 w4x1 mf32", PConvFwd<20, 20, 32, 4, 2, 9, 9, 64, 128, 32, 4, 1, 32>{grid(BB * 81, 128, 64, 32, 1), a1, W1, W1, a2, BB * 81}, f2);
      run1("conv2_fwd t128x64 w4x1 mf32", PConvFwd<20, 20, 32, 4, 2, 9, 9, 64, 128, 64, 4, 1, 32>{grid(BB * 81, 128, 64, 64, 1), a1, W1, W1, a2, BB * 81}, f2);
      run1("conv3_fwd t64x64 w2x2 mf32", PConvFwd<9, 9, 64, 3, 1, 7, 7, 64, 64, 64, 2, 2, 32>{grid(BB * 49, 64, 64, 64, 1), a2, W2, W2, a3, BB * 49}, f3);
      run1("conv3_fwd t128x32 w4x1 mf32", PConvFwd<9, 9, 64, 3, 1, 7, 7, 64, 128, 32, 4, 1, 32>{grid(BB * 49, 128, 64, 32, 1), a2, W2, W2, a3, BB * 49}, f3);
      run1("fc1_fwd t64x64 w2x2 mf32", PFc1FwdT<64, 64, 2, 2, 32>{grid(BB, 64, 512, 64, 1), a3, W3, W3, a4, BB}, f1);
      run1("fc1_fwd t32x128 w1x4 mf32", PFc1FwdT<32, 128, 1, 4, 32>{grid(BB, 32, 512, 128, 1), a3, W3, W3, a4, BB}, f1);
      if (BB > 1024) continue;
      run1("fc1_dgrad t64x64 w2x2 mf32", PFc1DgradT<64, 64, 2, 2, 32>{grid(BB, 64, 3136, 64, 1), dz4, W3, a3, dz3, BB}, f1);
      run1("fc1_dgrad t128x32 w4x1 mf32", PFc1DgradT<128, 32, 4, 1, 32>{grid(BB, 128, 3136, 32, 1), dz4, W3, a3, dz3, BB}, f1);
      run1("conv3_dgrad t64x64 w2x2 mf32", PConv3DgradT<64, 64, 2, 2, 32>{grid(BB * 81, 64, 64, 64, 1), dz3, W2, a2, dz2, BB * 81}, f3);
      run1("conv3_dgrad t128x32 w4x1 mf32", PConv3DgradT<128, 32, 4, 1, 32>{grid(BB * 81, 128, 64, 32, 1), dz3, W2, a2, dz2, BB * 81}, f3);
      run1("conv2_dgrad t128x32 w4x1 mf32", PConv2DgradT<128, 32, 4, 1, 32>{grid(BB * 100, 128, 32, 32, 4), dz2, W1, a1, dz1, BB * 100}, f2);
    }
#undef V
  }
  printf("--- generic GEMM (A row-major, B row-major)\n");
  {
    const int M = 8192, N = 4096, K = 4096;
    float* A = dbuf((size_t)65536 * 4 * 256, 20);
    float* B = dbuf((size_t)K * N, 21);
    float* C = dbuf((size_t)M * N, 22);
    gen32p<64, 64, 2, 2>(M, N, K, A, B, C);
    gen32p<128, 64, 2, 2>(M, N, K, A, B, C);
    gen32p<128, 128, 2, 2>(M, N, K, A, B, C);
    gen32p<64, 64, 2, 2>(65536, 64, 512, A, B, C);
    gen32p<128, 64, 2, 2>(65536, 64, 512, A, B, C);
    gen32p<128, 64, 4, 1>(65536, 64, 512, A, B, C);
    gen<64, 64, 2, 2>(M, N, K, A, B, C);
    gen32<64, 64, 2, 2, 36>(M, N, K, A, B, C);
    gen32<128, 64, 2, 2, 36>(M, N, K, A, B, C);
    gen32<128, 128, 2, 2, 36>(M, N, K, A, B, C);
    gen32<64, 64, 2, 2, 40>(M, N, K, A, B, C);
    gen32<64, 64, 2, 2, 36>(65536, 64, 512, A, B, C);
    gen32<128, 64, 2, 2, 36>(65536, 64, 512, A, B, C);
    gen<64, 64, 2, 2>(65536, 64, 512, A, B, C);
    gen<128, 64, 2, 2>(65536, 64, 512, A, B, C);
    gen<64, 32, 4, 1>(65536 * 4, 32, 256, A, B, C);
    gen<128, 32, 4, 1>(65536 * 4, 32, 256, A, B, C);
  }
  return 0;
}
