// Do fp32 MFMA and fp32 VALU FMA execute together?  Every SIMD runs one (or two) waves of independent
// v_mfma_f32_16x16x4_f32 chains and/or one (or two) waves of independent v_fma_f32 chains; the launch time gives each
// pipe's rate alone and side by side.  If the side-by-side rate is near the sum, a GEMM can give part of its outputs to
// the VALU (a fmaf chain in k order is bit for bit what the MFMA computes: scripts/mfma_f32_probe.hip).
//   hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize scripts/coexec_probe.hip -o coexec_probe && ./coexec_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));        \
      return 1;                                                                       \
    }                                                                                 \
  } while (0)

// mode bit 0: the first half of the block's waves run MFMA chains; bit 1: the second half run VALU chains (plain
// v_fma_f32 when pk == 0, v_pk_fma_f32 when pk == 1).  Waves not given work exit at once.
template <int PK>
__global__ __launch_bounds__(1024) void k_coexec(int mode, int iters_m, int iters_v, float seed, float* out) {
  const int wave = threadIdx.x >> 6, half = (blockDim.x >> 6) / 2;
  float s = 0.0f;
  if (wave < half) {
    if (!(mode & 1)) return;
    f32x4 acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    const float a = seed + threadIdx.x * 1e-7f, b = seed - threadIdx.x * 1e-7f;
    for (int it = 0; it < iters_m; ++it) {
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  } else {
    if (!(mode & 2)) return;
    if (PK) {
      f32x2 acc[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[i] = f32x2{(float)i, (float)-i};
      const f32x2 a = f32x2{seed + threadIdx.x * 1e-7f, seed}, b = f32x2{1.0f - threadIdx.x * 1e-9f, 0.999f};
      for (int it = 0; it < iters_v; ++it) {
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[i] = __builtin_elementwise_fma(a, acc[i], b);
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) s += acc[i][0] + acc[i][1];
    } else {
      float acc[32];
#pragma unroll
      for (int i = 0; i < 32; ++i) acc[i] = (float)i;
      const float a = seed + threadIdx.x * 1e-7f, b = 1.0f - threadIdx.x * 1e-9f;
      for (int it = 0; it < iters_v; ++it) {
#pragma unroll
        for (int i = 0; i < 32; ++i) acc[i] = fmaf(a, acc[i], b);
      }
#pragma unroll
      for (int i = 0; i < 32; ++i) s += acc[i];
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// one wave per SIMD: MFMA chains with V independent VALU fmas after every MFMA (the same wave) - the price of a
// VALU instruction inside an fp32 MFMA loop
template <int V>
__global__ __launch_bounds__(256) void k_inter(int iters, float seed, float* out) {
  f32x4 acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
  float x[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) x[i] = (float)i;
  const float a = seed + threadIdx.x * 1e-7f, b = seed - threadIdx.x * 1e-7f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
#pragma unroll
      for (int v = 0; v < V; ++v) x[(i * V + v) & 15] = fmaf(a, x[(i * V + v) & 15], b);
    }
  }
  float s = 0.0f;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
#pragma unroll
  for (int i = 0; i < 16; ++i) s += x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int V>
static int run_inter(int blocks, float* out, hipEvent_t e0, hipEvent_t e1) {
  const int iters = 40000;
  for (int rep = 0; rep < 2; ++rep) {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_inter<V>, dim3(blocks), dim3(256), 0, 0, iters, 1.0f + rep, out);
    CK(hipGetLastError());
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0.0f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double cyc = ms * 1e-3 * 2.4e9 / (8.0 * iters);   // cycles per MFMA at 2.4 GHz
    printf("interleaved: %d VALU fma per MFMA rep %d: %.3f ms, %.1f cycles per (MFMA + %d VALU), MFMA %.1f TF\n", V, rep, ms, cyc,
           V, 8.0 * 2048.0 * iters * blocks * 4 / ms / 1e9);
  }
  return 0;
}

int main(int argc, char** argv) {
  const int wps = argc > 1 ? atoi(argv[1]) : 1;   // waves of each kind per SIMD
  int dev = 0, cus = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const int threads = 2 * 4 * wps * 64;   // wps MFMA waves + wps VALU waves per SIMD
  const int blocks = cus;
  float* out = nullptr;
  CK(hipMalloc(&out, (size_t)blocks * threads * sizeof(float)));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int iters_m = 40000, iters_v = 40000;
  // flops per launch of each part: MFMA 8 x 2048 per iteration per wave; VALU 32 fma x 64 lanes x 2 (pk: 16 x 2 fma)
  const double f_m = 8.0 * 2048.0 * iters_m * blocks * 4 * wps;
  const double f_v = 32.0 * 64.0 * 2.0 * iters_v * blocks * 4 * wps;
  if (wps == 1) {
    if (run_inter<0>(blocks, out, e0, e1) || run_inter<1>(blocks, out, e0, e1) || run_inter<2>(blocks, out, e0, e1) ||
        run_inter<4>(blocks, out, e0, e1) || run_inter<8>(blocks, out, e0, e1))
      return 1;
  }
  for (int pk = 0; pk < 2; ++pk)
    for (int mode = 1; mode <= 3; ++mode)
      for (int rep = 0; rep < 3; ++rep) {
        CK(hipEventRecord(e0));
        if (pk) hipLaunchKernelGGL(k_coexec<1>, dim3(blocks), dim3(threads), 0, 0, mode, iters_m, iters_v, 1.0f + rep, out);
        else hipLaunchKernelGGL(k_coexec<0>, dim3(blocks), dim3(threads), 0, 0, mode, iters_m, iters_v, 1.0f + rep, out);
        CK(hipGetLastError());
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0.0f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double fm = (mode & 1) ? f_m : 0.0, fv = (mode & 2) ? f_v : 0.0;
        printf("%s waves/SIMD %d mode %s rep %d: %.3f ms  MFMA %.1f TF  VALU %.1f TF  sum %.1f TF\n", pk ? "pk_fma" : "fma   ", wps,
               mode == 1 ? "mfma " : (mode == 2 ? "valu " : "both "), rep, ms, fm / ms / 1e9, fv / ms / 1e9, (fm + fv) / ms / 1e9);
      }
  return 0;
}
