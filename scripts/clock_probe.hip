// Shader clock under a chip-wide fp32 MFMA load: every wave of a full grid runs independent v_mfma_f32_16x16x4_f32
// chains; lane 0 of each wave records s_memtime (shader clock) and s_memrealtime (100 MHz constant clock) around its
// loop.  Prints the effective clock and the achieved fp32 MFMA rate, i.e. the peak the fp32 kernels can reach on
// this box (the 157.3 TFLOP/s of MI355X_MICROARCH.md assumes the 2.4 GHz peak engine clock).
//   hipcc --offload-arch=gfx950 -O3 scripts/clock_probe.hip -o clock_probe && ./clock_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));        \
      return 1;                                                                       \
    }                                                                                 \
  } while (0)

__global__ __launch_bounds__(256) void k_mfma_load(int iters, float seed, float* out, unsigned long long* stamps) {
  f32x4 acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
  const float a = seed + threadIdx.x * 1e-7f, b = seed - threadIdx.x * 1e-7f;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0.0f;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  const int w = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
  if ((threadIdx.x & 63) == 0) {
    out[w] = s;
    stamps[4 * w + 0] = t0;
    stamps[4 * w + 1] = t1;
    stamps[4 * w + 2] = r0;
    stamps[4 * w + 3] = r1;
  }
}

int main(int argc, char** argv) {
  const int wps = argc > 1 ? atoi(argv[1]) : 2;   // waves per SIMD
  int dev = 0, cus = 0, wall_khz = 0, clk_khz = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  CK(hipDeviceGetAttribute(&wall_khz, hipDeviceAttributeWallClockRate, dev));
  CK(hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, dev));
  printf("%d CUs, s_memrealtime %d kHz, reported peak engine clock %d MHz\n", cus, wall_khz, clk_khz / 1000);
  const int blocks = cus * wps, waves = blocks * 4;   // wps waves per SIMD, 8 independent chains each
  float* out = nullptr;
  unsigned long long* st = nullptr;
  CK(hipMalloc(&out, waves * sizeof(float)));
  CK(hipMalloc(&st, waves * 4 * sizeof(unsigned long long)));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int rep = 0; rep < 4; ++rep) {
    const int iters = 80000 / wps;   // 8 MFMAs per iteration (~20 ms per launch)
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_mfma_load, dim3(blocks), dim3(256), 0, 0, iters, 1.0f + rep, out, st);
    CK(hipGetLastError());
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0.0f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<unsigned long long> h(waves * 4);
    CK(hipMemcpy(h.data(), st, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    double ratio = 0.0;
    for (int w = 0; w < waves; ++w) ratio += (double)(h[4 * w + 1] - h[4 * w]) / (double)(h[4 * w + 3] - h[4 * w + 2]);
    ratio /= waves;
    const double flop = 2.0 * 16 * 16 * 4 * 8.0 * iters * waves;
    printf("%d waves/SIMD rep %d: %.3f ms, %.1f TFLOP/s fp32 MFMA, shader clock %.0f MHz (s_memtime / s_memrealtime x its rate)\n", wps, rep, ms,
           flop / ms / 1e9, ratio * wall_khz / 1000.0);
  }
  return 0;
}
