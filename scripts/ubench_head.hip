// Microbenchmark of the fp32 dense-3 head (k_head32 of qnet32.hip) taken apart: operand loads alone, the MFMA chain
// alone, and both, at B = 1024 and 8192.  Dev tool:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o scripts/ubench_head scripts/ubench_head.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); std::exit(1); } } while (0)

// V: 0 = loads + chain (as shipped), 1 = loads only (sum), 2 = chain only (register operands), 3 = loads + chain with
// the 16 samples of a wave spread as 4 k-quarters (4 chains, wrong order: a bound on what splitting k would give)
template <int V>
__global__ __launch_bounds__(256) void k_head(const float* a4, const float* w4, int B, float* out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int s0 = (blockIdx.x * 4 + wave) * 16;
  if (s0 >= B) return;
  const int j = lane & 15, g = lane >> 4, n = lane & 15;
  const int b = s0 + j;
  const float* x = a4 + (size_t)b * 512 + g;
  f32x4 acc = f32x4{0, 0, 0, 0};
  if (V == 2) {
    float xv = x[0], wv = w4[g * 3 + (n < 3 ? n : 0)];
#pragma unroll
    for (int t = 0; t < 128; ++t) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wv, xv, acc, 0, 0, 0);
  } else {
    float xv[128];
#pragma unroll
    for (int t = 0; t < 128; ++t) xv[t] = x[4 * t];
    if (V == 1) {
      float s = 0;
#pragma unroll
      for (int t = 0; t < 128; ++t) s += xv[t];
      acc[0] = s;
    } else {
      const float* wp = w4 + g * 3 + (n < 3 ? n : 0);
#pragma unroll
      for (int t0 = 0; t0 < 128; t0 += 32) {
        float wv[32];
#pragma unroll
        for (int i = 0; i < 32; ++i) wv[i] = wp[(t0 + i) * 12];
#pragma unroll
        for (int i = 0; i < 32; ++i) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(n < 3 ? wv[i] : 0.0f, xv[t0 + i], acc, 0, 0, 0);
      }
    }
  }
  if (g == 0) out[b] = acc[0] + acc[1] + acc[2];
}

// one wave per 4 samples: x loaded as float4 rows (coalesced 2 KB per sample), q by VALU fmaf chains (the same
// k-ordered chain per output), then no MFMA at all
__global__ __launch_bounds__(256) void k_head_valu(const float* a4, const float* w4, int B, float* out) {
  __shared__ float ws[512 * 3];
  for (int i = threadIdx.x; i < 1536; i += 256) ws[i] = w4[i];
  __syncthreads();
  const int b = blockIdx.x * 256 + threadIdx.x;   // one sample per thread
  if (b >= B) return;
  const float* x = a4 + (size_t)b * 512;
  float q0 = 0, q1 = 0, q2 = 0;
#pragma unroll 8
  for (int k = 0; k < 512; k += 4) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(x + k);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      q0 = fmaf(v[e], ws[(k + e) * 3 + 0], q0);
      q1 = fmaf(v[e], ws[(k + e) * 3 + 1], q1);
      q2 = fmaf(v[e], ws[(k + e) * 3 + 2], q2);
    }
  }
  out[b] = q0 + q1 + q2;
}

template <class F>
static double time_us(F f, int reps = 30) {
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

int main() {
  const int Bmax = 8192;
  float *a4, *w4, *out;
  CK(hipMalloc(&a4, (size_t)Bmax * 512 * 4));
  CK(hipMalloc(&w4, 1539 * 4));
  CK(hipMalloc(&out, Bmax * 4));
  std::vector<float> h((size_t)Bmax * 512);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 2654435761u) % 1000) * 1e-3f;
  CK(hipMemcpy(a4, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(w4, h.data(), 1539 * 4, hipMemcpyHostToDevice));
  for (int B : {1024, 8192}) {
    const dim3 g((B + 63) / 64), blk(256);
    std::printf("B %5d  shipped %7.2f us  loads-only %7.2f us  chain-only %7.2f us  valu %7.2f us\n", B,
                time_us([&] { hipLaunchKernelGGL(k_head<0>, g, blk, 0, 0, a4, w4, B, out); }),
                time_us([&] { hipLaunchKernelGGL(k_head<1>, g, blk, 0, 0, a4, w4, B, out); }),
                time_us([&] { hipLaunchKernelGGL(k_head<2>, g, blk, 0, 0, a4, w4, B, out); }),
                time_us([&] { hipLaunchKernelGGL(k_head_valu, dim3((B + 255) / 256), blk, 0, 0, a4, w4, B, out); }));
  }
  std::printf("empty launch %7.2f us\n", time_us([&] { hipLaunchKernelGGL(k_head<2>, dim3(1), dim3(64), 0, 0, a4, w4, 0, out); }));
  return 0;
}
