// What sets the conv weight-gradient chunk reduction's time (k_wreduce32, ~11 us for ~26 MB at B = 1024)?
// The same two-level chain (groups of 16 chunks, then over the groups) over a conv3-sized slab (64 chunks x 36,928
// outputs) in two layouts:
//   A chunk-major  [z][e]            (shipped: each wave reads 256 B from 64 rows 147 KB apart)
//   B block-major  [e / 64][z][64]   (each wave reads its 64 outputs' 64 chunks as one 16 KB run)
// and a plain streaming copy-reduce of the same bytes as the bandwidth reference.
//   hipcc --offload-arch=gfx950 -O3 scripts/wred_probe.hip -o scripts/wred_probe && ./scripts/wred_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

constexpr int kG = 16;

// one output per lane; waves per block W; the lane's 64 chunks in 4 groups, all loads issued at once
template <bool BLOCKMAJOR>
__global__ __launch_bounds__(256) void k_red(const float* slab, int count, int nz, float* out) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= count) return;
  const int ng = nz / kG;
  float t = 0.0f;
  for (int q0 = 0; q0 < ng; q0 += 4) {
    float v[4][kG];
#pragma unroll
    for (int qq = 0; qq < 4; ++qq)
#pragma unroll
      for (int j = 0; j < kG; ++j) {
        const int z = (q0 + qq) * kG + j;
        size_t idx = BLOCKMAJOR ? ((size_t)(e >> 6) * nz + z) * 64 + (e & 63) : (size_t)z * count + e;
        v[qq][j] = q0 + qq < ng ? slab[idx] : 0.0f;
      }
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
      float s = 0.0f;
#pragma unroll
      for (int j = 0; j < kG; ++j) s = __fadd_rn(s, v[qq][j]);
      t = __fadd_rn(t, s);
    }
  }
  out[e] = t;
}

// the shipped form: 1024-thread blocks of 64 outputs x 16 group waves
__global__ __launch_bounds__(1024) void k_red_shipped(const float* slab, int count, int nz, float* out) {
  __shared__ float gs[128 * 64];
  const int o = threadIdx.x & 63, g0 = threadIdx.x >> 6;
  const int e = blockIdx.x * 64;
  const bool live = e + o < count;
  const int ng = nz / kG;
  const float* p = slab + e + (live ? o : 0);
  for (int q = g0; q < ng; q += 16) {
    float v[kG];
#pragma unroll
    for (int j = 0; j < kG; ++j) v[j] = p[(size_t)(q * kG + j) * count];
    float t = 0.0f;
#pragma unroll
    for (int j = 0; j < kG; ++j) t = __fadd_rn(t, v[j]);
    gs[q * 64 + o] = t;
  }
  __syncthreads();
  if (g0 != 0 || !live) return;
  float t = 0.0f;
  for (int q = 0; q < ng; ++q) t = __fadd_rn(t, gs[q * 64 + o]);
  out[e + o] = t;
}

// streaming reference: each thread sums 16 float4 of a contiguous run
__global__ __launch_bounds__(256) void k_stream(const float4* x, size_t n4, float* out) {
  const size_t t = (size_t)blockIdx.x * 256 + threadIdx.x, st = (size_t)gridDim.x * 256;
  float s = 0.0f;
  for (size_t i = t; i < n4; i += st) {
    const float4 v = x[i];
    s += v.x + v.y + v.z + v.w;
  }
  out[t] = s;
}

int main() {
  const int count = 577 * 64, nz = 64, reps = 20;
  const size_t n = (size_t)count * nz;
  float *a = nullptr, *b = nullptr, *oa = nullptr, *ob = nullptr, *os = nullptr;
  CK(hipMalloc(&a, n * 4));
  CK(hipMalloc(&b, n * 4));
  CK(hipMalloc(&oa, count * 4));
  CK(hipMalloc(&ob, count * 4));
  CK(hipMalloc(&os, 1 << 22));
  std::vector<float> h(n), hb(n);
  for (size_t i = 0; i < n; ++i) h[i] = (float)((i * 2654435761u) % 1000) * 1e-3f - 0.5f;
  for (int z = 0; z < nz; ++z)
    for (int e = 0; e < count; ++e) hb[((size_t)(e >> 6) * nz + z) * 64 + (e & 63)] = h[(size_t)z * count + e];
  CK(hipMemcpy(a, h.data(), n * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(b, hb.data(), n * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  // a 256 MB buffer written between reps evicts the slabs from L2 / MALL, as in place (the slabs come from HBM there too)
  float* junk = nullptr;
  const size_t nj = (size_t)64 << 20;
  CK(hipMalloc(&junk, nj * 4));
  auto timeit = [&](const char* name, auto launch) -> int {
    float tot = 0.0f, best = 1e9f;
    for (int r = 0; r < reps; ++r) {
      CK(hipMemsetAsync(junk, r, nj * 4));
      CK(hipEventRecord(e0));
      launch();
      CK(hipGetLastError());
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0.0f;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (r >= 2) tot += ms;
      if (ms < best) best = ms;
    }
    const float avg = tot / (reps - 2);
    printf("%-28s avg %.2f us  best %.2f us  %.2f TB/s\n", name, avg * 1e3f, best * 1e3f, n * 4.0 / (avg * 1e-3) / 1e12);
    return 0;
  };
  const int nb = (count + 255) / 256;
  if (timeit("shipped (1024 thr, [z][e])", [&] { hipLaunchKernelGGL(k_red_shipped, dim3(count / 64), dim3(1024), 0, 0, a, count, nz, oa); }) ||
      timeit("lane-all-groups [z][e]", [&] { hipLaunchKernelGGL(k_red<false>, dim3(nb), dim3(256), 0, 0, a, count, nz, ob); }) ||
      timeit("lane-all-groups [e/64][z][64]", [&] { hipLaunchKernelGGL(k_red<true>, dim3(nb), dim3(256), 0, 0, b, count, nz, ob); }) ||
      timeit("stream", [&] { hipLaunchKernelGGL(k_stream, dim3(1024), dim3(256), 0, 0, (const float4*)a, n / 4, os); }))
    return 1;
  std::vector<float> ra(count), rb(count);
  CK(hipMemcpy(ra.data(), oa, count * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(rb.data(), ob, count * 4, hipMemcpyDeviceToHost));
  int bad = 0;
  for (int e = 0; e < count; ++e) bad += ra[e] != rb[e];
  printf("mismatches %d\n", bad);
  return bad != 0;
}
