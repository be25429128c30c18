// conv1 fp32 weight-gradient / forward probe (development tool, not part of the product): where the time of
// k_conv1_wgrad32 / k_conv1_fwd32 goes at B = 1024.  Variants of the weight-gradient structure (MODE: 0 as shipped,
// 1 no MFMA loop, 2 no reload after the first sample, 3 loop only), frame sets (live: every step non-zero, band: rows
// 16..47 non-zero, zero: null table) and frame placement (packed: consecutive frames, scattered: random frames of a
// 7 GB replay-sized buffer, as the learner's sampled batches are).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I include -I q-learning_amd/csrc scripts/c1_probe.hip \
//         -o scripts/c1_probe && ./scripts/c1_probe
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

// k_conv1_wgrad32 with parts switched off (MODE) and the chunk size SC as a parameter
template <int MODE, int SC>
__global__ __launch_bounds__(256, 2) void k_c1w(const uint8_t* const* table, const float* dz1, int B, int nz, float* slab, int skip) {
  extern __shared__ __attribute__((aligned(16))) uint32_t c1w[];
  float* dzs = reinterpret_cast<float*>(c1w + 4 * kC1SlotDw);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int z = blockIdx.x % nz, hh = blockIdx.x / nz;
  const int g = lane >> 4, l15 = lane & 15;
  const int b0 = z * SC;
  const int nb = min(SC, B - b0);
  const int ao = (l15 & 3) * kC1SlotDw + (2 * wave + (l15 >> 3)) * 21 + ((l15 >> 2) & 1);
  uint4 pf[14];
  auto prefetch = [&](int b) {
    const C1Ptrs f = c1_ptrs(table, b);
    const uint64_t zp = (uint64_t)(gbyte*)q32_zero4;
    const uint64_t dzb = (uint64_t)(dz1 + (size_t)b * 400 * 32 + hh * 16);
#pragma unroll
    for (int j = 0; j < 14; ++j) {
      const int q = tid + 256 * j;
      const bool isf = q < kC1Chunks, isd = !isf && q < kC1Chunks + kC1DzChunks;
      const int qf = isf ? q : 0, slot = qf / 441, pos = qf - slot * 441;
      const int e = isd ? q - kC1Chunks : 0, r = e >> 2, part = e & 3;
      const uint64_t fp = (uint64_t)c1_slot(f, slot);
      const uint64_t fa = fp ? fp + (uint64_t)(pos * 16) : zp;
      const uint64_t da = dzb + (uint64_t)((r * 32 + part * 4) * 4);
      const u32x4v v = *(gu4*)(isf ? fa : (isd ? da : zp));
      pf[j] = uint4{v.x, v.y, v.z, v.w};
    }
  };
  auto stage = [&]() {
#pragma unroll
    for (int j = 0; j < 14; ++j) {
      const int q = tid + 256 * j;
      if (q < kC1Chunks) c1_put(c1w, q, pf[j]);
      else if (q < kC1Chunks + kC1DzChunks) *reinterpret_cast<uint4*>(dzs + (q - kC1Chunks) * 4) = pf[j];
    }
  };
  f32x4 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = zero4();
  float bsum = 0.0f;
  prefetch(b0);
  if (MODE == 3) {
    stage();
    __syncthreads();
  }
  for (int bl = 0; bl < nb; ++bl) {
    if (MODE != 3) {
      __syncthreads();
      stage();
      __syncthreads();
      if (bl + 1 < nb && (MODE != 2)) prefetch(b0 + bl + 1);
    }
    if (MODE != 1) {
#pragma unroll 10
      for (int rs = 0; rs < 100; ++rs) {
        const int r = 4 * rs + g, oh = r / 20, ow = r - oh * 20;
        const float bv = dzs[r * 16 + l15];
        const uint32_t px = c1w[ao + 84 * oh + ow];
        if (!skip || __builtin_amdgcn_ballot_w64(px != 0u) != 0)
#pragma unroll
          for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(ubyte(px, t), bv, acc[t], 0, 0, 0);
        if (wave == 0) bsum = __fadd_rn(bsum, bv);
      }
    }
  }
  float* out = slab + (size_t)z * 257 * 32;
  const int oc = hh * 16 + l15;
  if (wave == 0) {
    const float c1 = __shfl(bsum, lane + 16), c2 = __shfl(bsum, lane + 32), c3 = __shfl(bsum, lane + 48);
    if (g == 0) out[256 * 32 + oc] = __fadd_rn(__fadd_rn(__fadd_rn(bsum, c1), c2), c3);
  }
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rho = 4 * g + i, kh = 2 * wave + (rho >> 3), kw = 4 * ((rho >> 2) & 1) + t, c = rho & 3;
      out[(size_t)((kh * 8 + kw) * 4 + c) * 32 + oc] = acc[t][i];
    }
}

int main(int argc, char** argv) {
  const int B = 1024;
  // frames: packed (B * 4 consecutive 7056-byte frames) and scattered (random 16-byte-aligned frames in 7 GB)
  const size_t big = (size_t)7 << 30;
  uint8_t* pool = nullptr;
  CK(hipMalloc(&pool, big));
  std::mt19937_64 rng(7);
  std::vector<uint8_t> live(7056, 7), band(7056, 0);
  // s2d chunk layout (441 chunks of 16 B: 4 x 4 pixel blocks); band: image rows 16..47 non-zero
  for (int c = 0; c < 441; ++c) {
    const int bx = c / 21;
    if (bx >= 4 && bx < 12)
      for (int i = 0; i < 16; ++i) band[c * 16 + i] = 9;
  }
  std::vector<const uint8_t*> packed(B * 4), scat(B * 4);
  std::vector<size_t> offs(B * 4);
  for (int i = 0; i < B * 4; ++i) {
    packed[i] = pool + (size_t)i * 7056;
    const size_t lo = (size_t)B * 4 * 7056 + 8192, hi = big - 8192;   // past the packed frames, 7056 + pad below the end
    offs[i] = lo + (rng() % ((hi - lo) / 16)) * 16;
    scat[i] = pool + offs[i];
  }
  const uint8_t** tp = nullptr;
  const uint8_t** ts = nullptr;
  const uint8_t** tz = nullptr;
  CK(hipMalloc(&tp, B * 4 * sizeof(void*)));
  CK(hipMalloc(&ts, B * 4 * sizeof(void*)));
  CK(hipMalloc(&tz, B * 4 * sizeof(void*)));
  CK(hipMemcpy(tp, packed.data(), B * 4 * sizeof(void*), hipMemcpyHostToDevice));
  CK(hipMemcpy(ts, scat.data(), B * 4 * sizeof(void*), hipMemcpyHostToDevice));
  CK(hipMemset(tz, 0, B * 4 * sizeof(void*)));
  auto fill = [&](const std::vector<uint8_t>& img) {
    for (int i = 0; i < B * 4; ++i) {
      CK(hipMemcpy((void*)packed[i], img.data(), 7056, hipMemcpyHostToDevice));
      CK(hipMemcpy((void*)scat[i], img.data(), 7056, hipMemcpyHostToDevice));
    }
  };
  float *dz1 = nullptr, *slab = nullptr, *a1 = nullptr, *w = nullptr;
  CK(hipMalloc(&dz1, (size_t)B * 12800 * 4));
  CK(hipMalloc(&a1, (size_t)B * 12800 * 4));
  CK(hipMalloc(&slab, (size_t)B * 257 * 32 * 4));   // one 257 x 32 slab per chunk; chunk size 1 has B of them
  CK(hipMalloc(&w, 8192 * 4 + 128));
  CK(hipMemset(dz1, 0, (size_t)B * 12800 * 4));
  CK(hipMemset(w, 0, 8192 * 4 + 128));
  const int lds = kC1Frames + 400 * 16 * 4;
  CK(hipFuncSetAttribute((const void*)k_conv1_wgrad32, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  CK(hipFuncSetAttribute((const void*)k_conv1_fwd32<0>, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * kC1Frames));
#define SETL(M, S) CK(hipFuncSetAttribute((const void*)k_c1w<M, S>, hipFuncAttributeMaxDynamicSharedMemorySize, lds))
  SETL(0, 4); SETL(1, 4); SETL(2, 4); SETL(3, 4); SETL(0, 8); SETL(0, 2); SETL(0, 1);
  for (int i = 0; i < B * 4; ++i)
    if (scat[i] < pool || scat[i] + 7056 > pool + big || packed[i] + 7056 > pool + big) { fprintf(stderr, "frame out of range\n"); return 1; }
  const char* fnames[2] = {"live", "band"};
  for (int f = 0; f < 2; ++f) {
    fill(f == 0 ? live : band);
    for (int place = 0; place < 3; ++place) {
      const uint8_t* const* t = place == 0 ? tp : place == 1 ? ts : tz;
      const char* pn = place == 0 ? "packed" : place == 1 ? "scattered" : "zero";
      if (place == 2 && f == 1) continue;
      printf("--- frames %s %s\n", place == 2 ? "zero" : fnames[f], pn);
      const int nz = B / 4;
      const double us_w = time_us([&] { hipLaunchKernelGGL(k_conv1_wgrad32, dim3(2 * nz), dim3(kC1WgradThreads), lds, 0, t, dz1, B, nz, slab, 1); });
      const double us_f = time_us([&] { hipLaunchKernelGGL(k_conv1_fwd32<0>, dim3(512), dim3(256), 2 * kC1Frames, 0, t, B, w, w + 8192, a1, 1, C1Lists{}); });
      printf("  shipped: wgrad %7.2f us  fwd %7.2f us\n", us_w, us_f);
      for (int skip = 0; skip < 2; ++skip) {
        const double m0 = time_us([&] { hipLaunchKernelGGL((k_c1w<0, 4>), dim3(2 * nz), dim3(256), lds, 0, t, dz1, B, nz, slab, skip); });
        const double m1 = time_us([&] { hipLaunchKernelGGL((k_c1w<1, 4>), dim3(2 * nz), dim3(256), lds, 0, t, dz1, B, nz, slab, skip); });
        const double m2 = time_us([&] { hipLaunchKernelGGL((k_c1w<2, 4>), dim3(2 * nz), dim3(256), lds, 0, t, dz1, B, nz, slab, skip); });
        const double m3 = time_us([&] { hipLaunchKernelGGL((k_c1w<3, 4>), dim3(2 * nz), dim3(256), lds, 0, t, dz1, B, nz, slab, skip); });
        printf("  skip %d: wgrad copy %7.2f | no loop %7.2f | no reload %7.2f | loop only %7.2f us\n", skip, m0, m1, m2, m3);
      }
      for (int sc : {8, 4, 2, 1})   // every launch's slab chunks inside the allocation
        if ((size_t)(B / sc) * 257 * 32 > (size_t)B * 257 * 32) { fprintf(stderr, "slab too small\n"); return 1; }
      const double c8 = time_us([&] { hipLaunchKernelGGL((k_c1w<0, 8>), dim3(2 * (B / 8)), dim3(256), lds, 0, t, dz1, B, B / 8, slab, 1); });
      const double c2 = time_us([&] { hipLaunchKernelGGL((k_c1w<0, 2>), dim3(2 * (B / 2)), dim3(256), lds, 0, t, dz1, B, B / 2, slab, 1); });
      const double c1 = time_us([&] { hipLaunchKernelGGL((k_c1w<0, 1>), dim3(2 * B), dim3(256), lds, 0, t, dz1, B, B, slab, 1); });
      printf("  chunk 8 / 2 / 1 samples per block: %7.2f / %7.2f / %7.2f us\n", c8, c2, c1);
    }
  }
  printf("ok\n");
  return 0;
}
