// Which change of commit 25c5694 fixed the frame_sparsity read-back?  The diagnostic's pattern,
// replayed back to back (a big call, then a small one, as qlx_learner_frame_sparsity does: the train batch, then the
// acting frames) under four read-back variants, every call checked against the count it must return:
//   0  hipMallocAsync + memset + kernel + hipMemcpyAsync D2H into pageable (stack) memory + hipFreeAsync + stream sync
//      (the round-5 code before 25c5694)
//   1  hipMallocAsync / hipFreeAsync, D2H into pinned memory (hipHostMalloc)
//   2  hipMalloc / hipFree per call, hipMemcpyAsync D2H into pageable memory, stream sync, then hipFree
//   3  a persistent device counter + a persistent pinned host buffer, all on the stream (the round-6 product code)
// Prints one line per variant: calls, wrong read-backs, and the first wrong value.
//   hipcc -O2 --offload-arch=gfx950 scripts/readback_probe.hip -o scripts/readback_probe && ./scripts/readback_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                        \
    }                                                                                      \
  } while (0)

// per "sample" b: 400 + 400 + 81 + 49 units of LDS work, counted as in k_frame_sparsity (per-block LDS sum, then one
// global atomic per counter); the counts are known: cnt[k] = n * per[k]
__global__ __launch_bounds__(256) void k_count(const unsigned char* data, int n, unsigned long long* cnt) {
  __shared__ int tot[4];
  __shared__ unsigned int buf[1764];
  int mine[4] = {0, 0, 0, 0};
  for (int b = blockIdx.x; b < n; b += gridDim.x) {
    __syncthreads();
    for (int q = threadIdx.x; q < 1764; q += blockDim.x) buf[q] = data[((size_t)b * 1764 + q) & ((1u << 24) - 1)];
    __syncthreads();
    for (int i = threadIdx.x; i < 400; i += blockDim.x) {
      unsigned int o = 0u;
      for (int l = 0; l < 64; ++l) o |= buf[(i * 7 + l * 13) % 1764];
      mine[0] += o != 0xFFFFFFFFu;
      mine[1] += 1;
    }
    for (int p = threadIdx.x; p < 130; p += blockDim.x) mine[p < 81 ? 2 : 3] += 1;
  }
  if (threadIdx.x < 4) tot[threadIdx.x] = 0;
  __syncthreads();
  for (int k = 0; k < 4; ++k) atomicAdd(&tot[k], mine[k]);
  __syncthreads();
  if (threadIdx.x < 4) atomicAdd(cnt + threadIdx.x, (unsigned long long)tot[threadIdx.x]);
}

static int g_grid = 1024;

static bool check(const unsigned long long* h, int n) {
  const unsigned long long per[4] = {400, 400, 81, 49};
  for (int k = 0; k < 4; ++k)
    if (h[k] != per[k] * (unsigned long long)n) return false;
  return true;
}

static void call(int variant, const unsigned char* data, int n, hipStream_t s, unsigned long long* d_keep,
                 unsigned long long* h_pinned, unsigned long long out[4]) {
  const dim3 grid(n < g_grid ? n : g_grid);
  if (variant == 0 || variant == 1) {
    unsigned long long* d = nullptr;
    CK(hipMallocAsync((void**)&d, 4 * sizeof(unsigned long long), s));
    CK(hipMemsetAsync(d, 0, 4 * sizeof(unsigned long long), s));
    hipLaunchKernelGGL(k_count, grid, dim3(256), 0, s, data, n, d);
    CK(hipGetLastError());
    unsigned long long h[4];
    unsigned long long* dst = variant == 0 ? h : h_pinned;
    CK(hipMemcpyAsync(dst, d, 4 * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    CK(hipFreeAsync(d, s));
    CK(hipStreamSynchronize(s));
    std::memcpy(out, dst, sizeof(h));
  } else if (variant == 2) {
    unsigned long long* d = nullptr;
    CK(hipMalloc((void**)&d, 4 * sizeof(unsigned long long)));
    CK(hipMemsetAsync(d, 0, 4 * sizeof(unsigned long long), s));
    hipLaunchKernelGGL(k_count, grid, dim3(256), 0, s, data, n, d);
    CK(hipGetLastError());
    unsigned long long h[4];
    CK(hipMemcpyAsync(h, d, sizeof(h), hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    CK(hipFree(d));
    std::memcpy(out, h, sizeof(h));
  } else {
    CK(hipMemsetAsync(d_keep, 0, 4 * sizeof(unsigned long long), s));
    hipLaunchKernelGGL(k_count, grid, dim3(256), 0, s, data, n, d_keep);
    CK(hipGetLastError());
    CK(hipMemcpyAsync(h_pinned, d_keep, 4 * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    std::memcpy(out, h_pinned, 4 * sizeof(unsigned long long));
  }
}

int main(int argc, char** argv) {
  const int pairs = argc > 1 ? std::atoi(argv[1]) : 300;
  int dev = 0;
  CK(hipSetDevice(dev));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, dev));
  g_grid = 4 * prop.multiProcessorCount;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  unsigned char* data = nullptr;
  CK(hipMalloc(&data, 1u << 24));
  CK(hipMemset(data, 1, 1u << 24));
  unsigned long long *d_keep = nullptr, *h_pinned = nullptr;
  CK(hipMalloc((void**)&d_keep, 4 * sizeof(unsigned long long)));
  CK(hipHostMalloc((void**)&h_pinned, 4 * sizeof(unsigned long long), hipHostMallocDefault));
  CK(hipDeviceSynchronize());
  const int sizes[2] = {65536, 8192};   // C3: U x B sampled states, then n_envs acting frames
  for (int v = 0; v < 4; ++v) {
    int wrong[2] = {0, 0};
    unsigned long long first_bad[4] = {0, 0, 0, 0};
    for (int i = 0; i < pairs; ++i)
      for (int c = 0; c < 2; ++c) {
        unsigned long long h[4];
        call(v, data, sizes[c], s, d_keep, h_pinned, h);
        if (!check(h, sizes[c])) {
          if (wrong[0] + wrong[1] == 0) std::memcpy(first_bad, h, sizeof(h));
          ++wrong[c];
        }
      }
    std::printf("variant %d: %d pairs, wrong first-call %d, wrong second-call %d, first bad [%llu %llu %llu %llu]\n", v, pairs,
                wrong[0], wrong[1], first_bad[0], first_bad[1], first_bad[2], first_bad[3]);
    std::fflush(stdout);
  }
  CK(hipFree(data));
  CK(hipFree(d_keep));
  CK(hipHostFree(h_pinned));
  CK(hipStreamDestroy(s));
  return 0;
}
