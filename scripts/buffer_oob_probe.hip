// Range check of raw buffer loads on gfx950: does the SGPR offset (soffset) count toward the num_records bound?  A buffer
// of 64 floats (value i + 1) with num_records = 256 bytes; each lane loads voffset = 4 * lane with soffset 0, 128, 256 and
// 4096 (the memory past the 256 bytes holds 1000 + i).  Prints, per soffset, how many lanes read 0.
//   hipcc --offload-arch=gfx950 -O3 scripts/buffer_oob_probe.hip -o buffer_oob_probe && ./buffer_oob_probe
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void k_probe(const float* a, float* out) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)a, (short)0, 256, 0x00020000);
  const int soffs[4] = {0, 128, 256, 4096};
#pragma unroll
  for (int i = 0; i < 4; ++i)
    out[i * 64 + threadIdx.x] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, threadIdx.x * 4, soffs[i], 0));
}

int main() {
  float h[4096];
  for (int i = 0; i < 4096; ++i) h[i] = i < 64 ? (float)(i + 1) : (float)(1000 + i);
  float *d = nullptr, *o = nullptr;
  if (hipMalloc(&d, sizeof(h)) != hipSuccess || hipMalloc(&o, 256 * sizeof(float)) != hipSuccess) return 1;
  hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, d, o);
  float r[256];
  if (hipMemcpy(r, o, sizeof(r), hipMemcpyDeviceToHost) != hipSuccess) return 1;
  const int soffs[4] = {0, 128, 256, 4096};
  for (int i = 0; i < 4; ++i) {
    int zeros = 0;
    for (int l = 0; l < 64; ++l) zeros += r[i * 64 + l] == 0.0f;
    printf("soffset %4d: %2d of 64 lanes read 0 (lane 0 = %.0f, lane 63 = %.0f)\n", soffs[i], zeros, r[i * 64], r[i * 64 + 63]);
  }
  return 0;
}
