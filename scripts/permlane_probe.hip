// Probe (development tool): which element of __builtin_amdgcn_permlane{16,32}_swap holds which row on gfx950.
//   hipcc --offload-arch=gfx950 -O3 scripts/permlane_probe.hip -o scripts/permlane_probe && ./scripts/permlane_probe
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* o) {
  const unsigned v = threadIdx.x;
  const auto a = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  const auto b = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  o[threadIdx.x * 4 + 0] = a[0];
  o[threadIdx.x * 4 + 1] = a[1];
  o[threadIdx.x * 4 + 2] = b[0];
  o[threadIdx.x * 4 + 3] = b[1];
}
int main() {
  unsigned* d;
  hipMalloc(&d, 64 * 16);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  unsigned h[256];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int l : {0, 5, 16, 21, 32, 48}) printf("lane %2d: p16[0]=%2u p16[1]=%2u p32[0]=%2u p32[1]=%2u\n", l, h[l * 4], h[l * 4 + 1], h[l * 4 + 2], h[l * 4 + 3]);
  return 0;
}
