// Probe: is v_mfma_f32_16x16x4_f32 / 32x32x2_f32 bit-for-bit a k-ordered fmaf chain (lane group 0 first)?
// And are sqrtf / division correctly rounded in device code?  Decides the fp32 Q-net's reduction order.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off scripts/mfma_f32_probe.hip -o /tmp/probe && /tmp/probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// 16x16 tile, K = 4 * nk: A [16][K], B [K][16] row-major, C init [16][16]
__global__ void k16(const float* A, const float* B, const float* C, int nk, float* D) {
  const int l = threadIdx.x;
  f32x4 acc;
  for (int r = 0; r < 4; ++r) acc[r] = C[((l >> 4) * 4 + r) * 16 + (l & 15)];
  const int K = 4 * nk;
  for (int t = 0; t < nk; ++t) {
    const float a = A[(l & 15) * K + 4 * t + (l >> 4)];
    const float b = B[(4 * t + (l >> 4)) * 16 + (l & 15)];
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
  }
  for (int r = 0; r < 4; ++r) D[((l >> 4) * 4 + r) * 16 + (l & 15)] = acc[r];
}

// 32x32 tile, K = 2 * nk
__global__ void k32(const float* A, const float* B, const float* C, int nk, float* D) {
  const int l = threadIdx.x;
  f32x16 acc;
  for (int r = 0; r < 16; ++r) acc[r] = C[((r & 3) + 8 * (r >> 2) + 4 * (l >> 5)) * 32 + (l & 31)];
  const int K = 2 * nk;
  for (int t = 0; t < nk; ++t) {
    const float a = A[(l & 31) * K + 2 * t + (l >> 5)];
    const float b = B[(2 * t + (l >> 5)) * 32 + (l & 31)];
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
  }
  for (int r = 0; r < 16; ++r) D[((r & 3) + 8 * (r >> 2) + 4 * (l >> 5)) * 32 + (l & 31)] = acc[r];
}

__global__ void kmath(const float* x, const float* y, int n, float* s_def, float* s_rn, float* d_def, float* d_rn) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  s_def[i] = sqrtf(x[i]);
  s_rn[i] = __fsqrt_rn(x[i]);
  d_def[i] = x[i] / y[i];
  d_rn[i] = __fdiv_rn(x[i], y[i]);
}

static int check(int T, int nk, bool reversed_groups, bool exactsum, const std::vector<float>& A, const std::vector<float>& B,
                 const std::vector<float>& C, const std::vector<float>& D) {
  const int G = T == 16 ? 4 : 2;
  const int K = G * nk;
  int bad = 0;
  for (int i = 0; i < T; ++i)
    for (int j = 0; j < T; ++j) {
      float acc = C[i * T + j];
      for (int t = 0; t < nk; ++t) {
        if (exactsum) {   // products summed exactly (double), one rounding per instruction
          double s = acc;
          for (int g = 0; g < G; ++g) s += (double)A[i * K + G * t + g] * (double)B[(G * t + g) * T + j];
          acc = (float)s;
        } else {
          for (int gg = 0; gg < G; ++gg) {
            const int g = reversed_groups ? G - 1 - gg : gg;
            acc = std::fmaf(A[i * K + G * t + g], B[(G * t + g) * T + j], acc);
          }
        }
      }
      uint32_t u, v;
      std::memcpy(&u, &acc, 4);
      std::memcpy(&v, &D[i * T + j], 4);
      bad += u != v;
    }
  return bad;
}

int main() {
  std::mt19937 rng(12345);
  std::uniform_real_distribution<float> U(-1.0f, 1.0f);
  for (int T : {16, 32}) {
    for (int nk : {1, 64, 784}) {
      for (int zeroC : {0, 1}) {
        const int G = T == 16 ? 4 : 2, K = G * nk;
        std::vector<float> A(T * K), B(K * T), C(T * T), D(T * T);
        for (auto& v : A) v = U(rng);
        for (auto& v : B) v = U(rng) * 1e-3f;
        for (auto& v : C) v = zeroC ? 0.0f : U(rng);
        float *dA, *dB, *dC, *dD;
        hipMalloc(&dA, A.size() * 4); hipMalloc(&dB, B.size() * 4); hipMalloc(&dC, C.size() * 4); hipMalloc(&dD, D.size() * 4);
        hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
        hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice);
        hipMemcpy(dC, C.data(), C.size() * 4, hipMemcpyHostToDevice);
        if (T == 16) hipLaunchKernelGGL(k16, dim3(1), dim3(64), 0, 0, dA, dB, dC, nk, dD);
        else hipLaunchKernelGGL(k32, dim3(1), dim3(64), 0, 0, dA, dB, dC, nk, dD);
        hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost);
        printf("T=%d nk=%d zeroC=%d: mismatches vs chain(g asc)=%d chain(g desc)=%d exact-sum=%d of %d\n", T, nk, zeroC,
               check(T, nk, false, false, A, B, C, D), check(T, nk, true, false, A, B, C, D), check(T, nk, false, true, A, B, C, D),
               T * T);
        hipFree(dA); hipFree(dB); hipFree(dC); hipFree(dD);
      }
    }
  }
  // sqrt / div rounding
  const int n = 1 << 20;
  std::vector<float> x(n), y(n), o[4];
  std::uniform_real_distribution<float> P(1e-12f, 10.0f);
  for (int i = 0; i < n; ++i) { x[i] = P(rng) * P(rng); y[i] = P(rng); }
  float *dx, *dy, *d[4];
  hipMalloc(&dx, n * 4); hipMalloc(&dy, n * 4);
  for (int k = 0; k < 4; ++k) { hipMalloc(&d[k], n * 4); o[k].resize(n); }
  hipMemcpy(dx, x.data(), n * 4, hipMemcpyHostToDevice);
  hipMemcpy(dy, y.data(), n * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(kmath, dim3(n / 256), dim3(256), 0, 0, dx, dy, n, d[0], d[1], d[2], d[3]);
  for (int k = 0; k < 4; ++k) hipMemcpy(o[k].data(), d[k], n * 4, hipMemcpyDeviceToHost);
  int bad[4] = {0, 0, 0, 0};
  for (int i = 0; i < n; ++i) {
    const float s = std::sqrt(x[i]), q = x[i] / y[i];
    bad[0] += std::memcmp(&s, &o[0][i], 4) != 0;
    bad[1] += std::memcmp(&s, &o[1][i], 4) != 0;
    bad[2] += std::memcmp(&q, &o[2][i], 4) != 0;
    bad[3] += std::memcmp(&q, &o[3][i], 4) != 0;
  }
  printf("sqrtf mismatches %d, __fsqrt_rn %d, div %d, __fdiv_rn %d of %d\n", bad[0], bad[1], bad[2], bad[3], n);
  return 0;
}
