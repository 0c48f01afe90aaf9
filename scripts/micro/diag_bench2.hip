// Microbenchmark of the 32x32 diagonal-block factor + inverse variants of
// chol.h on gfx950: cycles per call (one wave, 20 calls) and the max
// deviation of L^-1 from the plain recurrence (diagnostics only).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 diag_bench2.hip -o diag_bench2
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>

#include "../../safer2-recommender_amd/csrc/chol.h"
using namespace frecsys_hip;

template <int V>
__global__ void __launch_bounds__(64) bench(const float* A, unsigned long long* cyc, float* Linv) {
  __shared__ __attribute__((aligned(16))) float tile[1024], src[1024];
  const int lane = threadIdx.x;
  for (int i = lane; i < 1024; i += 64) src[sw(i >> 5, i & 31)] = A[i];
  unsigned long long t0 = 0, t1 = 0;
  bool ok = true;
  for (int it = 0; it < 21; ++it) {
    for (int i = lane; i < 1024; i += 64) tile[i] = src[i];
    wave_lds_sync();
    if (it == 1) t0 = clock64();
    if constexpr (V == 0) ok = diag_factor_inv_lds((lds_float*)tile, lane);
    else ok = diag_factor_inv_blk((lds_float*)tile, lane);
    wave_lds_sync();
  }
  t1 = clock64();
  if (lane == 0) cyc[0] = (t1 - t0) / 20;
  for (int i = lane; i < 1024; i += 64) Linv[i] = tile[sw(i >> 5, i & 31)];
  if (lane == 0 && !ok) cyc[1] = 1;
}

int main() {
  float hA[1024];
  // SPD test matrix with a realistic spread: B B^T / 32 + 1e-3 I
  unsigned s = 12345;
  float B[32][32];
  for (int i = 0; i < 32; ++i)
    for (int j = 0; j < 32; ++j) {
      s = s * 1664525u + 1013904223u;
      B[i][j] = (float)((s >> 8) & 0xFFFF) / 65536.0f - 0.5f;
    }
  for (int i = 0; i < 32; ++i)
    for (int j = 0; j < 32; ++j) {
      double t = 0;
      for (int k = 0; k < 32; ++k) t += (double)B[i][k] * B[j][k];
      hA[i * 32 + j] = (float)(t / 32.0 + (i == j ? 1e-2 : 0.0));
    }
  float *dA, *dL;
  unsigned long long* dc;
  hipMalloc(&dA, 4096);
  hipMalloc(&dL, 3 * 4096);
  hipMalloc(&dc, 3 * 16);
  hipMemset(dc, 0, 48);
  hipMemcpy(dA, hA, 4096, hipMemcpyHostToDevice);
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(bench<0>, dim3(1), dim3(64), 0, 0, dA, dc, dL);
    hipLaunchKernelGGL(bench<1>, dim3(1), dim3(64), 0, 0, dA, dc + 2, dL + 1024);
  }
  unsigned long long hc[6];
  float hL[3 * 1024];
  hipMemcpy(hc, dc, 48, hipMemcpyDeviceToHost);
  hipMemcpy(hL, dL, 3 * 4096, hipMemcpyDeviceToHost);
  const char* names[2] = {"lds (plain)", "blk (16+16)"};
  for (int v = 0; v < 2; ++v) {
    double md = 0, mx = 0;
    for (int i = 0; i < 1024; ++i) {
      md = fmax(md, fabs((double)hL[v * 1024 + i] - hL[i]));
      mx = fmax(mx, fabs((double)hL[i]));
    }
    // residual of L^-1 A L^-T - I
    double res = 0;
    const float* Li = hL + v * 1024;
    for (int i = 0; i < 32; ++i)
      for (int j = 0; j < 32; ++j) {
        double t = 0;
        for (int k = 0; k < 32; ++k)
          for (int l = 0; l < 32; ++l) t += (double)Li[i * 32 + k] * hA[k * 32 + l] * Li[j * 32 + l];
        res = fmax(res, fabs(t - (i == j ? 1.0 : 0.0)));
      }
    printf("%-12s %6llu cycles  fail=%llu  max|dLinv| %.3g (max|Linv| %.3g)  max|Linv A Linv^T - I| %.3g\n",
           names[v], hc[2 * v], hc[2 * v + 1], md, mx, res);
  }
  return 0;
}
