// Microbenchmark: cycles of one diag_factor_inv / tile_pqT / lds_barrier on
// gfx950 (one workgroup; diagnostics only).
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../safer2-recommender_amd/csrc/chol.h"
using namespace frecsys_hip;

__global__ void __launch_bounds__(256) bench(unsigned long long* out, float* sink) {
  __shared__ float tile[1024], t2[1024];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lo = lane & 31, hi = lane >> 5;
  for (int i = tid; i < 1024; i += 256) {
    const int r = i >> 5, c = i & 31;
    t2[sw(r, c)] = (r == c ? 40.0f : 0.0f) + 1.0f / (1 + r + c);
  }
  lds_barrier();
  unsigned long long t0 = clock64();
  for (int it = 0; it < 20; ++it) {
    if (wave == 0) {
      for (int i = lane; i < 1024; i += 64) tile[i] = t2[i];
      wave_lds_sync();
      diag_factor_inv<FRECSYS_DIAG_BLK != 0>(tile, lane);
    }
    lds_barrier();
  }
  unsigned long long t1 = clock64();
  f32x16 acc = f32x16{0.f};
  for (int it = 0; it < 20; ++it) {
    f32x16 u = tile_pqT(tile, t2, lo, hi);
    acc += u;
    wave_lds_sync();
  }
  unsigned long long t2c = clock64();
  for (int it = 0; it < 100; ++it) lds_barrier();
  unsigned long long t3 = clock64();
  if (tid == 0) {
    out[0] = (t1 - t0) / 20;
    out[1] = (t2c - t1) / 20;
    out[2] = (t3 - t2c) / 100;
  }
  float s = 0;
  for (int q = 0; q < 16; ++q) s += acc[q];
  sink[tid] = s + tile[tid];
}

int main() {
  unsigned long long* d;
  float* sink;
  hipMalloc(&d, 64);
  hipMalloc(&sink, 4096);
  hipLaunchKernelGGL(bench, dim3(1), dim3(256), 0, 0, d, sink);
  hipLaunchKernelGGL(bench, dim3(1), dim3(256), 0, 0, d, sink);
  unsigned long long h[3];
  hipMemcpy(h, d, 24, hipMemcpyDeviceToHost);
  printf("diag_factor_inv (+tile copy) %llu cycles, tile_pqT %llu cycles, lds_barrier %llu cycles\n",
         h[0], h[1], h[2]);
  return 0;
}
