// Issue-rate check of v_mfma_f32_32x32x16_bf16 on gfx950 (diagnostics): one
// wave issuing 6 * ITER MFMAs as (a) one dependent chain on one accumulator,
// (b) round-robin over 2 / 4 independent accumulators, cycles per MFMA by
// s_memtime-free clock64 deltas.  hipcc --offload-arch=gfx950 -O3 mfma_dep.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int NACC>
__global__ void __launch_bounds__(64) dep_kernel(const bf16x8* in, float* out, long long* cyc,
                                                 int iters) {
  const int lane = threadIdx.x;
  bf16x8 a = in[lane], b = in[64 + lane];
  f32x16 acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = f32x16{0.f};
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int p = 0; p < 24; ++p) {
      const int i = p % NACC;
      acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[i], 0, 0, 0);
    }
  }
  float s = 0.0f;
#pragma unroll
  for (int i = 0; i < NACC; ++i)
#pragma unroll
    for (int q = 0; q < 16; ++q) s += acc[i][q];
  const long long t1 = clock64();
  out[lane] = s;
  if (lane == 0) cyc[0] = t1 - t0;
}

int main() {
  bf16x8* in;
  float* out;
  long long* cyc;
  (void)hipMalloc(&in, 128 * sizeof(bf16x8));
  (void)hipMalloc(&out, 64 * sizeof(float));
  (void)hipMalloc(&cyc, sizeof(long long));
  (void)hipMemset(in, 0, 128 * sizeof(bf16x8));
  const int iters = 1000;
  for (int rep = 0; rep < 2; ++rep) {
    long long c;
    hipLaunchKernelGGL(dep_kernel<1>, dim3(1), dim3(64), 0, 0, in, out, cyc, iters);
    (void)hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
    printf("1 accumulator (dependent chain): %.1f cycles per MFMA\n", (double)c / (24.0 * iters));
    hipLaunchKernelGGL(dep_kernel<2>, dim3(1), dim3(64), 0, 0, in, out, cyc, iters);
    (void)hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
    printf("2 accumulators: %.1f cycles per MFMA\n", (double)c / (24.0 * iters));
    hipLaunchKernelGGL(dep_kernel<4>, dim3(1), dim3(64), 0, 0, in, out, cyc, iters);
    (void)hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
    printf("4 accumulators: %.1f cycles per MFMA\n", (double)c / (24.0 * iters));
  }
  return 0;
}
