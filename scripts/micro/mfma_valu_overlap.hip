// Does one wave per SIMD overlap its own VALU with its MFMAs?  A loop of
// NM v_mfma_f32_32x32x16_bf16 (4 independent accumulators) and NV independent
// VALU ops (the split sequence of the wide SYRK: cvt_pk / shift / sub), with
// the VALU interleaved between the MFMAs by scheduling-group barriers.
// Prints cycles per iteration for (NM, NV) = (8, 0), (0, NV), (8, NV).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ unsigned pk(float a, float b) {
  const bf16x2 v = {(__bf16)a, (__bf16)b};
  unsigned u = __builtin_bit_cast(unsigned, v);
  asm("" : "+v"(u));
  return u;
}

template <int NM, int NSPLIT>
__global__ void __launch_bounds__(256) k(const float* in, float* out, long long* cyc, int iters) {
  const int lane = threadIdx.x & 63;
  bf16x8 a = {}, b = {};
  for (int i = 0; i < 8; ++i) { a[i] = (__bf16)in[lane + i]; b[i] = (__bf16)in[lane + 8 + i]; }
  f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
  float x[8];
  for (int i = 0; i < 8; ++i) x[i] = in[lane * 8 + i];
  unsigned acc = 0;
  long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int s = 0; s < NSPLIT; ++s) {  // one split of 8 values per s (~44 VALU)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float x0 = x[2 * e] + s, x1 = x[2 * e + 1];
        const unsigned H = pk(x0, x1);
        const float r0 = x0 - __uint_as_float(H << 16), r1 = x1 - __uint_as_float(H & 0xffff0000u);
        const unsigned M = pk(r0, r1);
        const float s0 = r0 - __uint_as_float(M << 16), s1 = r1 - __uint_as_float(M & 0xffff0000u);
        acc ^= H ^ M ^ pk(s0, s1);
      }
    }
#pragma unroll
    for (int m = 0; m < NM / 4; ++m) {
      c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c3, 0, 0, 0);
    }
    if constexpr (NM > 0 && NSPLIT > 0) {
      constexpr int VPER = (NSPLIT * 44 + NM - 1) / NM;
#pragma unroll
      for (int m = 0; m < NM; ++m) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, VPER, 0);
      }
    }
    x[0] += 1.0f;
  }
  long long t1 = clock64();
  float s = 0;
  for (int i = 0; i < 16; ++i) s += c0[i] + c1[i] + c2[i] + c3[i];
  out[blockIdx.x * 256 + threadIdx.x] = s + (float)acc;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int NM, int NS>
void run(const float* in, float* out, long long* cyc, int iters) {
  const int nb = 256;
  hipLaunchKernelGGL((k<NM, NS>), dim3(nb), dim3(256), 0, 0, in, out, cyc, iters);
  hipDeviceSynchronize();
  long long h[256];
  hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
  double m = 0;
  for (int i = 0; i < nb; ++i) m += h[i];
  printf("NM %2d splits %d (~%3d VALU): %.1f cycles / iteration\n", NM, NS, NS * 44, m / nb / iters);
}

int main() {
  float *in, *out;
  long long* cyc;
  hipMalloc(&in, 1 << 20);
  hipMalloc(&out, 1 << 20);
  hipMalloc(&cyc, 4096);
  hipMemset(in, 0, 1 << 20);
  const int it = 2000;
  run<8, 0>(in, out, cyc, it);
  run<0, 1>(in, out, cyc, it);
  run<8, 1>(in, out, cyc, it);
  run<12, 1>(in, out, cyc, it);
  run<24, 1>(in, out, cyc, it);
  run<24, 2>(in, out, cyc, it);
  run<0, 2>(in, out, cyc, it);
  return 0;
}
