// The off-diagonal SYRK role's MFMA pattern alone: 4 x 4 tiles (16
// accumulators, 256 registers -> AGPRs), 6 v_mfma_f32_32x32x16_bf16 per tile
// and step (mfma_x6 order: one dependent chain per tile), operands from 8
// fragments x 3 pieces; optionally the 8 splits (fp32 -> 3 bf16 pieces) of
// the next step's fragments beside them.  Cycles per step.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x16 x6(const bf16x8 (&a)[3], const bf16x8 (&b)[3], f32x16 c) {
  c = mfma(a[2], b[0], c);
  c = mfma(a[0], b[2], c);
  c = mfma(a[1], b[1], c);
  c = mfma(a[1], b[0], c);
  c = mfma(a[0], b[1], c);
  c = mfma(a[0], b[0], c);
  return c;
}
__device__ __forceinline__ unsigned pk(float a, float b) {
  const bf16x2 v = {(__bf16)a, (__bf16)b};
  unsigned u = __builtin_bit_cast(unsigned, v);
  asm("" : "+v"(u));
  return u;
}
__device__ __forceinline__ void split(const float* x, bf16x8 (&f)[3]) {
  unsigned wh[4], wm[4], wl[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float x0 = x[2 * e], x1 = x[2 * e + 1];
    const unsigned H = pk(x0, x1);
    const float r0 = x0 - __uint_as_float(H << 16), r1 = x1 - __uint_as_float(H & 0xffff0000u);
    const unsigned M = pk(r0, r1);
    const float s0 = r0 - __uint_as_float(M << 16), s1 = r1 - __uint_as_float(M & 0xffff0000u);
    wh[e] = H; wm[e] = M; wl[e] = pk(s0, s1);
  }
  f[0] = __builtin_bit_cast(bf16x8, wh);
  f[1] = __builtin_bit_cast(bf16x8, wm);
  f[2] = __builtin_bit_cast(bf16x8, wl);
}

__device__ __forceinline__ void glds16(const void* src, unsigned dst) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(dst)
      : "memory");
}
template <bool SPLIT, int NG, int TBL = 471355, int MODE = 0>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
    k(const float* in, float* out, long long* cyc, int iters, const float* table, const int* rows) {
  __shared__ __attribute__((aligned(16))) char lds[65536];
  const unsigned lbase = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)lds;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  float4 sink[8];
  const int lane = threadIdx.x & 63;
  bf16x8 F[2][8][3];
  float x[8];
  for (int i = 0; i < 8; ++i) x[i] = in[lane * 8 + i];
  for (int f = 0; f < 8; ++f) split(x, F[0][f]), split(x, F[1][f]);
  f32x16 acc[16];
  for (int t = 0; t < 16; ++t) acc[t] = f32x16{0.f};
  long long t0 = clock64();
  for (int it = 0; it < iters; it += 2) {
#pragma unroll
    for (int p = 0; p < 2; ++p) {
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        if constexpr (NG > 0) {
          if (s < NG) {
            const int r = __builtin_amdgcn_readfirstlane(rows[(it * 8 + s + 64 * blockIdx.x) & 0xfffff] % TBL);
            const float* src = table + (size_t)r * 512 + 256 * (s & 1) + 4 * (threadIdx.x & 63);
            if constexpr (MODE == 0) {
              glds16(src, __builtin_amdgcn_readfirstlane(lbase + ((wave * 8 + s) & 63) * 1024));
            } else {
              float4 v;
              asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(src) : "memory");
              sink[s & 7] = v;
            }
          }
          if (s == 7) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        }
        if (SPLIT) {
          x[0] += 1.0f;
          split(x, F[1 - p][s]);
        }
#pragma unroll
        for (int t = 2 * s; t < 2 * s + 2; ++t) acc[t] = x6(F[p][t >> 2], F[p][4 + (t & 3)], acc[t]);
        if (SPLIT) {
#pragma unroll
          for (int m = 0; m < 12; ++m) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
          }
        }
      }
    }
  }
  long long t1 = clock64();
  float sum = 0;
  for (int t = 0; t < 16; ++t)
    for (int i = 0; i < 16; ++i) sum += acc[t][i];
  if constexpr (MODE == 1) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (int i = 0; i < 8; ++i) sum += sink[i].x;
  }
  out[blockIdx.x * 256 + threadIdx.x] = sum;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <bool S, int NG, int TBL = 471355, int MODE = 0>
void run(const float* in, float* out, long long* cyc, int iters, const float* table, const int* rows) {
  hipLaunchKernelGGL((k<S, NG, TBL, MODE>), dim3(256), dim3(256), 0, 0, in, out, cyc, iters, table, rows);
  hipDeviceSynchronize();
  long long h[256];
  hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
  double m = 0;
  for (int i = 0; i < 256; ++i) m += h[i];
  printf("96 MFMAs / step, splits %d, row loads %d (%s, table %d rows): %.1f cycles / step\n", (int)S * 8, NG, MODE ? "global_load_dwordx4" : "LDS-DMA", TBL, m / 256 / iters);
}

int main() {
  float *in, *out;
  long long* cyc;
  hipMalloc(&in, 1 << 20);
  hipMalloc(&out, 1 << 20);
  hipMalloc(&cyc, 4096);
  hipMemset(in, 0, 1 << 20);
  float* table;
  int* rows;
  hipMalloc(&table, (size_t)471355 * 2048);
  hipMalloc(&rows, 4 << 20);
  hipMemset(table, 0, (size_t)471355 * 2048);
  int* hr = new int[1 << 20];
  unsigned st = 12345;
  for (int i = 0; i < (1 << 20); ++i) { st = st * 1103515245u + 12345u; hr[i] = (st >> 8) % 471355; }
  hipMemcpy(rows, hr, 4 << 20, hipMemcpyHostToDevice);
  run<false, 0>(in, out, cyc, 400, table, rows);
  run<false, 8>(in, out, cyc, 400, table, rows);
  run<false, 8, 2048>(in, out, cyc, 400, table, rows);
  run<false, 8, 471355, 1>(in, out, cyc, 400, table, rows);
  run<false, 8, 2048, 1>(in, out, cyc, 400, table, rows);
  run<true, 8, 471355, 1>(in, out, cyc, 400, table, rows);
  return 0;
}
