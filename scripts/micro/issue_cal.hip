// Calibration of single-wave instruction costs on gfx950 in clock64 cycles
// (diagnostics only).  Build: hipcc --offload-arch=gfx950 -O3 issue_cal.hip -o issue_cal
#include <hip/hip_runtime.h>
#include <cstdio>

#define KEEP(v) asm volatile("" : "+v"(v))
__global__ void __launch_bounds__(64) cal(float* out, unsigned long long* cyc, float seed) {
  const int lane = threadIdx.x;
  float x = seed + lane, y = x * 0.5f, z = x * 0.25f, w = x * 0.125f;
  unsigned long long t0, t1;
  t0 = clock64();
  t1 = clock64();
  cyc[0] = t1 - t0;  // overhead
  t0 = clock64();
#pragma unroll
  for (int i = 0; i < 256; ++i) { x = __builtin_fmaf(x, 0.999f, 0.001f); KEEP(x); }
  t1 = clock64();
  cyc[1] = t1 - t0;
  t0 = clock64();
#pragma unroll
  for (int i = 0; i < 256; ++i) {
    y = __builtin_fmaf(y, 0.999f, 0.001f); KEEP(y);
    z = __builtin_fmaf(z, 0.999f, 0.001f); KEEP(z);
    w = __builtin_fmaf(w, 0.999f, 0.001f); KEEP(w);
    x = __builtin_fmaf(x, 0.999f, 0.001f); KEEP(x);
  }
  t1 = clock64();
  cyc[2] = t1 - t0;
  t0 = clock64();
#pragma unroll
  for (int i = 0; i < 256; ++i) {
    float b = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), i & 63));
    x = __builtin_fmaf(x, b, 0.001f); KEEP(x);
  }
  t1 = clock64();
  cyc[3] = t1 - t0;
  t0 = clock64();
#pragma unroll
  for (int i = 0; i < 256; ++i) { y = __builtin_amdgcn_rsqf(y); KEEP(y); }
  t1 = clock64();
  cyc[4] = t1 - t0;
  // per-column chain: t -> readlane(t, k) -> rsq -> mul -> readlane(a, k+1) -> fma -> sub
  t0 = clock64();
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    const float piv = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(z), i & 31));
    const float a = z * __builtin_amdgcn_rsqf(piv);
    const float b = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(a), (i + 1) & 31));
    z = w - a * b; KEEP(z);
  }
  t1 = clock64();
  cyc[5] = t1 - t0;
  // LDS write -> read round trip (same wave)
  __shared__ float sh[64];
  t0 = clock64();
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    sh[lane] = w;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    w = sh[(lane + 1) & 63] + 1.0f;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  t1 = clock64();
  cyc[6] = t1 - t0;
  out[lane] = x + y + z + w;
}

int main() {
  float* o;
  unsigned long long* c;
  (void)hipMalloc(&o, 256);
  (void)hipMalloc(&c, 64);
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(cal, dim3(1), dim3(64), 0, 0, o, c, 1.0f);
  unsigned long long h[7];
  (void)hipMemcpy(h, c, 56, hipMemcpyDeviceToHost);
  const double ov = (double)h[0];
  printf("clock64 pair %llu | dep fma %.2f | 4 chains %.2f/op | readlane+fma %.2f | rsq %.2f | column chain %.2f | lds w->r %.2f\n",
         h[0], (h[1] - ov) / 256, (h[2] - ov) / 1024, (h[3] - ov) / 256, (h[4] - ov) / 256, (h[5] - ov) / 64, (h[6] - ov) / 64);
  return 0;
}
