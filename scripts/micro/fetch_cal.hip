// FETCH_SIZE calibration of this code's access widths (diagnostics):
// MI355X_MICROARCH.md says FETCH_SIZE reports half the bytes of 16-B/lane
// streaming reads and leaves other widths uncalibrated.  Three kernels read a
// 1.2 GB buffer (past the 256 MiB Infinity Cache) exactly once:
//   k16: float4 per lane, streaming;
//   k4 : one float per lane, 64 lanes = 256 contiguous bytes (the row
//        gathers of wide_syrk2_kernel / solve_tiled_kernel);
//   kg4: the same 4-B/lane reads over whole 2-KB rows in a random row order
//        (a gather of a 0.97 GB table: the MSD item half-step's pattern).
// rocprofv3 --pmc FETCH_SIZE -- ./fetch_cal  -> FETCH_SIZE per dispatch vs the
// printed byte count gives the factor per width.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
#include <random>

__global__ void k16(const float4* __restrict__ x, size_t n4, float* out) {
  float acc = 0.f;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
    const float4 v = x[i];
    acc += v.x + v.y + v.z + v.w;
  }
  if (acc == 1234.5f) out[0] = acc;
}
__global__ void k4(const float* __restrict__ x, size_t n, float* out) {
  float acc = 0.f;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) acc += x[i];
  if (acc == 1234.5f) out[0] = acc;
}
// one wave per row visit: 512 floats per row, lane reads 8 floats (4 B each)
__global__ void kg4(const float* __restrict__ x, const int* __restrict__ rows, int nrows, float* out) {
  const int w = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  float acc = 0.f;
  for (int r = w; r < nrows; r += gridDim.x * 4) {
    const float* p = x + (size_t)rows[r] * 512;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += p[64 * j + lane];
  }
  if (acc == 1234.5f) out[0] = acc;
}

int main() {
  const size_t rows = 600000, n = rows * 512;  // 1.23 GB
  float *x, *out;
  int* perm;
  hipMalloc(&x, n * 4);
  hipMalloc(&out, 4);
  hipMalloc(&perm, rows * 4);
  hipMemset(x, 0, n * 4);
  std::vector<int> p(rows);
  for (size_t i = 0; i < rows; ++i) p[i] = (int)i;
  std::shuffle(p.begin(), p.end(), std::mt19937(3));
  hipMemcpy(perm, p.data(), rows * 4, hipMemcpyHostToDevice);
  for (int it = 0; it < 2; ++it) {
    hipLaunchKernelGGL(k16, dim3(4096), dim3(256), 0, 0, (const float4*)x, n / 4, out);
    hipLaunchKernelGGL(k4, dim3(4096), dim3(256), 0, 0, x, n, out);
    hipLaunchKernelGGL(kg4, dim3(4096), dim3(256), 0, 0, x, perm, (int)rows, out);
  }
  hipDeviceSynchronize();
  printf("bytes read per dispatch: %zu (k16, k4, kg4; kg4 + %zu B of row ids)\n", n * 4, rows * 4);
  return 0;
}
