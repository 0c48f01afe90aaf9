// Correctness check of diag_factor_inv: L L^T = A and L^-1 L = I (host).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <random>
#include "../../safer2-recommender_amd/csrc/chol.h"
using namespace frecsys_hip;
__global__ void run(const float* A, float* Linv, float* Lrow, int* ok) {
  __shared__ float tile[1024];
  const int lane = threadIdx.x;
  for (int i = lane; i < 1024; i += 64) tile[sw(i >> 5, i & 31)] = A[i];
  __syncthreads();
  ok[0] = diag_factor_inv<FRECSYS_DIAG_BLK != 0>(tile, lane);
  __syncthreads();
  for (int i = lane; i < 1024; i += 64) Linv[i] = tile[sw(i >> 5, i & 31)];
}
int main() {
  std::mt19937 g(3);
  std::normal_distribution<double> nd;
  double B[32][40];
  for (auto& row : B) for (double& x : row) x = nd(g);
  float A[1024];
  for (int i = 0; i < 32; ++i)
    for (int j = 0; j < 32; ++j) {
      double s = (i == j) ? 2.0 : 0.0;
      for (int k = 0; k < 40; ++k) s += B[i][k] * B[j][k];
      A[i * 32 + j] = (float)s;
    }
  float *dA, *dL, *dR; int* dok;
  hipMalloc(&dA, 4096); hipMalloc(&dL, 4096); hipMalloc(&dR, 4096); hipMalloc(&dok, 4);
  hipMemcpy(dA, A, 4096, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(run, dim3(1), dim3(64), 0, 0, dA, dL, dR, dok);
  float Li[1024]; int ok;
  hipMemcpy(Li, dL, 4096, hipMemcpyDeviceToHost);
  hipMemcpy(&ok, dok, 4, hipMemcpyDeviceToHost);
  // check Linv * A * Linv^T = I
  double err = 0;
  for (int i = 0; i < 32; ++i)
    for (int j = 0; j < 32; ++j) {
      double s = 0;
      for (int k = 0; k < 32; ++k)
        for (int l = 0; l < 32; ++l) s += (double)Li[i * 32 + k] * A[k * 32 + l] * Li[j * 32 + l];
      err = std::max(err, std::fabs(s - (i == j)));
    }
  double up = 0;
  for (int i = 0; i < 32; ++i) for (int j = i + 1; j < 32; ++j) up = std::max(up, (double)std::fabs(Li[i * 32 + j]));
  printf("ok %d  max|Linv A Linv^T - I| = %.3e  upper max %.3e\n", ok, err, up);
  return 0;
}
