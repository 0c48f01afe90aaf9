// probe_eig -- times rocSOLVER symmetric eigensolvers on a d x d Gramian
// (the per-half-step eigendecomposition the dual solve path needs).
// Build: hipcc --offload-arch=gfx950 -O2 scripts/probe_eig.cpp -lrocsolver -lrocblas
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

#define CK(x) do { auto e_ = (x); if (e_) { printf("err %d at %d\n", (int)e_, __LINE__); return 1; } } while (0)

template <typename T>
static double check(const std::vector<double>& G, const std::vector<T>& Q, const std::vector<T>& w, int n) {
  // column-major Q: Q[i + j*n] = eigvec j component i
  double num = 0, den = 0, orth = 0;
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < n; ++i) {
      double gq = 0;
      for (int k = 0; k < n; ++k) gq += G[i + k * n] * (double)Q[k + j * n];
      double r = gq - (double)w[j] * (double)Q[i + j * n];
      num += r * r;
      den += G[i + j * n] * G[i + j * n];
    }
  for (int a = 0; a < n; a += 7)
    for (int b = 0; b < n; ++b) {
      double s = 0;
      for (int k = 0; k < n; ++k) s += (double)Q[k + a * n] * (double)Q[k + b * n];
      orth = std::max(orth, std::fabs(s - (a == b)));
    }
  printf("   resid %.3e  orth %.3e  wmin %.4g wmax %.4g\n", std::sqrt(num / den), orth,
         (double)w[0], (double)w[n - 1]);
  return 0;
}

template <typename T>
static int run(rocblas_handle h, const char* name, int which, int n, const std::vector<double>& G) {
  std::vector<T> A(n * n);
  for (int i = 0; i < n * n; ++i) A[i] = (T)G[i];
  T *dA, *dW, *dE, *dR;
  rocblas_int *dInfo, *dSweeps;
  hipMalloc(&dA, sizeof(T) * n * n);
  hipMalloc(&dW, sizeof(T) * n);
  hipMalloc(&dE, sizeof(T) * n);
  hipMalloc(&dR, sizeof(T));
  hipMalloc(&dInfo, 4);
  hipMalloc(&dSweeps, 4);
  double best = 1e30;
  for (int rep = 0; rep < 6; ++rep) {
    hipMemcpy(dA, A.data(), sizeof(T) * n * n, hipMemcpyHostToDevice);
    hipDeviceSynchronize();
    auto t0 = std::chrono::steady_clock::now();
    rocblas_status s;
    if (which == 0) {
      if constexpr (sizeof(T) == 4) s = rocsolver_ssyevd(h, rocblas_evect_original, rocblas_fill_lower, n, dA, n, dW, dE, dInfo);
      else s = rocsolver_dsyevd(h, rocblas_evect_original, rocblas_fill_lower, n, dA, n, dW, dE, dInfo);
    } else if (which == 1) {
      if constexpr (sizeof(T) == 4) s = rocsolver_ssyevj(h, rocblas_esort_ascending, rocblas_evect_original, rocblas_fill_lower, n, dA, n, 0.0f, dR, 20, dSweeps, dW, dInfo);
      else s = rocsolver_dsyevj(h, rocblas_esort_ascending, rocblas_evect_original, rocblas_fill_lower, n, dA, n, 0.0, dR, 20, dSweeps, dW, dInfo);
    } else {
      if constexpr (sizeof(T) == 4) s = rocsolver_ssyevdj(h, rocblas_evect_original, rocblas_fill_lower, n, dA, n, dW, dInfo);
      else s = rocsolver_dsyevdj(h, rocblas_evect_original, rocblas_fill_lower, n, dA, n, dW, dInfo);
    }
    hipDeviceSynchronize();
    auto t1 = std::chrono::steady_clock::now();
    if (s) { printf("%s status %d\n", name, (int)s); return 1; }
    double ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
    if (rep > 0) best = std::min(best, ms);
  }
  std::vector<T> Q(n * n), w(n);
  hipMemcpy(Q.data(), dA, sizeof(T) * n * n, hipMemcpyDeviceToHost);
  hipMemcpy(w.data(), dW, sizeof(T) * n, hipMemcpyDeviceToHost);
  int info;
  hipMemcpy(&info, dInfo, 4, hipMemcpyDeviceToHost);
  printf("%-8s n=%d  best %.3f ms  info %d\n", name, n, best, info);
  check(G, Q, w, n);
  hipFree(dA); hipFree(dW); hipFree(dE); hipFree(dR); hipFree(dInfo); hipFree(dSweeps);
  return 0;
}

int main() {
  rocblas_handle h;
  CK(rocblas_create_handle(&h));
  for (int n : {256, 512}) {
    std::mt19937 rng(7);
    std::normal_distribution<double> nd(0, 0.3);
    const int m = 20000;
    std::vector<double> V((size_t)m * n), G((size_t)n * n, 0.0);
    for (auto& x : V) x = nd(rng);
    for (int r = 0; r < m; ++r)
      for (int i = 0; i < n; ++i) {
        double vi = V[(size_t)r * n + i];
        for (int j = 0; j <= i; ++j) G[i + j * n] += vi * V[(size_t)r * n + j];
      }
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < i; ++j) G[j + i * n] = G[i + j * n];
    run<float>(h, "ssyevd", 0, n, G);
    run<double>(h, "dsyevd", 0, n, G);
    run<float>(h, "ssyevj", 1, n, G);
    run<double>(h, "dsyevj", 1, n, G);
    run<float>(h, "ssyevdj", 2, n, G);
    run<double>(h, "dsyevdj", 2, n, G);
  }
  return 0;
}
