// ComputeXi / Evaluate timing of the host smoothed-quantile Newton (safer2.h)
// with the pool in include/frecsys/parallel.h.  Build (from the repo root):
//   g++ -O3 -std=c++17 -I include -I safer2-recommender_amd/include -pthread \
//     scripts/micro/xi.cc -o scripts/micro/xi_new -Lsafer2-recommender_amd/frecsys_hip \
//     -lfrecsys_hip -Wl,-rpath,$ORIGIN/../../safer2-recommender_amd/frecsys_hip
// (xi_old: the same against the previous parallel.h).
#include <chrono>
#include <cstdio>
#include <random>
#include <vector>
#include "frecsys/safer2.h"
int main() {
  std::mt19937 g(1);
  std::gamma_distribution<float> gd(2.0f, 0.5f);
  const int n = 11667;
  std::vector<float> loss(n);
  for (auto& v : loss) v = gd(g);
  frecsys::quantile::Smoother sm{0.3f, 0.18f, false};
  float xi = 1.0f;
  auto t0 = std::chrono::steady_clock::now();
  int evals = 0;
  for (int rep = 0; rep < 20; ++rep) {
    float x = xi;
    for (int t = 0; t < 5; ++t) x += sm.Direction(x, loss.data(), n);
  }
  auto t1 = std::chrono::steady_clock::now();
  printf("ComputeXi (5 iters, n=%d): %.3f ms\n", n, std::chrono::duration<double, std::milli>(t1 - t0).count() / 20);
  // single evaluate
  t0 = std::chrono::steady_clock::now();
  for (int rep = 0; rep < 200; ++rep) sm.Evaluate(1.0f, loss.data(), n);
  t1 = std::chrono::steady_clock::now();
  printf("Evaluate: %.3f us\n", std::chrono::duration<double, std::micro>(t1 - t0).count() / 200);
  // serial erfc cost
  t0 = std::chrono::steady_clock::now();
  double s = 0;
  for (int rep = 0; rep < 20; ++rep) for (int i = 0; i < n; ++i) s += std::erfc(-(double)(loss[i] - 1.0f) * 0.7);
  t1 = std::chrono::steady_clock::now();
  printf("serial erfc per sample: %.1f ns (%g)\n", std::chrono::duration<double, std::nano>(t1 - t0).count() / 20 / n, s);
}
