// Timing of the wide tridiagonalisation alone (diagnostics): the persistent
// one-launch kernel vs the per-step launches (FRECSYS_TRIDIAG_STEPS=1), same
// input, outputs compared bit for bit.  Links libfrecsys_hip.so's internal
// launcher through the kernels.h interface.
// hipcc --offload-arch=gfx950 -O3 -std=c++17 -I safer2-recommender_amd/csrc -c <this> -o t.o;
// hipcc --offload-arch=gfx950 t.o -L safer2-recommender_amd/frecsys_hip -lfrecsys_hip
//   -Wl,-rpath,$ORIGIN/../../safer2-recommender_amd/frecsys_hip -o tridiag_wide_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "kernels.h"
using namespace frecsys_hip;

int main(int argc, char** argv) {
  for (int n : {512, 1024}) {
    std::vector<float> G((size_t)n * n, 0.0f);
    srand(7);
    const int R = 2 * n;
    std::vector<float> X((size_t)R * n);
    for (auto& x : X) x = (rand() / (float)RAND_MAX - 0.5f) * 0.1f;
    for (int r = 0; r < R; ++r)
      for (int i = 0; i < n; ++i) {
        const float xi = X[(size_t)r * n + i];
        for (int j = 0; j < n; ++j) G[(size_t)i * n + j] += xi * X[(size_t)r * n + j];
      }
    float *dG, *dd, *de, *dV, *dt, *work;
    hipMalloc(&dG, 4ull * n * n);
    hipMalloc(&dd, 4 * n);
    hipMalloc(&de, 4 * n);
    hipMalloc(&dV, 4ull * n * n);
    hipMalloc(&dt, 4 * n);
    hipMalloc(&work, 4 * wide_tridiag_work_floats(n));
    hipMemcpy(dG, G.data(), 4ull * n * n, hipMemcpyHostToDevice);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    std::vector<float> ref;
    for (int variant = 0; variant < 4; ++variant) {
      const int steps = variant == 2;
      setenv("FRECSYS_TRIDIAG_STEPS", steps ? "1" : "0", 1);
      setenv("FRECSYS_TRIDIAG_FENCE", variant == 1 ? "1" : "0", 1);
      setenv("FRECSYS_TRIDIAG_TAGGED", variant == 3 ? "1" : "0", 1);  // default on in the library
      float best = 1e9f;
      for (int it = 0; it < 5; ++it) {
        hipEventRecord(a);
        launch_wide_tridiag(dG, n, dd, de, dV, dt, work, 0);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
      }
      std::vector<float> o(2 * n);
      hipMemcpy(o.data(), dd, 4 * n, hipMemcpyDeviceToHost);
      hipMemcpy(o.data() + n, de, 4 * n, hipMemcpyDeviceToHost);
      if (variant == 0) ref = o;
      const char* name[4] = {"persistent", "persistent+fences", "step launches", "tagged"};
      printf("n=%d %s: %.3f ms (%.2f us/step) %s\n", n, name[variant], best, best * 1e3 / n,
             memcmp(o.data(), ref.data(), 8 * n) == 0 ? "bit-identical" : "DIFFERS");
    }
  }
  return 0;
}
