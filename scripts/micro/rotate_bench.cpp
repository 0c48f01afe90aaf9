// Timing of the basis rotation Y = X B alone (diagnostics): rotate_kernel
// (FRECSYS_ROT_RT=0) vs rotate_rt_kernel (RT row tiles per wave, X loads P
// steps ahead), at
// the two rotations the MSD / ML-20M epochs run (471,355 x 512 and
// 116,677 x 256), outputs compared bit for bit.  Links libfrecsys_hip.so's
// internal launchers through the kernels.h interface.
// hipcc --offload-arch=gfx950 -O3 -std=c++17 -I safer2-recommender_amd/csrc -c <this> -o r.o;
// hipcc --offload-arch=gfx950 r.o -L safer2-recommender_amd/frecsys_hip -lfrecsys_hip
//   -Wl,-rpath,$ORIGIN/../../safer2-recommender_amd/frecsys_hip -o rotate_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "kernels.h"
using namespace frecsys_hip;

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e_ = (x);                                               \
    if (e_ != hipSuccess) {                                            \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));          \
      return 1;                                                        \
    }                                                                  \
  } while (0)

int main() {
  struct Case { int64_t n; int dp; };
  for (Case cs : {Case{471355, 512}, Case{116677, 256}}) {
    const int64_t n = cs.n;
    const int dp = cs.dp;
    std::vector<float> X((size_t)n * dp), B((size_t)dp * dp);
    srand(11);
    for (auto& x : X) x = (rand() / (float)RAND_MAX - 0.5f);
    for (auto& x : B) x = (rand() / (float)RAND_MAX - 0.5f) * 0.1f;
    float *dX, *dB, *dY;
    void* img;
    CK(hipMalloc(&dX, 4 * X.size()));
    CK(hipMalloc(&dY, 4 * X.size()));
    CK(hipMalloc(&dB, 4 * B.size()));
    CK(hipMalloc(&img, basis_split_bytes(dp)));
    CK(hipMemcpy(dX, X.data(), 4 * X.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, B.data(), 4 * B.size(), hipMemcpyHostToDevice));
    CK(launch_split_basis(dB, dp, 0, img, 0));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<float> ref, out(X.size());
    // RT 0: rotate_kernel (one step ahead); rtp = RT * 10 + P for rotate_rt_kernel
    for (int rtp : {0, 12, 14, 22, 24}) {
      const int rt = rtp / 10;
      char b1[8], b2[8];
      snprintf(b1, sizeof b1, "%d", rt);
      snprintf(b2, sizeof b2, "%d", rtp % 10);
      setenv("FRECSYS_ROT_RT", b1, 1);
      setenv("FRECSYS_ROT_P", b2, 1);
      float best = 1e9f;
      for (int it = 0; it < 5; ++it) {
        CK(hipEventRecord(a));
        CK(launch_rotate(dX, nullptr, 0, n, img, dY, dp, 0));
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (ms < best) best = ms;
      }
      CK(hipMemcpy(out.data(), dY, 4 * out.size(), hipMemcpyDeviceToHost));
      if (rtp == 0) ref = out;
      const double flops = 2.0 * n * dp * dp, bytes = 8.0 * n * dp;
      printf("n=%lld dp=%d RT=%d P=%d: %.3f ms (%.1f TFLOP/s algorithmic, %.2f TB/s X+Y) %s\n",
             (long long)n, dp, rt, rtp % 10, best, flops / best / 1e9, bytes / best / 1e9,
             memcmp(out.data(), ref.data(), 4 * out.size()) == 0 ? "bit-identical" : "DIFFERS");
    }
    CK(hipFree(dX));
    CK(hipFree(dY));
    CK(hipFree(dB));
    CK(hipFree(img));
  }
  return 0;
}
