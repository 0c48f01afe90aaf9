// loss.hip -- per-user loss on gfx950.
//
// Replaces ComputeUserLoss / ComputeLoss (ials.h:70-86 + 367-408,
// safer2.h:85-101 + 558-596): l_u = (1/h) sum_j (x_j . u - 1)^2
// + beta u^T G u, halved for ERM-MF / CVaR-MF / SAFER2.  One wave per user:
// the history rows are gathered by groups of lanes (float4 per lane, one
// row per group), dot products reduced inside the group; u^T G u reads G
// rows coalesced from L2 with u staged in LDS.
#include <hip/hip_runtime.h>

#include "common.h"
#include "kernels.h"

namespace frecsys_hip {

namespace {

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
  return v;
}

constexpr int pow2_at_least(int x) {
  int p = 1;
  while (p < x) p <<= 1;
  return p;
}

template <int Dp>
__global__ void __launch_bounds__(256) user_loss_kernel(LossArgs a) {
  constexpr int WPB = 4;
  constexpr int LPR = pow2_at_least(Dp / 4) > 64 ? 64 : pow2_at_least(Dp / 4);
  constexpr int RPP = 64 / LPR;
  __shared__ __attribute__((aligned(16))) float su[WPB][Dp];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t idx = (int64_t)blockIdx.x * WPB + wave;
  if (idx >= a.n_rows) return;
  const int64_t e = a.row_lo + idx;
  const int64_t p0 = a.row_ptr[e];
  const int64_t h = a.row_ptr[e + 1] - p0;
  if (h == 0) return;
  const int g = lane / LPR, c4 = lane % LPR;
  const bool has = c4 < Dp / 4;
  float4 u4 = make_float4(0.f, 0.f, 0.f, 0.f);
  if (has) {
    u4 = *reinterpret_cast<const float4*>(a.U + e * Dp + 4 * c4);
    if (g == 0) *reinterpret_cast<float4*>(&su[wave][4 * c4]) = u4;
  }
  float sq = 0.0f;
  for (int64_t k0 = 0; k0 < h; k0 += RPP) {
    const int64_t k = k0 + g;
    float d = 0.0f;
    if (k < h && has) {
      const int id = a.col[p0 + k];
      const float4 x = *reinterpret_cast<const float4*>(a.V + (int64_t)id * Dp + 4 * c4);
      d = x.x * u4.x + x.y * u4.y + x.z * u4.z + x.w * u4.w;
    }
#pragma unroll
    for (int off = LPR / 2; off >= 1; off >>= 1) d += __shfl_xor(d, off);
    if (c4 == 0 && k < h) {
      const float t = d - 1.0f;
      sq = (float)((double)sq + (double)t * (double)t);
    }
  }
  sq = wave_sum(sq);
  float loss = sq / (float)h;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  float ir = 0.0f;
  for (int j = lane; j < Dp; j += 64) {
    float t = 0.0f;
    for (int i = 0; i < Dp; ++i) t += su[wave][i] * a.G[i * Dp + j];
    ir += t * su[wave][j];
  }
  ir = wave_sum(ir);
  loss += a.beta * ir;
  if (a.half) loss = (float)((double)loss / 2.0);
  if (lane == 0) a.out[e] = loss;
}

template <int Dp>
hipError_t launch(const LossArgs& a, hipStream_t s) {
  const unsigned nb = (unsigned)((a.n_rows + 3) / 4);
  hipLaunchKernelGGL(user_loss_kernel<Dp>, dim3(nb), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_user_loss(int Dp, const LossArgs& a, hipStream_t s) {
  if (a.n_rows <= 0) return hipSuccess;
  switch (Dp) {
    case 8: return launch<8>(a, s);
    case 16: return launch<16>(a, s);
    case 32: return launch<32>(a, s);
    case 64: return launch<64>(a, s);
    case 96: return launch<96>(a, s);
    case 128: return launch<128>(a, s);
    case 160: return launch<160>(a, s);
    case 192: return launch<192>(a, s);
    case 224: return launch<224>(a, s);
    case 256: return launch<256>(a, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace frecsys_hip
