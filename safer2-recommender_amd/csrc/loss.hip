// loss.hip -- per-user loss on gfx950.
//
// Replaces ComputeUserLoss / ComputeLoss (ials.h:70-86 + 367-408,
// safer2.h:85-101 + 558-596): l_u = (1/h) sum_j (x_j . u - 1)^2
// + beta u^T G u, halved for ERM-MF / CVaR-MF / SAFER2.
//
// Dp >= 32: two passes.  quad_kernel computes q_u = u^T G u for 64 users per
// workgroup as an MFMA product U G (U rows in LDS, G streamed by 32-row
// slabs) with a row-dot epilogue -- G is read once per 64 users instead of
// once per user.  loss_gather_kernel: one wave per user, eight lanes per
// history row and eight rows in flight (8 x float4 per lane), dot products
// reduced by DPP inside each 8-lane group.
// Dp = 8, 16: user_loss_kernel, one wave per user, u^T G u from L2.
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
  if (a.raw) {
    if (lane == 0) a.out[e] = sq;
    return;
  }
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


// Sum inside groups of 8 consecutive lanes (every lane gets its group's sum).
__device__ __forceinline__ float group8_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, false));
  return v;
}

// q[r] = u_r^T G u_r for rows row_lo .. row_lo + n_rows - 1.
template <int NCT>
__global__ void __launch_bounds__(256) quad_kernel(LossArgs a) {
  constexpr int Dp = 32 * NCT, XS = Dp + 1;
  constexpr int NTILE = 2 * NCT, MT = (NTILE + 3) / 4;
  __shared__ float xs[64 * XS];
  __shared__ float bs[32 * Dp];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lo = lane & 31, hi = lane >> 5;
  const int64_t base = (int64_t)blockIdx.x * 64;
  for (int s = tid; s < 64 * (Dp / 4); s += 256) {
    const int rr = s / (Dp / 4), c4 = s % (Dp / 4);
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (base + rr < a.n_rows)
      v = *reinterpret_cast<const float4*>(a.U + (a.row_lo + base + rr) * Dp + 4 * c4);
    float* d = xs + rr * XS + 4 * c4;
    d[0] = v.x;
    d[1] = v.y;
    d[2] = v.z;
    d[3] = v.w;
  }
  f32x16 acc[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) acc[m] = f32x16{0.f};
  for (int c = 0; c < NCT; ++c) {
    __syncthreads();
    for (int s = tid; s < 32 * (Dp / 4); s += 256) {
      const int kk = s / (Dp / 4), c4 = s % (Dp / 4);
      *reinterpret_cast<float4*>(bs + kk * Dp + 4 * c4) =
          *reinterpret_cast<const float4*>(a.G + (int64_t)(32 * c + kk) * Dp + 4 * c4);
    }
    __syncthreads();
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const int t = wave + 4 * m;
      if (t < NTILE) {
        const int R = t & 1, C = t >> 1;
#pragma unroll
        for (int s = 0; s < 16; ++s) {
          const int kk = 2 * s + hi;
          acc[m] = mfma32(xs[(32 * R + lo) * XS + 32 * c + kk], bs[kk * Dp + 32 * C + lo], acc[m]);
        }
      }
    }
  }
  __syncthreads();
  // (U G)[r][c] * U[r][c] in place (each element has one owner), then row sums
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int t = wave + 4 * m;
    if (t < NTILE) {
      const int R = t & 1, C = t >> 1;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        float* x = xs + (32 * R + acc_row(q, hi)) * XS + 32 * C + lo;
        *x = acc[m][q] * *x;
      }
    }
  }
  __syncthreads();
  if (tid < 64 && base + tid < a.n_rows) {
    float qv = 0.0f;
    const float* x = xs + tid * XS;
    for (int c = 0; c < Dp; ++c) qv += x[c];
    a.quad[a.row_lo + base + tid] = qv;
  }
}

// One wave per user: 8 groups of 8 lanes, one history row per group per
// step, each lane 8 float4 of the row (the group reads 128 contiguous
// bytes per instruction).
template <int Dp>
__global__ void __launch_bounds__(256) loss_gather_kernel(LossArgs a) {
  constexpr int WPB = 4, Q = Dp / 32;  // float4 per lane per row
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t idx = (int64_t)blockIdx.x * WPB + wave;
  if (idx >= a.n_rows) return;
  const int64_t e = a.row_lo + idx;
  const int64_t p0 = a.row_ptr[e];
  const int64_t h = a.row_ptr[e + 1] - p0;
  if (h == 0) return;
  const int g = lane >> 3, c = lane & 7;
  float4 u4[Q];
#pragma unroll
  for (int q = 0; q < Q; ++q)
    u4[q] = *reinterpret_cast<const float4*>(a.U + e * Dp + 4 * (c + 8 * q));
  float sq = 0.0f;
  for (int64_t k0 = 0; k0 < h; k0 += 8) {
    const int64_t k = k0 + g;
    float d = 0.0f;
    if (k < h) {
      const int id = a.col[p0 + k];
      const float* x = a.V + (int64_t)id * Dp;
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const float4 v = *reinterpret_cast<const float4*>(x + 4 * (c + 8 * q));
        d += v.x * u4[q].x + v.y * u4[q].y + v.z * u4[q].z + v.w * u4[q].w;
      }
    }
    d = group8_sum(d);
    if (c == 0 && k < h) {
      const float t = d - 1.0f;
      sq = (float)((double)sq + (double)t * (double)t);
    }
  }
  sq = wave_sum(sq);
  if (a.raw) {
    if (lane == 0) a.out[e] = sq;
    return;
  }
  float qv;
  if (a.quad_parts > 0) {  // u^T G u from the rotation kernel's column-block partials
    qv = 0.0f;
    for (int b = 0; b < a.quad_parts; ++b) qv += a.quad[(int64_t)b * a.n_rows + idx];
  } else {
    qv = a.quad[e];
  }
  float loss = sq / (float)h + a.beta * qv;
  if (a.half) loss = (float)((double)loss / 2.0);
  if (lane == 0) a.out[e] = loss;
}

template <int NCT>
hipError_t launch2(const LossArgs& a, hipStream_t s) {
  constexpr int Dp = 32 * NCT;
  const unsigned nq = (unsigned)((a.n_rows + 63) / 64);
  if (!a.raw && a.quad_parts > 0) {
    // u^T G u as (U G) .* U on the bf16 matrix cores (fp32-accurate split
    // products; spectral.hip rotate_kernel with the row-dot epilogue): 4x
    // the rate of quad_kernel's f32 MFMA at Dp = 256
    hipError_t e = launch_split_basis(a.G, Dp, 0, a.gsplit, s);
    if (e != hipSuccess) return e;
    e = launch_rotate_quad(a.U, a.row_lo, a.n_rows, a.gsplit, a.quad, Dp, s);
    if (e != hipSuccess) return e;
  } else if (!a.raw) {
    hipLaunchKernelGGL(quad_kernel<NCT>, dim3(nq), dim3(256), 0, s, a);
  }
  const unsigned nb = (unsigned)((a.n_rows + 3) / 4);
  if (a.ev_gather) (void)hipEventRecord(a.ev_gather, s);
  hipLaunchKernelGGL(loss_gather_kernel<Dp>, dim3(nb), dim3(256), 0, s, a);
  return hipGetLastError();
}

template <int Dp>
hipError_t launch(const LossArgs& a, hipStream_t s) {
  const unsigned nb = (unsigned)((a.n_rows + 3) / 4);
  hipLaunchKernelGGL(user_loss_kernel<Dp>, dim3(nb), dim3(256), 0, s, a);
  return hipGetLastError();
}

// ||X[r] - Y[r]||^2 (Y may be null: ||X[r]||^2), one wave per row.
__global__ void __launch_bounds__(256) row_norm2_kernel(const float* __restrict__ X,
                                                        const float* __restrict__ Y, int64_t n,
                                                        int Dp, float* __restrict__ out) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= n) return;
  float s = 0.0f;
  for (int j = lane; j < Dp; j += 64) {
    const float v = Y ? X[r * Dp + j] - Y[r * Dp + j] : X[r * Dp + j];
    s += v * v;
  }
  s = wave_sum(s);
  if (lane == 0) out[r] = s;
}

// sum_ij A_ij B_ij in double, one workgroup.
__global__ void __launch_bounds__(256) gram_dot_kernel(const float* __restrict__ A,
                                                       const float* __restrict__ B, int Dp,
                                                       double* __restrict__ dot) {
  __shared__ double red[256];
  double s = 0.0;
  for (int64_t i = threadIdx.x; i < (int64_t)Dp * Dp; i += 256) s += (double)A[i] * (double)B[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) dot[0] = red[0];
}

}  // namespace

hipError_t launch_row_norm2(const float* X, int64_t n, int Dp, float* out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(row_norm2_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, s, X,
                     (const float*)nullptr, n, Dp, out);
  return hipGetLastError();
}

hipError_t launch_row_diff2(const float* X, const float* Y, int64_t n, int Dp, float* out,
                            hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(row_norm2_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, s, X, Y, n,
                     Dp, out);
  return hipGetLastError();
}

hipError_t launch_gram_dot(const float* A, const float* B, int Dp, double* dot, hipStream_t s) {
  hipLaunchKernelGGL(gram_dot_kernel, dim3(1), dim3(256), 0, s, A, B, Dp, dot);
  return hipGetLastError();
}

hipError_t launch_user_loss(int Dp, const LossArgs& a, hipStream_t s) {
  if (a.n_rows <= 0) return hipSuccess;
  if (wide_dim(Dp)) return launch_wide_user_loss(Dp, a, s);
  switch (Dp) {
    case 8: return launch<8>(a, s);
    case 16: return launch<16>(a, s);
    case 32: return launch2<1>(a, s);
    case 64: return launch2<2>(a, s);
    case 96: return launch2<3>(a, s);
    case 128: return launch2<4>(a, s);
    case 160: return launch2<5>(a, s);
    case 192: return launch2<6>(a, s);
    case 224: return launch2<7>(a, s);
    case 256: return launch2<8>(a, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace frecsys_hip
