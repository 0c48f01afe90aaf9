// spectral.hip -- the per-half-step basis change of the history-space
// solve (dual.hip): G = Q T Q^T with Q orthogonal and T tridiagonal, and
// the rotations X -> X Q (other side, before the solve) and X' -> X' Q^T
// (solved rows, after it).
//
// The reference has no counterpart (it forms every d x d normal matrix,
// ials.h:101-131); this is the MI355X re-design that lets the short-history
// entities solve an h x h system instead.
//
//  tridiag_kernel  one workgroup, 16 waves: Householder reduction of the
//                  lower-packed matrix held in LDS (Dp(Dp+1)/2 floats, 129 KB
//                  at Dp = 256), LAPACK sytd2 conventions (v(k+1) = 1).
//  form_q_kernel   Q = H_0 ... H_{n-3}, one wave per column of Q.
//  rot_gemm_kernel 64 rows x Dp columns per workgroup, v_mfma_f32_32x32x2_f32,
//                  the row block in LDS and Q streamed through LDS by 32-row
//                  slabs; optional entity list for gather/scatter.
#include <hip/hip_runtime.h>

#include "common.h"
#include "kernels.h"

namespace frecsys_hip {

namespace {

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// packed lower index, i >= j
__device__ __forceinline__ int pk(int i, int j) { return i * (i + 1) / 2 + j; }

__global__ void __launch_bounds__(1024)
    tridiag_kernel(const float* __restrict__ G, int n, float* tdiag, float* toff, float* Vh,
                   float* tau_out) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int np = n * (n + 1) / 2;
  float* P = sm;
  float* v = P + np;
  float* p = v + n;
  float* part = p + n;      // [4][256]
  float* sc = part + 1024;  // [0..1] tau slots, [4..7] dot partials
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = wave; i < n; i += 16)
    for (int j = lane; j <= i; j += 64) P[pk(i, j)] = G[(int64_t)i * n + j];
  __syncthreads();
  for (int k = 0; k < n - 2; ++k) {
    const int m = n - k - 1;
    if (wave == 0) {
      // reflector for column k below the diagonal (LAPACK slarfg)
      const float x0 = P[pk(k + 1, k)];
      float s = 0.0f;
      for (int i = k + 2 + lane; i < n; i += 64) {
        const float x = P[pk(i, k)];
        s += x * x;
      }
      s = wave_sum(s);
      float tau = 0.0f, beta = x0, scal = 0.0f;
      if (s > 0.0f) {
        const float nrm = sqrtf(x0 * x0 + s);
        beta = x0 >= 0.0f ? -nrm : nrm;
        tau = (beta - x0) / beta;
        scal = 1.0f / (x0 - beta);
      }
      for (int i = k + 1 + lane; i < n; i += 64) {
        const float vi = (i == k + 1) ? 1.0f : P[pk(i, k)] * scal;
        v[i] = vi;
        Vh[(int64_t)k * n + i] = vi;
      }
      if (lane == 0) {
        sc[k & 1] = tau;
        tdiag[k] = P[pk(k, k)];
        toff[k] = beta;
        tau_out[k] = tau;
      }
    }
    __syncthreads();
    const float tau = sc[k & 1];
    if (tau == 0.0f) continue;  // column already reduced: A22 unchanged
    // p = tau * A22 v, four threads per row
    const int ro = tid >> 2, t = tid & 3;
    const int i = k + 1 + ro;
    float acc = 0.0f;
    if (i < n) {
      for (int j = k + 1 + t; j < n; j += 4) acc += P[j <= i ? pk(i, j) : pk(j, i)] * v[j];
    }
    part[t * 256 + ro] = acc;
    __syncthreads();
    float dp = 0.0f;
    if (tid < m) {
      const int ii = k + 1 + tid;
      const float pi = tau * ((part[tid] + part[256 + tid]) + (part[512 + tid] + part[768 + tid]));
      p[ii] = pi;
      dp = pi * v[ii];
    }
    dp = wave_sum(dp);
    if (lane == 0 && wave < 4) sc[4 + wave] = dp;
    __syncthreads();
    const float K = 0.5f * tau * ((sc[4] + sc[5]) + (sc[6] + sc[7]));
    // A22 -= v w^T + w v^T,  w = p - K v
    if (i < n) {
      const float vi = v[i], wi = p[i] - K * vi;
      for (int j = k + 1 + t; j <= i; j += 4) {
        const float vj = v[j], wj = p[j] - K * vj;
        P[pk(i, j)] -= vi * wj + wi * vj;
      }
    }
    __syncthreads();
  }
  if (tid == 0) {
    tdiag[n - 2] = P[pk(n - 2, n - 2)];
    tdiag[n - 1] = P[pk(n - 1, n - 1)];
    toff[n - 2] = P[pk(n - 1, n - 2)];
    toff[n - 1] = 0.0f;
    tau_out[n - 2] = 0.0f;
    tau_out[n - 1] = 0.0f;
  }
}

// One wave per column c of Q: q = H_0 (H_1 (... H_{n-3} e_c)); H_k leaves
// columns c <= k alone, so the product starts at k = min(c-1, n-3).
__global__ void __launch_bounds__(256)
    form_q_kernel(const float* __restrict__ Vh, const float* __restrict__ tau, int n, float* Q) {
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (c >= n) return;  // no barriers below
  float q[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) q[r] = (lane + 64 * r == c) ? 1.0f : 0.0f;
  int k = c - 1 < n - 3 ? c - 1 : n - 3;
  float vn[4];
  auto load = [&](int kk, float* dst) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = lane + 64 * r;
      dst[r] = (kk >= 0 && row > kk && row < n) ? Vh[(int64_t)kk * n + row] : 0.0f;
    }
  };
  load(k, vn);
  for (; k >= 0; --k) {
    float vk[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) vk[r] = vn[r];
    const float t = tau[k];
    load(k - 1, vn);  // prefetch the next reflector under this one's reduction
    if (t == 0.0f) continue;
    float d = 0.0f;
#pragma unroll
    for (int r = 0; r < 4; ++r) d += vk[r] * q[r];
    d = wave_sum(d) * t;
#pragma unroll
    for (int r = 0; r < 4; ++r) q[r] -= d * vk[r];
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = lane + 64 * r;
    if (row < n) Q[(int64_t)row * n + c] = q[r];
  }
}

// Y = X B, B = Q or Q^T; 64 rows per workgroup, 4 waves, tiles of 32x32.
template <int NCT>
__global__ void __launch_bounds__(256)
    rot_gemm_kernel(const float* __restrict__ X, const QueueRec* __restrict__ rows, int64_t r0,
                    int64_t n, const float* __restrict__ Q, int trans, float* __restrict__ Y) {
  constexpr int Dp = 32 * NCT, XS = Dp + 1;
  constexpr int NTILE = 2 * NCT, MT = (NTILE + 3) / 4;
  __shared__ float xs[64 * XS];
  __shared__ float bs[32 * Dp];
  __shared__ int64_t rid[64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lo = lane & 31, hi = lane >> 5;
  const int64_t base = (int64_t)blockIdx.x * 64;
  if (tid < 64) {
    const int64_t r = base + tid;
    rid[tid] = r < n ? (rows ? (int64_t)rows[r].entity : r0 + r) : -1;
  }
  __syncthreads();
  for (int s = tid; s < 64 * (Dp / 4); s += 256) {
    const int rr = s / (Dp / 4), c4 = s % (Dp / 4);
    const int64_t id = rid[rr];
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (id >= 0) v = *reinterpret_cast<const float4*>(X + id * Dp + 4 * c4);
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
    __syncthreads();  // xs ready / previous slab consumed
    if (!trans) {
      for (int s = tid; s < 32 * (Dp / 4); s += 256) {
        const int kk = s / (Dp / 4), c4 = s % (Dp / 4);
        *reinterpret_cast<float4*>(bs + kk * Dp + 4 * c4) =
            *reinterpret_cast<const float4*>(Q + (int64_t)(32 * c + kk) * Dp + 4 * c4);
      }
    } else {  // bs[kk][j] = Q[j][32c + kk]
      for (int s = tid; s < Dp * 8; s += 256) {
        const int j = s >> 3, k4 = s & 7;
        const float4 v = *reinterpret_cast<const float4*>(Q + (int64_t)j * Dp + 32 * c + 4 * k4);
        bs[(4 * k4 + 0) * Dp + j] = v.x;
        bs[(4 * k4 + 1) * Dp + j] = v.y;
        bs[(4 * k4 + 2) * Dp + j] = v.z;
        bs[(4 * k4 + 3) * Dp + j] = v.w;
      }
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
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int t = wave + 4 * m;
    if (t < NTILE) {
      const int R = t & 1, C = t >> 1;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int64_t id = rid[32 * R + acc_row(q, hi)];
        if (id >= 0) Y[id * Dp + 32 * C + lo] = acc[m][q];
      }
    }
  }
}

template <int NCT>
hipError_t launch_rot(const float* X, const QueueRec* rows, int64_t r0, int64_t n,
                      const float* Q, int trans, float* Y, hipStream_t s) {
  const unsigned nb = (unsigned)((n + 63) / 64);
  hipLaunchKernelGGL(rot_gemm_kernel<NCT>, dim3(nb), dim3(256), 0, s, X, rows, r0, n, Q, trans, Y);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_tridiag(const float* G, int Dp, float* tdiag, float* toff, float* Vh,
                          float* tau, hipStream_t s) {
  if (Dp < 4 || Dp > 256) return hipErrorInvalidValue;
  const size_t bytes = sizeof(float) * ((size_t)Dp * (Dp + 1) / 2 + 2 * Dp + 1024 + 8);
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)tridiag_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr = true;
  }
  hipLaunchKernelGGL(tridiag_kernel, dim3(1), dim3(1024), bytes, s, G, Dp, tdiag, toff, Vh, tau);
  return hipGetLastError();
}

hipError_t launch_form_q(const float* Vh, const float* tau, int Dp, float* Q, hipStream_t s) {
  if (Dp < 4 || Dp > 256) return hipErrorInvalidValue;
  hipLaunchKernelGGL(form_q_kernel, dim3((unsigned)((Dp + 3) / 4)), dim3(256), 0, s, Vh, tau, Dp,
                     Q);
  return hipGetLastError();
}

hipError_t launch_rot_gemm(const float* X, const QueueRec* rows, int64_t r0, int64_t n,
                           const float* Q, int trans, float* Y, int Dp, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  switch (Dp) {
    case 64: return launch_rot<2>(X, rows, r0, n, Q, trans, Y, s);
    case 96: return launch_rot<3>(X, rows, r0, n, Q, trans, Y, s);
    case 128: return launch_rot<4>(X, rows, r0, n, Q, trans, Y, s);
    case 160: return launch_rot<5>(X, rows, r0, n, Q, trans, Y, s);
    case 192: return launch_rot<6>(X, rows, r0, n, Q, trans, Y, s);
    case 224: return launch_rot<7>(X, rows, r0, n, Q, trans, Y, s);
    case 256: return launch_rot<8>(X, rows, r0, n, Q, trans, Y, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace frecsys_hip
