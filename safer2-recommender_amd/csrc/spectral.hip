// spectral.hip -- the per-half-step basis change of the history-space
// solve (dual.hip): G = Q T Q^T with Q orthogonal and T tridiagonal, and
// the rotations X -> X Q (other side, before the solve) and X' -> X' Q^T
// (solved rows, after it).
//
// The reference has no counterpart (it forms every d x d normal matrix,
// ials.h:101-131); this is the MI355X re-design that lets the short-history
// entities solve an h x h system instead.
//
//  tridiag_kernel  one workgroup, 16 waves: Householder reduction with the
//                  matrix in registers (an 8 x 8 block per thread), LAPACK
//                  sytd2 conventions (v(k+1) = 1).
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

// Sum over a full wave with DPP row ops (no LDS round trips); every lane
// gets the total.
__device__ __forceinline__ float wave_sum_dpp(float v) {
  auto dpp = [](float x, int ctrl, int row_mask) -> float {
    switch (ctrl) {  // the control word must be a compile-time constant
      case 0xB1: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0xB1, 0xF, 0xF, false));
      case 0x4E: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x4E, 0xF, 0xF, false));
      case 0x141: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x141, 0xF, 0xF, false));
      case 0x140: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x140, 0xF, 0xF, false));
      case 0x142: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x142, 0xA, 0xF, false));
      default: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x143, 0xC, 0xF, false));
    }
    (void)row_mask;
  };
  v += dpp(v, 0xB1, 0xF);   // quad_perm [1,0,3,2]
  v += dpp(v, 0x4E, 0xF);   // quad_perm [2,3,0,1]
  v += dpp(v, 0x141, 0xF);  // row_half_mirror
  v += dpp(v, 0x140, 0xF);  // row_mirror: 16-lane row sums
  v += dpp(v, 0x142, 0xA);  // row_bcast15 into rows 1, 3
  v += dpp(v, 0x143, 0xC);  // row_bcast31 into rows 2, 3: lane 63 = total
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

// Householder tridiagonalisation, register-resident: the 1024 threads hold
// the FULL symmetric matrix (zero-padded to 256) as 8 x 8 blocks; thread
// t owns block row bi = t & 31 of block column bj = t >> 5, so the owners
// of one block column are 32 lanes of one wave.  Step k (LAPACK sytd2,
// lower): the wave owning column k forms the reflector v (v_{k+1} = 1),
// tau, beta right after its own update of step k-1 and publishes v;
// p = tau A v (8x8 block products, partial row sums reduced through LDS,
// v^T A v reduced alongside for K); w = p - K v, K = (tau/2) v.p;
// A -= v w^T + w v^T on the whole matrix -- v is zero on rows <= k, so this
// is exactly H A H and the trailing block sees the textbook arithmetic.
// Three barriers per step.
__global__ void __launch_bounds__(1024)
    tridiag_kernel(const float* __restrict__ G, int n, float* tdiag, float* toff, float* Vh,
                   float* tau_out) {
  __shared__ float vs[2][256];
  __shared__ float ps[256];
  __shared__ float part[32 * 257];
  __shared__ float red[2][16];
  __shared__ float tsh[2];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int bi = tid & 31, bj = tid >> 5;
  const int r0 = 8 * bi, c0 = 8 * bj;
  float A[8][8];
#pragma unroll
  for (int r = 0; r < 8; ++r)
#pragma unroll
    for (int c = 0; c < 8; ++c)
      A[r][c] = (r0 + r < n && c0 + c < n) ? G[(int64_t)(r0 + r) * n + c0 + c] : 0.0f;

  // reflector for column k, by the wave that owns it (lanes of block col k>>3)
  auto reflector = [&](int k) {
    const int kb = k >> 3, cc = k & 7;
    if (wave != (kb >> 1)) return;
    const bool mine = bj == kb;  // my half of the wave holds column k
    float x[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      float t = 0.0f;
#pragma unroll
      for (int c = 0; c < 8; ++c) t = (c == cc) ? A[r][c] : t;
      x[r] = mine ? t : 0.0f;
    }
    float s = 0.0f, x0 = 0.0f, dkk = 0.0f;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int i = r0 + r;
      if (i >= k + 2) s += x[r] * x[r];
      if (i == k + 1) x0 = x[r];
      if (i == k) dkk = x[r];
    }
    s = wave_sum_dpp(s);
    x0 = wave_sum_dpp(x0);
    dkk = wave_sum_dpp(dkk);
    float tau = 0.0f, beta = x0, scal = 0.0f;
    if (s > 0.0f) {
      const float nrm = sqrtf(x0 * x0 + s);
      beta = x0 >= 0.0f ? -nrm : nrm;
      tau = (beta - x0) / beta;
      scal = 1.0f / (x0 - beta);
    }
    float* v = vs[k & 1];
    if (mine) {
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const int i = r0 + r;
        float vi = 0.0f;
        if (i == k + 1) vi = 1.0f;
        else if (i > k + 1) vi = x[r] * scal;
        v[i] = tau != 0.0f ? vi : 0.0f;
        if (i > k && i < n) Vh[(int64_t)k * n + i] = vi;
      }
    }
    if (lane == 0) {
      tsh[k & 1] = tau;
      tdiag[k] = dkk;
      toff[k] = beta;
      tau_out[k] = tau;
    }
  };

  if (n > 2) reflector(0);
  __syncthreads();
  for (int k = 0; k < n - 2; ++k) {
    const float tau = tsh[k & 1];
    const float* v = vs[k & 1];
    if (tau != 0.0f) {
      // p partials over my 8 columns; v^T (A v) partial for K
      float vc[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) vc[c] = v[c0 + c];
      float vav = 0.0f;
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        float acc = 0.0f;
#pragma unroll
        for (int c = 0; c < 8; ++c) acc += A[r][c] * vc[c];
        part[bj * 257 + r0 + r] = acc;
        vav += v[r0 + r] * acc;
      }
      vav = wave_sum_dpp(vav);
      if (lane == 0) red[k & 1][wave] = vav;
      __syncthreads();
      if (tid < 256) {
        float acc = 0.0f;
#pragma unroll 8
        for (int j = 0; j < 32; ++j) acc += part[j * 257 + tid];
        ps[tid] = tau * acc;
      }
      float vAv = 0.0f;
#pragma unroll
      for (int w = 0; w < 16; ++w) vAv += red[k & 1][w];
      const float K = 0.5f * tau * tau * vAv;
      __syncthreads();
      // A -= v w^T + w v^T
      float wc[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) wc[c] = ps[c0 + c] - K * vc[c];
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const float vr = v[r0 + r];
        const float wr = ps[r0 + r] - K * vr;
#pragma unroll
        for (int c = 0; c < 8; ++c) A[r][c] -= vr * wc[c] + wr * vc[c];
      }
    }
    if (k + 1 < n - 2) reflector(k + 1);
    __syncthreads();
  }
  // the last 2 x 2 block
#pragma unroll
  for (int r = 0; r < 8; ++r)
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int i = r0 + r, j = c0 + c;
      if (i == n - 2 && j == n - 2) tdiag[n - 2] = A[r][c];
      if (i == n - 1 && j == n - 1) tdiag[n - 1] = A[r][c];
      if (i == n - 1 && j == n - 2) toff[n - 2] = A[r][c];
    }
  if (tid == 0) {
    toff[n - 1] = 0.0f;
    tau_out[n - 2] = 0.0f;
    tau_out[n - 1] = 0.0f;
  }
}

// One wave per column c of Q: q = H_0 (H_1 (... H_{n-3} e_c)); H_k leaves
// columns c <= k alone, so the product starts at k = min(c-1, n-3).
// RPL = rows per lane (n <= 64 * RPL).
template <int RPL>
__global__ void __launch_bounds__(256)
    form_q_kernel(const float* __restrict__ Vh, const float* __restrict__ tau, int n, float* Q) {
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (c >= n) return;  // no barriers below
  float q[RPL];
#pragma unroll
  for (int r = 0; r < RPL; ++r) q[r] = (lane + 64 * r == c) ? 1.0f : 0.0f;
  int k = c - 1 < n - 3 ? c - 1 : n - 3;
  float vn[RPL];
  auto load = [&](int kk, float* dst) {
#pragma unroll
    for (int r = 0; r < RPL; ++r) {
      const int row = lane + 64 * r;
      dst[r] = (kk >= 0 && row > kk && row < n) ? Vh[(int64_t)kk * n + row] : 0.0f;
    }
  };
  load(k, vn);
  for (; k >= 0; --k) {
    float vk[RPL];
#pragma unroll
    for (int r = 0; r < RPL; ++r) vk[r] = vn[r];
    const float t = tau[k];
    load(k - 1, vn);  // prefetch the next reflector under this one's reduction
    if (t == 0.0f) continue;
    float d = 0.0f;
#pragma unroll
    for (int r = 0; r < RPL; ++r) d += vk[r] * q[r];
    d = wave_sum(d) * t;
#pragma unroll
    for (int r = 0; r < RPL; ++r) q[r] -= d * vk[r];
  }
#pragma unroll
  for (int r = 0; r < RPL; ++r) {
    const int row = lane + 64 * r;
    if (row < n) Q[(int64_t)row * n + c] = q[r];
  }
}

// Y = X B, B = Q or Q^T; 64 rows per workgroup, 4 waves, tiles of 32x32.
template <int NCT>
__global__ void __launch_bounds__(256)
    rot_gemm_kernel(const float* __restrict__ X, const QueueRec* __restrict__ rows, int64_t r0,
                    int64_t n, const float* __restrict__ Q, int trans, float* __restrict__ Y,
                    int x_blocked) {
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
  if (x_blocked) {  // rows = positions base .. base+63 = one 64-position block
    const float* xb = X + base * Dp;
    for (int s = tid; s < 64 * Dp; s += 256) xs[(s & 63) * XS + (s >> 6)] = xb[s];
  } else {
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
                      const float* Q, int trans, float* Y, hipStream_t s, int xb) {
  const unsigned nb = (unsigned)((n + 63) / 64);
  hipLaunchKernelGGL(rot_gemm_kernel<NCT>, dim3(nb), dim3(256), 0, s, X, rows, r0, n, Q, trans, Y,
                     xb);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_tridiag(const float* G, int Dp, float* tdiag, float* toff, float* Vh,
                          float* tau, hipStream_t s, float* work) {
  if (wide_dim(Dp)) return launch_wide_tridiag(G, Dp, tdiag, toff, Vh, tau, work, s);
  if (Dp < 4 || Dp > 256) return hipErrorInvalidValue;
  hipLaunchKernelGGL(tridiag_kernel, dim3(1), dim3(1024), 0, s, G, Dp, tdiag, toff, Vh, tau);
  return hipGetLastError();
}

hipError_t launch_form_q(const float* Vh, const float* tau, int Dp, float* Q, hipStream_t s) {
  if (Dp < 4 || Dp > 1024) return hipErrorInvalidValue;
  const dim3 grid((unsigned)((Dp + 3) / 4));
  if (Dp <= 256)
    hipLaunchKernelGGL(form_q_kernel<4>, grid, dim3(256), 0, s, Vh, tau, Dp, Q);
  else if (Dp <= 512)
    hipLaunchKernelGGL(form_q_kernel<8>, grid, dim3(256), 0, s, Vh, tau, Dp, Q);
  else
    hipLaunchKernelGGL(form_q_kernel<16>, grid, dim3(256), 0, s, Vh, tau, Dp, Q);
  return hipGetLastError();
}

hipError_t launch_rot_gemm(const float* X, const QueueRec* rows, int64_t r0, int64_t n,
                           const float* Q, int trans, float* Y, int Dp, hipStream_t s,
                           int x_blocked) {
  if (n <= 0) return hipSuccess;
  if (wide_dim(Dp)) return launch_wide_rot(X, rows, r0, n, Q, trans, Y, Dp, s, x_blocked);
  switch (Dp) {
    case 64: return launch_rot<2>(X, rows, r0, n, Q, trans, Y, s, x_blocked);
    case 96: return launch_rot<3>(X, rows, r0, n, Q, trans, Y, s, x_blocked);
    case 128: return launch_rot<4>(X, rows, r0, n, Q, trans, Y, s, x_blocked);
    case 160: return launch_rot<5>(X, rows, r0, n, Q, trans, Y, s, x_blocked);
    case 192: return launch_rot<6>(X, rows, r0, n, Q, trans, Y, s, x_blocked);
    case 224: return launch_rot<7>(X, rows, r0, n, Q, trans, Y, s, x_blocked);
    case 256: return launch_rot<8>(X, rows, r0, n, Q, trans, Y, s, x_blocked);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace frecsys_hip
