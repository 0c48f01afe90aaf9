// topk.hip -- fold-in scoring and top-K ranking on gfx950 (SURVEY 8(f)
// rank 1): the reference's EvaluateDatasetInternal / EvaluateUser
// (recommender.h:78-199) scores every item for a held-out user with a GEMV
// per user on a host thread, sets the user's fold-in history to lowest()
// and takes the top max_k by nth_element + stable_sort.  Here, per batch of
// held-out users:
//   score_kernel    S = U_eval V^T, 64 users x 128 items per workgroup,
//                   v_mfma_f32_32x32x2_f32, K in 32-wide slabs through LDS;
//   exclude_kernel  S[u][j] = lowest() for j in u's fold-in history;
//   topk_kernel     one workgroup per user: 4-pass 8-bit radix select of the
//                   k-th largest score key over the row, collect the keys
//                   above it and the lowest-index ties at it, bitonic sort
//                   of the <= 1024 candidates by (score desc, item asc).
// Ties are broken by item id (the reference's nth_element leaves their
// order unspecified).
#include <hip/hip_runtime.h>

#include <cfloat>

#include "common.h"
#include "kernels.h"

namespace frecsys_hip {

namespace {

constexpr int SB = 128;  // items per workgroup tile

__global__ void __launch_bounds__(256)
    score_kernel(const float* __restrict__ X, int64_t r0, int64_t n, const float* __restrict__ Y,
                 int64_t m, int Dp, float* __restrict__ S) {
  __shared__ float xs[64 * 33];
  __shared__ float ys[32 * (SB + 1)];
  const int tid = threadIdx.x, lane = tid & 63, lo = lane & 31, hi = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t base = (int64_t)blockIdx.x * 64;
  const int64_t j0 = (int64_t)blockIdx.y * SB;
  const int R = wave & 1, Cs = (wave >> 1) * 2;
  f32x16 acc[2] = {f32x16{0.f}, f32x16{0.f}};
  const int NC = (Dp + 31) >> 5;
  for (int c = 0; c < NC; ++c) {
    __syncthreads();
    for (int s = tid; s < 64 * 32; s += 256) {
      const int rr = s >> 5, kk = s & 31, col = 32 * c + kk;
      const int64_t row = base + rr;
      xs[rr * 33 + kk] = (row < n && col < Dp) ? X[(r0 + row) * Dp + col] : 0.0f;
    }
    for (int s = tid; s < 32 * SB; s += 256) {
      const int j = s >> 5, kk = s & 31, col = 32 * c + kk;
      const int64_t it = j0 + j;
      ys[kk * (SB + 1) + j] = (it < m && col < Dp) ? Y[it * Dp + col] : 0.0f;
    }
    __syncthreads();
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int C = Cs + t;
#pragma unroll
      for (int s2 = 0; s2 < 16; ++s2) {
        const int kk = 2 * s2 + hi;
        acc[t] = mfma32(xs[(32 * R + lo) * 33 + kk], ys[kk * (SB + 1) + 32 * C + lo], acc[t]);
      }
    }
  }
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int64_t it = j0 + 32 * (Cs + t) + lo;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int64_t row = base + 32 * R + acc_row(q, hi);
      if (row < n && it < m) S[row * m + it] = acc[t][q];
    }
  }
}

// S[u][j] = lowest() for every j of row u's history (EVAL CSR rows r0..).
__global__ void __launch_bounds__(64)
    exclude_kernel(const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ col,
                   int64_t r0, int64_t m, float* __restrict__ S) {
  const int64_t u = blockIdx.x;
  const int64_t p0 = row_ptr[r0 + u], p1 = row_ptr[r0 + u + 1];
  for (int64_t k = p0 + threadIdx.x; k < p1; k += 64) S[u * m + col[k]] = -FLT_MAX;
}

__device__ __forceinline__ uint32_t score_key(float x) {
  const uint32_t u = __float_as_uint(x);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);  // monotone in x
}

// One workgroup per row: the k best items, score descending, item ascending.
__global__ void __launch_bounds__(256)
    topk_kernel(const float* __restrict__ S, int64_t m, int k, int32_t* __restrict__ out) {
  __shared__ unsigned hist[256];
  __shared__ uint32_t ckey[1024];
  __shared__ int32_t cidx[1024];
  __shared__ unsigned sh[4];
  __shared__ unsigned scan[256];
  const int tid = threadIdx.x;
  const float* s = S + (int64_t)blockIdx.x * m;
  uint32_t prefix = 0, mask = 0;
  unsigned remaining = (unsigned)k;
  for (int shift = 24; shift >= 0; shift -= 8) {
    hist[tid] = 0;
    __syncthreads();
    for (int64_t i = tid; i < m; i += 256) {
      const uint32_t key = score_key(s[i]);
      if ((key & mask) == prefix) atomicAdd(&hist[(key >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (tid == 0) {
      unsigned cum = 0, sel = 0;
      for (int d = 255; d >= 0; --d) {
        if (cum + hist[d] >= remaining) {
          sel = (unsigned)d;
          break;
        }
        cum += hist[d];
      }
      sh[0] = sel;
      sh[1] = remaining - cum;
    }
    __syncthreads();
    prefix |= sh[0] << shift;
    mask |= 255u << shift;
    remaining = sh[1];
    __syncthreads();
  }
  // prefix = the k-th largest key; (k - remaining) keys lie above it and the
  // `remaining` lowest-index keys equal to it complete the k
  const unsigned n_gt = (unsigned)k - remaining;
  if (tid == 0) sh[2] = 0;
  __syncthreads();
  const int64_t chunk = (m + 255) / 256;
  const int64_t c0 = tid * chunk, c1 = c0 + chunk < m ? c0 + chunk : m;
  unsigned n_eq = 0;
  for (int64_t i = c0; i < c1; ++i) {
    const uint32_t key = score_key(s[i]);
    if (key > prefix) {
      const unsigned p = atomicAdd(&sh[2], 1u);
      ckey[p] = key;
      cidx[p] = (int32_t)i;
    } else if (key == prefix) {
      ++n_eq;
    }
  }
  scan[tid] = n_eq;
  __syncthreads();
  for (int o = 1; o < 256; o <<= 1) {  // inclusive scan of the tie counts
    const unsigned v = tid >= o ? scan[tid - o] : 0u;
    __syncthreads();
    scan[tid] += v;
    __syncthreads();
  }
  unsigned pos = scan[tid] - n_eq;  // ties before my chunk
  for (int64_t i = c0; i < c1 && pos < remaining; ++i) {
    if (score_key(s[i]) == prefix) {
      ckey[n_gt + pos] = prefix;
      cidx[n_gt + pos] = (int32_t)i;
      ++pos;
    }
  }
  int np = 1;
  while (np < k) np <<= 1;
  for (int i = k + tid; i < np; i += 256) {
    ckey[i] = 0u;
    cidx[i] = 0x7fffffff;
  }
  __syncthreads();
  // bitonic sort, "before" = larger key, then smaller index
  for (int size = 2; size <= np; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = tid; i < np; i += 256) {
        const int j = i ^ stride;
        if (j > i) {
          const bool up = (i & size) == 0;
          const uint32_t ka = ckey[i], kb = ckey[j];
          const int32_t ia = cidx[i], ib = cidx[j];
          const bool a_first = ka > kb || (ka == kb && ia < ib);
          if (up ? !a_first : a_first) {
            ckey[i] = kb;
            ckey[j] = ka;
            cidx[i] = ib;
            cidx[j] = ia;
          }
        }
      }
      __syncthreads();
    }
  }
  for (int i = tid; i < k; i += 256) out[(int64_t)blockIdx.x * k + i] = cidx[i];
}

}  // namespace

hipError_t launch_eval_topk(const float* X, int64_t r0, int64_t n, const float* Y, int64_t m,
                            int Dp, const int64_t* row_ptr, const int32_t* col, int k, float* S,
                            int32_t* out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if (k < 1 || k > 1024 || k > m) return hipErrorInvalidValue;
  hipLaunchKernelGGL(score_kernel, dim3((unsigned)((n + 63) / 64), (unsigned)((m + SB - 1) / SB)),
                     dim3(256), 0, s, X, r0, n, Y, m, Dp, S);
  hipLaunchKernelGGL(exclude_kernel, dim3((unsigned)n), dim3(64), 0, s, row_ptr, col, r0, m, S);
  hipLaunchKernelGGL(topk_kernel, dim3((unsigned)n), dim3(256), 0, s, S, m, k, out);
  return hipGetLastError();
}

}  // namespace frecsys_hip
