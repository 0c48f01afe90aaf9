// pp.hip -- iALS++ / SAFER2++ subspace block step on gfx950 (SURVEY 8(f)
// rank 2; reference ialspp.h: Step :351-424 with ProjectBlock :85-145, and
// PredictDataset :480-520; safer2pp.h: StepU / StepV :449-653 with ProjectU
// :97-160 and ProjectV :162-216).
//
// Per block of columns [s, s+bw) (bw = block_size <= 128) and per entity
// (one workgroup each, LPT queue order):
//   A = w*G[s:e, s:e] + lam*I + sum_j x_j,b x_j,b^T     (bw x bw, MFMA SYRK)
//   r = sum_j x_j,b (pred_j - 1) + w*G[s:e, :] u + lam*u_b
//   u_b <- u_b - A^-1 r                                 (chol_solve_tiles)
//   pred_j += (u_b' - u_b) . x_j,b                      (the entity's own ratings)
// SAFER2++ U: A = (S/h + w*Gl)*omega + lam*I, r = (sum x (pred-1))*omega/h
// + w*omega*Glg u + lam*u_b; V: rows weighted by nu_u (staged scaled by
// sqrt(nu)), G = the omega-weighted user Gramian.
// The block is padded to 32-column tiles (identity on the padded diagonal).
// pred is the device-resident prediction vector indexed by rating index
// (position of the tuple in the training file); each rating belongs to one
// entity per side, so the per-entity updates never race.
#include <hip/hip_runtime.h>

#include "chol.h"
#include "common.h"
#include "kernels.h"

namespace frecsys_hip {

namespace {

template <int TB>
struct PPCfg {
  static constexpr int BWP = 32 * TB;               // padded block width
  static constexpr int NT = TB * (TB + 1) / 2;
  static constexpr int MT = (NT + 3) / 4;           // tiles per wave (4 waves)
  static constexpr int TILES = NT * 1024;
  static constexpr int STAGE = 32 * BWP;
};

template <int TB>
__global__ void __launch_bounds__(256) pp_block_kernel(PPArgs a) {
  using C = PPCfg<TB>;
  constexpr int BWP = C::BWP, NT = C::NT, MT = C::MT;
  __shared__ __attribute__((aligned(16))) float tiles[C::TILES];
  __shared__ float stage[C::STAGE];
  __shared__ float us[1024];
  __shared__ int ids[32];
  __shared__ float coef[32], ssc[32];
  __shared__ float bvec[BWP], xvec[BWP];
  __shared__ float part[4 * 32];
  __shared__ float red[4];
  __shared__ int flag[1];
  const int tid = threadIdx.x, lane = tid & 63, lo = lane & 31, hi = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const QueueRec rec = a.order[blockIdx.x];
  const int64_t e = rec.entity, h = rec.h, p0 = rec.p0;
  if (h == 0) {  // untouched entity: its residual slot is read by the host sum
    if (tid == 0 && a.resid) a.resid[blockIdx.x] = 0.0f;
    return;
  }
  const int Dp = a.Dp, s0 = a.start, bw = a.bw, kind = a.kind;
  const bool uk = kind == KIND_WEIGHTED_U, vk = kind == KIND_WEIGHTED_V;
  // RegularizationValue (ialspp.h:313-318) / User-, ItemRegularizationValue
  // (safer2pp.h:425-436)
  const float lam = entity_lambda(kind, a.reg, a.reg_exp, a.w, a.alpha, h, a.n_other,
                                  a.entity_reg, e);
  const float omega = (uk && a.entity_weight) ? a.entity_weight[e] : 1.0f;
  const float hf = (float)h;
  // U: accumulate S + h*w*Gl, then A = acc * (omega/h) + lam*I
  const float gsc = uk ? hf * a.w : a.w;
  for (int c = tid; c < Dp; c += 256) us[c] = a.E[e * Dp + c];
  if (tid == 0) flag[0] = 0;

  f32x16 acc[MT];
  int aoff[MT], boff[MT];
  bool valid[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int t = wave + 4 * m;
    valid[m] = t < NT;
    int I = 0;
    while ((I + 1) * (I + 2) / 2 <= t) ++I;
    const int J = t - I * (I + 1) / 2;
    aoff[m] = 32 * I + lo;
    boff[m] = 32 * J + lo;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int gi = 32 * I + acc_row(q, hi), gj = 32 * J + lo;
      float v = 0.0f;
      if (valid[m]) {
        if (gi < bw && gj < bw)
          v = gsc * a.G[(int64_t)(s0 + gi) * Dp + s0 + gj] + (gi == gj && !uk ? lam : 0.0f);
        else if (gi == gj)
          v = 1.0f;  // padded coordinate: identity
      }
      acc[m][q] = v;
    }
  }
  float bacc = 0.0f;
  for (int64_t k0 = 0; k0 < h; k0 += 32) {
    __syncthreads();
    if (tid < 32) {
      const int64_t k = k0 + tid;
      int id = -1;
      float cf = 0.0f, sa = 0.0f;
      if (k < h) {
        id = a.col[p0 + k];
        cf = a.pred[a.rix ? a.rix[p0 + k] : p0 + k] - 1.0f;
        sa = 1.0f;
        if (vk) {  // row staged scaled by sqrt(nu): rhs weight nu / sqrt(nu)
          sa = sqrtf(a.other_weight[id]);
          cf *= sa;
        }
      }
      ids[tid] = id;
      coef[tid] = cf;
      ssc[tid] = sa;
    }
    __syncthreads();
    for (int i = tid; i < C::STAGE; i += 256) {
      const int r = i / BWP, cc = i % BWP;
      const int id = ids[r];
      stage[i] = (id >= 0 && cc < bw) ? a.X[(int64_t)id * Dp + s0 + cc] * ssc[r] : 0.0f;
    }
    __syncthreads();
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      if (valid[m]) {
#pragma unroll
        for (int s2 = 0; s2 < 16; ++s2) {
          const float* rowp = stage + (2 * s2 + hi) * BWP;
          acc[m] = mfma32(rowp[aoff[m]], rowp[boff[m]], acc[m]);
        }
      }
    }
    if (tid < bw) {
#pragma unroll 8
      for (int r = 0; r < 32; ++r) bacc += coef[r] * stage[r * BWP + tid];
    }
  }
  __syncthreads();
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    if (valid[m]) {
      const int I = (aoff[m] - lo) >> 5, J = (boff[m] - lo) >> 5;
      float* tile = tiles + tidx(I, J) * 1024;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int gi = 32 * I + acc_row(q, hi), gj = 32 * J + lo;
        float v = acc[m][q];
        if (uk && gi < bw && gj < bw) v = v * (omega / hf) + (gi == gj ? lam : 0.0f);
        tile[sw(acc_row(q, hi), lo)] = v;
      }
    }
  }
  if (tid < BWP) {
    float r = 0.0f;
    if (tid < bw) {
      const float* g = a.G + (int64_t)(s0 + tid) * Dp;
      float t = 0.0f;
      for (int c = 0; c < Dp; ++c) t += g[c] * us[c];
      // ialspp.h:134-137; safer2pp.h:143-147, 210-212
      r = uk ? bacc * (omega / hf) + a.w * t * omega + lam * us[s0 + tid]
             : bacc + a.w * t + lam * us[s0 + tid];
    }
    bvec[tid] = r;
  }
  __syncthreads();
  chol_solve_tiles<TB, 4>(tiles, bvec, xvec, part, flag, tid, 0);
  // new block (ialspp.h:141), residual, and the entity's predictions
  float d2 = 0.0f;
  if (tid < bw) {
    const float nw = us[s0 + tid] - xvec[tid];
    const float dl = nw - us[s0 + tid];
    xvec[tid] = dl;  // own element only
    a.E[e * Dp + s0 + tid] = nw;
    d2 = dl * dl;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) d2 += __shfl_xor(d2, o);
  if (lane == 0) red[wave] = d2;
  __syncthreads();
  if (tid == 0 && a.resid) a.resid[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
  for (int64_t k = wave; k < h; k += 4) {  // ialspp.h:400-404
    const int id = a.col[p0 + k];
    float t = 0.0f;
    // explicit fma: pp_refresh_kernel repeats this sum bit for bit
    for (int c = lane; c < bw; c += 64) t = __builtin_fmaf(xvec[c], a.X[(int64_t)id * Dp + s0 + c], t);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o);
    if (lane == 0) a.pred[a.rix ? a.rix[p0 + k] : p0 + k] += t;
  }
  if (tid == 0 && flag[0]) atomicMin(a.fail, (unsigned long long)(e + 1));
}

// pred[rix[k]] = X[col[k]] . E[row], one wave per row (PredictDataset).
__global__ void __launch_bounds__(256) pp_predict_kernel(PPArgs a, const int64_t* row_ptr,
                                                         int64_t n_rows) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= n_rows) return;
  const int Dp = a.Dp;
  const float* u = a.E + r * Dp;
  for (int64_t k = row_ptr[r]; k < row_ptr[r + 1]; ++k) {
    const float* x = a.X + (int64_t)a.col[k] * Dp;
    float t = 0.0f;
    for (int c = lane; c < Dp; c += 64) t += x[c] * u[c];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o);
    if (lane == 0) a.pred[a.rix ? a.rix[k] : k] = t;
  }
}

// Sharded block step (world > 1): the prediction updates of the rows other
// ranks solved, replayed from the all-gathered rows -- dl = new - old of the
// block (old: [n][bw] snapshot taken before the step), then per rating the
// same per-lane fma chain and butterfly sum as pp_block_kernel, so every
// rank's prediction vector is bitwise the single-rank one.  One wave per row
// of [0, n) outside [lo, hi).
__global__ void __launch_bounds__(256) pp_refresh_kernel(PPArgs a, const int64_t* row_ptr,
                                                         const float* old, int64_t n, int64_t lo,
                                                         int64_t hi) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= n || (r >= lo && r < hi)) return;
  const int Dp = a.Dp, s0 = a.start, bw = a.bw;
  float dl[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int c = lane + 64 * j;
    dl[j] = c < bw ? a.E[r * Dp + s0 + c] - old[r * bw + c] : 0.0f;
  }
  for (int64_t k = row_ptr[r]; k < row_ptr[r + 1]; ++k) {
    const float* x = a.X + (int64_t)a.col[k] * Dp + s0;
    float t = 0.0f;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int c = lane + 64 * j;
      if (c < bw) t = __builtin_fmaf(dl[j], x[c], t);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o);
    if (lane == 0) a.pred[a.rix ? a.rix[k] : k] += t;
  }
}

}  // namespace

hipError_t launch_pp_refresh(const PPArgs& a, const int64_t* row_ptr, const float* old,
                             int64_t n, int64_t lo, int64_t hi, hipStream_t s) {
  if (n <= 0 || (lo == 0 && hi >= n)) return hipSuccess;
  hipLaunchKernelGGL(pp_refresh_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, s, a,
                     row_ptr, old, n, lo, hi);
  return hipGetLastError();
}

hipError_t launch_pp_step(const PPArgs& a, hipStream_t s) {
  if (a.n_rows <= 0) return hipSuccess;
  if (a.bw < 1 || a.bw > 128 || a.Dp > 1024) return hipErrorInvalidValue;
  const int tb = (a.bw + 31) / 32;
  const dim3 g((unsigned)a.n_rows), b(256);
  switch (tb) {
    case 1: hipLaunchKernelGGL(pp_block_kernel<1>, g, b, 0, s, a); break;
    case 2: hipLaunchKernelGGL(pp_block_kernel<2>, g, b, 0, s, a); break;
    case 3: hipLaunchKernelGGL(pp_block_kernel<3>, g, b, 0, s, a); break;
    default: hipLaunchKernelGGL(pp_block_kernel<4>, g, b, 0, s, a); break;
  }
  return hipGetLastError();
}

hipError_t launch_pp_predict(const PPArgs& a, const int64_t* row_ptr, int64_t n_rows,
                             hipStream_t s) {
  if (n_rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(pp_predict_kernel, dim3((unsigned)((n_rows + 3) / 4)), dim3(256), 0, s, a,
                     row_ptr, n_rows);
  return hipGetLastError();
}

}  // namespace frecsys_hip
