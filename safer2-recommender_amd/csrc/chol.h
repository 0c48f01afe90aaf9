// chol.h -- blocked Cholesky solve on LDS-resident 32x32 tiles, shared by
// the d-space solve (solve.hip: A is d x d) and the history-space solve
// (dual.hip: S is h x h).  Internal header.
#pragma once

#include "common.h"

namespace frecsys_hip {

__device__ __forceinline__ float rdlane(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

// ---------------------------------------------------------------------
// 32x32 diagonal block: Cholesky factor AND its inverse by one wave.
//
// Lanes 0..31 own row r of A (becoming row r of L); lanes 32..63 own column
// j = lane-32 of the identity (becoming column j of L^-1).  Both halves run
// the same left-looking update at step k,
//     t = a[k] - sum_{m<k} a[m] * L[k][m],
// which for a row of A is the Cholesky update and for a column of the
// identity is forward substitution L x = e_j; then a[k] = t / L[k][k] (lane
// k itself takes the pivot sqrt).  Row k of L (lane k's registers) reaches
// every lane by v_readlane -- no LDS round trip on the serial chain; the dot
// product runs in 4 partial chains.  On return L^-1 (lower, upper zeroed)
// is in the swizzled tile.  Not inlined: two inlined copies (first panel +
// lookahead) overflow the SGPRs and the spills push the kernels to 256
// VGPRs (occupancy 1-2); as a call it costs nothing measurable.
// ---------------------------------------------------------------------
typedef __attribute__((address_space(3))) float lds_float;

__device__ __noinline__ bool diag_factor_inv_lds(lds_float* tile, int lane) {
  const int r = lane & 31;
  const bool fl = lane < 32;
  float a[32];
#pragma unroll
  for (int c = 0; c < 32; ++c) {
    const float t = tile[sw(r, c)];  // both halves read (no divergent loads)
    a[c] = fl ? t : (c == r ? 1.0f : 0.0f);
  }
  bool ok = true;
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    float p0 = 0.f, p1 = 0.f, p2 = 0.f, p3 = 0.f;
#pragma unroll
    for (int m = 0; m < k; m += 4) {
      // broadcasts first, then the FMAs: no SGPR-hazard nop per pair
      const float b0 = rdlane(a[m], k);
      const float b1 = m + 1 < k ? rdlane(a[m + 1], k) : 0.0f;
      const float b2 = m + 2 < k ? rdlane(a[m + 2], k) : 0.0f;
      const float b3 = m + 3 < k ? rdlane(a[m + 3], k) : 0.0f;
      p0 += a[m] * b0;
      if (m + 1 < k) p1 += a[m + 1] * b1;
      if (m + 2 < k) p2 += a[m + 2] * b2;
      if (m + 3 < k) p3 += a[m + 3] * b3;
    }
    const float t = a[k] - ((p0 + p1) + (p2 + p3));
    const float piv = rdlane(t, k);
    ok = ok && (piv > 0.0f);
    // v_rsq_f32 (1 ulp) instead of the IEEE sqrt + divide sequences on the
    // serial chain
    const float rd = __builtin_amdgcn_rsqf(piv);
    a[k] = (lane == k) ? piv * rd : t * rd;
  }
  // lanes 32..63: column j of L^-1 -> tile element (k, j), k >= j
  const int j = r;
#pragma unroll
  for (int k = 0; k < 32; ++k)
    if (!fl) tile[sw(k, j)] = (k >= j) ? a[k] : 0.0f;
  return ok;
}

__device__ __forceinline__ bool diag_factor_inv(float* tile, int lane) {
  return diag_factor_inv_lds((lds_float*)tile, lane);
}

// One 32x32 MFMA product u = P Q^T of two LDS tiles (P, Q swizzled).
__device__ __forceinline__ f32x16 tile_pqT(const float* P, const float* Q, int lo, int hi) {
  f32x16 u = f32x16{0.f};
#pragma unroll
  for (int s = 0; s < 16; ++s) u = mfma32(P[sw(lo, 2 * s + hi)], Q[sw(lo, 2 * s + hi)], u);
  return u;
}

// ---------------------------------------------------------------------
// Solve A x = b for the SPD matrix whose lower T(T+1)/2 tiles sit in LDS
// (tile (I, J) at tiles + tidx(I, J) * 1024, swizzled), NW waves.
//
// Right-looking blocked Cholesky with lookahead: diagonal tiles become
// L_pp^-1 (diag_factor_inv); the panel TRSM is an MFMA product with
// L_pp^-1 and the right-hand side rides along (y_p = L_pp^-1 b_p); wave 0
// updates and factors tile (p+1, p+1) while the other waves finish panel
// p's trailing update.  Back substitution x = L^-T y with one GEMV wave per
// tile and the stored inverses.
//
// In: tiles, bvec[32T] = b, a __syncthreads() since they were written.
// Out: xvec[32T] = x; bvec = y; *flag = 1 on a non-positive pivot.
// Scratch: part[NW * 32].  Ends with a __syncthreads().
// debug_skip masks (ablation only): 2 diag, 4 TRSM, 8 trailing, 16 back.
// ---------------------------------------------------------------------
template <int T, int NW>
__device__ __forceinline__ void chol_solve_tiles(float* tiles, float* bvec, float* xvec,
                                                 float* part, int* flag, int tid,
                                                 int debug_skip) {
  static_assert(T - 1 < NW || T == 1, "back substitution needs one wave per tile");
  const int lane = tid & 63, lo = lane & 31, hi = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (wave == 0 && !(debug_skip & 2)) {
    if (!diag_factor_inv(tiles, lane) && lane == 0) flag[0] = 1;
  }
  lds_barrier();
#pragma unroll 1
  for (int p = 0; p < T; ++p) {
    const float* Tpp = tiles + tidx(p, p) * 1024;
    const int npan = T - 1 - p;
    // TRSM by MFMA: L_Ip = A_Ip (L_pp^-1)^T ; y_p = L_pp^-1 b_p
    if (!(debug_skip & 4)) {
      for (int t = wave; t < npan; t += NW) {
        float* Aip = tiles + tidx(p + 1 + t, p) * 1024;
        const f32x16 u = tile_pqT(Aip, Tpp, lo, hi);
#pragma unroll
        for (int q = 0; q < 16; ++q) Aip[sw(acc_row(q, hi), lo)] = u[q];
      }
      if (wave == (npan % NW) && hi == 0) {
        float y = 0.0f;
#pragma unroll 8
        for (int k = 0; k < 32; ++k) y += Tpp[sw(lo, k)] * bvec[32 * p + k];
        xvec[lo] = y;  // staged; copied into bvec after the barrier
      }
    }
    lds_barrier();
    if (tid < 32) bvec[32 * p + tid] = xvec[tid];
    if (p < T - 1) {
      const int nb = 32 * npan;
      if (tid >= 64 && tid < 64 + nb) {  // b_J -= L_Jp y_p (y_p still in xvec)
        const int t2 = tid - 64;
        const int J = p + 1 + (t2 >> 5), r = t2 & 31;
        const float* L = tiles + tidx(J, p) * 1024;
        float t = 0.0f;
#pragma unroll 8
        for (int k = 0; k < 32; ++k) t += L[sw(r, k)] * xvec[k];
        bvec[32 * J + r] -= t;
      }
      // trailing update A_IJ -= L_Ip L_Jp^T; tile (p+1, p+1) is index 0
      const int ntr = npan * (npan + 1) / 2;
      if (wave == 0) {
        float* A11 = tiles + tidx(p + 1, p + 1) * 1024;
        const float* L1 = tiles + tidx(p + 1, p) * 1024;
        if (!(debug_skip & 8)) {
          const f32x16 u = tile_pqT(L1, L1, lo, hi);
#pragma unroll
          for (int q = 0; q < 16; ++q) A11[sw(acc_row(q, hi), lo)] -= u[q];
        }
        if (!(debug_skip & 2)) {
          if (!diag_factor_inv(A11, lane) && lane == 0) flag[0] = 1;
        }
      } else {
        for (int tt = wave; tt < ntr && !(debug_skip & 8); tt += NW - 1) {
          int Ir = 0;
          while ((Ir + 1) * (Ir + 2) / 2 <= tt) ++Ir;
          const int Jr = tt - Ir * (Ir + 1) / 2;
          const int I = p + 1 + Ir, J = p + 1 + Jr;
          const f32x16 u = tile_pqT(tiles + tidx(I, p) * 1024, tiles + tidx(J, p) * 1024, lo, hi);
          float* Aij = tiles + tidx(I, J) * 1024;
#pragma unroll
          for (int q = 0; q < 16; ++q) Aij[sw(acc_row(q, hi), lo)] -= u[q];
        }
      }
    }
    lds_barrier();
  }

  // ---- back substitution x = L^-T y with the stored L_pp^-1 ----
  // r_p = y_p - sum_{q>p} L_qp^T x_q   (one wave per q, partials in LDS)
  // x_p = (L_pp^-1)^T r_p
#pragma unroll 1
  for (int p = T - 1; p >= 0 && !(debug_skip & 16); --p) {
    const int nq = T - 1 - p;  // < NW: one q per wave
    if (wave < nq) {
      const int q = p + 1 + wave;
      const float* L = tiles + tidx(q, p) * 1024;
      float pr = 0.0f;
#pragma unroll 4
      for (int m = 16 * hi; m < 16 * hi + 16; ++m) pr += L[sw(m, lo)] * xvec[32 * q + m];
      pr += __shfl_xor(pr, 32);
      if (hi == 0) part[wave * 32 + lo] = pr;
    }
    lds_barrier();
    if (wave == 0) {
      float r = bvec[32 * p + lo];
      for (int w = 0; w < nq; ++w) r -= part[w * 32 + lo];
      const float* Tpp = tiles + tidx(p, p) * 1024;
      float x = 0.0f;
#pragma unroll
      for (int i = 0; i < 32; ++i) x += Tpp[sw(i, lo)] * rdlane(r, i);
      if (hi == 0) xvec[32 * p + lo] = x;
    }
    lds_barrier();
  }
}

}  // namespace frecsys_hip
