// chol.h -- blocked Cholesky solve on LDS-resident 32x32 tiles, shared by
// the d-space solve (solve.hip: A is d x d) and the history-space solve
// (dual.hip: S is h x h).  Internal header.
#pragma once

#include "common.h"

// With 8 waves: the wave that runs the forward substitution (Y, B of the
// chain's next block).  Waves w and w + 4 share a SIMD, so 4 leaves the
// chain wave's SIMD without a worker's tile products beside it.
constexpr int kCholYWave = 4;
// A worker raises its issue priority (1; the chain runs at 2) over the
// worker that shares its SIMD for the panel-p tasks of block rows
// I <= p + 1 + kCholWPrio -- the ones that feed the chain's next block
// (S(p+2, p), U(p+2, p+1, p), U(p+2, p+2, p)).
constexpr int kCholWPrio = 1;

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

// Lanes 0..31: row r of the swizzled tile; lanes 32..63: column r of the
// identity.  The row as 8 granule reads (conflict-free, see common.h sw);
// G = 1: every value pinned in its own register before the select below
// (the register-capped callers), else the select may be folded into the
// loads' uses.  Both halves read: no divergent loads.
template <int G>
__device__ __forceinline__ void load_factor_rows(const lds_float* tile, int r, bool fl,
                                                 float (&a)[32]) {
  typedef __attribute__((address_space(3))) const f32x4v lds_f32x4c;
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    const f32x4v v = *reinterpret_cast<lds_f32x4c*>(tile + r * 32 + (((g ^ (r >> 1)) & 7) << 2));
#pragma unroll
    for (int t = 0; t < 4; ++t) a[4 * g + t] = v[t];
  }
  if constexpr (G == 1) {
#pragma unroll
    for (int c = 0; c < 32; ++c) asm volatile("" : "+v"(a[c]));
  }
#pragma unroll
  for (int c = 0; c < 32; ++c) a[c] = fl ? a[c] : (c == r ? 1.0f : 0.0f);
}

__device__ __forceinline__ bool diag_factor_inv_lds_body(lds_float* tile, int lane) {
  const int r = lane & 31;
  const bool fl = lane < 32;
  float a[32];
  load_factor_rows<1>(tile, r, fl, a);
  // pivot test on the scalar unit: piv > 0 and not NaN <=> its bits as an
  // int lie in (0, 0x7f800000]
  int pmin = 0x7fffffff, pmax = 0;
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
    const int pi = __builtin_amdgcn_readfirstlane(__float_as_int(piv));
    pmin = min(pmin, pi);
    pmax = max(pmax, pi);
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
  return pmin > 0 && pmax <= 0x7f800000;
}
__device__ __noinline__ bool diag_factor_inv_lds(lds_float* tile, int lane) {
  return diag_factor_inv_lds_body(tile, lane);
}

// Blocked form of the same factor + inverse: columns 0..15 by the
// recurrence above (rows 16..31 come out as L21), then the cross terms of
// every lane's columns 16..31 -- sum_{m<16} L[16+c][m] v[m], the Schur
// update A22 -= L21 L21^T for the rows and the L21 X1 coupling for the
// inverse columns alike -- as one 64 x 16 x 16 product on the matrix cores
// (16 v_mfma_f32_16x16x4_f32, operands through the tile, whose values are
// in registers by then), and columns 16..31 by the recurrence over
// m in [16, k) only.  256 v_readlane + 256 FMAs of the serial chain become
// MFMAs.
// The factor from rows already in registers (a: lanes 0..31 row r of A,
// lanes 32..63 column r of the identity); L^-1 goes to the tile.
__device__ __forceinline__ bool diag_factor_inv_blk_regs(float (&a)[32], lds_float* tile,
                                                         int lane) {
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  const int r = lane & 31;
  const bool fl = lane < 32;
  // pivot test without a vector compare per column: piv > 0 and not NaN
  // <=> its bits as an int lie in (0, 0x7f800000]
  int pmin = 0x7fffffff, pmax = 0;
  auto column = [&](int k, int m0) {  // column k from the terms m in [m0, k)
    // two partial sums (one v_pk_fma_f32 per pair of terms, one add to
    // combine): this one wave's instruction count is the chain's bound
    float p0 = 0.f, p1 = 0.f;
#pragma unroll
    for (int m = m0; m < k; m += 2) {
      const float b0 = rdlane(a[m], k);
      const float b1 = m + 1 < k ? rdlane(a[m + 1], k) : 0.0f;
      p0 += a[m] * b0;
      if (m + 1 < k) p1 += a[m + 1] * b1;
    }
    const float t = a[k] - (p0 + p1);
    const float piv = rdlane(t, k);
    const int pi = __builtin_amdgcn_readfirstlane(__float_as_int(piv));
    pmin = min(pmin, pi);
    pmax = max(pmax, pi);
    a[k] = t * __builtin_amdgcn_rsqf(piv);  // lane k: t = piv -> sqrt(piv)
  };
#pragma unroll
  for (int k = 0; k < 16; ++k) column(k, 0);
  // ---- cross terms on the matrix cores ----
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  lds_float* U = tile;  // [64][16]: lane l's a[0..15]; rows 16..31 = L21
#pragma unroll
  for (int m = 0; m < 16; m += 4)
    *reinterpret_cast<__attribute__((address_space(3))) f32x4*>(U + lane * 16 + m) =
        f32x4{a[m], a[m + 1], a[m + 2], a[m + 3]};
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  const int li = lane & 15, lk = lane >> 4;
  f32x4 w[4] = {f32x4{0.f}, f32x4{0.f}, f32x4{0.f}, f32x4{0.f}};
#pragma unroll
  for (int k0 = 0; k0 < 4; ++k0) {
    // A[i][k] = L21[i][4k0+k], B[k][n] = U[16nb+n][4k0+k]; D[c'][n] -> W[16nb+n][c']
    const float av = U[(16 + li) * 16 + 4 * k0 + lk];
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
      const float bv = U[(16 * nb + li) * 16 + 4 * k0 + lk];
      w[nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, w[nb], 0, 0, 0);
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // U's reads done before W overwrites it
#pragma unroll
  for (int nb = 0; nb < 4; ++nb)
    *reinterpret_cast<__attribute__((address_space(3))) f32x4*>(U + (16 * nb + li) * 16 + 4 * lk) =
        w[nb];
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int c = 0; c < 16; c += 4) {
    const f32x4 x = *reinterpret_cast<const __attribute__((address_space(3))) f32x4*>(
        U + lane * 16 + c);
    a[16 + c] -= x[0];
    a[17 + c] -= x[1];
    a[18 + c] -= x[2];
    a[19 + c] -= x[3];
  }
#pragma unroll
  for (int k = 16; k < 32; ++k) column(k, 16);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  const int j = r;
  const bool ok = pmin > 0 && pmax <= 0x7f800000;
  if (ok) {
    // entries k < j of column j of L^-1 came out of the recurrence as +-0
    // (zero inputs times finite factors): stored as they are
#pragma unroll
    for (int k = 0; k < 32; ++k)
      if (!fl) tile[sw(k, j)] = a[k];
  } else {
#pragma unroll
    for (int k = 0; k < 32; ++k)
      if (!fl) tile[sw(k, j)] = (k >= j) ? a[k] : 0.0f;
  }
  return ok;
}
// The same from the chain's updated diagonal tile in MFMA accumulator layout
// (c[q] = element (acc_row(q, hi), lo)): lane lo takes COLUMN lo of the
// updated tile (its own 16 values and lane lo+32's, one v_permlane32_swap
// each) as row lo.  The tile is symmetric in exact arithmetic only -- the
// split-bf16 product's (i, j) and (j, i) terms accumulate in different
// orders -- so this factors the transposed lower triangle and agrees with a
// factor of the stored tile to rounding, not bitwise.  A call, as
// diag_factor_inv_blk (the accumulator travels in 16 VGPRs).
__device__ __noinline__ bool diag_factor_inv_acc(f32x16 c, lds_float* tile) {
  const int lane = __lane_id();
  const int r = lane & 31;
  const bool fl = lane < 32;
  float a[32];
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const auto sv = __builtin_amdgcn_permlane32_swap(__float_as_uint(c[q]),
                                                     __float_as_uint(c[q]), false, false);
    const int c0 = acc_row(q, 0), c1 = acc_row(q, 1);
    a[c0] = fl ? c[q] : (c0 == r ? 1.0f : 0.0f);
    a[c1] = fl ? __uint_as_float(sv[1]) : (c1 == r ? 1.0f : 0.0f);
  }
  return diag_factor_inv_blk_regs(a, tile, lane);
}
// As a call: the register cost counts once, not per call site.
__device__ __noinline__ bool diag_factor_inv_blk(lds_float* tile, int lane) {
  float a[32];
  load_factor_rows<8>(tile, lane & 31, lane < 32, a);
  return diag_factor_inv_blk_regs(a, tile, lane);
}

// BLK = true for kernels with a register budget above ~150 VGPRs (the
// blocked form needs more registers than the plain one; a call counts
// toward the caller's allocation, so a capped kernel would lose occupancy).
template <bool BLK = false>
__device__ __forceinline__ bool diag_factor_inv(float* tile, int lane) {
  if constexpr (BLK) return diag_factor_inv_blk((lds_float*)tile, lane);
  return diag_factor_inv_lds((lds_float*)tile, lane);
}

// One 32x32 MFMA product u = P Q^T of two LDS tiles (P, Q swizzled).
// Lane (lo, hi) supplies k = 2s + hi of row lo: with the granule swizzle,
// one b128 read of row lo's columns 4g .. 4g+3 serves s = 2g and 2g + 1.
__device__ __forceinline__ f32x16 tile_pqT(const float* P, const float* Q, int lo, int hi) {
  f32x16 u = f32x16{0.f};
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    const f32x4v pv = row_gran(P, lo, g), qv = row_gran(Q, lo, g);
    u = mfma32(hi ? pv[1] : pv[0], hi ? qv[1] : qv[0], u);
    u = mfma32(hi ? pv[3] : pv[2], hi ? qv[3] : qv[2], u);
  }
  return u;
}

// The same product with fp32-accurate split operands (common.h mfma_x6):
// lane (lo, hi) takes k = 16 g + 8 hi + j of row lo of P and of Q, splits
// them into three bf16 pieces in registers, and 2 x 6 v_mfma_f32_32x32x16_bf16
// (32 cycles each) replace 16 v_mfma_f32_32x32x2_f32 (64 cycles each).
// SAME: P == Q (one operand split, used on both sides).
template <bool SAME = false>
__device__ __forceinline__ f32x16 tile_pqT_x6(const float* P, const float* Q, int lo, int hi) {
  f32x16 u = f32x16{0.f};
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    float pv[8], qv[8];
#pragma unroll
    for (int h2 = 0; h2 < 2; ++h2) {
      const f32x4v p4 = row_gran(P, lo, 4 * g + 2 * hi + h2);
#pragma unroll
      for (int t = 0; t < 4; ++t) pv[4 * h2 + t] = p4[t];
      if (!SAME) {
        const f32x4v q4 = row_gran(Q, lo, 4 * g + 2 * hi + h2);
#pragma unroll
        for (int t = 0; t < 4; ++t) qv[4 * h2 + t] = q4[t];
      }
    }
    bf16x8 pf[3], qf[3];
    split3x8(pv, pf);
    if (SAME) {
      u = mfma_x6(pf, pf, u);
    } else {
      split3x8(qv, qf);
      u = mfma_x6(pf, qf, u);
    }
  }
  return u;
}

// ---------------------------------------------------------------------
// Barrier-phased solve (pp.hip's block steps, TB <= 4 tiles): A x = b for
// the SPD matrix whose lower T(T+1)/2 tiles sit in LDS (tile (I, J) at
// tiles + tidx(I, J) * 1024, swizzled), NW waves.
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
  if (wave == 0 && !FRECSYS_SKIP(debug_skip, 2)) {
    if (!diag_factor_inv(tiles, lane) && lane == 0) flag[0] = 1;
  }
  lds_barrier();
#pragma unroll 1
  for (int p = 0; p < T; ++p) {
    const float* Tpp = tiles + tidx(p, p) * 1024;
    const int npan = T - 1 - p;
    // TRSM by MFMA: L_Ip = A_Ip (L_pp^-1)^T ; y_p = L_pp^-1 b_p
    if (!FRECSYS_SKIP(debug_skip, 4)) {
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
        if (!FRECSYS_SKIP(debug_skip, 8)) {
          const f32x16 u = tile_pqT(L1, L1, lo, hi);
#pragma unroll
          for (int q = 0; q < 16; ++q) A11[sw(acc_row(q, hi), lo)] -= u[q];
        }
        if (!FRECSYS_SKIP(debug_skip, 2)) {
          if (!diag_factor_inv(A11, lane) && lane == 0) flag[0] = 1;
        }
      } else {
        for (int tt = wave; tt < ntr && !FRECSYS_SKIP(debug_skip, 8); tt += NW - 1) {
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
  for (int p = T - 1; p >= 0 && !FRECSYS_SKIP(debug_skip, 16); --p) {
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

// ---------------------------------------------------------------------
// Dataflow solve (the d-space and history-space kernels): A x = b for the
// SPD matrix whose lower T(T+1)/2 tiles sit in LDS (tile (I, J) at
// tiles + tidx(I, J) * 1024, swizzled), NW waves.
// In: tiles, bvec[32T] = b, a barrier since they were written.
// Out: xvec[32T] = x; bvec = y; *flag = 1 on a non-positive pivot; the
// diagonal tiles hold L_pp^-1.  Scratch: part[] holds 2T + T(T+1)/2 + 2
// ints and 32 floats.  Ends with a barrier.
// Blocked Cholesky with the diagonal tiles inverted (the panel TRSM is an
// MFMA product with L_pp^-1); the factorisation and both substitutions are
// tile tasks
//   F(p)      factor + invert diagonal tile (p, p)
//   Y(p)      y_p = L_pp^-1 b_p                       (b_p fully updated)
//   S(I, p)   TRSM  L_Ip = A_Ip (L_pp^-1)^T                       (I > p)
//   B(I, p)   b_I -= L_Ip y_p                                     (I > p)
//   U(I,J,p)  A_IJ -= L_Ip L_Jp^T                         (p < J <= I)
// ordered by LDS version counters instead of workgroup barriers: ver(I,J)
// = updates applied to tile (I, J), +1 once final (TRSM'd / factored);
// bver(I) = updates applied to b_I; yver = y blocks published.  Wave 0
// runs only the critical chain
//   F(p), Y(p) -> S(p+1, p), B(p+1, p) -> U(p+1, p+1, p) -> F(p+1), ...
// (at raised issue priority); the other waves take the remaining S+B and
// U tasks of each panel round-robin, next-column tiles first.  Every wave
// walks its tasks in one global order (panel by panel: chain, S+B, U by
// column) in which each task's dependencies come earlier, so the waits
// cannot deadlock.  The backward sweep x = L^-T y runs the same way after
// one barrier: wave 0 publishes x_q = L_qq^-T (r_q - L_{q+1,q}^T x_{q+1}),
// the workers fold x_q into r_p (p <= q - 2, each r_p owned by one worker,
// rcnt(p) = x blocks folded in).
// debug_skip masks (ablation only): 2 diag, 4 TRSM, 8 trailing.
// ---------------------------------------------------------------------
typedef __attribute__((address_space(3))) int lds_int;

__device__ __forceinline__ int ld_ver(const int* f) {
  return __builtin_amdgcn_readfirstlane(*(volatile lds_int*)(f));
}
__device__ __forceinline__ void wait_ver(const int* f, int v) {
  if (ld_ver(f) < v) {
    do {
      __builtin_amdgcn_s_sleep(1);
    } while (ld_ver(f) < v);
  }
  asm volatile("" ::: "memory");
}
// publish: all of this wave's LDS writes land before the counter
__device__ __forceinline__ void set_ver(int* f, int v, int lane) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (lane == 0) *(volatile lds_int*)(f) = v;
  asm volatile("" ::: "memory");
}

// One wave: sum_m M(lo, m) v[m] (TR: M(m, lo)) of a swizzled tile and a
// 32-vector in LDS; lane (lo, hi) takes half hi of m, both halves get the
// total.
template <bool TR>
__device__ __forceinline__ float tile_gemv(const float* M, const float* v, int lo, int hi) {
  float s0 = 0.0f, s1 = 0.0f;
  if constexpr (!TR) {
    // row lo's columns 16 hi .. +15 as four granule reads
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4v x = row_gran(M, lo, 4 * hi + g);
      const int m0 = 16 * hi + 4 * g;
      s0 += x[0] * v[m0];
      s1 += x[1] * v[m0 + 1];
      s0 += x[2] * v[m0 + 2];
      s1 += x[3] * v[m0 + 3];
    }
  } else {
#pragma unroll
    for (int m = 0; m < 16; m += 2) {
      const int m0 = 16 * hi + m;
      s0 += M[TR ? sw(m0, lo) : sw(lo, m0)] * v[m0];
      s1 += M[TR ? sw(m0 + 1, lo) : sw(lo, m0 + 1)] * v[m0 + 1];
    }
  }
  const float s = s0 + s1;
  return s + __shfl_xor(s, 32);
}

template <int T, int NW, bool BLK = true>
__device__ __forceinline__ void chol_solve_df(float* tiles, float* bvec, float* xvec,
                                              float* part, int* flag, int tid, int debug_skip,
                                              unsigned long long* prof = nullptr) {
  static_assert(NW >= 2, "one chain wave and at least one worker");
  constexpr int NT = T * (T + 1) / 2;
  // split-bf16 tile products (common.h mfma_x6, fp32-accurate) where the
  // register budget allows the blocked diagonal factor (BLK), and then the
  // chain's next diagonal update fused into its factor (diag_factor_inv_acc)
  constexpr bool X6 = BLK;
  constexpr bool FUSE = BLK;
  const unsigned long long t0 = prof ? clock64() : 0;
  const int lane = tid & 63, lo = lane & 31, hi = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  int* ver = reinterpret_cast<int*>(part);
  int* bver = ver + NT;
  int* rcnt = bver + T;
  int* yver = rcnt + T;
  int* xver = yver + 1;
  float* rbuf = part + ((NT + 2 * T + 2 + 3) & ~3);  // 32 floats: wave 0's r_p
  if (tid < NT + 2 * T + 2) ver[tid] = 0;
  lds_barrier();

  auto trsm = [&](int I, int p) {  // S(I, p)
    float* Aip = tiles + tidx(I, p) * 1024;
    if (!FRECSYS_SKIP(debug_skip, 4)) {
      const f32x16 u = X6 ? tile_pqT_x6(Aip, tiles + tidx(p, p) * 1024, lo, hi)
                          : tile_pqT(Aip, tiles + tidx(p, p) * 1024, lo, hi);
#pragma unroll
      for (int q = 0; q < 16; ++q) Aip[sw(acc_row(q, hi), lo)] = u[q];
    }
    set_ver(ver + tidx(I, p), p + 1, lane);
  };
  auto bupd = [&](int I, int p) {  // B(I, p): L_Ip final, y_p published
    wait_ver(bver + I, p);
    const float t = tile_gemv<false>(tiles + tidx(I, p) * 1024, bvec + 32 * p, lo, hi);
    if (hi == 0) bvec[32 * I + lo] -= t;
    set_ver(bver + I, p + 1, lane);
  };
  auto update = [&](int I, int J, int p) {  // U(I, J, p)
    float* Aij = tiles + tidx(I, J) * 1024;
    if (!FRECSYS_SKIP(debug_skip, 8)) {
      const float* Li = tiles + tidx(I, p) * 1024;
      const float* Lj = tiles + tidx(J, p) * 1024;
      const f32x16 u = !X6     ? tile_pqT(Li, Lj, lo, hi)
                       : I == J ? tile_pqT_x6<true>(Li, Li, lo, hi)
                                : tile_pqT_x6(Li, Lj, lo, hi);
#pragma unroll
      for (int q = 0; q < 16; ++q) Aij[sw(acc_row(q, hi), lo)] -= u[q];
    }
    set_ver(ver + tidx(I, J), p + 1, lane);
  };
  auto factor = [&](int p) {  // F(p)
    float* Tpp = tiles + tidx(p, p) * 1024;
    if (!FRECSYS_SKIP(debug_skip, 2)) {
      if (!diag_factor_inv<BLK>(Tpp, lane) && lane == 0) flag[0] = 1;
    }
    set_ver(ver + tidx(p, p), p + 1, lane);
  };
  auto ysolve = [&](int p) {  // Y(p): L_pp^-1 published, b_p final (bver(p) = p)
    const float y = tile_gemv<false>(tiles + tidx(p, p) * 1024, bvec + 32 * p, lo, hi);
    wave_lds_sync();
    if (hi == 0) bvec[32 * p + lo] = y;
    set_ver(yver, p + 1, lane);
  };
  // with 8 waves the forward substitution (Y, and B of the next block) runs
  // on its own wave behind the chain instead of on it
  constexpr bool YW = NW >= 8;
  constexpr int YWAVE = YW ? kCholYWave : -1;
  constexpr int NWK = YW ? NW - 2 : NW - 1;  // worker waves
  // worker slot s (0 .. NWK-1) -> wave: every wave but 0 and YWAVE, in order
  auto wk_wave = [&](int s) { return YW ? s + 1 + (s + 1 >= YWAVE ? 1 : 0) : s + 1; };

  if (wave == 0) {
    // ---- the critical chain (issue priority over the worker on its SIMD) ----
    __builtin_amdgcn_s_setprio(2);
    // diagnostics (prof): chain cycles in waits / TRSM / update / factor
    unsigned long long tw = 0, ts = 0, tu = 0, tf = 0, tc = prof ? clock64() : 0;
    auto lap = [&](unsigned long long& acc) {
      if (prof) {
        const unsigned long long t = clock64();
        acc += t - tc;
        tc = t;
      }
    };
#pragma unroll 1
    for (int p = -1; p + 1 < T; ++p) {  // one factor call site
      if constexpr (FUSE) {
        float* Tnn = tiles + tidx(p + 1, p + 1) * 1024;
        bool ok = true;
        if (p >= 0) {
          wait_ver(ver + tidx(p + 1, p), p);  // all of panel < p's updates
          lap(tw);
          trsm(p + 1, p);
          if (!YW) bupd(p + 1, p);
          lap(ts);
          wait_ver(ver + tidx(p + 1, p + 1), p);
          lap(tw);
          // A_nn - L_np L_np^T, element (acc_row(q, hi), lo); by symmetry
          // lane lo's row lo is its own 16 values + lane lo+32's
          const float* Lnp = tiles + tidx(p + 1, p) * 1024;
          f32x16 u = f32x16{0.f};
          if (!FRECSYS_SKIP(debug_skip, 8)) u = tile_pqT_x6<true>(Lnp, Lnp, lo, hi);
#pragma unroll
          for (int q = 0; q < 16; ++q) u[q] = Tnn[sw(acc_row(q, hi), lo)] - u[q];
          lap(tu);
          if (!FRECSYS_SKIP(debug_skip, 2)) ok = diag_factor_inv_acc(u, (lds_float*)Tnn);
        } else {
          if (!FRECSYS_SKIP(debug_skip, 2)) ok = diag_factor_inv_blk((lds_float*)Tnn, lane);
        }
        if (!ok && lane == 0) flag[0] = 1;
        set_ver(ver + tidx(p + 1, p + 1), p + 2, lane);
      } else {
        if (p >= 0) {
          wait_ver(ver + tidx(p + 1, p), p);  // all of panel < p's updates
          lap(tw);
          trsm(p + 1, p);
          if (!YW) bupd(p + 1, p);
          lap(ts);
          wait_ver(ver + tidx(p + 1, p + 1), p);
          lap(tw);
          update(p + 1, p + 1, p);
          lap(tu);
        }
        factor(p + 1);
      }
      if (!YW) ysolve(p + 1);
      lap(tf);
    }
    if (prof && lane == 0) {
      atomicAdd(prof + 11, tw);
      atomicAdd(prof + 12, ts);
      atomicAdd(prof + 13, tu);
      atomicAdd(prof + 14, tf);
    }
    __builtin_amdgcn_s_setprio(0);
    if (prof && lane == 0) atomicAdd(prof + 5, clock64() - t0);
  } else if (YW && wave == YWAVE) {
    // ---- the forward substitution along the chain ----
#pragma unroll 1
    for (int p = 0; p < T; ++p) {
      wait_ver(ver + tidx(p, p), p + 1);  // F(p)
      wait_ver(bver + p, p);             // b_p final
      ysolve(p);
      if (p + 1 < T) {
        wait_ver(ver + tidx(p + 1, p), p + 1);  // S(p+1, p)
        bupd(p + 1, p);
      }
    }
  } else {
    // ---- workers: the rest of each panel, round-robin ----
    int k = 0;
    unsigned long long tww = 0;  // diagnostics (prof): cycles in waits
    auto wwait = [&](const int* f, int v) {
      if (prof) {
        const unsigned long long t = clock64();
        wait_ver(f, v);
        tww += clock64() - t;
      } else {
        wait_ver(f, v);
      }
    };
    auto wprio = [&](bool c) {
      if (c) __builtin_amdgcn_s_setprio(1);
      else __builtin_amdgcn_s_setprio(0);
    };
#pragma unroll 1
    for (int p = 0; p + 1 < T; ++p) {
#pragma unroll 1
      for (int I = p + 2; I < T; ++I, ++k) {  // S(I, p), B(I, p)
        if (wk_wave(k % NWK) != wave) continue;
        wwait(ver + tidx(p, p), p + 1);
        wwait(ver + tidx(I, p), p);
        wprio(I <= p + 1 + kCholWPrio);
        trsm(I, p);
        wwait(yver, p + 1);
        bupd(I, p);
      }
#pragma unroll 1
      for (int J = p + 1; J < T; ++J) {  // U(I, J, p), column by column
#pragma unroll 1
        for (int I = (J == p + 1 ? p + 2 : J); I < T; ++I, ++k) {
          if (wk_wave(k % NWK) != wave) continue;
          wwait(ver + tidx(I, p), p + 1);
          wwait(ver + tidx(J, p), p + 1);
          wwait(ver + tidx(I, J), p);
          wprio(I <= p + 1 + kCholWPrio);
          update(I, J, p);
        }
      }
    }
    __builtin_amdgcn_s_setprio(0);
    if (prof && lane == 0) {
      atomicAdd(prof + 6, (clock64() - t0) / NWK);
      atomicAdd(prof + 15, tww / NWK);
    }
  }
  lds_barrier();
  if (prof && tid == 0) atomicAdd(prof + 7, clock64() - t0);

  // ---- backward: x = L^-T y; bvec holds y and, per block, r_p ----
  if (wave == 0) {
    __builtin_amdgcn_s_setprio(2);
#pragma unroll 1
    for (int p = T - 1; p >= 0; --p) {
      float r = bvec[32 * p + lo];
      if (p + 1 < T) {
        wait_ver(rcnt + p, T - 2 - p);  // x_q, q >= p + 2, folded in by a worker
        r = bvec[32 * p + lo] -
            tile_gemv<true>(tiles + tidx(p + 1, p) * 1024, xvec + 32 * (p + 1), lo, hi);
      }
      if (hi == 0) rbuf[lo] = r;
      wave_lds_sync();
      const float x = tile_gemv<true>(tiles + tidx(p, p) * 1024, rbuf, lo, hi);
      if (hi == 0) xvec[32 * p + lo] = x;
      set_ver(xver, T - p, lane);
    }
    __builtin_amdgcn_s_setprio(0);
  } else {
#pragma unroll 1
    for (int q = T - 1; q >= 2; --q) {
#pragma unroll 1
      for (int p = 0; p + 2 <= q; ++p) {
        if (1 + p % (NW - 1) != wave) continue;
        wait_ver(xver, T - q);
        const float t = tile_gemv<true>(tiles + tidx(q, p) * 1024, xvec + 32 * q, lo, hi);
        if (hi == 0) bvec[32 * p + lo] -= t;
        set_ver(rcnt + p, T - q, lane);
      }
    }
  }
  lds_barrier();
}

}  // namespace frecsys_hip
