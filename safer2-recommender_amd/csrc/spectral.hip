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
//  rotate_kernel   Y = X Q / X Q^T on the bf16 matrix cores (3-piece splits,
//                  fp32-accurate), Q split once per basis (split_basis_kernel);
//                  optional entity list for the scatter; also the u^T G u
//                  partials of the wide user loss.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <type_traits>

#include "chol.h"
#include "common.h"
#include "kernels.h"

namespace frecsys_hip {

namespace {

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

// DPP row operations (within 16-lane rows).
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
constexpr int DPP_XOR1 = 0xB1;         // quad_perm [1,0,3,2]
constexpr int DPP_XOR2 = 0x4E;         // quad_perm [2,3,0,1]
constexpr int DPP_ROR8 = 0x128;        // row_ror:8 (= lane ^ 8 in a 16-lane row)
constexpr int DPP_ROR4 = 0x124;
constexpr int DPP_HALF_MIRROR = 0x141; // lane i <- 7 - i within each 8 (flips bit 2)
// Sum over a 16-lane DPP row; every lane of the row gets it.
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp<DPP_ROR8>(v);
  v += dpp<DPP_ROR4>(v);
  v += dpp<DPP_XOR2>(v);
  v += dpp<DPP_XOR1>(v);
  return v;
}

// Per-phase cycle counters of tridiag_kernel, per wave (diagnostics:
// scripts/micro/tridiag_prof.hip builds with -DFRECSYS_TRIDIAG_PROF).
#ifdef FRECSYS_TRIDIAG_PROF
__device__ unsigned long long g_tri_prof[16][8];  // [wave][phase]
#define TRI_PROF_DECL unsigned long long tp_last = clock64(), tp_acc[6] = {0, 0, 0, 0, 0, 0};
#define TRI_PROF_MARK(i)                      \
  {                                           \
    const unsigned long long t_ = clock64();  \
    tp_acc[i] += t_ - tp_last;                \
    tp_last = t_;                             \
  }
#define TRI_PROF_FLUSH \
  if (lane == 0)       \
    for (int i = 0; i < 6; ++i) g_tri_prof[wave][i] = tp_acc[i];
#else
#define TRI_PROF_DECL
#define TRI_PROF_MARK(i)
#define TRI_PROF_FLUSH
#endif

// Householder tridiagonalisation (LAPACK sytd2 conventions, v(k+1) = 1),
// register-resident in one workgroup of 8 waves (2 per SIMD, so 256
// registers per lane): the symmetric matrix (zero-padded to 256) as 8 x 16
// blocks, thread (wave w, lane l) owning rows 8 (4w + l/16) .. +7 and
// columns 16 (l % 16) .. +15 -- each group of 8 rows lives in one 16-lane DPP
// row.  Every reduction of a step is a handful of DPP ops inside one wave:
//  * p = tau A v: each thread's 8 row partials are reduce-scattered over its
//    16 lanes (row_ror:8, row_half_mirror, quad perms), one LDS store per row;
//  * reflector k+1 is formed from ROW k+1 of the (symmetric) matrix, held by
//    one 16-lane group (norm, x0, diagonal by 16-lane sums), right after that
//    wave has updated this one row -- its latency hides under the rest of
//    the update.
// Column pairs run on v_pk_fma_f32.  Two LDS-only barriers per step (p
// published, v published): the reflector's global stores (Vh, T, tau) are
// never waited on inside the loop.  K = (tau/2) v.p is formed by every wave
// from the published p.  Step k only needs the trailing block
// [k+1:, k+1:], so waves whose 32 rows are all <= k skip its arithmetic.
// With Q != nullptr, workgroups 1 .. n/32 form the rows of Q while the
// reduction runs (common.h qrows_worker): at the start of step k the first n
// threads store v_k (its LDS copy, tau-masked) and tau_k as tagged words
// (vt, tt), so no form-Q launch follows.
__global__ void __launch_bounds__(512)
    tridiag_kernel(const float* __restrict__ G, int n, float* tdiag, float* toff, float* Vh,
                   float* tau_out, float* Q, bf16x8* img_q, bf16x8* img_qt,
                   unsigned long long* vt, unsigned long long* tt, unsigned* tcount) {
  typedef float f2 __attribute__((ext_vector_type(2)));  // v_pk_fma_f32 operands
  __shared__ __attribute__((aligned(16))) float vs[2][256];
  __shared__ __attribute__((aligned(16))) float ps[256];
  __shared__ float tsh[2];
  if (blockIdx.x > 0) {  // Q-row worker (reflectors k = 0 .. n-3)
    qrows_worker<256, 512>(blockIdx.x - 1, n, n - 2, vt, tt, Q, img_q, img_qt, &vs[0][0], tsh,
                           tcount);
    return;
  }
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int rb = 4 * wave + (lane >> 4);  // row block (8 rows)
  const int cb = lane & 15;               // column block (16 columns)
  const int r0 = 8 * rb, c0 = 16 * cb;
  f2 A[8][8];  // A[r][j] = columns c0 + 2j, c0 + 2j + 1 of row r0 + r
#pragma unroll
  for (int r = 0; r < 8; ++r)
#pragma unroll
    for (int c = 0; c < 16; c += 4) {
      float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
      if (r0 + r < n && c0 + c < n) g = *reinterpret_cast<const float4*>(G + (int64_t)(r0 + r) * n + c0 + c);
      A[r][c / 2] = f2{g.x, g.y};
      A[r][c / 2 + 1] = f2{g.z, g.w};
    }

  // reflector for column k (= row k), by the 16-lane group holding row k;
  // the row inside the 8 x 16 block, k & 7, is a compile-time constant RR
  // (the step loop is unrolled by 8) so A stays in registers
  auto reflector = [&](int k, auto rr_c) {
    constexpr int RR = decltype(rr_c)::value;
    if (wave != (k >> 5)) return;  // wave-uniform
    const bool mine = rb == (k >> 3);
    float s = 0.0f, x0 = 0.0f, dkk = 0.0f;
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      const int j = c0 + c;
      const float x = A[RR][c >> 1][c & 1];
      if (j >= k + 2) s += x * x;
      if (j == k + 1) x0 = x;
      if (j == k) dkk = x;
    }
    s = row16_sum(s);
    x0 = row16_sum(x0);
    dkk = row16_sum(dkk);
    float tau = 0.0f, beta = x0, scal = 0.0f;
    if (s > 0.0f) {
      const float nrm = sqrtf(x0 * x0 + s);
      beta = x0 >= 0.0f ? -nrm : nrm;
      tau = (beta - x0) / beta;
      scal = 1.0f / (x0 - beta);
    }
    if (mine) {
      float* v = vs[k & 1];
#pragma unroll
      for (int c = 0; c < 16; c += 4) {  // 16-B LDS and global stores
        float4 t, g;
        float* tp = &t.x;
        float* gp = &g.x;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int j = c0 + c + e;
          float vj = 0.0f;
          if (j == k + 1) vj = 1.0f;
          else if (j > k + 1) vj = A[RR][(c + e) >> 1][(c + e) & 1] * scal;
          gp[e] = vj;  // Vh row k: entries j <= k are never read (form_q masks them)
          tp[e] = tau != 0.0f ? vj : 0.0f;
        }
        *reinterpret_cast<float4*>(v + c0 + c) = t;
        if (c0 + c < n) *reinterpret_cast<float4*>(Vh + (int64_t)k * n + c0 + c) = g;
      }
      if (cb == 0) {
        tsh[k & 1] = tau;
        tdiag[k] = dkk;
        toff[k] = beta;
        tau_out[k] = tau;
      }
    }
  };

  if (n > 2) reflector(0, std::integral_constant<int, 0>{});
  __syncthreads();
  TRI_PROF_DECL
  auto step = [&](int k, auto rr_next) {
    constexpr int RN = decltype(rr_next)::value;  // row of reflector k+1 in its block
    TRI_PROF_MARK(0)
    const float tau = tsh[k & 1];
    const float* v = vs[k & 1];
    if (Q) {  // reflector k for the Q-row workers, from its LDS copy (published at step k)
      if (tid > k && tid < n) tstore(vt + (size_t)k * n + tid, (unsigned)k + 1, v[tid]);
      if (tid == 0) tstore(tt + k, (unsigned)k + 1, tau);
    }
    const bool active = 32 * wave + 31 >= k + 1;  // wave-uniform: rows > k present
    const bool owner = wave == ((k + 1) >> 5);    // forms reflector k+1 inside its update
    f2 vc[8];
    if (tau != 0.0f && active) {
#pragma unroll
      for (int c = 0; c < 16; c += 4) {
        const float4 t = *reinterpret_cast<const float4*>(v + c0 + c);
        vc[c / 2] = f2{t.x, t.y};
        vc[c / 2 + 1] = f2{t.z, t.w};
      }
      // row partials of A v over my 16 columns
      float pr[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        f2 acc = A[r][0] * vc[0];
#pragma unroll
        for (int j = 1; j < 8; ++j) acc = A[r][j] * vc[j] + acc;
        pr[r] = acc.x + acc.y;
      }
      // reduce-scatter of the 8 row sums over the 16 lanes
      const int b3 = (lane >> 3) & 1, b2 = (lane >> 2) & 1, b1 = (lane >> 1) & 1;
      float q4[4], q2[2];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float keep = b3 ? pr[4 + i] : pr[i];
        const float send = b3 ? pr[i] : pr[4 + i];
        q4[i] = keep + dpp<DPP_ROR8>(send);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const float keep = b2 ? q4[2 + i] : q4[i];
        const float send = b2 ? q4[i] : q4[2 + i];
        q2[i] = keep + dpp<DPP_HALF_MIRROR>(send);
      }
      float q1 = (b1 ? q2[1] : q2[0]) + dpp<DPP_XOR2>(b1 ? q2[0] : q2[1]);
      q1 += dpp<DPP_XOR1>(q1);
      if ((lane & 1) == 0) ps[r0 + 4 * b3 + 2 * b2 + b1] = tau * q1;
    }
    TRI_PROF_MARK(1)
    lds_barrier();
    TRI_PROF_MARK(2)
    bool reflected = false;
    if (tau != 0.0f && active) {
      // K = (tau / 2) v.p over the whole vector, by every wave
      const float4 pv = *reinterpret_cast<const float4*>(ps + 4 * lane);
      const float4 vv = *reinterpret_cast<const float4*>(v + 4 * lane);
      const float K = 0.5f * tau * wave_sum_dpp(pv.x * vv.x + pv.y * vv.y + pv.z * vv.z + pv.w * vv.w);
      const f2 K2 = f2{K, K};
      f2 wc[8];
#pragma unroll
      for (int c = 0; c < 16; c += 4) {
        const float4 t = *reinterpret_cast<const float4*>(ps + c0 + c);
        wc[c / 2] = f2{t.x, t.y} - K2 * vc[c / 2];
        wc[c / 2 + 1] = f2{t.z, t.w} - K2 * vc[c / 2 + 1];
      }
      float vr[8], wr[8];
#pragma unroll
      for (int r = 0; r < 8; r += 4) {
        const float4 a4 = *reinterpret_cast<const float4*>(v + r0 + r);
        const float4 b4 = *reinterpret_cast<const float4*>(ps + r0 + r);
        vr[r] = a4.x, vr[r + 1] = a4.y, vr[r + 2] = a4.z, vr[r + 3] = a4.w;
        wr[r] = b4.x - K * a4.x, wr[r + 1] = b4.y - K * a4.y;
        wr[r + 2] = b4.z - K * a4.z, wr[r + 3] = b4.w - K * a4.w;
      }
      // A -= v w^T + w v^T, two packed FMAs per column pair; row RN first,
      // so the owner forms reflector k+1 before the other 7 rows
      auto upd = [&](int r) {
        const f2 nv = f2{-vr[r], -vr[r]}, nw = f2{-wr[r], -wr[r]};
#pragma unroll
        for (int j = 0; j < 8; ++j) A[r][j] = nw * vc[j] + (nv * wc[j] + A[r][j]);
      };
      upd(RN);
      if (owner && k + 1 < n - 2) {
        __builtin_amdgcn_s_setprio(2);
        reflector(k + 1, rr_next);
        __builtin_amdgcn_s_setprio(0);
        reflected = true;
      }
#pragma unroll
      for (int r = 0; r < 8; ++r)
        if (r != RN) upd(r);
    }
    TRI_PROF_MARK(3)
    if (!reflected && k + 1 < n - 2) reflector(k + 1, rr_next);  // tau == 0 step
    TRI_PROF_MARK(4)
    lds_barrier();
    TRI_PROF_MARK(5)
  };
  for (int kb = 0; kb < n - 2; kb += 8) {
    step(kb + 0, std::integral_constant<int, 1>{});
    if (kb + 1 < n - 2) step(kb + 1, std::integral_constant<int, 2>{});
    if (kb + 2 < n - 2) step(kb + 2, std::integral_constant<int, 3>{});
    if (kb + 3 < n - 2) step(kb + 3, std::integral_constant<int, 4>{});
    if (kb + 4 < n - 2) step(kb + 4, std::integral_constant<int, 5>{});
    if (kb + 5 < n - 2) step(kb + 5, std::integral_constant<int, 6>{});
    if (kb + 6 < n - 2) step(kb + 6, std::integral_constant<int, 7>{});
    if (kb + 7 < n - 2) step(kb + 7, std::integral_constant<int, 0>{});
  }
  TRI_PROF_FLUSH
  // the last 2 x 2 block
#pragma unroll
  for (int r = 0; r < 8; ++r)
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      const int i = r0 + r, j = c0 + c;
      const float x = A[r][c >> 1][c & 1];
      if (i == n - 2 && j == n - 2) tdiag[n - 2] = x;
      if (i == n - 1 && j == n - 1) tdiag[n - 1] = x;
      if (i == n - 1 && j == n - 2) toff[n - 2] = x;
    }
  if (tid == 0) {
    toff[n - 1] = 0.0f;
    tau_out[n - 2] = 0.0f;
    tau_out[n - 1] = 0.0f;
  }
}

// Q = H_0 H_1 ... H_{n-3}: one wave per column c of Q, q = H_0 (H_1 (...
// H_{n-3} e_c)); H_k leaves columns c <= k alone, so the product starts at
// k = min(c-1, n-3).  The reflectors are staged through LDS FQ_KB at a time
// by all 8 waves of the workgroup, the next block's loads issued into
// registers before the current block is applied (one memory round trip per
// block would otherwise sit on the chain: 16 per basis at n = 256), then
// applied from LDS.  The epilogue writes Q and, from the 8 columns staged in
// LDS, this workgroup's granules of the split images of Q and Q^T that the
// rotations read (split_basis_kernel's layout; no separate launches).
// RPL = rows per lane (n <= 64 * RPL).
constexpr int FQ_KB = 16;
template <int RPL>
__global__ void __launch_bounds__(512)
    form_q_kernel(const float* __restrict__ Vh, const float* __restrict__ tau, int n, float* Q,
                  bf16x8* __restrict__ img_q, bf16x8* __restrict__ img_qt) {
  constexpr int ROWS = 64 * RPL;
  constexpr int PER = FQ_KB * ROWS / 512;  // staged values per thread and block
  __shared__ __attribute__((aligned(16))) float vsh[FQ_KB][ROWS];
  __shared__ float tsh[FQ_KB];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = blockIdx.x * 8 + wave;
  const int c_first = blockIdx.x * 8;
  float q[RPL];
#pragma unroll
  for (int r = 0; r < RPL; ++r) q[r] = (lane + 64 * r == c) ? 1.0f : 0.0f;
  const int kstart = c < n ? (c - 1 < n - 3 ? c - 1 : n - 3) : -1;
  // highest reflector any column of this workgroup needs
  int ktop = c_first + 7 - 1 < n - 3 ? c_first + 7 - 1 : n - 3;
  if (ktop >= n) ktop = n - 1;
  float pre[PER];
  float tpre = 0.0f;
  auto fetch = [&](int kb) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int s2 = threadIdx.x + 512 * i;
      const int kk = kb + s2 / ROWS, row = s2 % ROWS;
      pre[i] = (kb >= 0 && kk <= ktop && row > kk && row < n) ? Vh[(int64_t)kk * n + row] : 0.0f;
    }
    if (threadIdx.x < FQ_KB)
      tpre = (kb >= 0 && kb + (int)threadIdx.x <= ktop) ? tau[kb + threadIdx.x] : 0.0f;
  };
  const int kb0 = ktop >= 0 ? ktop - (ktop % FQ_KB) : -1;
  if (kb0 >= 0) fetch(kb0);
  for (int kb = kb0; kb >= 0; kb -= FQ_KB) {
    __syncthreads();  // previous block consumed
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int s2 = threadIdx.x + 512 * i;
      vsh[s2 / ROWS][s2 % ROWS] = pre[i];
    }
    if (threadIdx.x < FQ_KB) tsh[threadIdx.x] = tpre;
    __syncthreads();
    if (kb - FQ_KB >= 0) fetch(kb - FQ_KB);  // in flight while this block is applied
    for (int j = FQ_KB - 1; j >= 0; --j) {
      const int k = kb + j;
      if (k > kstart) continue;  // wave-uniform
      const float t = tsh[j];
      if (t == 0.0f) continue;
      float d = 0.0f;
#pragma unroll
      for (int r = 0; r < RPL; ++r) d += vsh[j][lane + 64 * r] * q[r];
      d = wave_sum_dpp(d) * t;
#pragma unroll
      for (int r = 0; r < RPL; ++r) q[r] -= d * vsh[j][lane + 64 * r];
    }
  }
  if (c < n) {
#pragma unroll
    for (int r = 0; r < RPL; ++r) {
      const int row = lane + 64 * r;
      if (row < n) Q[(int64_t)row * n + c] = q[r];
    }
  }
  if (!img_q) return;
  // split images (n a multiple of 32, so all 8 columns exist): the columns
  // through LDS, [8][n]
  __syncthreads();
  float* qs = &vsh[0][0];
#pragma unroll
  for (int r = 0; r < RPL; ++r) {
    const int row = lane + 64 * r;
    if (row < n) qs[wave * n + row] = q[r];
  }
  __syncthreads();
  const int NCT = n / 32;
  {  // image of Q: granule (s, hi) of column c = rows 16 s + 8 hi .. + 7
    const int C = c >> 5, lo = c & 31;
    for (int gi = lane; gi < n / 8; gi += 64) {
      const int sg = gi >> 1, hi = gi & 1;
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = qs[wave * n + 16 * sg + 8 * hi + j];
      bf16x8 f[3];
      split3x8(v, f);
#pragma unroll
      for (int p = 0; p < 3; ++p) img_q[((int64_t)(sg * NCT + C) * 3 + p) * 64 + 32 * hi + lo] = f[p];
    }
  }
  {  // image of Q^T: B[k][col] = Q[col][k], k = c_first .. c_first + 7 = one granule row
    const int sg = c_first >> 4, hi = (c_first >> 3) & 1;
    for (int col = threadIdx.x; col < n; col += 512) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = qs[j * n + col];
      bf16x8 f[3];
      split3x8(v, f);
      const int C = col >> 5, lo = col & 31;
#pragma unroll
      for (int p = 0; p < 3; ++p)
        img_qt[((int64_t)(sg * NCT + C) * 3 + p) * 64 + 32 * hi + lo] = f[p];
    }
  }
}

// ---- rotations on the bf16 matrix cores ----
// Y = X B (B = Q or Q^T), fp32-accurate: every product as common.h mfma_x6
// (3-piece bf16 splits).  B is split once per basis into its fragment image
// (split_basis_kernel): granule ((s * NCT + C) * 3 + p) * 64 + lane holds
// piece p of B[16s + 8hi .. +7][32C + lo] (lane = 32 hi + lo) -- one 1-KB
// coalesced load per wave and MFMA operand, L2-resident (Dp^2 * 6 bytes).
// X rows go straight from global memory into the A fragments (2 float4 per
// lane and k16 step, or 8 position-blocked scalars), so the kernel uses no
// LDS.  A workgroup: 4 waves, 64 rows x (2 or 4) 32-column tiles; the column
// blocks of one row block sit on one XCD (consecutive slots of its dispatch
// sequence) so X's rows are fetched from HBM once.
__global__ void __launch_bounds__(256)
    split_basis_kernel(const float* __restrict__ Q, int DP, int trans, bf16x8* __restrict__ out) {
  const int NCT = DP / 32, NS = DP / 16;
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (g >= (int64_t)NS * NCT * 64) return;
  const int lane = (int)(g & 63), lo = lane & 31, hi = lane >> 5;
  const int64_t sc = g >> 6;
  const int C = (int)(sc % NCT), s = (int)(sc / NCT);
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = 16 * s + 8 * hi + j, col = 32 * C + lo;
    v[j] = trans ? Q[(int64_t)col * DP + k] : Q[(int64_t)k * DP + col];
  }
  bf16x8 f[3];
  split3x8(v, f);
#pragma unroll
  for (int p = 0; p < 3; ++p) out[(sc * 3 + p) * 64 + lane] = f[p];
}

template <int DP>
__global__ void __launch_bounds__(256)
    rotate_kernel(const float* __restrict__ X, const QueueRec* __restrict__ rows, int64_t r0,
                  int64_t n, const bf16x8* __restrict__ Bs, float* __restrict__ Y, int x_blocked,
                  int ncb, float* __restrict__ qpart) {
  constexpr int NCT = DP / 32, NS = DP / 16;
  constexpr int CW = (DP % 128 == 0) ? 2 : 1;  // column tiles per wave
  constexpr int CB = 2 * CW;                   // column tiles per workgroup
  const int tid = threadIdx.x, lane = tid & 63, lo = lane & 31, hi = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // slot b -> XCD b % 8; the ncb column blocks of a row block on one XCD
  const int64_t bid = blockIdx.x, sx = bid >> 3;
  const int cbk = (int)(sx % ncb);
  const int64_t rblk = (sx / ncb) * 8 + (bid & 7);
  const int64_t base = rblk * 64;
  if (base >= n) return;
  const int R = wave & 1, cg = wave >> 1;
  const int C0 = cbk * CB + cg * CW;
  const int64_t pos = base + 32 * R + lo;  // my A row (position)
  const bool pv = pos < n;
  // X row: the entity rows[p] with a row list (forward rotation of a row
  // subset), else position r0 + p (x_blocked: the position-blocked layout)
  const int64_t xp = pv ? pos : base;
  const float* xr = X + (x_blocked ? 0 : (rows ? (int64_t)rows[xp].entity : r0 + xp) * DP);
  f32x16 acc[CW];
#pragma unroll
  for (int j = 0; j < CW; ++j) acc[j] = f32x16{0.f};
  auto load_a = [&](int s, float (&v)[8]) {
    const int k0 = 16 * s + 8 * hi;
    if (x_blocked) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = pv ? X[blk_v(pos, k0 + j, DP)] : 0.0f;
    } else {
      const float4 a = *reinterpret_cast<const float4*>(xr + k0);
      const float4 b = *reinterpret_cast<const float4*>(xr + k0 + 4);
      v[0] = a.x, v[1] = a.y, v[2] = a.z, v[3] = a.w;
      v[4] = b.x, v[5] = b.y, v[6] = b.z, v[7] = b.w;
      if (!pv) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = 0.0f;
      }
    }
  };
  float vn[8];
  load_a(0, vn);
  // B fragments (the Q pieces, L2-resident) one k-step ahead as well
  bf16x8 bn[CW][3];
  auto load_b = [&](int s) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < CW; ++j) {
      const int C = C0 + j < NCT ? C0 + j : NCT - 1;  // clamped: no branch around the loads
#pragma unroll
      for (int p = 0; p < 3; ++p) bn[j][p] = Bs[((int64_t)(s * NCT + C) * 3 + p) * 64 + lane];
    }
  };
  load_b(0);
#pragma unroll 2
  for (int s = 0; s < NS; ++s) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = vn[j];
    bf16x8 bf[CW][3];
#pragma unroll
    for (int j = 0; j < CW; ++j)
#pragma unroll
      for (int p = 0; p < 3; ++p) bf[j][p] = bn[j][p];
    if (s + 1 < NS) {  // next step's rows and Q pieces in flight
      load_a(s + 1, vn);
      load_b(s + 1);
    }
    bf16x8 af[3];
    split3x8(v, af);
#pragma unroll
    for (int j = 0; j < CW; ++j)
      if (C0 + j < NCT) acc[j] = mfma_x6(af, bf[j], acc[j]);  // wave-uniform
  }
  if (qpart) {
    // u^T B u partials of the user loss (B = G): row dots of (X B) with X
    // over this workgroup's column block, two waves per row half combined in
    // a fixed order -> qpart[column block][row]
    __shared__ float qred[2][64];
    float rs[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int64_t p = base + 32 * R + acc_row(q, hi);
      float sv = 0.0f;
      if (p < n) {  // explicit fma: the same rounding in rotate_lds_kernel
        const float* xp = X + (r0 + p) * DP + 32 * C0 + lo;
        if (CW == 2 && C0 + 1 < NCT) sv = __builtin_fmaf(acc[CW - 1][q], xp[32], acc[0][q] * xp[0]);
        else if (C0 < NCT) sv = acc[0][q] * xp[0];
      }
#pragma unroll
      for (int o = 16; o > 0; o >>= 1) sv += __shfl_xor(sv, o);  // the 32 columns of a half
      rs[q] = sv;
    }
    if (lo == 0) {
#pragma unroll
      for (int q = 0; q < 16; ++q) qred[cg][32 * R + acc_row(q, hi)] = rs[q];
    }
    __syncthreads();
    if (tid < 64 && base + tid < n) qpart[(int64_t)cbk * n + base + tid] = qred[0][tid] + qred[1][tid];
    return;
  }
#pragma unroll
  for (int j = 0; j < CW; ++j) {
    const int C = C0 + j;
    if (C >= NCT) continue;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int64_t p = base + 32 * R + acc_row(q, hi);
      if (p < n) {
        const int64_t id = rows ? (int64_t)rows[p].entity : r0 + p;
        Y[id * DP + 32 * C + lo] = acc[j][q];
      }
    }
  }
}

// ---- Cholesky basis: one M for every entity of the launch ----
constexpr int chol_basis_stage_tiles(int T) { return T <= 16 ? 16 : 7; }

// When every entity of a history-space launch has the same
// M = mu*G + lam*I (iALS with l2_reg_exp = 0: RegularizationValue,
// ials.h:310-315, is reg whatever the history; mu = unobserved_weight), the
// basis need not diagonalise G at all: with M = L L^T, W = X L^-T gives
// Xt M^-1 Xt^T = W_h W_h^T and x = L^-T (W_h^T z), so dual.hip runs
// unchanged on W with a unit LDL table (l = 0, D = 1) and the back rotation
// multiplies by L^-1.  One workgroup of 16 waves:
//  * right-looking blocked Cholesky over the 32x32 tiles of M in a global
//    workspace A (L2-resident): wave 0 factors and inverts the diagonal
//    tile (chol.h diag_factor_inv), the panel L_ip = A_ip L_pp^-T and the
//    trailing A_ij -= L_ip L_jp^T are f32 MFMA tile products (tile_pqT) over
//    LDS copies, one tile per wave;
//  * XT = L^-T by block rows of L: XT_ji = -(sum_{k=j}^{i-1} XT_jk L_ik^T)
//    L_ii^-T (X = L^-1: L_ii X_ij = -sum_k L_ik X_kj), XT_ii = L_ii^-T, one
//    tile j per wave of the first NS (16; 7 at Dp = 1024, where the panel of
//    31 tiles leaves room for 7 staging tiles in the 160 KB of LDS).
// status[0] = 1 when every pivot was positive, else 0 (dual_ldl_kernel turns
// 0 into the launch's failure flag: the call reruns on the d-space path).
template <int T>
__global__ void __launch_bounds__(1024)
    chol_basis_kernel(const float* __restrict__ G, float mu, float lam, float* __restrict__ A,
                      float* __restrict__ dinv, float* __restrict__ XT,
                      float* __restrict__ status) {
  constexpr int Dp = 32 * T, NW = 16, NS = chol_basis_stage_tiles(T);
  static_assert(NS < NW || T <= NW, "wave NW - 1 (XT's diagonal tiles) takes no tile j < T - 1");
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* panel = sm;               // [T-1] swizzled tiles: panel p / block row i of L
  float* D = sm + (T - 1) * 1024;  // L_pp^-1, swizzled
  float* stg = D + 1024;           // [NS] per-wave staging tile
  __shared__ int fail;
  const int tid = threadIdx.x, lane = tid & 63, lo = lane & 31, hi = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (tid == 0) fail = 0;
  for (int e4 = tid; e4 < Dp * Dp / 4; e4 += 1024) {  // A = mu*G + lam*I, XT = 0
    const int r = (4 * e4) / Dp, c = (4 * e4) % Dp;
    float4 g = reinterpret_cast<const float4*>(G)[e4];
    g.x = mu * g.x + (r == c ? lam : 0.0f);
    g.y = mu * g.y + (r == c + 1 ? lam : 0.0f);
    g.z = mu * g.z + (r == c + 2 ? lam : 0.0f);
    g.w = mu * g.w + (r == c + 3 ? lam : 0.0f);
    reinterpret_cast<float4*>(A)[e4] = g;
    reinterpret_cast<float4*>(XT)[e4] = float4{0.f, 0.f, 0.f, 0.f};
  }
  __syncthreads();
  // one wave: the 32x32 tile at src (ld Dp) into a swizzled LDS tile
  auto load_tile = [&](float* dst, const float* src) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e4 = lane + 64 * q, r = e4 >> 3, c = 4 * (e4 & 7);
      const float4 v = *reinterpret_cast<const float4*>(src + r * Dp + c);
      dst[sw(r, c)] = v.x;
      dst[sw(r, c + 1)] = v.y;
      dst[sw(r, c + 2)] = v.z;
      dst[sw(r, c + 3)] = v.w;
    }
  };
  for (int p = 0; p < T; ++p) {
    const int m = T - 1 - p;
    if (wave == 0) {
      load_tile(D, A + (32 * p) * Dp + 32 * p);
      if (!diag_factor_inv(D, lane) && lane == 0) fail = 1;
      for (int e = lane; e < 1024; e += 64) dinv[p * 1024 + e] = D[e];
    }
    __syncthreads();
    for (int s = wave; s < m; s += NW) {  // L_ip = A_ip L_pp^-T
      const int i = p + 1 + s;
      float* slot = panel + s * 1024;
      load_tile(slot, A + (32 * i) * Dp + 32 * p);
      const f32x16 u = tile_pqT(slot, D, lo, hi);
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int r = acc_row(q, hi);
        slot[sw(r, lo)] = u[q];
        A[(32 * i + r) * Dp + 32 * p + lo] = u[q];
      }
    }
    __syncthreads();
    for (int t = wave; t < m * (m + 1) / 2; t += NW) {  // A_ij -= L_ip L_jp^T
      int I = 0;
      while ((I + 1) * (I + 2) / 2 <= t) ++I;
      const int J = t - I * (I + 1) / 2;
      float* dst = A + (32 * (p + 1 + I)) * Dp + 32 * (p + 1 + J);
      float old[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) old[q] = dst[acc_row(q, hi) * Dp + lo];
      const f32x16 u = tile_pqT(panel + I * 1024, panel + J * 1024, lo, hi);
#pragma unroll
      for (int q = 0; q < 16; ++q) dst[acc_row(q, hi) * Dp + lo] = old[q] - u[q];
    }
    __syncthreads();
  }
  for (int i = 0; i < T; ++i) {
    for (int e = tid; e < i * 1024; e += 1024) {  // block row i of L, tiles k < i
      const int k = e >> 10, r = (e >> 5) & 31, c = e & 31;
      panel[k * 1024 + sw(r, c)] = A[(32 * i + r) * Dp + 32 * k + c];
    }
    D[tid] = dinv[i * 1024 + tid];
    __syncthreads();
    if (wave == NW - 1) {  // XT_ii = L_ii^-T (the tiles j < i go to waves < NS < NW - 1)
      for (int e = lane; e < 1024; e += 64) {
        const int r = e >> 5, c = e & 31;
        XT[(32 * i + c) * Dp + 32 * i + r] = D[sw(r, c)];
      }
    }
    for (int j = wave; wave < NS && j < i; j += NS) {
      f32x16 acc = f32x16{0.f};
      for (int k = j; k < i; ++k) {  // C^T = sum_k XT_jk L_ik^T
        const float* src = XT + (32 * j + lo) * Dp + 32 * k + hi;
        float pa[16];
#pragma unroll
        for (int s = 0; s < 16; ++s) pa[s] = src[2 * s];
        const float* Lk = panel + k * 1024;
#pragma unroll
        for (int g = 0; g < 8; ++g) {  // row lo of L_ik by granules (k = 2s + hi)
          const f32x4v l4 = row_gran(Lk, lo, g);
          acc = mfma32(pa[2 * g], hi ? l4[1] : l4[0], acc);
          acc = mfma32(pa[2 * g + 1], hi ? l4[3] : l4[2], acc);
        }
      }
      float* st = stg + wave * 1024;
#pragma unroll
      for (int q = 0; q < 16; ++q) st[sw(acc_row(q, hi), lo)] = acc[q];
      const f32x16 u = tile_pqT(st, D, lo, hi);  // XT_ji = -C^T L_ii^-T
#pragma unroll
      for (int q = 0; q < 16; ++q) XT[(32 * j + acc_row(q, hi)) * Dp + 32 * i + lo] = -u[q];
    }
    __syncthreads();
  }
  if (tid == 0) status[0] = fail ? 0.0f : 1.0f;
}

template <int T>
hipError_t launch_chol_basis_t(const float* G, float mu, float lam, float* work, float* XT,
                               float* status, hipStream_t s) {
  const size_t lds = (size_t)(T + chol_basis_stage_tiles(T)) * 1024 * sizeof(float);
  static bool attr = false;
  if (!attr) {
    hipError_t err = hipFuncSetAttribute((const void*)chol_basis_kernel<T>,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (err != hipSuccess) return err;
    attr = true;
  }
  float* A = work;
  float* dinv = work + (size_t)32 * T * 32 * T;
  hipLaunchKernelGGL(chol_basis_kernel<T>, dim3(1), dim3(1024), lds, s, G, mu, lam, A, dinv, XT,
                     status);
  return hipGetLastError();
}

// rotate_kernel with RT row tiles per wave (64 RT rows per workgroup) and
// the X rows loaded P k-steps ahead (a register ring): at the MSD shape the
// one-step-ahead loads of rotate_kernel left it waiting on HBM (MFMA busy
// ~0.27), and each B fragment now feeds RT tiles.  Same products in the same
// k order per output element as rotate_kernel: bit-identical.
template <int DP, int RT, int P>
__global__ void __launch_bounds__(256)
    rotate_rt_kernel(const float* __restrict__ X, const QueueRec* __restrict__ rows, int64_t r0,
                     int64_t n, const bf16x8* __restrict__ Bs, float* __restrict__ Y,
                     int x_blocked, int ncb) {
  constexpr int NCT = DP / 32, NS = DP / 16;
  static_assert(NS % P == 0, "k steps a multiple of the prefetch depth");
  constexpr int CW = (DP % 128 == 0) ? 2 : 1;
  constexpr int CB = 2 * CW;
  const int tid = threadIdx.x, lane = tid & 63, lo = lane & 31, hi = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t bid = blockIdx.x, sx = bid >> 3;
  const int cbk = (int)(sx % ncb);
  const int64_t rblk = (sx / ncb) * 8 + (bid & 7);
  const int64_t base = rblk * 64 * RT;
  if (base >= n) return;
  const int R = wave & 1, cg = wave >> 1;
  const int C0 = cbk * CB + cg * CW;
  int64_t pos[RT];
  bool pv[RT];
  const float* xr[RT];
#pragma unroll
  for (int t = 0; t < RT; ++t) {
    pos[t] = base + 32 * (R * RT + t) + lo;
    pv[t] = pos[t] < n;
    const int64_t xp = pv[t] ? pos[t] : base;
    xr[t] = X + (x_blocked ? 0 : (rows ? (int64_t)rows[xp].entity : r0 + xp) * DP);
  }
  f32x16 acc[RT][CW];
#pragma unroll
  for (int t = 0; t < RT; ++t)
#pragma unroll
    for (int j = 0; j < CW; ++j) acc[t][j] = f32x16{0.f};
  auto load_a = [&](int s, float (&v)[RT][8]) __attribute__((always_inline)) {
    const int k0 = 16 * s + 8 * hi;
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      if (x_blocked) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[t][j] = pv[t] ? X[blk_v(pos[t], k0 + j, DP)] : 0.0f;
      } else {
        const float4 a = *reinterpret_cast<const float4*>(xr[t] + k0);
        const float4 b = *reinterpret_cast<const float4*>(xr[t] + k0 + 4);
        v[t][0] = a.x, v[t][1] = a.y, v[t][2] = a.z, v[t][3] = a.w;
        v[t][4] = b.x, v[t][5] = b.y, v[t][6] = b.z, v[t][7] = b.w;
      }
    }
  };
  float va[P][RT][8];  // X ring: step s in slot s % P
#pragma unroll
  for (int u = 0; u < P - 1; ++u) load_a(u, va[u]);
  bf16x8 bn[CW][3];
  auto load_b = [&](int s) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < CW; ++j) {
      const int C = C0 + j < NCT ? C0 + j : NCT - 1;
#pragma unroll
      for (int p = 0; p < 3; ++p) bn[j][p] = Bs[((int64_t)(s * NCT + C) * 3 + p) * 64 + lane];
    }
  };
  load_b(0);
  for (int s0 = 0; s0 < NS; s0 += P) {
#pragma unroll
    for (int u = 0; u < P; ++u) {
      const int s = s0 + u;
      bf16x8 bf[CW][3];
#pragma unroll
      for (int j = 0; j < CW; ++j)
#pragma unroll
        for (int p = 0; p < 3; ++p) bf[j][p] = bn[j][p];
      if (s + P - 1 < NS) load_a(s + P - 1, va[(u + P - 1) % P]);
      if (s + 1 < NS) load_b(s + 1);
#pragma unroll
      for (int t = 0; t < RT; ++t) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = pv[t] ? va[u][t][j] : 0.0f;
        bf16x8 af[3];
        split3x8(v, af);
#pragma unroll
        for (int j = 0; j < CW; ++j)
          if (C0 + j < NCT) acc[t][j] = mfma_x6(af, bf[j], acc[t][j]);
      }
    }
  }
#pragma unroll
  for (int t = 0; t < RT; ++t)
#pragma unroll
    for (int j = 0; j < CW; ++j) {
      const int C = C0 + j;
      if (C >= NCT) continue;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int64_t p = base + 32 * (R * RT + t) + acc_row(q, hi);
        if (p < n) {
          const int64_t id = rows ? (int64_t)rows[p].entity : r0 + p;
          Y[id * DP + 32 * C + lo] = acc[t][j][q];
        }
      }
    }
}

// ---- Rotation GEMM from LDS-DMA stages (Dp = 256, 512, 1024) ----
// Y = X B for B given by its split image (Q, Q^T, or G for the u^T G u
// partials), the work of rotate_rt_kernel / rotate_kernel on a larger block:
// one workgroup of 8 waves per 256 x 256 block of Y; every k16 step, X's 256
// rows (fp32, 16 KB) and B's 24 granule-KB of the block's 8 column tiles
// arrive by LDS-DMA in a 3-stage ring two steps ahead (no VGPR staging, one
// barrier per step).  Wave w takes row tiles 2 (w >> 1), +1 x column tiles
// 4 (w & 1) .. +3: each B fragment set feeds two row tiles, each split A
// fragment four column tiles.  Per block and step 40 KB of intake for 384
// MFMAs, against 8 KB per wave and 24 MFMAs in rotate_rt_kernel (whose B
// fragments every wave fetched from L2 / MALL).  X rows land row-major with
// their 16-B quads XOR-swizzled by row / 4 (set on the DMA's source address,
// conflict-free b128 reads); position-blocked X (XB: the back rotation's
// out_rot) lands k-major, one k per DMA.  Every output element sees the same
// products in the same k order as the older kernels (mfma_x6 of split3x8(X)
// and the image's pieces), and the u^T G u partials the same sums per
// 128-column half: bit-identical.
constexpr int RL_ROWS = 256, RL_STG = 3;
constexpr int RL_A = RL_ROWS * 16 * 4;  // 16 KB: 256 rows x 16 k, fp32
constexpr int RL_B = 8 * 3 * 1024;      // 24 KB: 8 column tiles x 3 pieces x 64 granules
constexpr int RL_STAGE = RL_A + RL_B;
constexpr size_t RL_LDS = (size_t)RL_STG * RL_STAGE;  // 120 KB: one workgroup per CU

template <int DP, bool XB, bool QUAD>
__global__ void __launch_bounds__(512)
    rotate_lds_kernel(const float* __restrict__ X, const QueueRec* __restrict__ rows, int64_t r0,
                      int64_t n, const bf16x8* __restrict__ Bs, float* __restrict__ Y, int ncb,
                      float* __restrict__ qpart) {
  constexpr int NCT = DP / 32, NS = DP / 16;
  static_assert(DP % 256 == 0, "256-column blocks");
  extern __shared__ __attribute__((aligned(16))) char rl_lds[];
  const int tid = threadIdx.x, lane = tid & 63, lo = lane & 31, hi = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // slot b -> XCD b % 8; the ncb column blocks of a row block on one XCD
  const int64_t bid = blockIdx.x, sx = bid >> 3;
  const int cb = (int)(sx % ncb);
  const int64_t base = ((sx / ncb) * 8 + (bid & 7)) * RL_ROWS;
  if (base >= n) return;  // the whole workgroup
  const int C0 = 8 * cb;  // the block's first column tile
  const unsigned ring = lds_addr(rl_lds);
  const char* lds = rl_lds;
  (void)tid;

  // this wave's two A DMAs per step: d = 2 wave + i
  const float* asrc[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int d = 2 * wave + i;
    if constexpr (XB) {  // k-row d of the step: positions base + 4 lane .. +3
      const int64_t npos = (n + 63) / 64 * 64;  // out_rot's allocated positions
      int64_t p4 = base + 4 * lane;
      if (p4 >= npos) p4 = 0;
      asrc[i] = X + (((p4 >> 6) * DP + d) << 6) + (p4 & 63);
    } else {  // rows 16 d + lane / 4, quad lane & 3 of the swizzled row
      const int rr = 16 * d + (lane >> 2);
      const int64_t p = base + rr < n ? base + rr : base;
      const int64_t id = rows ? (int64_t)rows[p].entity : r0 + p;
      const int lq = (lane & 3) ^ ((rr >> 2) & 3);
      asrc[i] = X + id * DP + 4 * lq;
    }
  }
  const bf16x8* bsrc = Bs + (int64_t)C0 * 3 * 64 + lane;
  auto issue = [&](int s) __attribute__((always_inline)) {
    const unsigned st = ring + (unsigned)((s % RL_STG) * RL_STAGE);
#pragma unroll
    for (int i = 0; i < 2; ++i)
      glds16(asrc[i] + (XB ? (int64_t)s * 16 * 64 : (int64_t)s * 16),
             st + (unsigned)((2 * wave + i) * 1024));
    const bf16x8* bs = bsrc + (int64_t)s * NCT * 3 * 64;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int kb = 3 * wave + i;
      glds16(bs + kb * 64, st + (unsigned)(RL_A + kb * 1024));
    }
  };
  f32x16 acc[2][4];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[t][c] = f32x16{0.f};
  issue(0);
  if (NS > 1) issue(1);
  const int rbase = 64 * (wave >> 1), cw = 4 * (wave & 1);
#pragma unroll 1
  for (int s = 0; s < NS; ++s) {
    vm_wait(s + 1 < NS ? 5 : 0);  // this wave's DMAs of stage s (not s + 1's)
    w3_barrier();                 // every wave's stage s landed; stage s - 1 read
    if (s + 2 < NS) issue(s + 2);  // into the slot of stage s - 1
    const char* st = lds + (s % RL_STG) * RL_STAGE;
    bf16x8 af[2][3];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int r = rbase + 32 * t + lo;
      float v[8];
      if constexpr (XB) {
        const float* a = reinterpret_cast<const float*>(st);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = a[(8 * hi + j) * RL_ROWS + r];
      } else {
#pragma unroll
        for (int g = 0; g < 2; ++g) {
          const f32x4v x4 = *reinterpret_cast<const f32x4v*>(
              st + r * 64 + 16 * ((2 * hi + g) ^ ((r >> 2) & 3)));
#pragma unroll
          for (int j = 0; j < 4; ++j) v[4 * g + j] = x4[j];
        }
      }
      split3x8(v, af[t]);
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      bf16x8 bf[3];
#pragma unroll
      for (int p = 0; p < 3; ++p)
        bf[p] = *reinterpret_cast<const bf16x8*>(st + RL_A + (((cw + c) * 3 + p) * 64 + lane) * 16);
#pragma unroll
      for (int t = 0; t < 2; ++t) acc[t][c] = mfma_x6(af[t], bf, acc[t][c]);
    }
  }
  if constexpr (QUAD) {
    // u^T G u partials: per 128-column half (column tiles cw .. cw + 3 =
    // rotate_kernel's block 2 cb + (w & 1)) the row dots of its two 64-column
    // wave halves, each reduced over the lanes, then added in that order
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int64_t p = base + rbase + 32 * t + acc_row(q, hi);
        float sh[2];
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          float sv = 0.0f;
          if (p < n) {  // as rotate_kernel's pair of column tiles
            const float* xp = X + (r0 + p) * DP + 32 * (C0 + cw + 2 * hh) + lo;
            sv = __builtin_fmaf(acc[t][2 * hh + 1][q], xp[32], acc[t][2 * hh][q] * xp[0]);
          }
#pragma unroll
          for (int o = 16; o > 0; o >>= 1) sv += __shfl_xor(sv, o);
          sh[hh] = sv;
        }
        if (lo == 0 && p < n) qpart[(int64_t)(2 * cb + (wave & 1)) * n + p] = sh[0] + sh[1];
      }
    }
    return;
  }
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int col = 32 * (C0 + cw + c) + lo;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int64_t p = base + rbase + 32 * t + acc_row(q, hi);
        if (p < n) {
          const int64_t id = rows ? (int64_t)rows[p].entity : r0 + p;
          Y[id * DP + col] = acc[t][c][q];
        }
      }
    }
}

// FRECSYS_ROT_LDS=0: the register-fed rotation kernels only (A/B, bitwise
// tests; read at every launch)
#ifndef FRECSYS_ROT_LDS_DEFAULT
#define FRECSYS_ROT_LDS_DEFAULT 1
#endif
bool rotate_lds_on() {
  const char* v = getenv("FRECSYS_ROT_LDS");
  return v ? atoi(v) != 0 : FRECSYS_ROT_LDS_DEFAULT != 0;
}

// the LDS kernel takes a launch of at least one workgroup per CU (256-row
// blocks x Dp / 256 column blocks: 65,536 rows at Dp = 256, 16,384 at 1024);
// smaller ones leave most CUs idle there, and the register-fed kernels
// spread them wider
constexpr int64_t kRotLdsMinBlocks = 256;

template <int DP, bool XB, bool QUAD>
hipError_t launch_rotate_lds_t(const float* X, const QueueRec* rows, int64_t r0, int64_t n,
                               const bf16x8* Bs, float* Y, float* qpart, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    hipError_t err = hipFuncSetAttribute((const void*)rotate_lds_kernel<DP, XB, QUAD>,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)RL_LDS);
    if (err != hipSuccess) return err;
    attr = true;
  }
  const int ncb = DP / 256;
  const int64_t units = (n + RL_ROWS - 1) / RL_ROWS;
  const unsigned grid = (unsigned)(((units + 7) / 8) * 8 * ncb);
  hipLaunchKernelGGL((rotate_lds_kernel<DP, XB, QUAD>), dim3(grid), dim3(512), RL_LDS, s, X, rows,
                     r0, n, Bs, Y, ncb, qpart);
  return hipGetLastError();
}

// rotate_rt_kernel with 2 row tiles per wave and P = 2 k-steps of loads in
// flight: 1.95 vs 2.20 ms (rotate_kernel) for the 471,355 x 512 rotation,
// 0.138 vs 0.141 ms for 116,677 x 256, bit-identical; RT = 1 and P = 4
// measured no better (scripts/micro/rotate_bench.cpp).  (An LDS-staged GEMM
// form -- X block split once per workgroup, B's image copied to LDS, 128 x
// 128 blocks, two stages -- measured 2.97 ms: one workgroup per CU did not
// hide the loads.)  rotate_kernel remains for the rotations that also form
// the u^T G u partials.
template <int DP, int RT>
void launch_rotate_rtp(const float* X, const QueueRec* rows, int64_t r0, int64_t n,
                       const bf16x8* Bs, float* Y, hipStream_t s, int xb, int ncb) {
  const int64_t units = (n + 64 * RT - 1) / (64 * RT);
  const unsigned grid = (unsigned)(((units + 7) / 8) * 8 * ncb);
  hipLaunchKernelGGL((rotate_rt_kernel<DP, RT, 2>), dim3(grid), dim3(256), 0, s, X, rows, r0, n,
                     Bs, Y, xb, ncb);
}

template <int DP>
hipError_t launch_rotate_t(const float* X, const QueueRec* rows, int64_t r0, int64_t n,
                           const bf16x8* Bs, float* Y, hipStream_t s, int xb,
                           float* qpart = nullptr) {
  if constexpr (DP % 256 == 0) {
    if (rotate_lds_on() && (n / RL_ROWS) * (DP / 256) >= kRotLdsMinBlocks) {
      if (qpart) return launch_rotate_lds_t<DP, false, true>(X, nullptr, r0, n, Bs, nullptr, qpart, s);
      if (xb) return launch_rotate_lds_t<DP, true, false>(X, rows, r0, n, Bs, Y, nullptr, s);
      return launch_rotate_lds_t<DP, false, false>(X, rows, r0, n, Bs, Y, nullptr, s);
    }
  }
  constexpr int CBc = (DP % 128 == 0) ? 4 : 2;
  const int ncbc = (DP / 32 + CBc - 1) / CBc;
  if (!qpart) {
    launch_rotate_rtp<DP, 2>(X, rows, r0, n, Bs, Y, s, xb, ncbc);
    return hipGetLastError();
  }
  constexpr int CB = (DP % 128 == 0) ? 4 : 2;
  const int ncb = (DP / 32 + CB - 1) / CB;
  const int64_t units = (n + 63) / 64;
  const unsigned grid = (unsigned)(((units + 7) / 8) * 8 * ncb);
  hipLaunchKernelGGL(rotate_kernel<DP>, dim3(grid), dim3(256), 0, s, X, rows, r0, n, Bs, Y, xb,
                     ncb, qpart);
  return hipGetLastError();
}

}  // namespace

bool tridiag_forms_q(int Dp) {
  // Q rows (and their split images) formed inside the reduction's launch; a
  // separate form_q_kernel launch after it measured slower
  if (Dp < 64 || Dp % 32) return false;
  return wide_dim(Dp) ? wide_tridiag_tagged() : Dp <= 256;
}

size_t tridiag_work_floats(int Dp) {
  return wide_dim(Dp) ? wide_tridiag_work_floats(Dp) : (size_t)2 * Dp * Dp + 2 * (size_t)Dp;
}

hipError_t launch_tridiag(const float* G, int Dp, float* tdiag, float* toff, float* Vh,
                          float* tau, hipStream_t s, float* work, float* Q, void* img_q,
                          void* img_qt, unsigned* tcount) {
  if (Q && (!tridiag_forms_q(Dp) || !work)) return hipErrorInvalidValue;
  if ((img_q != nullptr) != (img_qt != nullptr) || (img_q && !Q)) return hipErrorInvalidValue;
  if (wide_dim(Dp)) return launch_wide_tridiag(G, Dp, tdiag, toff, Vh, tau, work, s, Q, img_q, img_qt, tcount);
  if (Dp < 4 || Dp > 256) return hipErrorInvalidValue;
  unsigned long long* vt = Q ? reinterpret_cast<unsigned long long*>(work) : nullptr;
  unsigned long long* tt = Q ? vt + (size_t)Dp * Dp : nullptr;
  if (Q) {
    hipError_t e = hipMemsetAsync(vt, 0, ((size_t)Dp * Dp + Dp) * sizeof(unsigned long long), s);
    if (e != hipSuccess) return e;
  }
  const unsigned grid = 1 + (Q ? (unsigned)(Dp / 32) : 0u);
  hipLaunchKernelGGL(tridiag_kernel, dim3(grid), dim3(512), 0, s, G, Dp, tdiag, toff, Vh, tau, Q,
                     reinterpret_cast<bf16x8*>(img_q), reinterpret_cast<bf16x8*>(img_qt), vt, tt,
                     tcount);
  return hipGetLastError();
}

hipError_t launch_form_q(const float* Vh, const float* tau, int Dp, float* Q, hipStream_t s,
                         void* img_q, void* img_qt) {
  if (Dp < 4 || Dp > 1024) return hipErrorInvalidValue;
  if ((img_q != nullptr) != (img_qt != nullptr) || (img_q && (Dp < 64 || Dp % 32)))
    return hipErrorInvalidValue;
  const dim3 grid((unsigned)((Dp + 7) / 8));
  bf16x8* a = reinterpret_cast<bf16x8*>(img_q);
  bf16x8* b = reinterpret_cast<bf16x8*>(img_qt);
  if (Dp <= 256)
    hipLaunchKernelGGL(form_q_kernel<4>, grid, dim3(512), 0, s, Vh, tau, Dp, Q, a, b);
  else if (Dp <= 512)
    hipLaunchKernelGGL(form_q_kernel<8>, grid, dim3(512), 0, s, Vh, tau, Dp, Q, a, b);
  else
    hipLaunchKernelGGL(form_q_kernel<16>, grid, dim3(512), 0, s, Vh, tau, Dp, Q, a, b);
  return hipGetLastError();
}

size_t basis_split_bytes(int Dp) { return (size_t)Dp * Dp * 3 * sizeof(__bf16); }

size_t chol_basis_work_floats(int Dp) { return (size_t)Dp * Dp + (size_t)(Dp / 32) * 1024; }

hipError_t launch_chol_basis(const float* G, int Dp, float mu, float lam, float* work, float* XT,
                             float* status, hipStream_t s) {
  switch (Dp) {
    case 64: return launch_chol_basis_t<2>(G, mu, lam, work, XT, status, s);
    case 96: return launch_chol_basis_t<3>(G, mu, lam, work, XT, status, s);
    case 128: return launch_chol_basis_t<4>(G, mu, lam, work, XT, status, s);
    case 160: return launch_chol_basis_t<5>(G, mu, lam, work, XT, status, s);
    case 192: return launch_chol_basis_t<6>(G, mu, lam, work, XT, status, s);
    case 224: return launch_chol_basis_t<7>(G, mu, lam, work, XT, status, s);
    case 256: return launch_chol_basis_t<8>(G, mu, lam, work, XT, status, s);
    case 512: return launch_chol_basis_t<16>(G, mu, lam, work, XT, status, s);
    case 1024: return launch_chol_basis_t<32>(G, mu, lam, work, XT, status, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_split_basis(const float* Q, int Dp, int trans, void* out, hipStream_t s) {
  if (Dp < 64 || Dp % 32 != 0) return hipErrorInvalidValue;
  const int64_t n = (int64_t)(Dp / 16) * (Dp / 32) * 64;
  hipLaunchKernelGGL(split_basis_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, Q, Dp,
                     trans, reinterpret_cast<bf16x8*>(out));
  return hipGetLastError();
}

hipError_t launch_rotate(const float* X, const QueueRec* rows, int64_t r0, int64_t n,
                         const void* bsplit, float* Y, int Dp, hipStream_t s, int x_blocked) {
  if (n <= 0) return hipSuccess;
  const bf16x8* B = reinterpret_cast<const bf16x8*>(bsplit);
  switch (Dp) {
    case 64: return launch_rotate_t<64>(X, rows, r0, n, B, Y, s, x_blocked);
    case 96: return launch_rotate_t<96>(X, rows, r0, n, B, Y, s, x_blocked);
    case 128: return launch_rotate_t<128>(X, rows, r0, n, B, Y, s, x_blocked);
    case 160: return launch_rotate_t<160>(X, rows, r0, n, B, Y, s, x_blocked);
    case 192: return launch_rotate_t<192>(X, rows, r0, n, B, Y, s, x_blocked);
    case 224: return launch_rotate_t<224>(X, rows, r0, n, B, Y, s, x_blocked);
    case 256: return launch_rotate_t<256>(X, rows, r0, n, B, Y, s, x_blocked);
    case 512: return launch_rotate_t<512>(X, rows, r0, n, B, Y, s, x_blocked);
    case 1024: return launch_rotate_t<1024>(X, rows, r0, n, B, Y, s, x_blocked);
    default: return hipErrorInvalidValue;
  }
}

namespace {
__global__ void __launch_bounds__(256) mark_rows_kernel(const QueueRec* __restrict__ order,
                                                        const int32_t* __restrict__ col,
                                                        uint8_t* __restrict__ mark) {
  const QueueRec r = order[blockIdx.x];
  for (int64_t k = threadIdx.x; k < r.h; k += 256) mark[col[r.p0 + k]] = 1;
}
}  // namespace

hipError_t launch_mark_rows(const QueueRec* order, int64_t n, const int32_t* col, uint8_t* mark,
                            hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(mark_rows_kernel, dim3((unsigned)n), dim3(256), 0, s, order, col, mark);
  return hipGetLastError();
}

hipError_t launch_rotate_quad(const float* X, int64_t r0, int64_t n, const void* bsplit,
                              float* qpart, int Dp, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const bf16x8* B = reinterpret_cast<const bf16x8*>(bsplit);
  switch (Dp) {
    case 64: return launch_rotate_t<64>(X, nullptr, r0, n, B, nullptr, s, 0, qpart);
    case 96: return launch_rotate_t<96>(X, nullptr, r0, n, B, nullptr, s, 0, qpart);
    case 128: return launch_rotate_t<128>(X, nullptr, r0, n, B, nullptr, s, 0, qpart);
    case 160: return launch_rotate_t<160>(X, nullptr, r0, n, B, nullptr, s, 0, qpart);
    case 192: return launch_rotate_t<192>(X, nullptr, r0, n, B, nullptr, s, 0, qpart);
    case 224: return launch_rotate_t<224>(X, nullptr, r0, n, B, nullptr, s, 0, qpart);
    case 256: return launch_rotate_t<256>(X, nullptr, r0, n, B, nullptr, s, 0, qpart);
    case 512: return launch_rotate_t<512>(X, nullptr, r0, n, B, nullptr, s, 0, qpart);
    case 1024: return launch_rotate_t<1024>(X, nullptr, r0, n, B, nullptr, s, 0, qpart);
    default: return hipErrorInvalidValue;
  }
}

int rotate_quad_parts(int Dp) {
  const int cb = (Dp % 128 == 0) ? 4 : 2;  // rotate_kernel's column tiles per workgroup
  return (Dp / 32 + cb - 1) / cb;
}

}  // namespace frecsys_hip
