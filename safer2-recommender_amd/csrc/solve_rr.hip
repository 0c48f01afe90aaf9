// solve_rr.hip -- d-space solve at Dp = 256 with A register-resident, two
// entities per CU.
//
// Replaces, like solve_tiled_kernel<8, false, true> (solve.hip), the
// Eigen-backed Project / ProjectU / ProjectV (ials.h:88-144,
// safer2.h:104-221) of one entity whose history is too long for the
// history-space path.  The tiled kernel keeps the 36 lower 32x32 tiles of A
// in LDS (155 KB) for its dataflow Cholesky, so a CU holds one entity and its
// MFMA pipes idle while the diagonal-factor chain (half of an entity's time)
// runs.  Here the tiles never leave the registers of the four waves that
// accumulate them:
//
//   * wave w owns block rows rA = 7 - w and rB = w of the lower triangle (9
//     tiles each: rows 7+0, 6+1, 5+2, 4+3): off-diagonal tile (rA, J) in
//     accumulator slot J, (rB, J) in slot 6 - J, the diagonal tiles (rA, rA)
//     and (rB, rB) in slots 7 and 8 -- every slot index is static once the
//     column loops are unrolled, and after the SYRK the two diagonal tiles
//     move to their LDS buffers (the factor reads them there), so the
//     Cholesky holds 7 tiles (112 VGPRs) beside the inlined diagonal factor;
//   * a tile is held TRANSPOSED in the 32x32 MFMA accumulator layout: lane
//     (lo, hi), register q = element (lo, acc_row(q, hi)), i.e. each lane
//     holds 16 entries of row lo.  That is exactly the operand layout of
//     v_mfma_f32_32x32x2_f32 with the k index permuted by acc_row, so
//     the SYRK (operands swapped), the panel TRSM L_Ip^T = L_pp^-1 A_Ip^T and
//     the trailing update A_IJ -= L_Ip L_Jp^T (as (L_Jp L_Ip^T)^T) all read
//     and write register tiles with no layout change;
//   * LDS holds only the gather stage during the SYRK, then the eight
//     diagonal inverses L_pp^-1 (chol.h diag_factor_inv_blk) and one panel
//     column of L_Ip rows: 66 KB, so two workgroups share a CU and one's SYRK
//     fills the MFMA pipes while the other's factor chain runs.
//
// Per step p: (owner of (p, p) factored it at the end of step p-1's update
// phase) TRSM of column p by the owners of (I, p), b_I -= L_Ip y_p alongside,
// panel rows to LDS; barrier; trailing updates, the owner of (p+1, p+1)
// updating and factoring that tile first (lookahead); barrier.  Backward
// x = L^-T y: the wave owning row q forms x_q = L_qq^-T r_q and folds
// L_qp^T x_q into r_p (p < q) through a per-wave LDS transpose; one barrier
// per q.
//
// SYRK: chunks of 16 history rows, one thread per column gathers its 16
// values, scales and splits them into three bf16 pieces (common.h split3,
// fp32-accurate products as in solve.hip) and writes the k-major granules the
// bf16 MFMA reads; two chunks of loads in flight, ids and row weights in a
// 4-slot ring three chunks ahead.
//
// Kinds: iALS, WEIGHTED_U, WEIGHTED_V (the CVaR-MF gradient kinds keep the
// tiled kernel).  Long histories start from the split kernel's slabs
// (solve.hip PARTIAL, raw accumulator layout, read transposed here).
// Opt-in (FRECSYS_RR=1): measured slower than the tiled kernel, see DESIGN 3.1.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "chol.h"
#include "common.h"
#include "kernels.h"

namespace frecsys_hip {

namespace {

constexpr int kT = 8, kDp = 256, kNTHR = 256, kR = 16, kRing = 4;
constexpr int kNT = kT * (kT + 1) / 2;
constexpr int kGran = 6 * kDp;            // 16-B granules per stage buffer: 3 pieces x 2 k-halves x Dp
constexpr int kStage = 2 * 4 * kGran;     // floats, two buffers
constexpr int kLD = 36;                   // padded row stride of the LDS tiles below
constexpr int kTileF = 32 * kLD;
constexpr int kDiag = 0;                  // [8] L_pp^-1, rows padded
constexpr int kPanel = 8 * kTileF;        // [7] rows of L_Ip, slot I-1
constexpr int kChol = kPanel + 7 * kTileF;
constexpr int kRegion0 = kStage > kChol ? kStage : kChol;
constexpr int kOffB = kRegion0;           // rhs, then y, then r
constexpr int kOffX = kOffB + kDp;        // x
constexpr int kOffSA = kOffX + kDp;       // ring: A-scale per row
constexpr int kOffBW = kOffSA + kRing * kR;
constexpr int kOffID = kOffBW + kRing * kR;
constexpr int kOffFlag = kOffID + kRing * kR;
constexpr int kTotal = kOffFlag + 4;
constexpr size_t kBytes = (size_t)kTotal * 4;
static_assert(kBytes <= 81920, "two workgroups per CU");

__device__ __forceinline__ int gran(int p, int hh, int c) { return (p * 2 + hh) * kDp + c; }

__device__ __forceinline__ int64_t vpos(int64_t k, int64_t h) {
  return k < h ? k : (h - 128 + (k - h));
}

// LDS tiles (diagonal inverses, panel, backward scratch): row-major with
// rows padded to 36 floats.  A lane's register-order row (columns
// acc_row(4k..4k+3, hi) = 8k + 4hi + 0..3) is four 16-B accesses at constant
// offsets from one base, a column read (fixed r, lanes over c) is
// contiguous, and neither needs per-element address registers (an XOR
// swizzle would: the hoisted addresses alone pushed the kernel past 256
// VGPRs).
typedef float f32x4 __attribute__((ext_vector_type(4)));

// Register tile (transposed layout) -> rows of an LDS tile.
__device__ __forceinline__ void put_rows(float* tile, const f32x16& t, int lo, int hi) {
  float* row = tile + lo * kLD + 4 * hi;
#pragma unroll
  for (int k = 0; k < 4; ++k)
    *reinterpret_cast<f32x4*>(row + 8 * k) = f32x4{t[4 * k], t[4 * k + 1], t[4 * k + 2], t[4 * k + 3]};
}
// Row lo of an LDS tile in register order (k = acc_row(s, hi)).
__device__ __forceinline__ f32x16 get_rows(const float* tile, int lo, int hi) {
  const float* row = tile + lo * kLD + 4 * hi;
  f32x16 t;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(row + 8 * k);
    t[4 * k] = v[0];
    t[4 * k + 1] = v[1];
    t[4 * k + 2] = v[2];
    t[4 * k + 3] = v[3];
  }
  return t;
}
// sum_m M(lo, m) v[m] (TR: M(m, lo)); lane half hi takes m in [16hi, 16hi+16),
// both halves get the total.
template <bool TR>
__device__ __forceinline__ float gemv_pad(const float* M, const float* v, int lo, int hi) {
  float s0 = 0.0f, s1 = 0.0f;
#pragma unroll
  for (int i = 0; i < 16; i += 2) {
    const int m = 16 * hi + i;
    s0 += M[TR ? m * kLD + lo : lo * kLD + m] * v[m];
    s1 += M[TR ? (m + 1) * kLD + lo : lo * kLD + m + 1] * v[m + 1];
  }
  const float s = s0 + s1;
  return s + __shfl_xor(s, 32);
}

// c + A B over the 32 permuted k: a[s] = A(lo, k), b[s] = B^T(lo, k) with
// k = acc_row(s, hi) -- both operands in register order.
__device__ __forceinline__ f32x16 mfma_rows(const f32x16& a, const f32x16& b, f32x16 c) {
#pragma unroll
  for (int s = 0; s < 16; ++s) c = mfma32(a[s], b[s], c);
  return c;
}

template <bool OFF64>
__global__ void __launch_bounds__(kNTHR) __attribute__((amdgpu_waves_per_eu(2, 2)))
solve_rr_kernel(SolveArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* stage = smem;
  float* diag = smem + kDiag;
  float* panel = smem + kPanel;
  float* bvec = smem + kOffB;
  float* xvec = smem + kOffX;
  float* ring_sa = smem + kOffSA;
  float* ring_bw = smem + kOffBW;
  int* ring_id = reinterpret_cast<int*>(smem + kOffID);
  int* flag = reinterpret_cast<int*>(smem + kOffFlag);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lo = lane & 31, hi = lane >> 5;
  const int rA = 7 - wave, rB = wave;  // my block rows
  const int kind = a.kind;
  const bool vk = is_v_kind(kind);

  const int qpos = blockIdx.x;
  int slab0 = 0, nslab = 0;
  if (qpos < a.n_split) {
    const int2 sp = a.split[qpos];
    slab0 = sp.x;
    nslab = sp.y;
  }
  const QueueRec rec = a.order[qpos];
  const int64_t e = rec.entity;
  const int64_t h = rec.h;
  const int64_t p0 = rec.p0;
  if (h == 0) return;
  int64_t extra = 0;
  if (vk && a.quirk && h > 128 && (h % 128) != 0) extra = 128 - (h % 128);
  const int64_t ntot = h + extra;
  const int64_t k1 = nslab > 0 ? 0 : ntot;  // split: the slabs hold the rows
  const int nchunks = (int)((k1 + kR - 1) / kR);

  auto ring_id_load = [&](int c) {
    const int64_t k = (int64_t)c * kR + tid;
    return k < k1 ? a.col[p0 + vpos(k, h)] : -1;
  };
  auto ring_weights = [&](int c, int id, float& sa, float& bw) {
    const int64_t k = (int64_t)c * kR + tid;
    sa = 0.0f;
    bw = 0.0f;
    if (k < k1) {
      if (vk) {
        const float nu = a.other_weight[id];
        sa = sqrtf(nu);
        bw = (k < h && sa > 0.0f) ? nu / sa : 0.0f;
      } else {
        sa = 1.0f;
        bw = 1.0f;
      }
    }
  };
  auto ring_store = [&](int c, int id, float sa, float bw) {
    const int s = (c % kRing) * kR + tid;
    ring_id[s] = id;
    ring_sa[s] = sa;
    ring_bw[s] = bw;
  };
  // thread = column tid of the chunk's 16 rows (branch-free: rows past the
  // history load row 0 and are zeroed by their scale)
  auto load_rows = [&](int c, float (&xr)[16]) {
    const int4* ids = reinterpret_cast<const int4*>(ring_id + (c % kRing) * kR);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int4 id4 = ids[q];
      const int id[4] = {id4.x, id4.y, id4.z, id4.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if constexpr (OFF64)
          xr[4 * q + j] = a.X[(int64_t)max(id[j], 0) * kDp + tid];
        else
          xr[4 * q + j] = a.X[(unsigned)max(id[j], 0) * (unsigned)kDp + (unsigned)tid];
      }
    }
  };
  float bpart = 0.0f;
  // scale chunk c's values in place (rhs part alongside)
  auto scale_rows = [&](int c, float (&xr)[16], bool live) {
    const int base = (c % kRing) * kR;
    float bsum = 0.0f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 s4 = reinterpret_cast<const float4*>(ring_sa + base)[q];
      const float4 w4 = reinterpret_cast<const float4*>(ring_bw + base)[q];
      const float sa[4] = {s4.x, s4.y, s4.z, s4.w}, bw[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        xr[4 * q + j] *= sa[j];
        bsum += bw[j] * xr[4 * q + j];
      }
    }
    bpart = live ? bpart + bsum : bpart;
  };
  // pieces of rows 8hh .. 8hh+7 -> the three granules of (hh, column tid)
  auto split_write = [&](int buf, const float (&xs)[16], int hh) {
    bf16x8 f[3];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      __bf16 ph, pm, pl;
      split3(xs[8 * hh + j], ph, pm, pl);
      f[0][j] = ph;
      f[1][j] = pm;
      f[2][j] = pl;
    }
    bf16x8* st = reinterpret_cast<bf16x8*>(stage) + buf * kGran;
#pragma unroll
    for (int p = 0; p < 3; ++p) st[gran(p, hh, tid)] = f[p];
  };

  if (tid == 0) flag[0] = 0;
  // diagnostics (FRECSYS_DUAL_PROF): wave 0's cycles per phase, summed
  unsigned long long t_prev = a.prof ? clock64() : 0;
  auto mark = [&](int ph) {
    if (a.prof && tid == 0) {
      const unsigned long long t = clock64();
      atomicAdd(a.prof + ph, t - t_prev);
      t_prev = t;
    }
  };
  if (tid < kR) {  // ring prologue
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      if (c < nchunks) {
        const int id = ring_id_load(c);
        float sa, bw;
        ring_weights(c, id, sa, bw);
        ring_store(c, id, sa, bw);
      }
    }
  }

  // ---- accumulators: slot s < rA tile (rA, s), rA <= s < 7 tile (rB, 6 - s),
  // slot 7 (rA, rA), slot 8 (rB, rB) ----
  const float hf = (float)h;
  const float omega = (is_u_kind(kind) && a.entity_weight) ? a.entity_weight[e] : 1.0f;
  const float lam = entity_lambda(kind, a.reg, a.reg_exp, a.w, a.alpha, h, a.n_other,
                                  a.entity_reg, e, a.lambda_is_reg);
  const float gscale = kind == KIND_IALS ? a.w : (is_u_kind(kind) ? hf * a.w : a.w);
  const float lam_d = kind == KIND_IALS ? lam : 0.0f;
  f32x16 acc[9];
  const size_t slab_floats = (size_t)kNT * 1024 + kDp;
  // slab element (lo, acc_row(q, hi)) of tile t: register q' / lane' of the
  // raw (untransposed) accumulator layout
  const int shi = (lo >> 2) & 1, sq = (lo & 3) + 4 * (lo >> 3);
#pragma unroll
  for (int s = 0; s < 9; ++s) {
    const int I = s < 7 ? (s < rA ? rA : rB) : (s == 7 ? rA : rB);
    const int J = s < 7 ? (s < rA ? s : 6 - s) : I;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int r = acc_row(q, hi);
      // element (32I + lo, 32J + r) = G(32J + r, 32I + lo): lanes coalesced
      acc[s][q] = gscale * a.G[(32 * J + r) * kDp + 32 * I + lo] +
                  ((I == J && lo == r) ? lam_d : 0.0f);
    }
    for (int si = 0; si < nslab; ++si) {
      const float* sl = a.slabs + (size_t)(slab0 + si) * slab_floats + tidx(I, J) * 1024;
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[s][q] += sl[sq * 64 + acc_row(q, hi) + 32 * shi];
    }
  }
  float bacc = 0.0f;
  for (int si = 0; si < nslab; ++si)
    bacc += a.slabs[(size_t)(slab0 + si) * slab_floats + kNT * 1024 + tid];
  lds_barrier();
  mark(0);

  // ---- SYRK: S^T tiles by split-bf16 MFMA ----
  // Step c: chunk c+1 (loaded during step c-1) is scaled, split and written
  // to stage buffer (c+1)&1, chunk c+2's row loads are issued into the same
  // registers, then chunk c's MFMAs run from buffer c&1 -- the loads stay in
  // flight through them (16 VGPRs beside the 144 of the tiles); the ring is
  // filled three chunks ahead.
  {
    float xr[16];
    if (nchunks > 0) {
      load_rows(0, xr);
      scale_rows(0, xr, true);
      split_write(0, xr, 0);
      split_write(0, xr, 1);
    }
    if (nchunks > 1) load_rows(1, xr);
    lds_barrier();
    for (int c = 0; c < nchunks; ++c) {
      const int buf = c & 1;
      const bool ring_more = (tid < kR) && (c + 3 < nchunks);
      int nid = -1;
      if (ring_more) nid = ring_id_load(c + 3);
      if (c + 1 < nchunks) {
        scale_rows(c + 1, xr, true);
        split_write(buf ^ 1, xr, 0);
        split_write(buf ^ 1, xr, 1);
      }
      if (c + 2 < nchunks) load_rows(c + 2, xr);
      const bf16x8* st = reinterpret_cast<const bf16x8*>(stage) + buf * kGran;
      auto frag = [&](int blk, bf16x8 (&f)[3]) {
#pragma unroll
        for (int p = 0; p < 3; ++p) f[p] = st[gran(p, hi, 32 * blk + lo)];
      };
      bf16x8 fa[3];
      frag(rA, fa);
#pragma unroll
      for (int J = 0; J < 8; ++J) {
        if (J <= 4 || J <= rA) {
          bf16x8 fj[3];
          frag(J, fj);
          if (J < 4 || J < rA) acc[J] = mfma_x6s(fj, fa, acc[J]);
          else acc[7] = mfma_x6s(fj, fa, acc[7]);  // J == rA
          if (J == 0 || (J <= 3 && J <= rB)) {
            bf16x8 fb[3];
            frag(rB, fb);
            if (J < 3 && J < rB) acc[6 - J] = mfma_x6s(fj, fb, acc[6 - J]);
            else acc[8] = mfma_x6s(fj, fb, acc[8]);  // J == rB
          }
        }
      }
      if (ring_more) {
        float nsa, nbw;
        ring_weights(c + 3, nid, nsa, nbw);
        ring_store(c + 3, nid, nsa, nbw);
      }
      lds_barrier();
    }
  }

  mark(1);
  // ---- epilogue: kind scaling, rhs ----
  const float us = omega / hf;
  if (kind != KIND_IALS) {
    const bool uk = is_u_kind(kind);
#pragma unroll
    for (int s = 0; s < 9; ++s) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const bool dg = s >= 7 && lo == acc_row(q, hi);
        float v = acc[s][q];
        v = uk ? v * us + (dg ? lam : 0.0f) : v + (dg ? lam : 0.0f);
        acc[s][q] = v;
      }
    }
  }
  {
    float b = bacc + bpart;
    if (is_u_kind(kind)) b *= us;
    bvec[tid] = b;
  }
  lds_barrier();  // stage dead: the diagonal / panel region is free
  put_rows(diag + rA * kTileF, acc[7], lo, hi);  // the diagonal tiles live in LDS from here
  put_rows(diag + rB * kTileF, acc[8], lo, hi);

  // ---- blocked Cholesky on the register tiles ----
  // diag[p] -> L_pp^-1 in place, then y_p = L_pp^-1 b_p (b_p final).  One
  // inlined copy (a call would clobber half of the VGPRs holding the tiles).
  auto factor = [&](int p) {
    float* dp = diag + p * kTileF;
    wave_lds_sync();
    if (!diag_factor_inv_blk_inl<kLD>((lds_float*)dp, lane) && lane == 0) flag[0] = 1;
    wave_lds_sync();
    const float y = gemv_pad<false>(dp, bvec + 32 * p, lo, hi);
    wave_lds_sync();
    if (hi == 0) bvec[32 * p + lo] = y;
  };
  // TRSM of tile (I, p) in place (register order), rows to the panel,
  // b_I -= L_Ip y_p
  // (A_Ip goes through its panel slot first, so that the product can land
  // in the tile's own registers: an MFMA result may not overlap its B
  // operand, and a fresh 16-register result per TRSM spilled the tiles)
  auto trsm = [&](int I, int p, f32x16& t) {
    float* ps = panel + (I - 1) * kTileF;
    put_rows(ps, t, lo, hi);
    wave_lds_sync();
    const f32x16 ai = get_rows(ps, lo, hi);
    const f32x16 li = get_rows(diag + p * kTileF, lo, hi);
    t = mfma_rows(li, ai, f32x16{0.f});
    wave_lds_sync();
    put_rows(ps, t, lo, hi);
    const float* y = bvec + 32 * p + 4 * hi;
    float d = 0.0f;
#pragma unroll
    for (int s = 0; s < 16; ++s) d += t[s] * y[(s & 3) + 8 * (s >> 2)];
    d += __shfl_xor(d, 32);
    if (hi == 0) bvec[32 * I + lo] -= d;
  };
  // A_IJ -= L_Ip L_Jp^T with L_Ip my register tile lip and L_Jp from the
  // panel (J != I), or A_II -= L_Ip L_Ip^T
  auto update = [&](int J, const f32x16& lip, f32x16& t) {
    f32x16 nj = get_rows(panel + (J - 1) * kTileF, lo, hi);
#pragma unroll
    for (int s = 0; s < 16; ++s) nj[s] = -nj[s];
    t = mfma_rows(nj, lip, t);
  };
  auto update_diag = [&](int I, const f32x16& lip) {  // A_II (LDS) -= L_Ip L_Ip^T
    f32x16 t = get_rows(diag + I * kTileF, lo, hi);
#pragma unroll
    for (int s = 0; s < 16; ++s) t = mfma32(-lip[s], lip[s], t);
    put_rows(diag + I * kTileF, t, lo, hi);
  };
  // Step bodies with static slot indices (P static), dispatched per step.
  auto trsm_col = [&](auto pc) {
    constexpr int P = decltype(pc)::value;
    if (P < rA) trsm(rA, P, acc[P]);
    if constexpr (P < 3)
      if (P < rB) trsm(rB, P, acc[6 - P]);
  };
  auto lookahead = [&](auto pc) {  // owner of (P+1, P+1): its last update
    constexpr int P = decltype(pc)::value;
    if constexpr (P + 1 < kT) {
      if (P + 1 == rA) update_diag(rA, acc[P]);
      if constexpr (P + 1 <= 3)
        if (P + 1 == rB) update_diag(rB, acc[6 - P]);
    }
  };
  auto rest = [&](auto pc) {  // the other trailing updates of step P
    constexpr int P = decltype(pc)::value;
#pragma unroll
    for (int J = P + 1; J < kT; ++J) {
      if (J < rA) update(J, acc[P], acc[J]);
      else if (J == rA && J != P + 1) update_diag(rA, acc[P]);
      if (J <= 3 && P < 2) {
        if (P < rB) {
          if (J < rB) update(J, acc[6 - P], acc[6 - J]);
          else if (J == rB && J != P + 1) update_diag(rB, acc[6 - P]);
        }
      }
    }
  };
  auto dispatch = [&](int p, auto fn) {
    switch (p) {
      case 0: fn(std::integral_constant<int, 0>{}); break;
      case 1: fn(std::integral_constant<int, 1>{}); break;
      case 2: fn(std::integral_constant<int, 2>{}); break;
      case 3: fn(std::integral_constant<int, 3>{}); break;
      case 4: fn(std::integral_constant<int, 4>{}); break;
      case 5: fn(std::integral_constant<int, 5>{}); break;
      case 6: fn(std::integral_constant<int, 6>{}); break;
      default: fn(std::integral_constant<int, 7>{}); break;
    }
  };

  mark(2);
  if (rB == 0) factor(0);  // tile (0, 0)
  lds_barrier();
#pragma unroll 1
  for (int p = 0; p < kT; ++p) {
    dispatch(p, trsm_col);
    lds_barrier();
    if (p == kT - 1) break;
    dispatch(p, lookahead);
    if (p + 1 == rA || p + 1 == rB) factor(p + 1);
    dispatch(p, rest);
    lds_barrier();
  }

  mark(3);
  // ---- backward: x = L^-T y; bvec holds y, becoming r ----
  float* scr = panel + wave * kTileF;
  auto fold = [&](int p, int q, const f32x16& lqp) {  // r_p -= L_qp^T x_q
    put_rows(scr, lqp, lo, hi);
    wave_lds_sync();
    const float d = gemv_pad<true>(scr, xvec + 32 * q, lo, hi);
    wave_lds_sync();
    if (hi == 0) bvec[32 * p + lo] -= d;
  };
#pragma unroll
  for (int q = kT - 1; q >= 0; --q) {
    if (q == rA || q == rB) {
      const float x = gemv_pad<true>(diag + q * kTileF, bvec + 32 * q, lo, hi);
      if (hi == 0) xvec[32 * q + lo] = x;
      wave_lds_sync();
#pragma unroll
      for (int p = q - 1; p >= 0; --p) {
        if (q == rA) fold(p, q, acc[p]);
        else if (q <= 3) fold(p, q, acc[6 - p]);
      }
    }
    lds_barrier();
  }
  mark(5);
  a.out[e * kDp + tid] = xvec[tid];
  if (tid == 0 && flag[0]) atomicMin(a.fail, (unsigned long long)(e + 1));
  if (a.prof && tid == 0) {
    atomicAdd(a.prof + 4, 1ull);
    atomicAdd(a.prof + 8, (unsigned long long)ntot);
  }
}

// FRECSYS_RR_LDS_KB: dynamic LDS per workgroup (>= the kernel's own), e.g.
// 96 to hold one workgroup per CU (experiments only).
size_t rr_lds_bytes() {
  static const size_t b = [] {
    const char* v = getenv("FRECSYS_RR_LDS_KB");
    const size_t want = v ? (size_t)atoi(v) * 1024 : 0;
    return want > kBytes ? (want > 163840 ? (size_t)163840 : want) : kBytes;
  }();
  return b;
}

template <bool OFF64>
hipError_t launch_rr_o(const SolveArgs& a, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    hipError_t err = hipFuncSetAttribute((const void*)solve_rr_kernel<OFF64>,
                                         hipFuncAttributeMaxDynamicSharedMemorySize,
                                         (int)rr_lds_bytes());
    if (err != hipSuccess) return err;
    attr = true;
  }
  hipLaunchKernelGGL((solve_rr_kernel<OFF64>), dim3((unsigned)a.n_rows), dim3(kNTHR),
                     rr_lds_bytes(), s, a);
  return hipGetLastError();
}

}  // namespace

bool solve_rr_enabled(int Dp, int kind) {
  // opt-in, read at every launch: measured slower than the tiled kernel
  const char* v = getenv("FRECSYS_RR");
  const bool on = v && atoi(v) != 0;
  return on && Dp == kDp && !is_grad_kind(kind) && syrk_split_bf16();
}

hipError_t launch_solve_rr(const SolveArgs& a, hipStream_t s) {
  if (a.n_rows <= 0) return hipSuccess;
  if (gather_off64(a.n_other, kDp)) return launch_rr_o<true>(a, s);
  return launch_rr_o<false>(a, s);
}

}  // namespace frecsys_hip
