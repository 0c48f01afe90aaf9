// solve.hip -- per-entity normal-equation assembly + SPD solve on gfx950.
//
// Replaces the Eigen-backed Project / ProjectU / ProjectV / ProjectU_eval
// (ials.h:88-144, safer2.h:104-221, erm_mf.h:91-210, cvar_mf.h:88-229) and
// the std::thread work queue of the Step* drivers (ials.h:317-365,
// safer2.h:437-555): one workgroup per entity, the whole entity on one CU.
//
// Tiled kernel (padded dim Dp = 32*T, T = 1..8):
//   1. gather: the entity's history rows of X (row-major, ld Dp) are pulled
//      in chunks of R rows by coalesced float4 loads into an LDS staging
//      ring (double buffered; the history ids + per-row scales run one chunk
//      further ahead in a 4-slot ring);
//   2. assembly: the lower T(T+1)/2 32x32 tiles of S = X_h^T D X_h are
//      accumulated in registers by v_mfma_f32_32x32x2_f32 (exact fp32), each
//      wave owning a fixed subset of tiles; the epilogue folds in w*G,
//      lambda and the per-kind scaling and writes A into LDS (XOR-swizzled
//      tiles, aliasing the staging ring that is dead by then);
//   3. solve: right-looking blocked Cholesky on the LDS tiles -- per panel a
//      32x32 diagonal factor that also yields L_pp^-1 (one wave, see
//      diag_factor_inv), the panel TRSM as MFMA products with L_pp^-1 (the
//      right-hand side rides along: y_p = L_pp^-1 b_p), MFMA trailing
//      updates; then x = L^-T y with one GEMV wave per tile and the stored
//      inverses.  Workgroup b takes entity order[b]: the rank's entities in
//      decreasing-history order, so the dispatcher starts the longest first
//      (LPT scheduling of a skewed workload).
//   CVaR-MF kinds skip 3 and take one gradient step with the full matrix
//   whose strict upper triangle lacks the observed term (cvar_mf.h:133).
//
// Small kernel (Dp = 8, 16): one wave per entity, VALU assembly, the dense
// solve by one lane (the reference's own tests run at dim 8).
#include <hip/hip_runtime.h>

#include <type_traits>

#include "chol.h"
#include "common.h"
#include "kernels.h"

// Super-block tile ownership of the split-bf16 SYRK at Dp = 256 (kSbPat):
// 2 in the split (PARTIAL) and the solve kernels, 1 (default) in the split
// kernel only, 0 nowhere (tile t to wave t % 8).  All three are bit-identical
// (scripts/sb_ab_cmd.sh).  Measured (ML-20M d = 256, serialised): split
// kernel 1.059 vs 1.086 ms/epoch; in the solve kernel the five ownership
// copies of the SYRK loop spill beside the Cholesky's registers (2.72 vs 2.21
// ms), so it keeps t % 8 there.
constexpr int kSyrkSB = 1;

namespace frecsys_hip {

namespace {

constexpr int kRing = 4;

// BF = true: the SYRK runs on the bf16 matrix cores with 3-piece split
// operands (common.h mfma_x6, fp32-accurate).  Chunks of R = 32 rows, staged
// as pieces in a k-major image: 16-B granule (piece p, row group g of 16,
// k-half hh, column c) holds rows 16g + 8hh .. +7 of column c -- exactly the
// bf16x8 fragment lane (c & 31, hh) of v_mfma_f32_32x32x16_bf16 reads; lanes
// read consecutive granules (no bank conflicts).  One thread per (column,
// row group) gathers its 16 values, splits them and writes 6 granules.
template <int T, bool BF>
struct TiledCfg {
  static constexpr int Dp = 32 * T;
  static constexpr int NT = T * (T + 1) / 2;
  static constexpr int NW = (T <= 2) ? 4 : 8;       // waves per workgroup
  static constexpr int NTHR = NW * 64;
  static constexpr int MT = (NT + NW - 1) / NW;     // tiles per wave (max)
  static constexpr int R = BF ? 32 : ((T <= 2) ? 16 : (T >= 8 ? 64 : 32));  // rows per chunk
  static constexpr int NSLOT = R * Dp / 4;          // float4 per chunk
  static constexpr int NQ = (NSLOT + NTHR - 1) / NTHR;
  static constexpr int GRAN = 12 * Dp;              // BF: 16-B granules per stage buffer
  // LDS carve (floats); every offset a multiple of 4 floats (16 B).
  static constexpr int TILES = NT * 1024;
  static constexpr int STAGE = BF ? 2 * 4 * GRAN : 2 * R * Dp;  // aliases TILES
  static constexpr int REGION0 = TILES > STAGE ? TILES : STAGE;
  static constexpr int OFF_B = REGION0;             // rhs, then y
  static constexpr int OFF_X = OFF_B + Dp;          // e (CVaR), then x
  static constexpr int OFF_LD = OFF_X + Dp;         // unswizzled L_pp copy
  static constexpr int OFF_SA = OFF_LD + 1024;      // ring: A-scale per row
  static constexpr int OFF_BW = OFF_SA + kRing * R; // ring: rhs weight per row
  static constexpr int OFF_ID = OFF_BW + kRing * R; // ring: row ids (int)
  static constexpr int OFF_FLAG = OFF_ID + kRing * R;
  static constexpr int TOTAL = OFF_FLAG + 4;
  static constexpr size_t BYTES = (size_t)TOTAL * 4;
  static_assert(BYTES <= 163840, "LDS budget");
  static_assert(R % 2 == 0, "row pairs");
  static_assert(!BF || 2 * Dp <= NTHR, "BF: one thread per (column, row group)");
};

// Granule index (16 B) of piece p, row group g, k-half hh, column c in one
// BF stage buffer.
template <int Dp>
__device__ __forceinline__ int bf_gran(int p, int g, int hh, int c) {
  return ((p * 2 + g) * 2 + hh) * Dp + c;
}

// Tile ownership of the split-bf16 SYRK at T = 8 ("super-blocks"): each
// wave reads the operand fragments of (at most) four column blocks X[0..3]
// per k step and reuses each for two or more of its tiles -- 12 granule
// reads per k step instead of 6 per tile (~2.5x less LDS fragment traffic).
// Waves 0..5 own the six off-diagonal 2x2 super-blocks of the 8x8 tile grid
// (block rows X0, X1 x block columns X2, X3), waves 6 and 7 diagonal tiles;
// the sub-diagonal and diagonal tiles left over go where their fragments
// are already loaded.  Tiles per wave 5,5,5,5,4,4,4,4: waves w and w+4
// (one SIMD) hold 9 between them, as tile t -> wave t % 8 did.
//   pattern 0: SB + (X1, X0)  waves 0, 1, 3      pattern 1: SB   waves 4, 5
//   pattern 2: SB + (X0, X0)  wave 2             pattern 3: (X0,X0) (X1,X0) (X1,X1) (X2,X2)  wave 6
//   pattern 4: (X0,X0) (X1,X1) (X2,X2) (X3,X3)   wave 7
// with SB = (X0,X2) (X0,X3) (X1,X2) (X1,X3); slot m = tile (X[pa[m]], X[pb[m]]).
struct SbPat {
  int n, pa[5], pb[5];
};
__device__ constexpr SbPat kSbPat[5] = {
    {5, {0, 0, 1, 1, 1}, {2, 3, 2, 3, 0}},
    {4, {0, 0, 1, 1, 0}, {2, 3, 2, 3, 0}},
    {5, {0, 0, 1, 1, 0}, {2, 3, 2, 3, 0}},
    {4, {0, 1, 1, 2, 0}, {0, 0, 1, 2, 0}},
    {4, {0, 1, 2, 3, 0}, {0, 1, 2, 3, 0}},
};
__device__ __forceinline__ int sb_pattern(int wave) {
  constexpr int pat[8] = {0, 0, 2, 0, 1, 1, 3, 4};
  return pat[wave];
}
__device__ __forceinline__ int sb_block(int wave, int x) {
  constexpr int blk[8][4] = {{2, 3, 0, 1}, {4, 5, 0, 1}, {4, 5, 2, 3}, {6, 7, 0, 1},
                             {6, 7, 2, 3}, {6, 7, 4, 5}, {0, 1, 2, 2}, {3, 5, 6, 7}};
  return blk[wave][x];
}

// Virtual history position k -> offset within the entity's CSR row: k < h
// are the real rows; with the tail quirk rows h .. h+extra-1 re-read the
// positions [h-128, h-r) (safer2.h:200-204).
__device__ __forceinline__ int64_t virt_pos(int64_t k, int64_t h) {
  return k < h ? k : (h - 128 + (k - h));
}

// PARTIAL = true: one workgroup per SplitWork item accumulates the SYRK of
// the history positions [k0, k1) of a long entity (and its rhs part) and
// writes the raw accumulators to a workspace slab (register layout: tile t,
// element (q, lane) at t*1024 + q*64 + lane; rhs at NT*1024).  The entity's
// own workgroup (PARTIAL = false, a.split[pos].y > 0) then starts from the
// sum of its slabs instead of gathering -- the longest histories (55K rows
// on the ML-20M item side) no longer serialise on one CU.
template <int T, bool PARTIAL, bool BF, bool OFF64 = false>
__global__ void __launch_bounds__((TiledCfg<T, BF>::NTHR))
    solve_tiled_kernel(SolveArgs a) {
  using C = TiledCfg<T, BF>;
  // SB: super-block tile ownership (sb_tile) for the split-bf16 SYRK at T = 8
  constexpr bool SB = BF && T == 8 && (kSyrkSB >= 2 || (PARTIAL && kSyrkSB >= 1));
  constexpr int Dp = C::Dp, NT = C::NT, NW = C::NW, NTHR = C::NTHR;
  constexpr int MT = C::MT;
  constexpr int R = C::R, NQ = C::NQ, NSLOT = C::NSLOT;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* tiles = smem;
  float* stage = smem;
  float* bvec = smem + C::OFF_B;
  float* xvec = smem + C::OFF_X;
  float* part = smem + C::OFF_LD;  // back-solve partial sums
  float* ring_sa = smem + C::OFF_SA;
  float* ring_bw = smem + C::OFF_BW;
  int* ring_id = reinterpret_cast<int*>(smem + C::OFF_ID);
  int* flag = reinterpret_cast<int*>(smem + C::OFF_FLAG);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform branches
  const int lo = lane & 31, hi = lane >> 5;
  const int kind = a.kind;
  const bool vk = is_v_kind(kind);

  // ---- one entity per workgroup, dispatched in LPT order (longest first) ----
  int qpos = blockIdx.x;
  int64_t k0 = 0, k1 = 0;
  int slab0 = 0, nslab = 0;
  if (PARTIAL) {
    const SplitWork wk = a.work[blockIdx.x];
    qpos = wk.pos;
    k0 = wk.k0;
    k1 = wk.k1;
    slab0 = wk.slab;
  } else if (qpos < a.n_split) {
    const int2 sp = a.split[qpos];
    slab0 = sp.x;
    nslab = sp.y;
  }
  const QueueRec rec = a.order[qpos];
  const int64_t e = rec.entity;
  const int64_t h = rec.h;
  const int64_t p0 = rec.p0;
  if (h == 0) return;  // not in by_user / by_item: untouched
  int64_t extra = 0;
  if (vk && a.quirk && h > 128 && (h % 128) != 0) extra = 128 - (h % 128);
  const int64_t ntot = h + extra;
  if (!PARTIAL) k1 = nslab > 0 ? 0 : ntot;  // split: the slabs hold the rows
  const int nchunks = (int)((k1 - k0 + R - 1) / R);

  auto ring_load = [&](int c, int& id, float& sa, float& bw) {
    const int64_t k = k0 + (int64_t)c * R + tid;
    id = -1;
    sa = 0.0f;
    bw = 0.0f;
    if (k < k1) {
      id = a.col[p0 + virt_pos(k, h)];
      if (vk) {
        // rows are staged pre-scaled by sa (the factor column sqrt(w) * cp_v,
        // safer2.h:192); the rhs weight w (safer2.h:190) is then applied as
        // w / sa to the scaled row
        const float nu = a.other_weight[id];
        sa = sqrtf(nu);
        bw = (k < h && sa > 0.0f) ? nu / sa : 0.0f;
      } else {
        sa = 1.0f;
        bw = 1.0f;
      }
    }
  };
  // the same in two halves for the BF loop: the id load issued ahead of the
  // chunk's row gathers, the (dependent) weights formed at the end of the
  // step -- a use of the id right after the gathers would wait (in-order
  // vmcnt) for those rows too, stalling wave 0 a full HBM latency per chunk
  auto ring_id_load = [&](int c) {
    const int64_t k = k0 + (int64_t)c * R + tid;
    return k < k1 ? a.col[p0 + virt_pos(k, h)] : -1;
  };
  auto ring_store = [&](int c, int id, float sa, float bw) {
    const int s = (c % kRing) * R + tid;
    ring_id[s] = id;
    ring_sa[s] = sa;
    ring_bw[s] = bw;
  };
  // BF gather: thread (column bc, row group bg) of the chunk
  // (row group wave-uniform when Dp is a multiple of 64; threads past 2*Dp
  // gather row group 0 again and never store -- branch-free loads)
  const int bc = tid % Dp;
  const bool bown = BF && tid < 2 * Dp;
  const int bg = bown ? tid / Dp : 0;
  float bpart = 0.0f;  // BF: this thread's rhs part for column bc
  auto load_bf = [&](int c, float (&xr)[16]) {
    if constexpr (BF) {
      const int4* ids = reinterpret_cast<const int4*>(ring_id + (c % kRing) * R + 16 * bg);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int4 id4 = ids[q];
        const int id[4] = {id4.x, id4.y, id4.z, id4.w};
        // no select on the loaded value: rows past the history have sa = 0
        // (split_bf), so the loads stay in flight through the MFMA phase
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          // 32-bit element offsets while rows x Dp < 2^32 (launch_tiled_v
          // dispatches OFF64 above that)
          if constexpr (OFF64)
            xr[4 * q + j] = a.X[(int64_t)max(id[j], 0) * Dp + bc];
          else
            xr[4 * q + j] = a.X[(unsigned)max(id[j], 0) * (unsigned)Dp + (unsigned)bc];
        }
      }
    }
  };
  // split_bf: the pieces of chunk c in registers (the math only, so it can
  // share a basic block with -- and be scheduled between -- the MFMAs of
  // the previous chunk); write_bf: the granule stores.  `live` = false
  // (past the last chunk) leaves the rhs part untouched.
  auto split_bf = [&](int c, const float (&xr)[16], bf16x8 (&f)[2][3], bool live) {
    if constexpr (BF) {
      // rows pre-scaled by sa (1 for non-V kinds, 0 past the history), rhs
      // weight bw per scaled row -- as the fp32 staging below
      const int base = (c % kRing) * R + 16 * bg;
      float sa[16], bw[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 s4 = reinterpret_cast<const float4*>(ring_sa + base)[q];
        const float4 w4 = reinterpret_cast<const float4*>(ring_bw + base)[q];
        sa[4 * q] = s4.x, sa[4 * q + 1] = s4.y, sa[4 * q + 2] = s4.z, sa[4 * q + 3] = s4.w;
        bw[4 * q] = w4.x, bw[4 * q + 1] = w4.y, bw[4 * q + 2] = w4.z, bw[4 * q + 3] = w4.w;
      }
      float bsum = 0.0f;
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float x = xr[8 * hh + j] * sa[8 * hh + j];
          bsum += bw[8 * hh + j] * x;
          v[j] = x;
        }
        split3x8(v, f[hh]);
      }
      bpart = live ? bpart + bsum : bpart;
    }
  };
  auto scale_bf = [&](int c, const float (&xr)[16], float (&xs)[16], bool live) {
    if constexpr (BF) {
      const int base = (c % kRing) * R + 16 * bg;
      float bsum = 0.0f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 s4 = reinterpret_cast<const float4*>(ring_sa + base)[q];
        const float4 w4 = reinterpret_cast<const float4*>(ring_bw + base)[q];
        const float sa[4] = {s4.x, s4.y, s4.z, s4.w}, bw[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          xs[4 * q + j] = xr[4 * q + j] * sa[j];
          bsum += bw[j] * xs[4 * q + j];
        }
      }
      bpart = live ? bpart + bsum : bpart;
    }
  };
  auto write_bf = [&](int buf, const bf16x8 (&f)[2][3]) {
    if constexpr (BF) {
      bf16x8* st = reinterpret_cast<bf16x8*>(stage) + buf * C::GRAN;
      if (bown) {
#pragma unroll
        for (int hh = 0; hh < 2; ++hh)
#pragma unroll
          for (int p = 0; p < 3; ++p) st[bf_gran<Dp>(p, bg, hh, bc)] = f[hh][p];
      }
    }
  };
  constexpr int NQR = BF ? 1 : NQ;
  float4 regs[NQR];
  auto load_data = [&](int c) {  // fp32 path
    {
      const int slot = c % kRing;
#pragma unroll
      for (int q = 0; q < NQR; ++q) {
        const int sidx = tid + q * NTHR;
        regs[q] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (NSLOT % NTHR == 0 || sidx < NSLOT) {
          const int r = sidx / (Dp / 4), c4 = sidx % (Dp / 4);
          const int id = ring_id[slot * R + r];
          if (id >= 0) regs[q] = *reinterpret_cast<const float4*>(a.X + (int64_t)id * Dp + 4 * c4);
        }
      }
    }
  };
  auto store_stage = [&](int buf, int c) {  // fp32 path
    {
      float* st = stage + buf * R * Dp;
      const int slot = c % kRing;
#pragma unroll
      for (int q = 0; q < NQR; ++q) {
        const int sidx = tid + q * NTHR;
        if (NSLOT % NTHR == 0 || sidx < NSLOT) {
          float4 v = regs[q];
          if (vk) {
            const float sc = ring_sa[slot * R + sidx / (Dp / 4)];
            v.x *= sc;
            v.y *= sc;
            v.z *= sc;
            v.w *= sc;
          }
          *reinterpret_cast<float4*>(st + 4 * sidx) = v;
        }
      }
    }
  };

  if (tid == 0) flag[0] = 0;
  // diagnostics (FRECSYS_DUAL_PROF): cycles per phase summed over entities
  unsigned long long t_prev = (!PARTIAL && a.prof) ? clock64() : 0;
  auto mark = [&](int ph) {
    if (!PARTIAL && a.prof && tid == 0) {
      const unsigned long long t = clock64();
      atomicAdd(a.prof + ph, t - t_prev);
      t_prev = t;
    }
  };
  if (tid < R) {  // ring prologue: the chunks the first iteration reads
#pragma unroll
    for (int c = 0; c < (BF ? 3 : 2); ++c) {
      if (c < nchunks) {
        int id;
        float sa, bw;
        ring_load(c, id, sa, bw);
        ring_store(c, id, sa, bw);
      }
    }
  }
  if (!PARTIAL && is_grad_kind(kind) && tid < Dp) xvec[tid] = a.E[e * Dp + tid];

  // ---- my tiles; accumulators start from the G part of A ----
  // (the G reads overlap the history gather that starts below)
  //  iALS: acc0 = w*G + lam*I        -> A = acc
  //  U:    acc0 = h*w*G              -> A = acc * (omega/h) + lam*I
  //  V:    acc0 = w*G                -> A = acc + lam*I
  //  CVaR: acc0 = 0 (the stale upper triangle needs S and G apart)
  const float hf = (float)h;
  const float omega = (is_u_kind(kind) && a.entity_weight) ? a.entity_weight[e] : 1.0f;
  const float lam =
      entity_lambda(kind, a.reg, a.reg_exp, a.w, a.alpha, h, a.n_other, a.entity_reg, e,
                    a.lambda_is_reg);
  const bool grad = is_grad_kind(kind);
  const float gscale = kind == KIND_IALS ? a.w : (is_u_kind(kind) ? hf * a.w : a.w);
  const float lam_d = kind == KIND_IALS ? lam : 0.0f;  // iALS: lambda rides in acc0
  f32x16 acc[MT];
  int aoff[MT], boff[MT];
  bool valid[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    int I = 0, J = 0;
    if constexpr (SB) {
      const SbPat& pt = kSbPat[sb_pattern(wave)];
      valid[m] = m < pt.n;
      I = sb_block(wave, pt.pa[m]);
      J = sb_block(wave, pt.pb[m]);
    } else {
      const int t = wave + m * NW;
      valid[m] = t < NT;
      while ((I + 1) * (I + 2) / 2 <= t) ++I;
      J = t - I * (I + 1) / 2;
    }
    aoff[m] = 32 * I + lo;
    boff[m] = 32 * J + lo;
    acc[m] = f32x16{0.f};
    if (!PARTIAL && valid[m] && !grad) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int gi = 32 * I + acc_row(q, hi), gj = 32 * J + lo;
        acc[m][q] = gscale * a.G[gi * Dp + gj] + (gi == gj ? lam_d : 0.0f);
      }
    }
  }
  int sbx[4] = {0, 0, 0, 0};  // SB: the wave's four column blocks
  if constexpr (SB) {
#pragma unroll
    for (int x = 0; x < 4; ++x) sbx[x] = sb_block(wave, x);
  }
  // split entity: add its slabs in slab order (deterministic)
  float bacc = 0.0f;
  const size_t slab_floats = (size_t)NT * 1024 + Dp;
  for (int sidx = 0; sidx < nslab; ++sidx) {
    const float* sl = a.slabs + (size_t)(slab0 + sidx) * slab_floats;
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      if (valid[m]) {
        const int t = tidx((aoff[m] - lo) >> 5, (boff[m] - lo) >> 5);
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[m][q] += sl[t * 1024 + q * 64 + lane];
      }
    }
    if (tid < Dp) bacc += sl[NT * 1024 + tid];
  }
  // The tiles leave the registers right after the SYRK loop (inside each
  // ownership pattern's copy of it, so the accumulators of the copies never
  // merge): PARTIAL -> the slab (raw accumulator layout), else -> A in the
  // swizzled LDS tiles (aliasing the then-dead stage; the loop's last
  // barrier ordered every stage read before these writes).
  // ---- epilogue: finish A into the swizzled LDS tiles ----
  // (the kind is dispatched once, outside the element loops: a per-element
  // kind test compiled into ~7 scalar branches per element, 15K cycles)
  const float us = omega / hf;
  auto write_tiles = [&](auto mode_c) __attribute__((always_inline)) {
    constexpr int MODE = decltype(mode_c)::value;  // 0 iALS, 1 U kinds, 2 V kinds, 3 CVaR
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      if (valid[m]) {
        const int I = (aoff[m] - lo) >> 5, J = (boff[m] - lo) >> 5;
        float* tile = tiles + tidx(I, J) * 1024;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int i = acc_row(q, hi);
          const bool dg = (32 * I + i) == (32 * J + lo);
          float v = acc[m][q];
          if constexpr (MODE == 1) v = v * us + (dg ? lam : 0.0f);
          if constexpr (MODE == 2) v = v + (dg ? lam : 0.0f);
          if constexpr (MODE == 3)
            v = assemble(kind, v, a.G[(32 * I + i) * Dp + 32 * J + lo], dg, a.w, lam, hf, omega);
          tile[sw(i, lo)] = v;
        }
      }
    }
  };
  auto store_tiles = [&]() __attribute__((always_inline)) {
    if constexpr (PARTIAL) {
      float* sl = a.slabs + (size_t)slab0 * slab_floats;
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        if (valid[m]) {
          const int t = tidx((aoff[m] - lo) >> 5, (boff[m] - lo) >> 5);
#pragma unroll
          for (int q = 0; q < 16; ++q) sl[t * 1024 + q * 64 + lane] = acc[m][q];
        }
      }
    } else {
      if (grad) write_tiles(std::integral_constant<int, 3>{});
      else if (is_u_kind(kind)) write_tiles(std::integral_constant<int, 1>{});
      else if (vk) write_tiles(std::integral_constant<int, 2>{});
      else write_tiles(std::integral_constant<int, 0>{});
    }
  };
  lds_barrier();
  mark(0);
  if constexpr (BF) {
    // two chunks of row loads in flight: iteration c runs the MFMAs of
    // chunk c, stages chunk c+1 (registers xcur, loaded one iteration ago)
    // and issues chunk c+2's loads into xnxt -- a full iteration of cover
    // for the gather latency; the ring is filled three chunks ahead
    float xa[16], xb[16];
    if (nchunks > 0) {
      load_bf(0, xa);
      bf16x8 f[2][3];
      split_bf(0, xa, f, true);
      write_bf(0, f);
    }
    if (nchunks > 1) load_bf(1, xa);
    lds_barrier();
    // the ring's weights trail its ids by one iteration: chunk c+3's id is
    // loaded at the top of step c and stored at its end (step c+1's row
    // gathers read it), its weight operand (other_weight[id], V kinds) is
    // issued then and its sa / bw stored at the end of step c+1 (step c+2
    // scales with them) -- so no wait at the end of a step is behind the row
    // gathers issued at its top (in-order vmcnt)
    float wpend = 0.0f;  // raw weight of chunk c+2 at the top of step c
    auto step = [&](int c, float (&xcur)[16], float (&xnxt)[16], auto pc)
                    __attribute__((always_inline)) {
      const int buf = c & 1;
      const bool ring_more = (tid < R) && (c + 3 < nchunks);
      int nid = -1;
      if (ring_more) nid = ring_id_load(c + 3);
      // unconditional (past the end it re-gathers the last chunk, whose ring
      // slot stays valid; the values are never staged): a conditional load
      // block here made the waitcnt pass wait (vmcnt) for these fresh rows
      // before this step's scaling and MFMAs
      load_bf(c + 2 < nchunks ? c + 2 : nchunks - 1, xnxt);
      const bool live = c + 1 < nchunks;
      // chunk c+1's staging math is spread over the issue gaps of this
      // chunk's MFMAs: scaled values (and the rhs part) first, then two
      // 3-piece splits after each mfma_x6 of the tiles every wave has
      float xs[16];
      scale_bf(c + 1, xcur, xs, live);
      bf16x8 f[2][3];
      constexpr int SLOTS = (NT / NW) * 2 > 0 ? (NT / NW) * 2 : 1;
      constexpr int PER = (16 + SLOTS - 1) / SLOTS;
      auto split_slot = [&](int slot) {
#pragma unroll
        for (int u = 0; u < PER; ++u) {
          const int j = slot * PER + u;
          if (j < 16) {
            __bf16 h, m, l;
            split3(xs[j], h, m, l);
            f[j >> 3][0][j & 7] = h;
            f[j >> 3][1][j & 7] = m;
            f[j >> 3][2][j & 7] = l;
          }
        }
        // keep this slot's pieces here (between the MFMAs), not sunk to
        // their stores after the loop
#pragma unroll
        for (int hh = 0; hh < 2; ++hh)
          if ((slot * PER) >> 3 == hh || (slot * PER + PER - 1) >> 3 == hh)
#pragma unroll
            for (int p = 0; p < 3; ++p) asm volatile("" : "+v"(f[hh][p]));
      };
      const bf16x8* st = reinterpret_cast<const bf16x8*>(stage) + buf * C::GRAN;
      if (SB && !FRECSYS_SKIP(a.debug_skip, 1)) {
        // the wave's column blocks' fragments, each feeding two or more
        // tiles (per-tile accumulation order as below: bit-identical)
        {
          constexpr SbPat P = kSbPat[decltype(pc)::value];
          constexpr int NX = decltype(pc)::value == 3 ? 3 : 4;
#pragma unroll
          for (int g = 0; g < 2; ++g) {
            bf16x8 fr[NX][3];
#pragma unroll
            for (int x = 0; x < NX; ++x)
#pragma unroll
              for (int p = 0; p < 3; ++p) fr[x][p] = st[bf_gran<Dp>(p, g, hi, 32 * sbx[x] + lo)];
#pragma unroll
            for (int m = 0; m < P.n; ++m) {
              acc[m] = mfma_x6s(fr[P.pa[m]], fr[P.pb[m]], acc[m]);
              if (m < 4) split_slot(4 * g + m);
            }
          }
        }
      } else if (!FRECSYS_SKIP(a.debug_skip, 1)) {
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          // tiles every wave has: no branch, one basic block with the splits
          if (m < NT / NW || valid[m]) {
#pragma unroll
            for (int g = 0; g < 2; ++g) {
              bf16x8 av[3], bv[3];
#pragma unroll
              for (int p = 0; p < 3; ++p) {
                av[p] = st[bf_gran<Dp>(p, g, hi, aoff[m])];
                bv[p] = st[bf_gran<Dp>(p, g, hi, boff[m])];
              }
              acc[m] = mfma_x6s(av, bv, acc[m]);
              if (m < NT / NW) split_slot(2 * m + g);
            }
          }
        }
        if constexpr (NT / NW == 0) split_slot(0);
      } else {
#pragma unroll
        for (int k = 0; k < SLOTS; ++k) split_slot(k);
      }
      if (live) write_bf(buf ^ 1, f);
      if (tid < R && c >= 1 && c + 2 < nchunks) {  // chunk c+2's sa / bw
        const int64_t k = k0 + (int64_t)(c + 2) * R + tid;
        float sa = 0.0f, bw = 0.0f;
        if (k < k1) {
          if (vk) {
            sa = sqrtf(wpend);
            bw = (k < h && sa > 0.0f) ? wpend / sa : 0.0f;
          } else {
            sa = 1.0f;
            bw = 1.0f;
          }
        }
        const int s = ((c + 2) % kRing) * R + tid;
        ring_sa[s] = sa;
        ring_bw[s] = bw;
      }
      if (ring_more) {
        ring_id[((c + 3) % kRing) * R + tid] = nid;
        if (vk) wpend = a.other_weight[max(nid, 0)];
      }
      lds_barrier();
    };
    // SB: one copy of the chunk loop per ownership pattern (the tiles'
    // accumulators then merge once, after the loop, not at every step)
    auto loop = [&](auto pc) __attribute__((always_inline)) {
      for (int c = 0; c < nchunks; c += 2) {
        step(c, xa, xb, pc);
        if (c + 1 < nchunks) step(c + 1, xb, xa, pc);
      }
      store_tiles();
    };
    if constexpr (SB) {
      switch (sb_pattern(wave)) {
        case 0: loop(std::integral_constant<int, 0>{}); break;
        case 1: loop(std::integral_constant<int, 1>{}); break;
        case 2: loop(std::integral_constant<int, 2>{}); break;
        case 3: loop(std::integral_constant<int, 3>{}); break;
        default: loop(std::integral_constant<int, 4>{}); break;
      }
    } else {
      loop(std::integral_constant<int, 0>{});
    }
  } else {
    if (nchunks > 0) {
      load_data(0);
      store_stage(0, 0);
    }
    lds_barrier();
    for (int c = 0; c < nchunks; ++c) {
      const int buf = c & 1;
      const bool more = c + 1 < nchunks;
      const bool ring_more = (tid < R) && (c + 2 < nchunks);
      if (more) load_data(c + 1);
      int nid = -1;
      float nsa = 0.f, nbw = 0.f;
      if (ring_more) ring_load(c + 2, nid, nsa, nbw);
      const float* st = stage + buf * R * Dp;
      const int slot = c % kRing;
      // tile-outer, row-pair-inner: one wave-uniform branch per tile and the
      // operand reads free to run ahead of the MFMAs
      if (!FRECSYS_SKIP(a.debug_skip, 1)) {
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          if (valid[m]) {
#pragma unroll
            for (int s = 0; s < R / 2; ++s) {
              const float* rowp = st + (2 * s + hi) * Dp;
              acc[m] = mfma32(rowp[aoff[m]], rowp[boff[m]], acc[m]);
            }
          }
        }
      }
      if (tid < Dp) {
#pragma unroll 4
        for (int r = 0; r < R; ++r) bacc += ring_bw[slot * R + r] * st[r * Dp + tid];
      }
      if (more) store_stage(buf ^ 1, c + 1);
      if (ring_more) ring_store(c + 2, nid, nsa, nbw);
      lds_barrier();
    }
    store_tiles();
  }
  mark(1);
  if constexpr (BF) {
    // rhs: the two row groups' parts of each column (the stage is dead)
    if (bown && bg == 1) part[bc] = bpart;
    lds_barrier();
    if (tid < Dp) bacc += bpart + part[tid];
    lds_barrier();
  }
  mark(9);

  if (PARTIAL) {  // the tiles went out in store_tiles
    if (tid < Dp) a.slabs[(size_t)slab0 * slab_floats + NT * 1024 + tid] = bacc;
    return;
  }

  mark(10);
  if (tid < Dp) {
    float b = bacc;
    if (is_u_kind(kind)) b *= us;  // rhs *= weight / history_size
    bvec[tid] = b;
  }
  lds_barrier();
  mark(2);

  if (grad) {
    // ---- CVaR-MF: one gradient step with the full (stale-upper) matrix ----
    if (tid < Dp) {
      const int i = tid, I = i >> 5, ri = i & 31;
      float y = 0.0f;
      for (int j = 0; j < Dp; ++j) {
        float aij;
        if (j <= i)
          aij = tiles[tidx(I, j >> 5) * 1024 + sw(ri, j & 31)];
        else
          aij = cvar_upper(kind, a.G[i * Dp + j], a.w, omega);
        y += aij * xvec[j];
      }
      a.out[e * Dp + i] = xvec[i] - a.eta * (y - bvec[i]);
    }
    return;
  }

  // ---- blocked right-looking Cholesky with lookahead + back-solve ----
  chol_solve_df<T, NW>(tiles, bvec, xvec, part, flag, tid, a.debug_skip, a.prof);
  mark(3);
  if (tid < Dp) a.out[e * Dp + tid] = xvec[tid];
  if (tid == 0 && flag[0]) atomicMin(a.fail, (unsigned long long)(e + 1));
  if (a.prof && tid == 0) {
    atomicAdd(a.prof + 4, 1ull);
    atomicAdd(a.prof + 8, (unsigned long long)ntot);
  }
}

// ---------------------------------------------------------------------
// Small dims (Dp = 8, 16): one wave per entity, 4 entities per workgroup.
// ---------------------------------------------------------------------
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int Dp>
__global__ void __launch_bounds__(256) solve_small_kernel(SolveArgs a) {
  constexpr int WPB = 4, CH = 64, PER = Dp * Dp / 64;
  __shared__ float sA[WPB][Dp * Dp];
  __shared__ float sX[WPB][CH * Dp];
  __shared__ float sB[WPB][Dp];
  __shared__ float sE[WPB][Dp];
  __shared__ float sSA[WPB][CH];
  __shared__ float sBW[WPB][CH];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t idx = (int64_t)blockIdx.x * WPB + wave;
  if (idx >= a.n_rows) return;  // no workgroup barrier below
  const int64_t e = a.row_lo + idx;
  const int64_t p0 = a.row_ptr[e];
  const int64_t h = a.row_ptr[e + 1] - p0;
  if (h == 0) return;
  const int kind = a.kind;
  const bool vk = is_v_kind(kind);
  int64_t extra = 0;
  if (vk && a.quirk && h > 128 && (h % 128) != 0) extra = 128 - (h % 128);
  const int64_t ntot = h + extra;
  float acc[PER];
#pragma unroll
  for (int t = 0; t < PER; ++t) acc[t] = 0.0f;
  float bacc = 0.0f;
  float* X = sX[wave];
  for (int64_t c0 = 0; c0 < ntot; c0 += CH) {
    const int64_t k = c0 + lane;
    int id = -1;
    float sa = 0.f, bw = 0.f;
    if (k < ntot) {
      id = a.col[p0 + virt_pos(k, h)];
      if (vk) {
        const float nu = a.other_weight[id];
        sa = sqrtf(nu);
        bw = (k < h) ? nu : 0.0f;
      } else {
        sa = 1.0f;
        bw = 1.0f;
      }
    }
    sSA[wave][lane] = sa;
    sBW[wave][lane] = bw;
#pragma unroll
    for (int d = 0; d < Dp; d += 4) {
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (id >= 0) v = *reinterpret_cast<const float4*>(a.X + (int64_t)id * Dp + d);
      *reinterpret_cast<float4*>(X + lane * Dp + d) = v;
    }
    wave_sync();
    const int cnt = (int)((ntot - c0) < CH ? (ntot - c0) : CH);
    for (int r = 0; r < cnt; ++r) {
      const float* x = X + r * Dp;
      const float s = sSA[wave][r];
#pragma unroll
      for (int t = 0; t < PER; ++t) {
        const int el = lane * PER + t, i = el / Dp, j = el % Dp;
        acc[t] += (s * x[i]) * (s * x[j]);
      }
      if (lane < Dp) bacc += sBW[wave][r] * x[lane];
    }
    wave_sync();
  }
  const float hf = (float)h;
  const float omega = (is_u_kind(kind) && a.entity_weight) ? a.entity_weight[e] : 1.0f;
  const float lam = entity_lambda(kind, a.reg, a.reg_exp, a.w, a.alpha, h, a.n_other,
                                  a.entity_reg, e, a.lambda_is_reg);
#pragma unroll
  for (int t = 0; t < PER; ++t) {
    const int el = lane * PER + t, i = el / Dp, j = el % Dp;
    sA[wave][el] = assemble(kind, acc[t], a.G[i * Dp + j], i == j, a.w, lam, hf, omega);
  }
  if (lane < Dp) {
    float b = bacc;
    if (is_u_kind(kind)) b *= (omega / hf);
    sB[wave][lane] = b;
    if (is_grad_kind(kind)) sE[wave][lane] = a.E[e * Dp + lane];
  }
  wave_sync();
  if (lane != 0) return;
  float* A = sA[wave];
  const float* b = sB[wave];
  if (is_grad_kind(kind)) {
    const float* ev = sE[wave];
    for (int i = 0; i < Dp; ++i) {
      float y = 0.0f;
      for (int j = 0; j < Dp; ++j) {
        const float aij = (j <= i) ? A[i * Dp + j] : cvar_upper(kind, a.G[i * Dp + j], a.w, omega);
        y += aij * ev[j];
      }
      a.out[e * Dp + i] = ev[i] - a.eta * (y - b[i]);
    }
    return;
  }
  bool ok = true;
  for (int j = 0; j < Dp; ++j) {  // left-looking LLT<Lower>
    float s = A[j * Dp + j];
    for (int k = 0; k < j; ++k) s -= A[j * Dp + k] * A[j * Dp + k];
    ok = ok && (s > 0.0f);
    const float ljj = sqrtf(s);
    A[j * Dp + j] = ljj;
    for (int i = j + 1; i < Dp; ++i) {
      float t = A[i * Dp + j];
      for (int k = 0; k < j; ++k) t -= A[i * Dp + k] * A[j * Dp + k];
      A[i * Dp + j] = t / ljj;
    }
  }
  float x[Dp];
  for (int i = 0; i < Dp; ++i) {
    float t = b[i];
    for (int k = 0; k < i; ++k) t -= A[i * Dp + k] * x[k];
    x[i] = t / A[i * Dp + i];
  }
  for (int i = Dp - 1; i >= 0; --i) {
    float t = x[i];
    for (int k = i + 1; k < Dp; ++k) t -= A[k * Dp + i] * x[k];
    x[i] = t / A[i * Dp + i];
  }
  for (int i = 0; i < Dp; ++i) a.out[e * Dp + i] = x[i];
  if (!ok) atomicMin(a.fail, (unsigned long long)(e + 1));
}

template <int T, bool PARTIAL, bool BF, bool OFF64>
hipError_t launch_tiled_o(const SolveArgs& a, hipStream_t s) {
  using C = TiledCfg<T, BF>;
  static bool attr = false;
  if (!attr) {
    hipError_t err = hipFuncSetAttribute((const void*)solve_tiled_kernel<T, PARTIAL, BF, OFF64>,
                                         hipFuncAttributeMaxDynamicSharedMemorySize,
                                         (int)C::BYTES);
    if (err != hipSuccess) return err;
    attr = true;
  }
  const int64_t n = PARTIAL ? a.n_work : a.n_rows;
  hipLaunchKernelGGL((solve_tiled_kernel<T, PARTIAL, BF, OFF64>), dim3((unsigned)n),
                     dim3(C::NTHR), C::BYTES, s, a);
  return hipGetLastError();
}

// The split-bf16 gathers use 32-bit element offsets while n_other * Dp <
// 2^32 (Dp = 256: 16.7M rows), 64-bit ones above (the fp32 staging path
// always uses 64-bit offsets).
template <int T, bool PARTIAL, bool BF>
hipError_t launch_tiled_v(const SolveArgs& a, hipStream_t s) {
  if constexpr (BF) {
    if (gather_off64(a.n_other, 32 * T)) return launch_tiled_o<T, PARTIAL, BF, true>(a, s);
  }
  return launch_tiled_o<T, PARTIAL, BF, false>(a, s);
}

template <int T, bool PARTIAL>
hipError_t launch_tiled(const SolveArgs& a, hipStream_t s) {
  return syrk_split_bf16() ? launch_tiled_v<T, PARTIAL, true>(a, s)
                           : launch_tiled_v<T, PARTIAL, false>(a, s);
}

template <int Dp>
hipError_t launch_small(const SolveArgs& a, hipStream_t s) {
  const unsigned nb = (unsigned)((a.n_rows + 3) / 4);
  hipLaunchKernelGGL(solve_small_kernel<Dp>, dim3(nb), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace

bool gather_off64(int64_t rows, int Dp) {
  if (rows * (int64_t)Dp >= ((int64_t)1 << 32)) return true;
  const char* v = getenv("FRECSYS_GATHER64");  // tests: force the 64-bit variants
  return v && atoi(v) != 0;
}

bool syrk_split_bf16() {
  static const bool on = [] {
    const char* v = getenv("FRECSYS_SYRK_F32");
    return !(v && atoi(v) != 0);
  }();
  return on;
}

int padded_dim(int dim) {
  if (dim <= 0) return 0;
  if (dim <= 8) return 8;
  if (dim <= 16) return 16;
  if (dim <= 256) return ((dim + 31) / 32) * 32;
  if (dim <= 512) return 512;
  if (dim <= 1024) return 1024;
  return 0;
}

hipError_t launch_solve(int Dp, const SolveArgs& a, hipStream_t s) {
  if (a.n_rows <= 0) return hipSuccess;
  switch (Dp) {
    case 8: return launch_small<8>(a, s);
    case 16: return launch_small<16>(a, s);
    case 32: return launch_tiled<1, false>(a, s);
    case 64: return launch_tiled<2, false>(a, s);
    case 96: return launch_tiled<3, false>(a, s);
    case 128: return launch_tiled<4, false>(a, s);
    case 160: return launch_tiled<5, false>(a, s);
    case 192: return launch_tiled<6, false>(a, s);
    case 224: return launch_tiled<7, false>(a, s);
    case 256:
      return launch_tiled<8, false>(a, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_split_syrk(int Dp, const SolveArgs& a, hipStream_t s) {
  if (a.n_work <= 0) return hipSuccess;
  switch (Dp) {
    case 32: return launch_tiled<1, true>(a, s);
    case 64: return launch_tiled<2, true>(a, s);
    case 96: return launch_tiled<3, true>(a, s);
    case 128: return launch_tiled<4, true>(a, s);
    case 160: return launch_tiled<5, true>(a, s);
    case 192: return launch_tiled<6, true>(a, s);
    case 224: return launch_tiled<7, true>(a, s);
    case 256: return launch_tiled<8, true>(a, s);
    default: return hipErrorInvalidValue;
  }
}

size_t split_slab_floats(int Dp) {
  const int T = Dp / 32;
  return (size_t)T * (T + 1) / 2 * 1024 + Dp;
}

// Diagnostics (frecsys_debug_diag_factor): one wave per 32x32 tile, the
// tile factored + inverted in LDS by the lane recurrence (blk = 0,
// diag_factor_inv_lds) or the MFMA-blocked factor (blk = 1,
// diag_factor_inv_blk) -- the two diagonal-block routines of chol.h.
__global__ void __launch_bounds__(64)
    debug_diag_kernel(const float* __restrict__ A, float* __restrict__ Linv, int* __restrict__ ok,
                      int blk) {
  __shared__ __attribute__((aligned(16))) float tile[1024];
  const int lane = threadIdx.x;
  const float* a = A + (int64_t)blockIdx.x * 1024;
  for (int i = lane; i < 1024; i += 64) tile[sw(i >> 5, i & 31)] = a[i];
  __syncthreads();
  const bool good = blk ? diag_factor_inv_blk((lds_float*)tile, lane)
                        : diag_factor_inv_lds((lds_float*)tile, lane);
  __syncthreads();
  for (int i = lane; i < 1024; i += 64) Linv[(int64_t)blockIdx.x * 1024 + i] = tile[sw(i >> 5, i & 31)];
  if (lane == 0) ok[blockIdx.x] = good ? 1 : 0;
}

hipError_t launch_debug_diag(const float* A, float* Linv, int* ok, int n, int blk, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(debug_diag_kernel, dim3((unsigned)n), dim3(64), 0, s, A, Linv, ok, blk);
  return hipGetLastError();
}

}  // namespace frecsys_hip
