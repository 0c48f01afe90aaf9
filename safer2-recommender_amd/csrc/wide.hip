// wide.hip -- the solve loop at d = 512 / 1024 (Dp > 256) on gfx950.
//
// At these widths a d x d normal matrix no longer fits one CU (1 MB / 4 MB
// fp32 against 160 KB of LDS), so the d-space solve of the reference's
// Project / ProjectU / ProjectV (ials.h:88-144, safer2.h:104-221,
// erm_mf.h:91-210, cvar_mf.h:182-229) is split across kernels with A in an
// HBM workspace, a bounded batch of entities at a time:
//
//   wide_syrk2_kernel<1> grid (entity, 256x256 block pair of A's lower
//                        triangle): the pair's 32x32 tiles accumulate
//                        X_h^T D X_h over the gathered history rows as
//                        split-bf16 MFMAs (fp32-accurate; rows staged through
//                        LDS as bf16 pieces, 16 per chunk, one chunk ahead),
//                        two-level accumulation, the G part of A added in the
//                        epilogue; the diagonal pairs also form b.
//   wide_chol_kernel     one workgroup (8 waves) per entity: left-looking
//                        blocked Cholesky over the workspace tiles -- row p
//                        of L staged in LDS, the diagonal tile updated,
//                        factored and inverted in LDS (diag_factor_inv), the
//                        panel tiles summed from the streamed L tiles and
//                        finished by MFMA with L_pp^-T, y = L^-1 b riding
//                        along, then x = L^-T y.
//   wide_grad_kernel     CVaR-MF's gradient step with the stale upper
//                        triangle (cvar_mf.h:133, 179).
//
// Most entities never come here: the history-space path (dual.hip) takes
// every h_eff <= 256 at any width.  Its basis at these widths:
//   tridiag_step_kernel  one launch per Householder step (no grid barrier):
//                        each workgroup finishes the previous step's rank-2
//                        update on its 16 columns (ping-pong copy of the
//                        matrix), re-forms the step's reflector from the
//                        updated row k itself, and writes its columns of
//                        p = tau A v for the next launch.
//   rotations            spectral.hip rotate_kernel (split-bf16), which also
//                        forms the u^T G u partials of the user loss.
// and the Gramian: wide_syrk2_kernel<0> (split-K over row blocks x block
// pairs) + wide_gram_reduce_kernel (fixed order, deterministic).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "chol.h"
#include "common.h"
#include "kernels.h"
#include "wide.h"

// waves per SIMD wide_chol_kernel<16> is compiled for (4: two workgroups per
// CU, 128 registers, 30.5 ms at MSD; 2: one workgroup, 256 registers,
// 32.1 ms); at Dp = 1024 row p of L alone takes 128 KB of LDS: 2.
constexpr int kWideCholWPE = 4;
// waves of wide_chol_kernel<16>: 8 (f32 panel products, two workgroups per
// CU); 4 with split-bf16 products (170 registers, two workgroups per CU)
// measured MSD 114.5-115.0 vs 114.1-114.5 ms, config 5 unchanged (round 6)
constexpr int kWideChol16NW = 8;

namespace frecsys_hip {

namespace {

constexpr int WB = 128;    // block-pair edge
constexpr int WR = 16;     // rows per staged chunk
// Leaves of a wide Gramian (kernels.h GramPlan): 768 rather than 256, so that
// a rank's two of the 16 groups at N = 8 still launch ~100 leaves x the block
// pairs (the 1,842-row leaves of 256 took 376 us for the MSD user Gramian on
// 96 workgroups); the leaf structure depends on n only (partition-independent)
constexpr int kWideGramLeaves = 768;

__device__ __forceinline__ void pair_of(int pidx, int& BI, int& BJ) {
  BI = 0;
  while ((BI + 1) * (BI + 2) / 2 <= pidx) ++BI;
  BJ = pidx - BI * (BI + 1) / 2;
}

__device__ __forceinline__ float block_sum(float v, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int tid = threadIdx.x, nw = blockDim.x >> 6;
  __syncthreads();
  if ((tid & 63) == 0) red[tid >> 6] = v;
  __syncthreads();
  float s = 0.0f;
  for (int w = 0; w < nw; ++w) s += red[w];
  return s;
}


// ---- SYRK of A (MODE 1) / partial Gramians (MODE 0) over 256 x 256 block
// pairs, fp32 products on the bf16 matrix cores ----
// One workgroup per (unit, block pair of A's lower triangle): MODE 1 unit =
// entity (the pair's tiles of X_h^T D X_h from the gathered history rows,
// plus the G part of A and its b in the epilogue), MODE 0 unit = row block
// of the Gramian.  Products as common.h mfma_x6 (3-piece bf16 splits,
// fp32-accurate).  A pair of 256-column blocks per workgroup: every gathered
// row is read 2x per entity at Dp = 512 (3 pairs), 4x at Dp = 1024 (10
// pairs) -- half the re-reads of 128-wide pairs.  512 threads:
//  * staging: one thread per staged column (512 for an off-diagonal pair:
//    block BI then block BJ; 256 x two row halves for a diagonal one) gathers
//    its 16 (8) rows of the chunk, scales them (sqrt(nu) for the V kinds,
//    the row weight on the B side of a weighted Gramian), splits them into
//    3 bf16 pieces and writes the k-major granules the MFMA lanes read
//    (granule (piece p, row half hh, column c) = rows 8hh..8hh+7 of c);
//  * MFMAs: wave w owns tile row w of an off-diagonal pair (8 tiles, its A
//    fragments shared), or tiles w, w+8, ... of a diagonal pair's 36.
// Chunks of 16 rows (one k16 step), double-buffered; the next chunk's rows
// are loaded one iteration ahead, row ids three ahead.  Two-level
// accumulation as wide_syrk_kernel (flush into the unit's output tiles
// every W2FLUSH chunks).
constexpr int WB2 = 256;
constexpr int W2R = 16;
// rows gathered W2AH chunks ahead of their staging (1: measured slower)
constexpr int W2AH = 2;
static_assert(W2AH == 1 || W2AH == 2, "one or two chunks ahead");
constexpr int W2RING = W2AH == 1 ? 4 : 8;
constexpr int W2FLUSH = 128;
constexpr int W2GRAN = 6 * 512;  // 16-B granules per stage buffer

__device__ __forceinline__ int g2(int p, int hh, int c) { return (p * 2 + hh) * 512 + c; }

int wide_pairs2(int Dp) {
  const int nb = Dp / WB2;
  return nb * (nb + 1) / 2;
}

template <int MODE, bool OFF64 = false>
__global__ void __launch_bounds__(512)
    wide_syrk2_kernel(SolveArgs a, GramArgs g, int Dp, int64_t rpb, int64_t pos0, float* ws,
                      int64_t n_units) {
  __shared__ __attribute__((aligned(16))) bf16x8 stage[2][W2GRAN];
  __shared__ __attribute__((aligned(16))) int ring_id[W2RING * W2R];
  __shared__ float2 ring_sb[W2RING * W2R];  // (row scale, rhs / B-side weight)
  __shared__ float bred[WB2];
  const int tid = threadIdx.x, lane = tid & 63, lo = lane & 31, hi = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int T = Dp >> 5, NT = T * (T + 1) / 2, NB = Dp / WB2;
  int64_t unit;
  int pidx;
  if (!xcd_unit(NB * (NB + 1) / 2, n_units, unit, pidx)) return;
  int BI, BJ;
  pair_of(pidx, BI, BJ);
  const bool dgp = BI == BJ;
  // a diagonal pair stages one block (A = B) unless its B side is weighted
  const bool same = dgp && !(MODE == 0 && g.w != nullptr);
  const int kind = a.kind;
  const bool vk = MODE >= 1 && is_v_kind(kind);

  // MODE 2 unit = one slab (rows [k0, k1) of a long history) of a.work;
  // MODE 1 units below a.n_split fold their slabs instead of gathering
  int64_t r0 = 0, nrow = 0, e = 0, h = 0, p0 = 0, kbase = 0, klim = 0;
  bool fin = false;
  if (MODE == 0) {
    r0 = g.row0 + unit * rpb;
    int64_t r1 = r0 + rpb;
    if (r1 > g.row0 + g.n) r1 = g.row0 + g.n;
    nrow = r1 > r0 ? r1 - r0 : 0;
    klim = nrow;
  } else {
    SplitWork sw{};
    if (MODE == 2) sw = a.work[unit];
    const QueueRec rec = a.order[MODE == 2 ? (int64_t)sw.pos : pos0 + unit];
    e = rec.entity;
    h = rec.h;
    p0 = rec.p0;
    if (h == 0) return;  // untouched entity (no barrier passed yet)
    int64_t extra = 0;
    if (vk && a.quirk && h > 128 && (h % 128) != 0) extra = 128 - (h % 128);
    nrow = h + extra;
    klim = nrow;
    if (MODE == 2) {
      kbase = sw.k0;
      klim = sw.k1;
    } else {
      fin = pos0 + unit < a.n_split;
    }
  }
  const int nchunks = fin ? 0 : (int)((klim - kbase + W2R - 1) / W2R);

  auto ring_load = [&](int c, int& id, float& sa, float& bw) __attribute__((always_inline)) {
    const int64_t k = kbase + (int64_t)c * W2R + tid;
    id = -1;
    sa = 0.0f;
    bw = 0.0f;
    if (k < klim) {
      if (MODE == 0) {
        id = (int)(r0 + k);
        sa = 1.0f;
        bw = g.w ? g.w[r0 + k] : 1.0f;  // weight of the B operand
      } else {
        id = a.col[p0 + wide_virt_pos(k, h)];
        if (vk) {  // rows pre-scaled by sqrt(nu); rhs weight nu / sqrt(nu) (safer2.h:190-192)
          const float nu = a.other_weight[id];
          sa = sqrtf(nu);
          bw = (k < h && sa > 0.0f) ? nu / sa : 0.0f;
        } else {
          sa = 1.0f;
          bw = 1.0f;
        }
      }
    }
  };
  // the same split in two stages for the main loop, every load unconditional
  // (past the end it re-reads the last row; the selects come at use): the
  // row id of chunk c, then its weight operand (other_weight[id] for the V
  // kinds, the row weight of a weighted Gramian), then the finished values
  auto ring_idl = [&](int c) __attribute__((always_inline)) {
    const int64_t k = kbase + (int64_t)c * W2R + tid;
    const int64_t kc = k < klim ? k : klim - 1;
    if (MODE == 0) return (int)(r0 + kc);
    return a.col[p0 + wide_virt_pos(kc, h)];
  };
  auto ring_wraw = [&](int c, int id) __attribute__((always_inline)) {
    const int64_t k = kbase + (int64_t)c * W2R + tid;
    const int64_t kc = k < klim ? k : klim - 1;
    if (MODE == 0) return g.w ? g.w[r0 + kc] : 1.0f;
    return vk ? a.other_weight[id] : 1.0f;
  };
  auto ring_fin = [&](int c, int& id, float w, float& sa, float& bw) __attribute__((always_inline)) {
    const int64_t k = kbase + (int64_t)c * W2R + tid;
    if (k >= klim) {
      id = -1;
      sa = 0.0f;
      bw = 0.0f;
    } else if (MODE == 0) {
      sa = 1.0f;
      bw = w;
    } else if (vk) {
      sa = sqrtf(w);
      bw = (k < h && sa > 0.0f) ? w / sa : 0.0f;
    } else {
      sa = 1.0f;
      bw = 1.0f;
    }
  };
  auto ring_store = [&](int c, int id, float sa, float bw) __attribute__((always_inline)) {
    const int sl = (c % W2RING) * W2R + tid;
    ring_id[sl] = id;
    ring_sb[sl] = make_float2(sa, bw);
  };
  const float* X = MODE == 0 ? g.X : a.X;
  // staging role: column sc of the staged image, rows 8*hh0 .. 8*hh0 + 8*nh - 1
  const int sc = same ? (tid & (WB2 - 1)) : tid;
  const int hh0 = same ? (tid >> 8) : 0;
  const int xcol = sc < WB2 ? WB2 * BI + sc : WB2 * BJ + (sc - WB2);
  const bool wside = MODE == 0 && !same && sc >= WB2;  // weighted B operand
  const bool bown = MODE >= 1 && dgp;                  // diagonal pairs form b
  // the staged rows of the next chunk, loaded one iteration before it is staged
  float xr0[16], xr1[W2AH == 2 ? 16 : 1];
  auto load = [&](int c, float (&xr)[16]) __attribute__((always_inline)) {
    const int base = (c % W2RING) * W2R + 8 * hh0;
    const int4* ids4 = reinterpret_cast<const int4*>(ring_id + base);  // base % 8 == 0
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (same && q >= 2) break;
      const int4 i4 = ids4[q];
      const int id[4] = {i4.x, i4.y, i4.z, i4.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        // no select on the loaded value (rows past the end have sa = 0): the
        // loads stay in flight through the MFMAs of the current chunk.  32-bit
        // element offsets while rows x Dp < 2^32 (OFF64 above: gather_off64)
        float v;
        if constexpr (OFF64)
          v = X[(int64_t)max(id[j], 0) * Dp + xcol];
        else
          v = X[(unsigned)max(id[j], 0) * (unsigned)Dp + (unsigned)xcol];
        xr[4 * q + j] = FRECSYS_SKIP(a.debug_skip, 32) ? 0.0f : v;
      }
    }
  };
  float bpart = 0.0f, btot = 0.0f;
  // staging math of one value (row r of the thread's column): scale, rhs
  // part, 3-piece split into the fragment being assembled
  auto stage_val = [&](const float (&xr)[16], int base, int r, bf16x8 (&f)[3], int j)
                       __attribute__((always_inline)) {
    // no contraction: x is the rounded fp32 product in every instantiation
    // (fused into split3's x - hi it would depend on the code around it)
#pragma clang fp contract(off)
    const float2 sb = ring_sb[base + r];
    float x = xr[r] * sb.x;
    if (bown) bpart += sb.y * x;
    if (wside) x *= sb.y;
    __bf16 ph, pm, pl;
    if (FRECSYS_SKIP(a.debug_skip, 1024)) {  // ablation: one conversion, no split
      ph = (__bf16)x;
      pm = ph;
      pl = ph;
    } else {
      split3(x, ph, pm, pl);
    }
    f[0][j] = ph;
    f[1][j] = pm;
    f[2][j] = pl;
  };
  // the whole chunk at once (prologue)
  auto stage_write = [&](const float (&xr)[16], int buf, int c) __attribute__((always_inline)) {
    const int base = (c % W2RING) * W2R + 8 * hh0;
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      if (same && hh > 0) break;
      bf16x8 f[3];
#pragma unroll
      for (int j = 0; j < 8; ++j) stage_val(xr, base, 8 * hh + j, f, j);
#pragma unroll
      for (int p = 0; p < 3; ++p) stage[buf][g2(p, hh0 + hh, sc)] = f[p];
    }
  };

  // tiles of this wave (block-local 32x32 tile coordinates): tile row I, all
  // 8 tile columns J (J <= I on a diagonal pair).  I = w for waves 0..3 and
  // 11 - w for 4..7, so the two waves of a SIMD (w, w + 4) hold rows
  // summing to 7: 9 tiles per SIMD on a diagonal pair, 16 on the others.
  constexpr int MT = 8;
  const int tI = wave < 4 ? wave : 11 - wave;
  auto tv = [&](int m) __attribute__((always_inline)) {  // wave-uniform
    return !dgp || m <= tI;
  };
  const int boff = same ? 0 : WB2;  // B operand columns in the staged image

  float* const otile0 = MODE == 0   ? g.partials + unit * NT * 1024
                        : MODE == 1 ? ws + unit * ((int64_t)NT * 1024 + Dp)
                                    : nullptr;  // MODE 2 never flushes (<= W2FLUSH chunks)
  auto otile = [&](int m) __attribute__((always_inline)) {
    return otile0 + (int64_t)tidx(8 * BI + tI, 8 * BJ + m) * 1024;
  };
  bool flushed = false;
  f32x16 acc[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) acc[m] = f32x16{0.f};
  auto flush = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      if (tv(m)) {  // wave-uniform
        float* t = otile(m);
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          float* pq = t + acc_row(q, hi) * 32 + lo;
          *pq = flushed ? *pq + acc[m][q] : acc[m][q];
        }
      }
      acc[m] = f32x16{0.f};
      __builtin_amdgcn_sched_barrier(0);
    }
    flushed = true;
  };

  if (tid < W2R) {
#pragma unroll
    for (int c = 0; c < 2 + W2AH; ++c)
      if (c < nchunks) {
        int id;
        float sa, bw;
        ring_load(c, id, sa, bw);
        ring_store(c, id, sa, bw);
      }
  }
  lds_barrier();
  if (nchunks > 0) {
    load(0, xr0);
    stage_write(xr0, 0, 0);
  }
  // ring pipeline of the wave-0 threads, issued at the end of each iteration
  // before the rows it gathers (so that waiting for those rows, in order,
  // never waits for a ring load younger than them): chunk x's id at the end
  // of iteration x-5, its weight operand at the end of x-4 (the id an
  // iteration old), the finished values stored at the end of x-3
  // (with W2AH = 2 every distance one chunk longer)
  int idA = -1, idB = -1;  // chunks c+3+W2AH (id in flight) and c+2+W2AH (id, weight)
  float wB = 0.0f;
  if (tid < W2R && nchunks > 2 + W2AH) {
    idB = ring_idl(2 + W2AH);
    wB = ring_wraw(2 + W2AH, idB);
  }
  if (tid < W2R && nchunks > 3 + W2AH) idA = ring_idl(3 + W2AH);
  if constexpr (W2AH == 2) {
    if (nchunks > 1) load(1, xr1);
    if (nchunks > 2) load(2, xr0);
  } else {
    if (nchunks > 1) load(1, xr0);
  }
  lds_barrier();

#ifdef FRECSYS_ABLATION
  // diagnostics (FRECSYS_DUAL_PROF, ablation builds): per-chunk phase cycles
  // of waves 0 and 7 (MFMA + staging loop, ring + row-load issue, barrier)
  const bool tprof = MODE == 1 && a.prof && lane == 0 && (wave == 0 || wave == 7);
  unsigned long long tp_t = tprof ? clock64() : 0, tp_acc[3] = {0, 0, 0};
  auto tp_mark = [&](int i) __attribute__((always_inline)) {
    if (tprof) {
      const unsigned long long t = clock64();
      tp_acc[i] += t - tp_t;
      tp_t = t;
    }
  };
#else
  auto tp_mark = [](int) {};
#endif
  // chunk c: the MFMAs of its tiles, with chunk c+1's staging math (rows
  // loaded one iteration ago) spread over the gaps between them -- a slice
  // of NV/8 values after each tile, a granule group stored once complete --
  // instead of a VALU phase of its own after the MFMAs
  // iteration c: xr holds chunk c+1 (staged now), and then takes chunk c+2
  auto body = [&](auto same_c, int c, float (&xr)[16]) __attribute__((always_inline)) {
      constexpr bool SAME = decltype(same_c)::value;
      constexpr int NV = SAME ? 8 : 16, PER = NV / MT;
      const int buf = c & 1;
      const bool live = c < nchunks;  // W2AH = 2: the loop runs an even count
      const bool more = c + 1 < nchunks;
      const bool ring_more = (tid < W2R) && (c + 2 + W2AH < nchunks);
      const bf16x8* st = stage[buf];
      bf16x8* sto = stage[buf ^ 1];
      const int nbase = ((c + 1) % W2RING) * W2R + 8 * hh0;
      // b's block boundary matches the tiles' (chunks <= c; chunk c+1 is
      // staged below), so 2048-row slabs fold into the same sums
      if ((c + 1) % W2FLUSH == 0 && more) {  // block-uniform
        btot += bpart;
        bpart = 0.0f;
      }
      // A fragments of the wave's tile row, shared by its tiles; B fragments
      // one tile ahead of their MFMAs
      bf16x8 af[3], bcur[3], fs[3];
      [[maybe_unused]] bf16x8 bnxt[W2AH == 2 ? 1 : 3];
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        af[p] = st[g2(p, hi, 32 * tI + lo)];
        bcur[p] = st[g2(p, hi, boff + lo)];
      }
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        if (tv(m) && live) {
          if constexpr (W2AH == 2) {
            // no second fragment set (the registers hold the second chunk
            // of rows): tile m+1's B fragments read after tile m's MFMAs
            if (!FRECSYS_SKIP(a.debug_skip, 1)) acc[m] = mfma_x6(af, bcur, acc[m]);
            if (m + 1 < MT) {
#pragma unroll
              for (int p = 0; p < 3; ++p) bcur[p] = st[g2(p, hi, boff + 32 * (m + 1) + lo)];
            }
          } else {
            if (m + 1 < MT) {
#pragma unroll
              for (int p = 0; p < 3; ++p) bnxt[p] = st[g2(p, hi, boff + 32 * (m + 1) + lo)];
            }
            if (!FRECSYS_SKIP(a.debug_skip, 1)) acc[m] = mfma_x6(af, bcur, acc[m]);
#pragma unroll
            for (int p = 0; p < 3; ++p) bcur[p] = bnxt[p];
          }
        }
        if (more) {  // block-uniform
#pragma unroll
          for (int u = 0; u < PER; ++u) {
            const int r = m * PER + u;
            stage_val(xr, nbase, r, fs, r & 7);
          }
          if ((m * PER + PER) % 8 == 0) {
            const int hh = (m * PER) >> 3;
#pragma unroll
            for (int p = 0; p < 3; ++p) sto[g2(p, hh0 + hh, sc)] = fs[p];
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      if ((c + 1) % W2FLUSH == 0 && more) flush();  // block-uniform
      tp_mark(0);
      // the ring slot first: its store waits (vmcnt) for the ring loads, and
      // placed after load(c+2) that wait -- in-order counters, a conditional
      // load between -- was vmcnt(0), wave 0 stalling on the rows it had just
      // requested (a full HBM latency per chunk, every wave behind it at the
      // barrier).  Chunk c+3's values were loaded an iteration ago.
      if (ring_more) {
        float sa, bw;
        int id = idB;
        ring_fin(c + 2 + W2AH, id, wB, sa, bw);
        ring_store(c + 2 + W2AH, id, sa, bw);
      }
      if (tid < W2R && c + 3 + W2AH < nchunks) {
        idB = idA;
        wB = ring_wraw(c + 3 + W2AH, idA);
      }
      if (tid < W2R && c + 4 + W2AH < nchunks) idA = ring_idl(c + 4 + W2AH);
      // unconditional (past the end it re-gathers the last chunk, whose ring
      // slot stays valid; never staged): a conditional load here made the
      // waitcnt pass flush vmcnt at the loop head, stalling on these rows
      load(c + 1 + W2AH < nchunks ? c + 1 + W2AH : nchunks - 1, xr);
      tp_mark(1);
      lds_barrier();
      tp_mark(2);
  };
  auto run = [&](auto same_c) __attribute__((always_inline)) {
    if constexpr (W2AH == 2) {
      // both register sets in one unconditional body pair (an odd count runs
      // one idle step): a conditional second step made the compiler wait for
      // every outstanding row load, one chunk of prefetch in effect
      for (int c = 0; c < nchunks; c += 2) {
        body(same_c, c, xr1);
        body(same_c, c + 1, xr0);
      }
    } else {
      for (int c = 0; c < nchunks; ++c) body(same_c, c, xr0);
    }
  };
  if (same) run(std::true_type{});
  else run(std::false_type{});
#ifdef FRECSYS_ABLATION
  if (tprof) {
    const int o = (wave == 7 ? 4 : 0) + (dgp ? 8 : 0);
    atomicAdd(a.prof + o + 0, tp_acc[0]);
    atomicAdd(a.prof + o + 1, tp_acc[1]);
    atomicAdd(a.prof + o + 2, tp_acc[2]);
    atomicAdd(a.prof + o + 3, (unsigned long long)nchunks);
  }
#endif
  if (flushed) {
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      if (tv(m)) {
        const float* t = otile(m);
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[m][q] += t[acc_row(q, hi) * 32 + lo];
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  // slab layout: tile t's accumulator q of lane l at t * 1024 + q * 64 + l
  // (coalesced); b partials of the diagonal pairs' threads after the tiles
  const size_t slab_floats = (size_t)NT * 1024 + 2 * (size_t)Dp;
  auto stile = [&](const float* sb, int m) __attribute__((always_inline)) {
    return sb + (int64_t)tidx(8 * BI + tI, 8 * BJ + m) * 1024 + lane;
  };
  if (MODE == 2) {
    float* sb = a.slabs + (size_t)a.work[unit].slab * slab_floats;
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      if (tv(m)) {
        float* t = const_cast<float*>(stile(sb, m));
#pragma unroll
        for (int q = 0; q < 16; ++q) t[q * 64] = acc[m][q];
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if (bown) sb[(size_t)NT * 1024 + WB2 * 2 * BI + tid] = bpart;
    return;
  }
  if (MODE == 1 && fin) {
    // the unsplit kernel's two-level sum: block sums folded left to right
    // (t = s_1, t = t + s_j, ..., s_last + t), b likewise from 0
    // (the next tile's slab values in flight under each add, across slabs)
    const int2 sp = a.split[pos0 + unit];
    f32x16 nx;
    auto lds_ = [&](int j, int m) __attribute__((always_inline)) {
      if (j < sp.y && tv(m)) {
        const float* t = stile(a.slabs + (size_t)(sp.x + j) * slab_floats, m);
#pragma unroll
        for (int q = 0; q < 16; ++q) nx[q] = t[q * 64];
      }
    };
    lds_(0, 0);
#pragma unroll 1
    for (int j = 0; j < sp.y; ++j) {
      const float* sb = a.slabs + (size_t)(sp.x + j) * slab_floats;
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const f32x16 v = nx;
        if (m + 1 < MT) lds_(j, m + 1);
        else lds_(j + 1, 0);
        if (tv(m)) acc[m] = j == 0 ? v : acc[m] + v;
        __builtin_amdgcn_sched_barrier(0);
      }
      if (bown) {
        const float bv = sb[(size_t)NT * 1024 + WB2 * 2 * BI + tid];
        if (j + 1 < sp.y) btot += bv;
        else bpart = bv;
      }
    }
  }
  bpart += btot;

  if (MODE == 0) {
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      if (tv(m)) {
        float* t = otile(m);
#pragma unroll
        for (int q = 0; q < 16; ++q) t[acc_row(q, hi) * 32 + lo] = acc[m][q];
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    return;
  }

  // epilogue: the G part and the per-kind finish of A (as solve.hip)
  const float hf = (float)h;
  const float omega = (is_u_kind(kind) && a.entity_weight) ? a.entity_weight[e] : 1.0f;
  const float lam = entity_lambda(kind, a.reg, a.reg_exp, a.w, a.alpha, h, a.n_other,
                                  a.entity_reg, e, a.lambda_is_reg);
  const bool grad = is_grad_kind(kind);
  const float gscale = kind == KIND_IALS ? a.w : (is_u_kind(kind) ? hf * a.w : a.w);
  const float us = omega / hf;
  // the kind is dispatched once, outside the element loops (a per-element
  // kind test compiles into scalar branches per element)
  auto finish = [&](auto mode_c) __attribute__((always_inline)) {
    constexpr int FM = decltype(mode_c)::value;  // 0 iALS, 1 U kinds, 2 V kinds, 3 CVaR
    // G values one tile ahead: tile m+1's loads are in flight while tile m
    // is finished and stored (one HBM round trip per epilogue, not one per tile)
    float gnx[16];
    auto ldg = [&](int m) __attribute__((always_inline)) {
      if (tv(m)) {
        const int I = 8 * BI + tI, J = 8 * BJ + m;
#pragma unroll
        for (int q = 0; q < 16; ++q)
          gnx[q] = a.G[(int64_t)(32 * I + acc_row(q, hi)) * Dp + 32 * J + lo];
      }
    };
    ldg(0);
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      float gcur[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) gcur[q] = gnx[q];
      if (m + 1 < MT) ldg(m + 1);
      if (tv(m)) {
        float* t = otile(m);
        const int I = 8 * BI + tI, J = 8 * BJ + m;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int i = acc_row(q, hi);
          const int gi = 32 * I + i, gj = 32 * J + lo;
          const bool dg = gi == gj;
          float v = acc[m][q];
          const float gv = gcur[q];
          if constexpr (FM == 3) {
            v = assemble(kind, v, gv, dg, a.w, lam, hf, omega);
          } else {
            float g0 = gscale * gv;
            if constexpr (FM == 0) g0 += dg ? lam : 0.0f;
            v = g0 + v;  // accumulators started from the G part in the fp32 kernels
            if constexpr (FM == 1) v = v * us + (dg ? lam : 0.0f);
            if constexpr (FM == 2) v = v + (dg ? lam : 0.0f);
          }
          t[i * 32 + lo] = v;
        }
      }
      __builtin_amdgcn_sched_barrier(0);  // two tiles' G loads live at a time
    }
  };
  if (grad) finish(std::integral_constant<int, 3>{});
  else if (is_u_kind(kind)) finish(std::integral_constant<int, 1>{});
  else if (vk) finish(std::integral_constant<int, 2>{});
  else finish(std::integral_constant<int, 0>{});
  if (bown) {  // b of this diagonal block: the two row halves of each column
    if (tid >= WB2) bred[sc] = bpart;
    lds_barrier();
    if (tid < WB2) {
      float b = bpart + bred[tid];
      if (is_u_kind(kind)) b *= us;  // rhs *= weight / history_size
      ws[unit * ((int64_t)NT * 1024 + Dp) + (int64_t)NT * 1024 + WB2 * BI + tid] = b;
    }
  }
}

__global__ void __launch_bounds__(256)
    wide_gram_reduce_kernel(const float* __restrict__ P, int64_t nblk, float* __restrict__ G,
                            int Dp) {
  const int64_t el = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (el >= (int64_t)Dp * Dp) return;
  const int gi = (int)(el / Dp), gj = (int)(el % Dp);
  if (gi < gj) return;
  const int T = Dp >> 5, NT = T * (T + 1) / 2;
  const int64_t off = (int64_t)tidx(gi >> 5, gj >> 5) * 1024 + (gi & 31) * 32 + (gj & 31);
  float s = 0.0f;
  for (int64_t b = 0; b < nblk; ++b) s += P[b * NT * 1024 + off];
  G[(int64_t)gi * Dp + gj] = s;
  G[(int64_t)gj * Dp + gi] = s;
}

// ---- back substitution x_p = L_pp^-T (y_p - sum_{q>p} L_qp^T x_q) over the
// factor in the workspace slot (diagonal tiles hold L_pp^-1), 8 waves.
// The substitutions of both Cholesky kernels use explicit fmaf: left to
// contraction, the compiler pairs some of these products into v_pk_mul_f32
// (rounded, then added) differently in each kernel, and the two kernels'
// y differed in the last bit in about one element in 500 ----
template <int T, int NW = 8>
__device__ __forceinline__ void wide_back_subst(float* slot, const float* yv, float* xv,
                                                float* part, int wave, int lo, int hi,
                                                int te = T) {
  auto gtile = [&](int I, int J) { return slot + (int64_t)tidx(I, J) * 1024; };
#pragma unroll 1
  for (int p = te - 1; p >= 0; --p) {
    // every workspace load of the step is issued before the first use (the
    // x-independent L values: one HBM round trip per step instead of one per
    // four values); the summation orders are unchanged
    float li[32];
    if (wave == 0) {
      const float* Li = gtile(p, p);
#pragma unroll
      for (int i = 0; i < 32; ++i) li[i] = Li[i * 32 + lo];
    }
    float pr = 0.0f;
    for (int q = p + 1 + wave; q < te; q += NW) {
      const float* L = gtile(q, p) + 16 * hi * 32 + lo;
      float lv[16];
#pragma unroll
      for (int mm = 0; mm < 16; ++mm) lv[mm] = L[mm * 32];
#pragma unroll
      for (int mm = 0; mm < 16; ++mm) pr = __builtin_fmaf(lv[mm], xv[32 * q + 16 * hi + mm], pr);
    }
    pr += __shfl_xor(pr, 32);
    if (hi == 0) part[wave * 32 + lo] = pr;
    lds_barrier();
    if (wave == 0) {
      float r = yv[32 * p + lo];
#pragma unroll
      for (int w = 0; w < NW; ++w) r -= part[w * 32 + lo];
      float x = 0.0f;
#pragma unroll
      for (int i = 0; i < 32; ++i) x = __builtin_fmaf(li[i], rdlane(r, i), x);
      if (hi == 0) xv[32 * p + lo] = x;
    }
    lds_barrier();
  }
}

// One workgroup (8 waves) per entity of the batch: A x = b with A's lower
// tiles in the entity's workspace slot (row-major 32x32 tiles, tidx order),
// left-looking blocked Cholesky.  Panel p
//   A  row p of L (tiles (p, q), q < p, final) into LDS, swizzled;
//   B  wave 0: D = A_pp - sum_q L_pq L_pq^T, factored + inverted in LDS
//      (diag_factor_inv) and L_pp^-1 stored back for the back substitution;
//      wave 1 first: r_p = b_p - sum_q L_pq y_q;
//      waves 1..7, tiles I > p round-robin: C_I = (A_Ip - sum_q L_Iq L_pq^T)^T
//      in accumulator registers, L_Iq streamed from the workspace straight
//      into MFMA operand registers (k-order of that product: lane half hi
//      takes k = 16 hi + s, i.e. 4 float4 loads of its row);
//   C  waves 1..7: L_Ip = C_I^T L_pp^-T, C_I used as the MFMA A operand as it
//      sits in the accumulators (k = acc_row(s, hi)); wave 0: y_p = L_pp^-1 r_p.
// Each tile of A is read once and each tile of L written once; L tiles are
// re-read by later panels: ~T^3/6 tile reads + T^2/2 writes per entity
// against ~T^3/3 reads and T^3/3 writes of a right-looking update sweep
// (round 2's kernel: MSD 174 GB of workspace traffic per epoch, 37 ms; this
// one 30.5 ms).  Compiled for two workgroups per CU (128 registers).
template <int T, int NW = 8>
__global__ void __launch_bounds__(64 * NW)
    __attribute__((amdgpu_waves_per_eu(NW == 4 ? 2 : (T == 16 ? kWideCholWPE : 2), 8)))
    wide_chol_kernel(SolveArgs a, int64_t pos0, float* ws, int slot_out) {
  constexpr int Dp = 32 * T, NT = T * (T + 1) / 2, NTHR = 64 * NW;
  typedef float f32x4v __attribute__((ext_vector_type(4)));
  extern __shared__ __attribute__((aligned(16))) float smem[];
  // LDS tiles of row p of L and of L_pp^-1 are row-major with a 33-float
  // row stride (lane lo reads row lo at immediate offsets, conflict-free);
  // the diagonal factor works on its own swizzled tile
  constexpr int LP = 33 * 32;
  float* rowL = smem;                   // [T-1][LP], row p of L
  float* dpad = rowL + (T - 1) * LP;    // L_pp^-1
  float* dinv = dpad + LP;              // swizzled factor tile
  float* yv = dinv + 1024;              // b, then y
  float* xv = yv + Dp;
  float* rv = xv + Dp;                  // r_p
  float* part = rv + 32;                // NW x 32 back-substitution partials
  int* flag = reinterpret_cast<int*>(part + NW * 32);
  const int tid = threadIdx.x, lane = tid & 63, lo = lane & 31, hi = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const QueueRec rec = a.order[pos0 + blockIdx.x];
  const int64_t e = rec.entity;
  if (rec.h == 0) return;
  // slot_out (the history-space wide bucket's S): only the tiles holding
  // the h_eff rows are factored -- the padding is the identity with a zero
  // rhs, so its solution is 0 (2: ProjectV with the tail quirk's rows)
  int te = T;
  if (slot_out) {
    int64_t heff = rec.h;
    if (slot_out == 2 && heff > 128 && (heff % 128) != 0) heff += 128 - (heff % 128);
    te = (int)min<int64_t>(T, (heff + 31) / 32);
  }
  float* slot = ws + (int64_t)blockIdx.x * ((int64_t)NT * 1024 + Dp);
  auto gtile = [&](int I, int J) { return slot + (int64_t)tidx(I, J) * 1024; };
  for (int i = tid; i < Dp; i += NTHR) yv[i] = slot[(int64_t)NT * 1024 + i];
  if (tid == 0) flag[0] = 0;
  __syncthreads();

  // C_I = (A_Ip - sum_{q<p} L_Iq L_pq^T)^T in accumulator registers: A_Ip^T
  // as its rows, L_Iq streamed from the workspace into operand registers
  // (k = 16 hi + s), a ring of PF tiles: the loads of tiles q+1 .. q+PF-1
  // in flight under the product of tile q (the loop unrolled by PF so that
  // every ring slot is a fixed set of registers)
  constexpr int PF = T == 16 ? 2 : 4;
  // T = 32: split-bf16 products (common.h mfma_x6, fp32-accurate) with the
  // operands split in registers; T = 16 keeps f32 MFMA (at 128 registers the
  // splits spill, and its time was unchanged)
  constexpr bool X6 = T == 32 || NW == 4;
  auto panel_sum = [&](int I, int p) __attribute__((always_inline)) {
    const float* Aip = gtile(I, p) + lo * 32 + 4 * hi;
    f32x16 c;
#pragma unroll
    for (int g = 0; g < 4; ++g) {  // row lo, columns acc_row(4g + j, hi)
      const f32x4v v = *reinterpret_cast<const f32x4v*>(Aip + 8 * g);
#pragma unroll
      for (int j = 0; j < 4; ++j) c[4 * g + j] = v[j];
    }
    f32x4v ring[PF][4];
    auto ld = [&](int q, f32x4v(&dst)[4]) __attribute__((always_inline)) {
      if constexpr (X6) {  // k = 16 g + 8 hi + t of row lo (the bf16 MFMA operand layout)
        const float* L = gtile(I, q) + lo * 32 + 8 * hi;
        dst[0] = *reinterpret_cast<const f32x4v*>(L);
        dst[1] = *reinterpret_cast<const f32x4v*>(L + 4);
        dst[2] = *reinterpret_cast<const f32x4v*>(L + 16);
        dst[3] = *reinterpret_cast<const f32x4v*>(L + 20);
      } else {  // k = 16 hi + s
        const f32x4v* L = reinterpret_cast<const f32x4v*>(gtile(I, q) + lo * 32 + 16 * hi);
#pragma unroll
        for (int j = 0; j < 4; ++j) dst[j] = L[j];
      }
    };
#pragma unroll
    for (int j = 0; j < PF - 1; ++j)
      if (j < p) ld(j, ring[j]);
#pragma unroll 1
    for (int q0 = 0; q0 < p; q0 += PF) {
#pragma unroll
      for (int j = 0; j < PF; ++j) {
        const int q = q0 + j;
        if (q < p) {
          if (q + PF - 1 < p) ld(q + PF - 1, ring[(j + PF - 1) % PF]);
          if constexpr (X6) {
            const float* P = rowL + q * LP + lo * 33 + 8 * hi;
#pragma unroll
            for (int g = 0; g < 2; ++g) {
              float pv[8], lv[8];
#pragma unroll
              for (int t = 0; t < 8; ++t) {
                pv[t] = -P[16 * g + t];
                lv[t] = ring[j][2 * g + (t >> 2)][t & 3];
              }
              bf16x8 pf[3], lf[3];
              split3x8(pv, pf);
              split3x8(lv, lf);
              c = mfma_x6(pf, lf, c);
            }
          } else {
            const float* P = rowL + q * LP + lo * 33 + 16 * hi;
#pragma unroll
            for (int s2 = 0; s2 < 16; ++s2) c = mfma32(-P[s2], ring[j][s2 >> 2][s2 & 3], c);
          }
        }
      }
    }
    return c;
  };

#pragma unroll 1
  for (int p = 0; p < te; ++p) {
    // ---- A: row p of L (the thread's loads issued four at a time, each
    // unconditional -- past the row it re-reads tile (p, 0) and drops it --
    // so a panel costs two HBM round trips, not one per float4) ----
    {
      constexpr int NA = ((T - 1) * 256 + NTHR - 1) / NTHR, NB = 4;
      const int n = p * 256;
#pragma unroll
      for (int k0 = 0; k0 < NA; k0 += NB) {
        if (tid + NTHR * k0 < n) {  // wave-uniform (n is a multiple of 256)
          float4 v[NB];
#pragma unroll
          for (int k = 0; k < NB; ++k) {
            const int i = tid + NTHR * (k0 + k);
            const int ii = i < n ? i : tid;
            const int q = ii >> 8, r = (ii >> 3) & 31, c = (ii & 7) * 4;
            v[k] = *reinterpret_cast<const float4*>(gtile(p, q) + r * 32 + c);
          }
#pragma unroll
          for (int k = 0; k < NB; ++k) {
            const int i = tid + NTHR * (k0 + k);
            if (i < n) {
              const int q = i >> 8, r = (i >> 3) & 31, c = (i & 7) * 4;
              float* t = rowL + q * LP + r * 33 + c;
              t[0] = v[k].x;
              t[1] = v[k].y;
              t[2] = v[k].z;
              t[3] = v[k].w;
            }
          }
        }
      }
    }
    __syncthreads();
    // ---- B ----
    f32x16 acc0;
    if (wave == 0) {
      const float* App = gtile(p, p);
      f32x16 d;
#pragma unroll
      for (int q = 0; q < 16; ++q) d[q] = App[acc_row(q, hi) * 32 + lo];
#pragma unroll 1
      for (int q = 0; q < p; ++q) {  // d -= L_pq L_pq^T
        if constexpr (X6) {
          const float* P = rowL + q * LP + lo * 33 + 8 * hi;  // k = 16 g + 8 hi + t
#pragma unroll
          for (int g = 0; g < 2; ++g) {
            float pv[8], nv[8];
#pragma unroll
            for (int t = 0; t < 8; ++t) {
              pv[t] = P[16 * g + t];
              nv[t] = -pv[t];
            }
            bf16x8 pf[3], nf[3];
            split3x8(pv, pf);
            split3x8(nv, nf);
            d = mfma_x6(nf, pf, d);
          }
        } else {
          const float* P = rowL + q * LP + lo * 33 + 16 * hi;  // k = 16 hi + s
#pragma unroll
          for (int s2 = 0; s2 < 16; ++s2) d = mfma32(-P[s2], P[s2], d);
        }
      }
      // opaque copies of the lane coordinates: the 48 swizzled / padded
      // addresses below are formed here with a few VALU ops each, not hoisted
      // out of the panel loop (at 128 registers they were spilled, and every
      // store of this chain-critical block then waited on a scratch reload)
      int lo_o, hi_o;
      asm volatile("v_mov_b32 %0, %1" : "=v"(lo_o) : "v"(lo));
      asm volatile("v_mov_b32 %0, %1" : "=v"(hi_o) : "v"(hi));
#pragma unroll
      for (int q = 0; q < 16; ++q) dinv[sw(acc_row(q, hi_o), lo_o)] = d[q];
      wave_lds_sync();
      if (!diag_factor_inv(dinv, lane) && lane == 0) flag[0] = 1;
      wave_lds_sync();
      float* Aw = gtile(p, p);  // L_pp^-1 for the back substitution, and its padded copy
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int r = 2 * i + hi_o;
        const float v = dinv[sw(r, lo_o)];
        Aw[r * 32 + lo_o] = v;
        dpad[r * 33 + lo_o] = v;
      }
    } else {
      if (wave == 1) {
        float r = 0.0f;
#pragma unroll 1
        for (int q = 0; q < p; ++q) {  // row lo of L_pq . y_q, k halves by hi
          const float* L = rowL + q * LP + lo * 33 + 16 * hi;
          const float* y = yv + 32 * q + 16 * hi;
#pragma unroll
          for (int k2 = 0; k2 < 16; ++k2) r = __builtin_fmaf(L[k2], y[k2], r);
        }
        r += __shfl_xor(r, 32);
        if (hi == 0) rv[lo] = yv[32 * p + lo] - r;
      }
      if (p + wave < te) acc0 = panel_sum(p + wave, p);  // first panel tile
    }
    __syncthreads();
    // ---- C ----
    if (wave == 0) {
      float y = 0.0f;
#pragma unroll
      for (int k2 = 0; k2 < 16; ++k2) y = __builtin_fmaf(dpad[lo * 33 + 16 * hi + k2], rv[16 * hi + k2], y);
      y += __shfl_xor(y, 32);
      if (hi == 0) yv[32 * p + lo] = y;
    } else {
      // first tile from its B-phase sum, the rest sum-then-finish (L_pp^-1 is ready)
#pragma unroll 1
      for (int I = p + wave; I < te; I += NW - 1) {
        const f32x16 cI = I == p + wave ? acc0 : panel_sum(I, p);
        f32x16 l = f32x16{0.f};
#pragma unroll
        for (int s2 = 0; s2 < 16; ++s2) l = mfma32(cI[s2], dpad[lo * 33 + acc_row(s2, hi)], l);
        float* Lw = gtile(I, p);
#pragma unroll
        for (int q = 0; q < 16; ++q) Lw[acc_row(q, hi) * 32 + lo] = l[q];
      }
    }
    __syncthreads();
  }
  wide_back_subst<T, NW>(slot, yv, xv, part, wave, lo, hi, te);
  // slot_out: the solution of slot b into out[Dp b ..) (the history-space
  // wide bucket's S systems), else into the entity's row
  const int64_t orow = slot_out ? (int64_t)blockIdx.x : e;
  for (int i = tid; i < Dp; i += NTHR) a.out[orow * Dp + i] = i < 32 * te ? xv[i] : 0.0f;
  if (tid == 0 && flag[0]) atomicMin(a.fail, (unsigned long long)(e + 1));
}

// ---- the same factorisation, two panels per pass (Dp = 1024) ----
// wide_chol_kernel streams L_Iq from the workspace once per product: at
// Dp = 1024 the working set (2.2 MB per entity, one entity per CU) lives in
// HBM, and its panel sums fetch 4 KB per 32x32x32 product -- ~157 GB per
// launch at config 5, 4.1 TB/s, MFMA busy 0.21.  Here panels p and p+1 are
// summed together, so every streamed L_Iq feeds two products:
//   U  waves 0..6 (workers) hold C_Ip^T and C_I,p+1^T for up to NI tiles
//      I >= p+2 each (more tiles: another pass over q); rows p and p+1 of L
//      come through LDS in chunks of QC tiles (LDS-DMA one chunk ahead), and
//      each chunk is split once into a negated 3-piece bf16 image that every
//      wave reads as MFMA operands (two barriers per chunk); L_Iq from the
//      workspace in a RING-deep register ring.  Wave 7 (the diagonal wave)
//      sums the diagonal block: A_pp, A_p+1,p, A_p+1,p+1 and the
//      forward-substitution dots r_p, r_p+1.
//   D  wave 7: L_pp^-1 (diag_factor_inv); | workers: L_Ip = C_Ip^T L_pp^-T;
//      L_p+1,p (into LDS);                | workers: C_I,p+1 -= L_Ip L_p+1,p^T;
//      L_p+1,p+1^-1, y_p, y_p+1;          | workers: L_I,p+1.
// Every product, operand split and summation runs in wide_chol_kernel<T>'s
// order on the same values (split-bf16 mfma_x6 sums over q ascending, the
// f32 finishes, the fmaf dot chains): bit-identical to it.
// Configuration (every one bit-identical): QC q tiles per staged chunk, NI
// tiles per worker per pass, RING workspace tiles in flight per worker, WPE
// waves per SIMD the registers are sized for.  Measured at config 5,
// streams serialised: <6, 2, 6, 2> (one workgroup per CU, 256 registers)
// 26.8 ms per launch; <2, 1, 2, 4> (two workgroups per CU, 128 registers,
// 66 KB of LDS each) 30.6 ms; the one-panel kernel 31.9 ms
// (profiles/r06/wide_chol2/)
template <int QC_, int NI_, int RING_, int WPE_>
struct Chol2Cfg {
  static constexpr int QC = QC_, NI = NI_, RING = RING_, WPE = WPE_;
  static constexpr int STAGE = 2 * QC * 1024;       // rows p, p+1 x QC tiles, fp32 (common.h sw)
  static constexpr int IMG = 2 * QC * 3 * 32 * 16;  // their -split images: [tile][piece][row][4 x 8 bf16]
  static_assert(QC % 2 == 0, "split units: QC / 2 per thread");
  static_assert(8 * 33 * 32 <= STAGE + IMG, "per-wave transpose scratch inside the stages");
};
typedef Chol2Cfg<6, 2, 6, 2> Chol2Wide;
constexpr int C2_NWK = 7;                // worker waves (wave 7: the diagonal wave)
template <int T, class CF>
struct Chol2Lds {  // offsets in floats
  static constexpr int Dp = 32 * T;
  static constexpr int STG = 0;             // CF::STAGE; with IMG the finishes' transpose scratch
  static constexpr int IMG = CF::STAGE;     // CF::IMG (floats)
  static constexpr int LX = IMG + CF::IMG;  // L_p+1,p (sw layout)
  static constexpr int DP0 = LX + 1024;     // L_pp^-1 (33-float rows)
  static constexpr int DP1 = DP0 + 33 * 32; // L_p+1,p+1^-1
  static constexpr int DINV = DP1 + 33 * 32;  // factor tile (sw)
  static constexpr int YV = DINV + 1024;
  static constexpr int XV = YV + Dp;
  static constexpr int RV = XV + Dp;        // r_p, r_p+1
  static constexpr int PART = RV + 64;      // back-substitution partials
  static constexpr int FLAG = PART + 8 * 32;
  static constexpr int FLOATS = FLAG + 4;
};

// -f for the three pieces of a split (sign bits: exact)
__device__ __forceinline__ void neg3(bf16x8 (&f)[3]) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    u32x4 u = __builtin_bit_cast(u32x4, f[i]);
    u ^= 0x80008000u;
    f[i] = __builtin_bit_cast(bf16x8, u);
  }
}

// Per-phase cycle counts of wide_chol2_kernel (diagnostics: build with
// -DFRECSYS_CHOL2_PROF; workgroups 0..3 print per wave: U products, U waits
// (DMA + chunk barriers), D work, D barrier waits, pass-start syncs)
#ifdef FRECSYS_CHOL2_PROF
#define C2P_DECL unsigned long long c2p_t = clock64(), c2p[5] = {0, 0, 0, 0, 0};
#define C2P(i)                               \
  {                                          \
    const unsigned long long t_ = clock64(); \
    c2p[i] += t_ - c2p_t;                    \
    c2p_t = t_;                              \
  }
#define C2P_FLUSH                                                                          \
  if (blockIdx.x < 4 && lane == 0)                                                         \
    printf("chol2 b%d w%d U %llu Uwait %llu D %llu Dwait %llu sync %llu\n", (int)blockIdx.x, \
           wave, c2p[0], c2p[1], c2p[2], c2p[3], c2p[4]);
#else
#define C2P_DECL
#define C2P(i)
#define C2P_FLUSH
#endif

template <int T, class CF>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(CF::WPE, CF::WPE)))
    wide_chol2_kernel(SolveArgs a, int64_t pos0, float* ws, int slot_out) {
  using LY = Chol2Lds<T, CF>;
  constexpr int C2_QC = CF::QC, C2_NI = CF::NI, C2_RING = CF::RING;
  constexpr int C2_NA = C2_NI > 2 ? C2_NI : 2;  // accumulator arrays (the diagonal wave uses 3)
  constexpr int C2_STAGE = CF::STAGE;
  constexpr int Dp = 32 * T, NT = T * (T + 1) / 2;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* stg = smem + LY::STG;
  float* img = smem + LY::IMG;
  float* lx = smem + LY::LX;
  float* dp0 = smem + LY::DP0;
  float* dp1 = smem + LY::DP1;
  float* dinv = smem + LY::DINV;
  float* yv = smem + LY::YV;
  float* xv = smem + LY::XV;
  float* rv = smem + LY::RV;
  float* part = smem + LY::PART;
  int* flag = reinterpret_cast<int*>(smem + LY::FLAG);
  const int tid = threadIdx.x, lane = tid & 63;
  // lo / hi are re-made opaque (fresh) at the top of each phase: otherwise the
  // compiler hoists dozens of lane-dependent LDS / workspace offsets out of
  // the pair loop and spills them
  int lo = lane & 31, hi = lane >> 5;
  auto fresh = [&]() __attribute__((always_inline)) {
    asm volatile("" : "+v"(lo));
    asm volatile("" : "+v"(hi));
  };
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool dw = wave == C2_NWK;
  const QueueRec rec = a.order[pos0 + blockIdx.x];
  const int64_t e = rec.entity;
  if (rec.h == 0) return;
  int te = T;
  if (slot_out) {
    int64_t heff = rec.h;
    if (slot_out == 2 && heff > 128 && (heff % 128) != 0) heff += 128 - (heff % 128);
    te = (int)min<int64_t>(T, (heff + 31) / 32);
  }
  float* slot = ws + (int64_t)blockIdx.x * ((int64_t)NT * 1024 + Dp);
  auto gtile = [&](int I, int J) { return slot + (int64_t)tidx(I, J) * 1024; };
  for (int i = tid; i < Dp; i += 512) yv[i] = slot[(int64_t)NT * 1024 + i];
  if (tid == 0) flag[0] = 0;
  C2P_DECL

  // row lo of an LDS tile (sw layout), columns 16 g + 8 hi + t: the bf16
  // MFMA operand's k order
  auto prow8 = [&](const float* t, int g, float (&v)[8]) __attribute__((always_inline)) {
    const f32x4v a0 = row_gran(t, lo, 4 * g + 2 * hi), a1 = row_gran(t, lo, 4 * g + 2 * hi + 1);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[j] = a0[j];
      v[4 + j] = a1[j];
    }
  };
  // row lo of L_Iq from the workspace in the same k order
  auto ld_op = [&](int I, int q, f32x4v(&dst)[4]) __attribute__((always_inline)) {
    const float* L = gtile(I, q) + lo * 32 + 8 * hi;
    dst[0] = *reinterpret_cast<const f32x4v*>(L);
    dst[1] = *reinterpret_cast<const f32x4v*>(L + 4);
    dst[2] = *reinterpret_cast<const f32x4v*>(L + 16);
    dst[3] = *reinterpret_cast<const f32x4v*>(L + 20);
  };
  // C^T of a panel tile as wide_chol_kernel's panel_sum starts it: A_IJ^T
  auto ld_panel = [&](int I, int J) __attribute__((always_inline)) {
    const float* Aip = gtile(I, J) + lo * 32 + 4 * hi;
    f32x16 c;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4v v = *reinterpret_cast<const f32x4v*>(Aip + 8 * g);
#pragma unroll
      for (int j = 0; j < 4; ++j) c[4 * g + j] = v[j];
    }
    return c;
  };
  auto ld_diag = [&](int P) __attribute__((always_inline)) {
    const float* App = gtile(P, P);
    f32x16 d;
#pragma unroll
    for (int q = 0; q < 16; ++q) d[q] = App[acc_row(q, hi) * 32 + lo];
    return d;
  };
  // C^T L^-T with L^-1 in a 33-float-row LDS tile (f32 MFMA, as wide_chol_kernel)
  auto finish = [&](const f32x16& c, const float* dpad) __attribute__((always_inline)) {
    f32x16 l = f32x16{0.f};
#pragma unroll
    for (int s2 = 0; s2 < 16; ++s2) l = mfma32(c[s2], dpad[lo * 33 + acc_row(s2, hi)], l);
    return l;
  };
  auto store_tile = [&](float* t, const f32x16& l) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < 16; ++q) t[acc_row(q, hi) * 32 + lo] = l[q];
  };
  // D: factor + invert the diagonal tile d (wave 7): L^-1 to the workspace
  // tile and the padded LDS copy
  auto factor = [&](const f32x16& d, float* Aw, float* dpad) __attribute__((always_inline)) {
    int lo_o, hi_o;  // opaque lane coordinates (wide_chol_kernel)
    asm volatile("v_mov_b32 %0, %1" : "=v"(lo_o) : "v"(lo));
    asm volatile("v_mov_b32 %0, %1" : "=v"(hi_o) : "v"(hi));
#pragma unroll
    for (int q = 0; q < 16; ++q) dinv[sw(acc_row(q, hi_o), lo_o)] = d[q];
    wave_lds_sync();
    // inlined (as a call, every worker accumulator live across it would be
    // saved to scratch around it)
    int ln = lane;
    asm volatile("" : "+v"(ln));
    if (!diag_factor_inv_lds_body((lds_float*)dinv, ln) && lane == 0) flag[0] = 1;
    wave_lds_sync();
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int r = 2 * i + hi_o;
      const float v = dinv[sw(r, lo_o)];
      Aw[r * 32 + lo_o] = v;
      dpad[r * 33 + lo_o] = v;
    }
  };
  // y_P = L_PP^-1 r (wave 7)
  auto fwd = [&](const float* dpad, const float* r, int P) __attribute__((always_inline)) {
    float y = 0.0f;
#pragma unroll
    for (int k2 = 0; k2 < 16; ++k2) y = __builtin_fmaf(dpad[lo * 33 + 16 * hi + k2], r[16 * hi + k2], y);
    y += __shfl_xor(y, 32);
    if (hi == 0) yv[32 * P + lo] = y;
  };
  __syncthreads();

  // rows p, p+1 of L (tiles q < p) through LDS in chunks of C2_QC tiles, by
  // LDS-DMA (no registers): 2 C2_QC tiles x 4 wave-instructions of 1 KB,
  // C2_DMA per wave; LDS position pos of a tile holds the granule that
  // common.h sw puts there.  Out-of-range tiles re-read tile p-1 (never read
  // back), so every wave issues exactly C2_DMA loads per chunk
  constexpr int C2_DMA = 2 * C2_QC * 4 / 8;
  auto stage_dma = [&](int p, bool two, int ch) __attribute__((always_inline)) {
    float* st = stg;
    int ln = lane;
    asm volatile("" : "+v"(ln));
#pragma unroll
    for (int k = 0; k < C2_DMA; ++k) {
      const int f = C2_DMA * wave + k;  // wave-uniform
      const int ti = f >> 2, i = f & 3;
      const int sel = ti >= C2_QC, qo = ti - C2_QC * sel;
      const int q = min(C2_QC * ch + qo, p - 1);
      const int pos = 64 * i + ln, r = pos >> 3, G = (pos & 7) ^ ((r >> 1) & 7);
      glds16(gtile(p + (two ? sel : 0), q) + r * 32 + 4 * G,
             lds_addr(st + sel * C2_QC * 1024 + qo * 1024 + 256 * i));
    }
  };
  // the chunk in the stage -> its negated 3-piece split image (each worker
  // would otherwise split the same rows for every tile it owns): unit =
  // (tile, row, 8 columns), 3 per thread; 16-B granule kg of a row sits at
  // kg ^ ((row >> 2) & 3) (lanes over rows read conflict-free)
  auto split_chunk = [&]() __attribute__((always_inline)) {
    int t = tid;
    asm volatile("" : "+v"(t));
#pragma unroll
    for (int u = 0; u < C2_QC / 2; ++u) {
      const int unit = t + 512 * u, ti = unit >> 7, r = (unit >> 2) & 31, kg = unit & 3;
      const float* src = stg + ti * 1024;
      const f32x4v a0 = row_gran(src, r, 2 * kg), a1 = row_gran(src, r, 2 * kg + 1);
      float v[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v[j] = a0[j];
        v[4 + j] = a1[j];
      }
      bf16x8 f[3];
      split3x8(v, f);
      neg3(f);
#pragma unroll
      for (int pc = 0; pc < 3; ++pc)
        *reinterpret_cast<bf16x8*>(img + (((ti * 3 + pc) * 32 + r) * 4 + (kg ^ ((r >> 2) & 3))) * 4) = f[pc];
    }
  };
  // -split(row lo of image tile ti), k = 16 g + 8 hi .. +7: the MFMA A operand
  auto img_frag = [&](int ti, int g, bf16x8(&f)[3]) __attribute__((always_inline)) {
    const int kg = 2 * g + hi;
#pragma unroll
    for (int pc = 0; pc < 3; ++pc)
      f[pc] = *reinterpret_cast<const bf16x8*>(img + (((ti * 3 + pc) * 32 + lo) * 4 + (kg ^ ((lo >> 2) & 3))) * 4);
  };
  // U for one role; every role runs the same barriers.  NV = -1: the
  // diagonal wave (d0 = c1[0], cx = c2[0], d1 = c1[1]); NV = 0..C2_NI: a
  // worker with NV tiles, all valid (the tile count is a compile-time
  // constant: no per-tile branches, so no register copies at the joins)
  auto uphase = [&](auto nv_c, int p, bool two, int tb, f32x16(&c1)[C2_NA], f32x16(&c2)[C2_NA],
                    float& r0, float& r1) __attribute__((always_inline)) {
    constexpr int NV = decltype(nv_c)::value;
    // ring: C2_RING workspace tiles in flight, D = C2_RING / NV steps of q
    // per block (the q loop unrolled by D, so every ring slot is static)
    constexpr int D = NV > 0 ? C2_RING / NV : 1;
    static_assert(NV <= 0 || (C2_RING % NV == 0 && C2_QC % D == 0), "ring blocks tile the chunks");
    const int nch = (p + C2_QC - 1) / C2_QC;
    f32x4v ring[NV > 0 ? NV : 1][D][4];
    // the first chunk before the ring's first loads: a worker's wait for it
    // then leaves those 4 NV D loads in flight
    if (nch > 0) stage_dma(p, two, 0);
    if constexpr (NV > 0) {
#pragma unroll
      for (int s = 0; s < NV; ++s) {
        c1[s] = ld_panel(p + 2 + tb + C2_NWK * s, p);
        c2[s] = ld_panel(p + 2 + tb + C2_NWK * s, p + 1);
        if (p > 0) {
#pragma unroll
          for (int d = 0; d < D; ++d) ld_op(p + 2 + tb + C2_NWK * s, min(d, p - 1), ring[s][d]);
        }
      }
    }
    if constexpr (NV == -1) {
      c1[0] = ld_diag(p);
      if (two) {
        c2[0] = ld_panel(p + 1, p);
        c1[1] = ld_diag(p + 1);
      }
    }
    C2P(0)
    vm_wait(NV > 0 && p > 0 ? 4 * NV * D : 0);
    lds_barrier();
    C2P(1)
#pragma unroll 1
    for (int ch = 0; ch < nch; ++ch) {
      const int q0 = C2_QC * ch, q1 = min(p, q0 + C2_QC);
      // the stage holds chunk ch: its image, and (diagonal wave) the
      // forward-substitution dots r_P -= L_Pq y_q, row lo, k = 16 hi + k2
      // (wide_chol_kernel's chain), which need the fp32 rows
      fresh();
      split_chunk();
      if constexpr (NV == -1) {
#pragma unroll 1
        for (int q = q0; q < q1; ++q) {
          const float* t0 = stg + (q - q0) * 1024;  // L_pq
          const float* t1 = t0 + C2_QC * 1024;      // L_p+1,q
#pragma unroll
          for (int G = 0; G < 4; ++G) {
            const f32x4v a0 = row_gran(t0, lo, 4 * hi + G);
#pragma unroll
            for (int j = 0; j < 4; ++j) r0 = __builtin_fmaf(a0[j], yv[32 * q + 16 * hi + 4 * G + j], r0);
          }
          if (two) {
#pragma unroll
            for (int G = 0; G < 4; ++G) {
              const f32x4v a1 = row_gran(t1, lo, 4 * hi + G);
#pragma unroll
              for (int j = 0; j < 4; ++j) r1 = __builtin_fmaf(a1[j], yv[32 * q + 16 * hi + 4 * G + j], r1);
            }
          }
        }
      }
      C2P(0)
      lds_barrier();  // the image is complete, the stage free
      C2P(1)
      if (ch + 1 < nch) stage_dma(p, two, ch + 1);
      if constexpr (NV == -1) {
#pragma unroll 1
        for (int q = q0; q < q1; ++q) {
          fresh();
#pragma unroll
          for (int g = 0; g < 2; ++g) {
            bf16x8 nf0[3], pf0[3];
            img_frag(q - q0, g, nf0);
#pragma unroll
            for (int i = 0; i < 3; ++i) pf0[i] = nf0[i];
            neg3(pf0);
            c1[0] = mfma_x6(nf0, pf0, c1[0]);
            if (two) {
              bf16x8 nf1[3], pf1[3];
              img_frag(C2_QC + q - q0, g, nf1);
#pragma unroll
              for (int i = 0; i < 3; ++i) pf1[i] = nf1[i];
              neg3(pf1);
              c2[0] = mfma_x6(nf0, pf1, c2[0]);
              c1[1] = mfma_x6(nf1, pf1, c1[1]);
            }
          }
        }
      } else if constexpr (NV > 0) {
#pragma unroll 1
        for (int qb = q0; qb < q1; qb += D) {
#pragma unroll
          for (int d = 0; d < D; ++d) {
            const int q = qb + d;
            fresh();
            if (q < q1) {  // wave-uniform; only the pair's last block is partial
#pragma unroll
              for (int s = 0; s < NV; ++s) {
#pragma unroll
                for (int g = 0; g < 2; ++g) {
                  float lv[8];
#pragma unroll
                  for (int t = 0; t < 8; ++t) lv[t] = ring[s][d][2 * g + (t >> 2)][t & 3];
                  bf16x8 lf[3], pf[3];
                  split3x8(lv, lf);
                  img_frag(q - q0, g, pf);
                  c1[s] = mfma_x6(pf, lf, c1[s]);
                  img_frag(C2_QC + q - q0, g, pf);
                  c2[s] = mfma_x6(pf, lf, c2[s]);
                  __builtin_amdgcn_sched_barrier(0);  // one (tile, g) of operands live at a time
                }
              }
            }
            // tile q + D into the slot just read; unconditional (past the end
            // it re-reads tile p-1), so that no register phi forms at the joins
#pragma unroll
            for (int s = 0; s < NV; ++s) ld_op(p + 2 + tb + C2_NWK * s, min(q + D, p - 1), ring[s][d]);
          }
        }
      }
      // chunk ch+1 landed: only this chunk's ring loads (4 per tile and step,
      // every step of a block issues them) may still be in flight
      C2P(0)
      if (ch + 1 < nch) vm_wait(NV > 0 ? 4 * NV * D * ((q1 - q0 + D - 1) / D) : 0);
      lds_barrier();
      C2P(1)
    }
  };
  // D for a worker with NV tiles (barriers B1-B3 only in the first pass,
  // where the diagonal wave produces what they wait for)
  auto wphase = [&](auto nv_c, int p, bool two, int tb, bool first, f32x16(&c1)[C2_NA],
                    f32x16(&c2)[C2_NA]) __attribute__((always_inline)) {
    constexpr int NV = decltype(nv_c)::value;
    float* scr = stg + wave * 33 * 32;  // the stages are free now
    C2P(2)
    if (first) lds_barrier();  // B1: L_pp^-1
    C2P(3)
    fresh();
#pragma unroll
    for (int s = 0; s < NV; ++s) {
      c1[s] = finish(c1[s], dp0);  // L_Ip
      store_tile(gtile(p + 2 + tb + C2_NWK * s, p), c1[s]);
    }
    if (two) {
      C2P(2)
      if (first) lds_barrier();  // B2: L_p+1,p
      C2P(3)
      // C_I,p+1 -= L_Ip L_p+1,p^T: L_Ip to operand order through the scratch
#pragma unroll
      for (int s = 0; s < NV; ++s) {
        fresh();
#pragma unroll
        for (int q = 0; q < 16; ++q) scr[acc_row(q, hi) * 33 + lo] = c1[s][q];
        wave_lds_sync();
#pragma unroll
        for (int g = 0; g < 2; ++g) {
          float lv[8], pv[8];
#pragma unroll
          for (int t = 0; t < 8; ++t) lv[t] = scr[lo * 33 + 16 * g + 8 * hi + t];
          bf16x8 lf[3], pf[3];
          split3x8(lv, lf);
          prow8(lx, g, pv);
          split3x8(pv, pf);
          neg3(pf);
          c2[s] = mfma_x6(pf, lf, c2[s]);
        }
        wave_lds_sync();
      }
      C2P(2)
      if (first) lds_barrier();  // B3: L_p+1,p+1^-1
      C2P(3)
      fresh();
#pragma unroll
      for (int s = 0; s < NV; ++s) store_tile(gtile(p + 2 + tb + C2_NWK * s, p + 1), finish(c2[s], dp1));
    }
  };
  // D for the diagonal wave: both factorisations through one inlined copy
  // of the factor (two copies overflow the SGPRs)
  auto dphase = [&](int p, bool two, f32x16(&c1)[C2_NA], f32x16(&c2)[C2_NA], float r0,
                    float r1) __attribute__((always_inline)) {
#pragma unroll 1
    for (int it = 0; it < (two ? 2 : 1); ++it) {
      fresh();
      if (it == 1) {
        wave_lds_sync();
        fwd(dp0, rv, p);
        wave_lds_sync();
#pragma unroll
        for (int g = 0; g < 2; ++g) {  // the q = p term of A_p+1,p+1
          float v[8];
          prow8(lx, g, v);
          bf16x8 pf[3], nf[3];
          split3x8(v, pf);
#pragma unroll
          for (int i = 0; i < 3; ++i) nf[i] = pf[i];
          neg3(nf);
          c1[1] = mfma_x6(nf, pf, c1[1]);
        }
#pragma unroll
        for (int G = 0; G < 4; ++G) {
          const f32x4v a1 = row_gran(lx, lo, 4 * hi + G);
#pragma unroll
          for (int j = 0; j < 4; ++j) r1 = __builtin_fmaf(a1[j], yv[32 * p + 16 * hi + 4 * G + j], r1);
        }
      }
      f32x16 dd;
#pragma unroll
      for (int q = 0; q < 16; ++q) dd[q] = it == 0 ? c1[0][q] : c1[1][q];
      factor(dd, gtile(p + it, p + it), it == 0 ? dp0 : dp1);
      float rr = it == 0 ? r0 : r1;
      rr += __shfl_xor(rr, 32);
      if (hi == 0) rv[32 * it + lo] = yv[32 * (p + it) + lo] - rr;
      if (it == 0) {
        C2P(2)
        lds_barrier();  // B1
        C2P(3)
        if (two) {
          fresh();
          const f32x16 l = finish(c2[0], dp0);  // L_p+1,p
          store_tile(gtile(p + 1, p), l);
#pragma unroll
          for (int q = 0; q < 16; ++q) lx[sw(acc_row(q, hi), lo)] = l[q];
          C2P(2)
          lds_barrier();  // B2
          C2P(3)
        }
      } else {
        C2P(2)
        lds_barrier();  // B3
        C2P(3)
      }
    }
    wave_lds_sync();
    if (two) fwd(dp1, rv + 32, p + 1);
    else fwd(dp0, rv, p);
  };
  typedef std::integral_constant<int, -1> DiagRole;
  typedef std::integral_constant<int, 0> Idle;
  typedef std::integral_constant<int, 1> One;
  typedef std::integral_constant<int, 2> Two;
  static_assert(C2_NI == 1 || C2_NI == 2, "role dispatch below");

#pragma unroll 1
  for (int p = 0; p < te; p += 2) {
    const bool two = p + 1 < te;
    const int nI = te - p - 2;  // tiles below the pair (workers have tiles only with two)
    const int npass = nI > C2_NWK * C2_NI ? (nI + C2_NWK * C2_NI - 1) / (C2_NWK * C2_NI) : 1;
#pragma unroll 1
    for (int pass = 0; pass < npass; ++pass) {
      C2P(2)
      __syncthreads();  // the last pass's workspace stores and scratch reads are done
      C2P(4)
      fresh();
      const int tb = C2_NWK * C2_NI * pass + wave;
      const bool first = pass == 0;
      const int nv = dw ? 0 : max(0, min(C2_NI, (nI - tb + C2_NWK - 1) / C2_NWK));
      // each role's registers are its own (shared arrays would meet at the
      // joins with undefined parts, which the compiler keeps as zeros)
      if (dw && first) {
        f32x16 c1[C2_NA], c2[C2_NA];
        float r0 = 0.0f, r1 = 0.0f;
        uphase(DiagRole{}, p, two, tb, c1, c2, r0, r1);
        dphase(p, two, c1, c2, r0, r1);
      } else if (C2_NI >= 2 && nv == 2) {
        f32x16 c1[C2_NA], c2[C2_NA];
        float r0 = 0.0f, r1 = 0.0f;
        uphase(std::integral_constant<int, (C2_NI >= 2 ? 2 : 1)>{}, p, two, tb, c1, c2, r0, r1);
        wphase(std::integral_constant<int, (C2_NI >= 2 ? 2 : 1)>{}, p, two, tb, first, c1, c2);
      } else if (nv == 1) {
        f32x16 c1[C2_NA], c2[C2_NA];
        float r0 = 0.0f, r1 = 0.0f;
        uphase(One{}, p, two, tb, c1, c2, r0, r1);
        wphase(One{}, p, two, tb, first, c1, c2);
      } else {
        f32x16 c1[C2_NA], c2[C2_NA];
        float r0 = 0.0f, r1 = 0.0f;
        uphase(Idle{}, p, two, tb, c1, c2, r0, r1);
        wphase(Idle{}, p, two, tb, first, c1, c2);
      }
    }
  }
  C2P(2)
  C2P_FLUSH
  __syncthreads();
  wide_back_subst<T, 8>(slot, yv, xv, part, wave, lo, hi, te);
  const int64_t orow = slot_out ? (int64_t)blockIdx.x : e;
  for (int i = tid; i < Dp; i += 512) a.out[orow * Dp + i] = i < 32 * te ? xv[i] : 0.0f;
  if (tid == 0 && flag[0]) atomicMin(a.fail, (unsigned long long)(e + 1));
}

// CVaR-MF: x = e - eta (A_full e - b), A_full's strict upper part the stale
// G part (cvar_upper); one workgroup per entity.
__global__ void __launch_bounds__(256)
    wide_grad_kernel(SolveArgs a, int Dp, int64_t pos0, float* ws) {
  __shared__ float ev[1024];
  const int T = Dp >> 5, NT = T * (T + 1) / 2;
  const QueueRec rec = a.order[pos0 + blockIdx.x];
  const int64_t e = rec.entity;
  if (rec.h == 0) return;
  const float* slot = ws + (int64_t)blockIdx.x * ((int64_t)NT * 1024 + Dp);
  const int kind = a.kind;
  const float omega = (is_u_kind(kind) && a.entity_weight) ? a.entity_weight[e] : 1.0f;
  for (int i = threadIdx.x; i < Dp; i += 256) ev[i] = a.E[e * Dp + i];
  __syncthreads();
  for (int i = threadIdx.x; i < Dp; i += 256) {
    float y = 0.0f;
    for (int j = 0; j < Dp; ++j) {
      float aij;
      if (j <= i)
        aij = slot[(int64_t)tidx(i >> 5, j >> 5) * 1024 + (i & 31) * 32 + (j & 31)];
      else
        aij = cvar_upper(kind, a.G[(int64_t)i * Dp + j], a.w, omega);
      y += aij * ev[j];
    }
    a.out[e * Dp + i] = ev[i] - a.eta * (y - slot[(int64_t)NT * 1024 + i]);
  }
}

// One Householder step k of G = Q T Q^T (LAPACK sytd2, lower; v(k+1) = 1).
// Ain holds the matrix after step k-1's reflection EXCEPT its rank-2
// update, which this launch applies: rows / columns >= k of
// A - v w^T - w v^T with v = reflector k-1 (Vh row k-1, tau[k-1]) and
// w = p + K v, K = -tau/2 p.v, p = pin (written by launch k-1).  Every
// workgroup re-forms row k of the updated matrix and reflector k from it;
// workgroup b then updates columns [16b, 16b+16) into Aout (rows >= k+1)
// and writes those columns of p_k = tau_k A v_k to pout.
template <int N>
__global__ void __launch_bounds__(256)
    tridiag_step_kernel(const float* __restrict__ Ain, float* __restrict__ Aout, int k,
                        const float* __restrict__ pin, float* __restrict__ pout,
                        float* __restrict__ Vh, float* __restrict__ tau,
                        float* __restrict__ tdiag, float* __restrict__ toff) {
  constexpr int n = N, CW = 16, NR = N / 16, NV = N / 256;
  const int c0 = blockIdx.x * CW;
  if (blockIdx.x != 0 && c0 + CW <= k + 1) return;  // whole workgroup, before any barrier
  __shared__ float vp[N], wv[N], vk[N];
  __shared__ float red[8];
  __shared__ float pc[16][CW + 1];
  const int tid = threadIdx.x;
  const int c = c0 + (tid & (CW - 1)), rg = tid >> 4;
  // ---- every global load of the step, issued at entry: the previous
  // reflector, p, row k, and this thread's strip of its column (rows rg,
  // rg + 16, ...) -- one memory round trip instead of a chain of them ----
  const float tp = k > 0 ? tau[k - 1] : 0.0f;
  float vpr[NV], pir[NV], akr[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int r = tid + 256 * j;
    vpr[j] = (k > 0 && r > k) ? Vh[(int64_t)(k - 1) * n + r] : 0.0f;
    pir[j] = r >= k ? pin[r] : 0.0f;
    akr[j] = r >= k ? Ain[(int64_t)k * n + r] : 0.0f;
  }
  const bool col_live = c >= k + 1 && c < n && k + 1 < n;
  float sreg[NR];
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    const int r = rg + 16 * i;
    sreg[i] = (col_live && r >= k + 1) ? Ain[(int64_t)r * n + c] : 0.0f;
  }
  // previous reflector and w
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int r = tid + 256 * j;
    float v = 0.0f;
    if (k > 0 && tp != 0.0f) v = r == k ? 1.0f : vpr[j];
    vp[r] = v;
  }
  __syncthreads();
  float d = 0.0f;
  if (tp != 0.0f) {
#pragma unroll
    for (int j = 0; j < NV; ++j) d += pir[j] * vp[tid + 256 * j];
  }
  d = block_sum(d, red);
  const float K = -0.5f * tp * d;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int r = tid + 256 * j;
    wv[r] = (tp != 0.0f && r >= k) ? pir[j] + K * vp[r] : 0.0f;
  }
  __syncthreads();
  // row k of the updated matrix -> reflector k
  const float vpk = vp[k], wk = wv[k];
  float xn = 0.0f;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int r = tid + 256 * j;
    if (r >= k) {
      const float ck = akr[j] - vpk * wv[r] - wk * vp[r];
      vk[r] = ck;
      if (r >= k + 2) xn += ck * ck;
    }
  }
  xn = block_sum(xn, red);  // (barriers inside: vk complete)
  const float dkk = vk[k];
  float beta = 0.0f, tk = 0.0f, scal = 0.0f;
  if (k + 1 < n) {
    const float alpha = vk[k + 1];
    if (xn == 0.0f) {
      beta = alpha;
      tk = 0.0f;
    } else {
      beta = -copysignf(sqrtf(alpha * alpha + xn), alpha);
      tk = (beta - alpha) / beta;
      scal = 1.0f / (alpha - beta);
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int r = tid + 256 * j;
    float v = 0.0f;
    if (r == k + 1) v = 1.0f;
    else if (r >= k + 2) v = tk != 0.0f ? vk[r] * scal : 0.0f;
    vk[r] = v;
  }
  __syncthreads();
  if (blockIdx.x == 0) {
    if (tid == 0) {
      tdiag[k] = dkk;
      toff[k] = k + 1 < n ? beta : 0.0f;
      tau[k] = tk;
    }
    if (k + 1 < n)
      for (int r = k + 1 + tid; r < n; r += 256) Vh[(int64_t)k * n + r] = vk[r];
  }
  if (k + 1 >= n) return;
  // my columns: finish step k-1's update (rows >= k+1) and p_k
  float pacc = 0.0f;
  if (col_live) {
    const float vpc = vp[c], wc = wv[c];
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      const int r = rg + 16 * i;
      if (r >= k + 1) {
        const float v = sreg[i] - vp[r] * wc - wv[r] * vpc;
        Aout[(int64_t)r * n + c] = v;
        pacc += v * vk[r];
      }
    }
  }
  pc[rg][tid & (CW - 1)] = pacc;
  __syncthreads();
  if (tid < CW) {
    const int cc = c0 + tid;
    float sum = 0.0f;
#pragma unroll
    for (int g2 = 0; g2 < 16; ++g2) sum += pc[g2][tid];
    if (cc >= k + 1 && cc < n) pout[cc] = tk * sum;
  }
}

// The same Householder sequence as tridiag_step_kernel in ONE launch: N/16
// persistent workgroups, each keeping its 16-column strip of the matrix in
// registers through all N steps.  Per step a workgroup reads p_{k-1} and
// row k of the matrix (pending update k-1 not yet applied) from a ping-pong
// exchange buffer, forms K, w_{k-1} and reflector k redundantly (every
// workgroup, as the step kernel does), applies update k-1 to its strip,
// publishes its slice of p_k = tau_k A v_k and its entries of row k+1, and
// meets the others at one grid barrier (a device-scope counter).  The strip
// never leaves the registers (the step kernel re-read and re-wrote the whole
// matrix per launch) and the host enqueues one launch instead of N (the
// d-space launch queued behind them waited for the enqueue).  Arithmetic,
// thread mapping and reduction orders are the step kernel's: bit-identical.
// The grid (32 / 64 workgroups of 256 threads) is far below one workgroup
// per CU, so every workgroup becomes resident even beside other kernels; a
// bounded wait sets *err instead of spinning forever.
__device__ __forceinline__ float xload(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void xstore(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int N>
__global__ void __launch_bounds__(256)
    tridiag_persist_kernel(const float* __restrict__ G, float* xbuf, unsigned* bar, int* err,
                           float* __restrict__ Vh, float* __restrict__ tau,
                           float* __restrict__ tdiag, float* __restrict__ toff, int fenced) {
  constexpr int n = N, CW = 16, NR = N / 16, NV = N / 256, NWG = N / CW;
  const int c0 = blockIdx.x * CW;
  const int tid = threadIdx.x;
  const int c = c0 + (tid & (CW - 1)), rg = tid >> 4;
  const bool writer = blockIdx.x == NWG - 1;  // its columns stay live to the end
  __shared__ float vp[N], wv[N], vk[N];
  __shared__ float red[8];
  __shared__ float pc[16][CW + 1];
  __shared__ float tsh;
  float sreg[NR];
#pragma unroll
  for (int i = 0; i < NR; ++i) sreg[i] = G[(int64_t)(rg + 16 * i) * n + c];
  for (int r = tid; r < N; r += 256) vp[r] = 0.0f;
  if (tid == 0) tsh = 0.0f;
  __syncthreads();
  for (int k = 0; k < n; ++k) {
    const bool live = c0 + CW > k + 1 || writer;  // workgroup-uniform
    float* pin = xbuf + (size_t)(k & 1) * 2 * N;
    float* pout = xbuf + (size_t)((k + 1) & 1) * 2 * N;
    if (live) {
      const float tp = tsh;
      float pir[NV], akr[NV];
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        const int r = tid + 256 * j;
        pir[j] = (k > 0 && r >= k) ? xload(pin + r) : 0.0f;
        akr[j] = r >= k ? (k == 0 ? G[r] : xload(pin + N + r)) : 0.0f;
      }
      float d = 0.0f;
      if (tp != 0.0f) {
#pragma unroll
        for (int j = 0; j < NV; ++j) d += pir[j] * vp[tid + 256 * j];
      }
      d = block_sum(d, red);
      const float K = -0.5f * tp * d;
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        const int r = tid + 256 * j;
        wv[r] = (tp != 0.0f && r >= k) ? pir[j] + K * vp[r] : 0.0f;
      }
      __syncthreads();
      const float vpk = vp[k], wk = wv[k];
      float xn = 0.0f;
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        const int r = tid + 256 * j;
        if (r >= k) {
          const float ck = akr[j] - vpk * wv[r] - wk * vp[r];
          vk[r] = ck;
          if (r >= k + 2) xn += ck * ck;
        }
      }
      xn = block_sum(xn, red);
      const float dkk = vk[k];
      float beta = 0.0f, tk = 0.0f, scal = 0.0f;
      if (k + 1 < n) {
        const float alpha = vk[k + 1];
        if (xn == 0.0f) {
          beta = alpha;
          tk = 0.0f;
        } else {
          beta = -copysignf(sqrtf(alpha * alpha + xn), alpha);
          tk = (beta - alpha) / beta;
          scal = 1.0f / (alpha - beta);
        }
      }
      __syncthreads();
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        const int r = tid + 256 * j;
        float v = 0.0f;
        if (r == k + 1) v = 1.0f;
        else if (r >= k + 2) v = tk != 0.0f ? vk[r] * scal : 0.0f;
        vk[r] = v;
      }
      __syncthreads();
      if (writer) {
        if (tid == 0) {
          tdiag[k] = dkk;
          toff[k] = k + 1 < n ? beta : 0.0f;
          tau[k] = tk;
        }
        if (k + 1 < n)
          for (int r = k + 1 + tid; r < n; r += 256) Vh[(int64_t)k * n + r] = vk[r];
      }
      if (k + 1 >= n) break;  // the last step: no update, no exchange (every workgroup)
      // finish update k-1 on my columns (rows >= k+1), p_k partials, row k+1
      const bool col_live = c >= k + 1 && c < n;
      float pacc = 0.0f;
      if (col_live) {
        const float vpc = vp[c], wc = wv[c];
#pragma unroll
        for (int i = 0; i < NR; ++i) {
          const int r = rg + 16 * i;
          if (r >= k + 1) {
            const float v = sreg[i] - vp[r] * wc - wv[r] * vpc;
            sreg[i] = v;
            pacc += v * vk[r];
          }
        }
#pragma unroll
        for (int i = 0; i < NR; ++i)
          if (rg + 16 * i == k + 1) xstore(pout + N + c, sreg[i]);  // row k+1, my column
      }
      pc[rg][tid & (CW - 1)] = pacc;
      __syncthreads();
      if (tid < CW) {
        const int cc = c0 + tid;
        float sum = 0.0f;
#pragma unroll
        for (int g2 = 0; g2 < 16; ++g2) sum += pc[g2][tid];
        if (cc >= k + 1 && cc < n) xstore(pout + cc, tk * sum);
      }
      // reflector k becomes the pending one
      for (int r = tid; r < N; r += 256) vp[r] = vk[r];
      if (tid == 0) tsh = tk;
    } else if (k + 1 >= n) {
      break;
    }
    // grid barrier (step k): the exchange stores above (agent-scope atomic
    // stores) are complete before the arrival -- every thread waits for its
    // own (vmcnt 0) -- and the reads after it are agent-scope atomic loads.
    // fenced != 0 (FRECSYS_TRIDIAG_FENCE=1, A/B) adds device-scope fences,
    // which write back / invalidate the whole L2 of the XCD each step.
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (tid == 0) {
      if (fenced) __threadfence();
      atomicAdd(bar, 1u);
      const unsigned target = (unsigned)(k + 1) * NWG;
      unsigned spins = 0;
      while (__hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(2);
        if (++spins > (1u << 22) ||
            __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
          atomicExch(err, 1);
          break;
        }
      }
      if (fenced) __threadfence();
    }
    __syncthreads();
  }
  // a timed-out barrier leaves a garbage basis: poison it so that every LDL
  // pivot of the history-space solve fails and the call reruns in d-space
  if (writer && tid == 0 && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
    tdiag[0] = __builtin_nanf("");
}

// The same kernel without the grid barrier: every exchanged value travels
// with the step that produced it, as one 64-bit word (tag << 32 | bits,
// tag = base + step + 1, base a per-launch epoch so a previous launch's words
// never match), stored and polled with agent-scope atomics.  A workgroup
// starts step k as soon as the values it reads -- p_{k-1} and row k, rows
// >= k -- carry step k's tag: no arrival counter, no second round trip,
// and workgroups whose columns are all finished leave.  Ping-pong buffers
// still suffice: a workgroup can only reach step k+1 (writing buffer k & 1)
// once every producer has finished step k, whose reads of buffer k & 1 came
// first.  Same arithmetic and order: bit-identical to the barrier kernel.
// With Q != nullptr the grid carries N/32 more workgroups that form the
// rows of Q as the reflectors are published (common.h qrows_worker; the
// writer stores v_k and tau_k as tagged words into vt / tt), so no form-Q
// launch follows the reduction.
template <int N>
__global__ void __launch_bounds__(256)
    tridiag_tagged_kernel(const float* __restrict__ G, unsigned long long* xb, unsigned base,
                          int* err, float* __restrict__ Vh, float* __restrict__ tau,
                          float* __restrict__ tdiag, float* __restrict__ toff, float* Q,
                          bf16x8* img_q, bf16x8* img_qt, unsigned long long* vt,
                          unsigned long long* tt, unsigned* tcount) {
  constexpr int n = N, CW = 16, NR = N / 16, NV = N / 256, NWG = N / CW;
  __shared__ float lbuf[3 * N];
  float* vp = lbuf;
  float* wv = lbuf + N;
  float* vk = lbuf + 2 * N;
  __shared__ float red[8];
  __shared__ float pc[16][CW + 1];
  __shared__ float tsh;
  if (blockIdx.x >= NWG) {  // Q-row worker (reflectors k = 0 .. n-2)
    qrows_worker<N, 256>(blockIdx.x - NWG, n, n - 1, vt, tt, Q, img_q, img_qt, lbuf, red, tcount);
    return;
  }
  const int c0 = blockIdx.x * CW;
  const int tid = threadIdx.x;
  const int c = c0 + (tid & (CW - 1)), rg = tid >> 4;
  const bool writer = blockIdx.x == NWG - 1;
  float sreg[NR];
#pragma unroll
  for (int i = 0; i < NR; ++i) sreg[i] = G[(int64_t)(rg + 16 * i) * n + c];
  for (int r = tid; r < N; r += 256) vp[r] = 0.0f;
  if (tid == 0) tsh = 0.0f;
  __syncthreads();
  for (int k = 0; k < n; ++k) {
    if (!(c0 + CW > k + 1 || writer)) return;  // my columns are final (workgroup-uniform)
    const unsigned long long* pin = xb + (size_t)(k & 1) * 2 * N;
    unsigned long long* pout = xb + (size_t)((k + 1) & 1) * 2 * N;
    const unsigned tin = base + (unsigned)k, tout = base + (unsigned)k + 1;
    const float tp = tsh;
    float pir[NV], akr[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int r = tid + 256 * j;
      pir[j] = (k > 0 && r >= k) ? tpoll(pin + r, tin, err, false, tcount) : 0.0f;
      akr[j] = r >= k ? (k == 0 ? G[r] : tpoll(pin + N + r, tin, err, false, tcount)) : 0.0f;
    }
    float d = 0.0f;
    if (tp != 0.0f) {
#pragma unroll
      for (int j = 0; j < NV; ++j) d += pir[j] * vp[tid + 256 * j];
    }
    d = block_sum(d, red);
    const float K = -0.5f * tp * d;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int r = tid + 256 * j;
      wv[r] = (tp != 0.0f && r >= k) ? pir[j] + K * vp[r] : 0.0f;
    }
    __syncthreads();
    const float vpk = vp[k], wk = wv[k];
    float xn = 0.0f;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int r = tid + 256 * j;
      if (r >= k) {
        const float ck = akr[j] - vpk * wv[r] - wk * vp[r];
        vk[r] = ck;
        if (r >= k + 2) xn += ck * ck;
      }
    }
    xn = block_sum(xn, red);
    const float dkk = vk[k];
    float beta = 0.0f, tk = 0.0f, scal = 0.0f;
    if (k + 1 < n) {
      const float alpha = vk[k + 1];
      if (xn == 0.0f) {
        beta = alpha;
        tk = 0.0f;
      } else {
        beta = -copysignf(sqrtf(alpha * alpha + xn), alpha);
        tk = (beta - alpha) / beta;
        scal = 1.0f / (alpha - beta);
      }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int r = tid + 256 * j;
      float v = 0.0f;
      if (r == k + 1) v = 1.0f;
      else if (r >= k + 2) v = tk != 0.0f ? vk[r] * scal : 0.0f;
      vk[r] = v;
    }
    __syncthreads();
    if (writer) {
      if (tid == 0) {
        tdiag[k] = dkk;
        toff[k] = k + 1 < n ? beta : 0.0f;
        tau[k] = tk;
        if (Q && k + 1 < n) tstore(tt + k, (unsigned)k + 1, tk);
      }
      if (k + 1 < n)
        for (int r = k + 1 + tid; r < n; r += 256) {
          Vh[(int64_t)k * n + r] = vk[r];
          if (Q) tstore(vt + (size_t)k * n + r, (unsigned)k + 1, vk[r]);
        }
    }
    if (k + 1 >= n) break;
    const bool col_live = c >= k + 1 && c < n;
    float pacc = 0.0f;
    if (col_live) {
      const float vpc = vp[c], wc = wv[c];
#pragma unroll
      for (int i = 0; i < NR; ++i) {
        const int r = rg + 16 * i;
        if (r >= k + 1) {
          const float v = sreg[i] - vp[r] * wc - wv[r] * vpc;
          sreg[i] = v;
          pacc += v * vk[r];
        }
      }
#pragma unroll
      for (int i = 0; i < NR; ++i)
        if (rg + 16 * i == k + 1) tstore(pout + N + c, tout, sreg[i]);  // row k+1, my column
    }
    pc[rg][tid & (CW - 1)] = pacc;
    __syncthreads();
    if (tid < CW) {
      const int cc = c0 + tid;
      float sum = 0.0f;
#pragma unroll
      for (int g2 = 0; g2 < 16; ++g2) sum += pc[g2][tid];
      if (cc >= k + 1 && cc < n) tstore(pout + cc, tout, tk * sum);
    }
    for (int r = tid; r < N; r += 256) vp[r] = vk[r];
    if (tid == 0) tsh = tk;
    __syncthreads();
  }
  if (writer && tid == 0 && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
    tdiag[0] = __builtin_nanf("");
}

// User loss at wide Dp: one wave per user, Dp/32 lanes per history row
// (8 float4 each), 64*32/Dp rows in flight; u^T G u from the rotate_kernel
// partials (one per 128-column block) summed in column-block order.
template <int Dp>
__global__ void __launch_bounds__(256) loss_gather_wide_kernel(LossArgs a) {
  constexpr int LPR = Dp / 32, NG = 64 / LPR, NB = Dp / WB;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t idx = (int64_t)blockIdx.x * 4 + wave;
  if (idx >= a.n_rows) return;
  const int64_t e = a.row_lo + idx;
  const int64_t p0 = a.row_ptr[e];
  const int64_t h = a.row_ptr[e + 1] - p0;
  if (h == 0) return;
  const int g = lane / LPR, c = lane % LPR;
  float4 u4[8];
#pragma unroll
  for (int q = 0; q < 8; ++q)
    u4[q] = *reinterpret_cast<const float4*>(a.U + e * Dp + 4 * (c + LPR * q));
  float sq = 0.0f;
  for (int64_t k0 = 0; k0 < h; k0 += NG) {
    const int64_t k = k0 + g;
    float d = 0.0f;
    if (k < h) {
      const int id = a.col[p0 + k];
      const float* x = a.V + (int64_t)id * Dp;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float4 v = *reinterpret_cast<const float4*>(x + 4 * (c + LPR * q));
        d += v.x * u4[q].x + v.y * u4[q].y + v.z * u4[q].z + v.w * u4[q].w;
      }
    }
#pragma unroll
    for (int o = LPR / 2; o > 0; o >>= 1) d += __shfl_xor(d, o);
    if (c == 0 && k < h) {
      const float t = d - 1.0f;
      sq = (float)((double)sq + (double)t * (double)t);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) sq += __shfl_xor(sq, o);
  if (a.raw) {
    if (lane == 0) a.out[e] = sq;
    return;
  }
  float qv = 0.0f;
#pragma unroll
  for (int b = 0; b < NB; ++b) qv += a.quad[(int64_t)b * a.n_rows + idx];
  float loss = sq / (float)h + a.beta * qv;
  if (a.half) loss = (float)((double)loss / 2.0);
  if (lane == 0) a.out[e] = loss;
}


// the two-panel Cholesky at Dp = 1024 (FRECSYS_WIDE_CHOL2=0: the one-panel
// kernel, A/B; bit-identical)
#ifndef FRECSYS_WIDE_CHOL2_DEFAULT
#define FRECSYS_WIDE_CHOL2_DEFAULT 1
#endif
bool wide_chol2_on() {
  const char* v = getenv("FRECSYS_WIDE_CHOL2");
  return v ? atoi(v) != 0 : FRECSYS_WIDE_CHOL2_DEFAULT != 0;
}

size_t wide_chol_lds_bytes(int Dp) {
  const int T = Dp >> 5;
  return sizeof(float) * ((size_t)T * 33 * 32 + 1024 + 2 * Dp + 32 + 8 * 32 + 4);
}



}  // namespace

bool wide_dim(int Dp) { return Dp == 512 || Dp == 1024; }

size_t wide_slot_floats(int Dp) {
  const int T = Dp >> 5;
  return (size_t)T * (T + 1) / 2 * 1024 + Dp;
}

int64_t wide_slab_rows() { return (int64_t)W2FLUSH * W2R; }

size_t wide_slab_floats(int Dp) {
  const int T = Dp >> 5;
  return (size_t)T * (T + 1) / 2 * 1024 + 2 * (size_t)Dp;
}

int64_t wide_rows_per_leaf(int64_t n) {
  int64_t rpl = (n + kWideGramLeaves - 1) / kWideGramLeaves;
  if (rpl < 256) rpl = 256;
  return (rpl + WR - 1) / WR * WR;
}

hipError_t launch_wide_gram_leaves(int Dp, const GramArgs& g, hipStream_t s) {
  if (!wide_dim(Dp)) return hipErrorInvalidValue;
  const int64_t nblk = (g.n + g.plan.rpl - 1) / g.plan.rpl;
  if (nblk <= 0) return hipSuccess;
  SolveArgs a{};
  if (gather_off64(g.row0 + g.n, Dp))
    hipLaunchKernelGGL((wide_syrk2_kernel<0, true>), dim3(xcd_grid(nblk, wide_pairs2(Dp))),
                       dim3(512), 0, s, a, g, Dp, g.plan.rpl, (int64_t)0, (float*)nullptr, nblk);
  else
    hipLaunchKernelGGL((wide_syrk2_kernel<0, false>), dim3(xcd_grid(nblk, wide_pairs2(Dp))),
                       dim3(512), 0, s, a, g, Dp, g.plan.rpl, (int64_t)0, (float*)nullptr, nblk);
  return hipGetLastError();
}

hipError_t launch_wide_gram_final(int Dp, const float* gslabs, int64_t ngroup, float* G,
                                  hipStream_t s) {
  hipLaunchKernelGGL(wide_gram_reduce_kernel, dim3((unsigned)(((int64_t)Dp * Dp + 255) / 256)),
                     dim3(256), 0, s, gslabs, ngroup, G, Dp);
  return hipGetLastError();
}

hipError_t launch_wide_chol_slots(const QueueRec* order, int64_t n, float* slots, float* out,
                                  unsigned long long* fail, int quirk_v, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  static bool attr = false;
  if (!attr) {
    hipError_t err = hipFuncSetAttribute((const void*)wide_chol_kernel<16, kWideChol16NW>,
                                         hipFuncAttributeMaxDynamicSharedMemorySize,
                                         (int)wide_chol_lds_bytes(512));
    if (err != hipSuccess) return err;
    attr = true;
  }
  SolveArgs a{};
  a.order = order;
  a.out = out;
  a.fail = fail;
  hipLaunchKernelGGL((wide_chol_kernel<16, kWideChol16NW>), dim3((unsigned)n),
                     dim3(64 * kWideChol16NW), wide_chol_lds_bytes(512), s, a, (int64_t)0, slots,
                     quirk_v ? 2 : 1);
  return hipGetLastError();
}

hipError_t launch_wide_solve(int Dp, const SolveArgs& a, float* ws, int64_t batch,
                             hipStream_t s, char* xsplit) {
  if (!wide_dim(Dp) || batch <= 0) return hipErrorInvalidValue;
  if (a.n_rows <= 0) return hipSuccess;
  const bool off64 = gather_off64(a.n_other, Dp);
  static bool attr = false;
  if (!attr) {
    hipError_t err = hipFuncSetAttribute((const void*)wide_chol_kernel<16, kWideChol16NW>,
                                hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)wide_chol_lds_bytes(512));
    if (err == hipSuccess)
      err = hipFuncSetAttribute((const void*)wide_chol_kernel<32>,
                                hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)wide_chol_lds_bytes(1024));
    if (err == hipSuccess)
      err = hipFuncSetAttribute((const void*)wide_chol2_kernel<32, Chol2Wide>,
                                hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)(sizeof(float) * Chol2Lds<32, Chol2Wide>::FLOATS));
    if (err != hipSuccess) return err;
    attr = true;
  }
  const bool chol2 = wide_chol2_on();
  const bool grad = is_grad_kind(a.kind);
  GramArgs g{};
  // the SYRK from the pre-split table (wide_syrk.hip; xsplit: its buffer,
  // wide_xsplit_bytes), or the register-staged wide_syrk2_kernel (nullptr)
  SolveArgs a3 = a;
  if (xsplit) {
    hipError_t e = launch_wide_presplit(Dp, a, xsplit, s);
    if (e != hipSuccess) return e;
    a3.xsplit = xsplit;
    if (a.n_work > 0) {
      if (a.n_split > std::min<int64_t>(batch, a.n_rows)) return hipErrorInvalidValue;
      e = launch_wide_syrk3(Dp, a3, 2, 0, a.n_work, ws, s);
      if (e != hipSuccess) return e;
    }
  }
  // the slabs of the long histories (all in the first batch) first
  if (a.n_work > 0 && !xsplit) {
    if (a.n_split > std::min<int64_t>(batch, a.n_rows)) return hipErrorInvalidValue;
    if (off64)
      hipLaunchKernelGGL((wide_syrk2_kernel<2, true>), dim3(xcd_grid(a.n_work, wide_pairs2(Dp))),
                         dim3(512), 0, s, a, g, Dp, (int64_t)0, (int64_t)0, ws, a.n_work);
    else
      hipLaunchKernelGGL((wide_syrk2_kernel<2, false>), dim3(xcd_grid(a.n_work, wide_pairs2(Dp))),
                         dim3(512), 0, s, a, g, Dp, (int64_t)0, (int64_t)0, ws, a.n_work);
  }
  for (int64_t s0 = 0; s0 < a.n_rows; s0 += batch) {
    const int64_t nb = std::min<int64_t>(batch, a.n_rows - s0);
    if (xsplit) {
      hipError_t e = launch_wide_syrk3(Dp, a3, 1, s0, nb, ws, s);
      if (e != hipSuccess) return e;
    } else if (off64)
      hipLaunchKernelGGL((wide_syrk2_kernel<1, true>), dim3(xcd_grid(nb, wide_pairs2(Dp))),
                         dim3(512), 0, s, a, g, Dp, (int64_t)0, s0, ws, nb);
    else
      hipLaunchKernelGGL((wide_syrk2_kernel<1, false>), dim3(xcd_grid(nb, wide_pairs2(Dp))),
                         dim3(512), 0, s, a, g, Dp, (int64_t)0, s0, ws, nb);
    if (grad)
      hipLaunchKernelGGL(wide_grad_kernel, dim3((unsigned)nb), dim3(256), 0, s, a, Dp, s0, ws);
    else if (Dp == 512)
      hipLaunchKernelGGL((wide_chol_kernel<16, kWideChol16NW>), dim3((unsigned)nb),
                         dim3(64 * kWideChol16NW), wide_chol_lds_bytes(Dp), s, a, s0, ws, 0);
    else if (chol2)
      hipLaunchKernelGGL((wide_chol2_kernel<32, Chol2Wide>), dim3((unsigned)nb), dim3(512),
                         (sizeof(float) * Chol2Lds<32, Chol2Wide>::FLOATS), s, a, s0, ws, 0);
    else
      hipLaunchKernelGGL(wide_chol_kernel<32>, dim3((unsigned)nb), dim3(512),
                         wide_chol_lds_bytes(Dp), s, a, s0, ws, 0);
  }
  return hipGetLastError();
}

// persistent kernel: exchange [2][2][Dp] + barrier counter + error flag; the
// step kernels (FRECSYS_TRIDIAG_STEPS=1, A/B): two Dp x Dp copies + two p
// (+ the tagged reflector words of the Q-row workers: 2 Dp^2 + 2 Dp floats more)
size_t wide_tridiag_work_floats(int Dp) { return (size_t)4 * Dp * Dp + 32 * (size_t)Dp; }

// default: the tagged exchange (2.48 vs 2.96 ms at 512, 7.40 vs 8.51 at
// 1024 alone, bit-identical; scripts/micro/tridiag_wide_bench.cpp);
// FRECSYS_TRIDIAG_TAGGED=0: the barrier kernel, FRECSYS_TRIDIAG_STEPS=1 one
// launch per step (A/B)
bool wide_tridiag_tagged() {
  const char* tv = getenv("FRECSYS_TRIDIAG_TAGGED");
  const char* sv = getenv("FRECSYS_TRIDIAG_STEPS");
  return (!tv || atoi(tv) != 0) && !(sv && atoi(sv) != 0);
}

bool tridiag_steps() {
  const char* v = getenv("FRECSYS_TRIDIAG_STEPS");
  return v && atoi(v) != 0;
}

hipError_t launch_wide_tridiag(const float* G, int Dp, float* tdiag, float* toff, float* Vh,
                               float* tau, float* work, hipStream_t s, float* Q, void* img_q,
                               void* img_qt, unsigned* tcount) {
  if (!wide_dim(Dp) || !work) return hipErrorInvalidValue;
  if (!tridiag_steps()) {
    float* xbuf = work;                                     // [2][2][Dp]
    unsigned* bar = reinterpret_cast<unsigned*>(work + 4 * (size_t)Dp);
    int* err = reinterpret_cast<int*>(work + 4 * (size_t)Dp + 1);
    hipError_t e = hipMemsetAsync(bar, 0, 2 * sizeof(float), s);
    if (e != hipSuccess) return e;
    const char* fv = getenv("FRECSYS_TRIDIAG_FENCE");
    const int fenced = fv && atoi(fv) != 0;
    const bool tagged = wide_tridiag_tagged();
    if (tagged) {  // tagged words [2][2][Dp] after the counters; cleared per launch
      unsigned long long* xb = reinterpret_cast<unsigned long long*>(work + 8 * (size_t)Dp);
      // with Q: the reflectors as tagged words vt [Dp][Dp], tt [Dp], cleared too
      unsigned long long* vt = xb + 4 * (size_t)Dp;
      unsigned long long* tt = vt + (size_t)Dp * Dp;
      const size_t words = 4 * (size_t)Dp + (Q ? (size_t)Dp * Dp + Dp : 0);
      e = hipMemsetAsync(xb, 0, words * sizeof(unsigned long long), s);
      if (e != hipSuccess) return e;
      const unsigned grid = (unsigned)(Dp / 16 + (Q ? Dp / 32 : 0));
      bf16x8* iq = reinterpret_cast<bf16x8*>(img_q);
      bf16x8* iqt = reinterpret_cast<bf16x8*>(img_qt);
      if (Dp == 512)
        hipLaunchKernelGGL(tridiag_tagged_kernel<512>, dim3(grid), dim3(256), 0, s, G, xb, 0u, err,
                           Vh, tau, tdiag, toff, Q, iq, iqt, vt, tt, tcount);
      else
        hipLaunchKernelGGL(tridiag_tagged_kernel<1024>, dim3(grid), dim3(256), 0, s, G, xb, 0u,
                           err, Vh, tau, tdiag, toff, Q, iq, iqt, vt, tt, tcount);
      return hipGetLastError();
    }
    if (Dp == 512)
      hipLaunchKernelGGL(tridiag_persist_kernel<512>, dim3(512 / 16), dim3(256), 0, s, G, xbuf, bar,
                         err, Vh, tau, tdiag, toff, fenced);
    else
      hipLaunchKernelGGL(tridiag_persist_kernel<1024>, dim3(1024 / 16), dim3(256), 0, s, G, xbuf,
                         bar, err, Vh, tau, tdiag, toff, fenced);
    return hipGetLastError();
  }
  const int n = Dp;
  float* A[2] = {work, work + (size_t)n * n};
  float* P[2] = {work + (size_t)2 * n * n, work + (size_t)2 * n * n + n};
  const unsigned nb = (unsigned)((n + 15) / 16);
  for (int k = 0; k < n; ++k) {
    const float* ain = k == 0 ? G : A[(k - 1) & 1];
    if (n == 512)
      hipLaunchKernelGGL(tridiag_step_kernel<512>, dim3(nb), dim3(256), 0, s, ain, A[k & 1], k,
                         (const float*)P[(k + 1) & 1], P[k & 1], Vh, tau, tdiag, toff);
    else
      hipLaunchKernelGGL(tridiag_step_kernel<1024>, dim3(nb), dim3(256), 0, s, ain, A[k & 1], k,
                         (const float*)P[(k + 1) & 1], P[k & 1], Vh, tau, tdiag, toff);
  }
  return hipGetLastError();
}


size_t wide_quad_floats(int Dp, int64_t rows) { return (size_t)(Dp / WB) * (size_t)rows; }

hipError_t launch_wide_user_loss(int Dp, const LossArgs& a, hipStream_t s) {
  if (!wide_dim(Dp)) return hipErrorInvalidValue;
  if (a.n_rows <= 0) return hipSuccess;
  if (!a.raw) {  // u^T G u partials: (U G) .* U on the bf16 matrix cores (spectral.hip)
    hipError_t e = launch_split_basis(a.G, Dp, 0, a.gsplit, s);
    if (e != hipSuccess) return e;
    e = launch_rotate_quad(a.U, a.row_lo, a.n_rows, a.gsplit, a.quad, Dp, s);
    if (e != hipSuccess) return e;
  }
  const unsigned nb = (unsigned)((a.n_rows + 3) / 4);
  if (a.ev_gather) (void)hipEventRecord(a.ev_gather, s);
  if (Dp == 512)
    hipLaunchKernelGGL(loss_gather_wide_kernel<512>, dim3(nb), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(loss_gather_wide_kernel<1024>, dim3(nb), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace frecsys_hip
