// wide_syrk.hip -- the d-space SYRK of A = X_h^T D X_h at Dp = 512 / 1024
// (the rank updates of Project / ProjectU / ProjectV at the wide dims:
// ials.h:101-131, safer2.h:133-150, 181-199, erm_mf.h, cvar_mf.h), its rows
// moved by LDS-DMA.
//
// The products are fp32-accurate split-bf16 MFMAs (common.h mfma_x6) on
// x~ = sa x (sa = sqrt(nu) on the V kinds, else 1).  What bounds this SYRK
// is the rate at which a CU can take in gathered rows (a row is an
// arbitrary one of the other side: each chunk of 16 rows is a gather from
// HBM or the Infinity Cache), so the rows travel as fp32 (2 KB per 512
// columns; a pre-split bf16 copy would be 3 KB) and are split into their
// three bf16 pieces in registers, after the operand read:
//
//   * LDS-DMA (global_load_lds_dwordx4, a per-lane source address = a row
//     gather) brings each chunk of 16 rows -- the two 256-column blocks the
//     workgroup reads, 2 KB per row -- into a 4-slot LDS ring three chunks
//     ahead of its MFMAs (two chunks = 64 KB in flight per CU).  The issues
//     are spread over the MFMAs; one barrier per chunk.  The row ids arrive
//     the same way (4-byte LDS-DMA, six chunks ahead), so the loop issues no
//     vector load the compiler would wait on.
//   * V kinds: the rows are read from a pre-scaled copy sa X (and the rhs
//     weights nu / sa from a table beside it), formed once per half-step
//     (wide_prescale_kernel); the other kinds read X itself.
//   * Two kinds of workgroup per unit, both reading 512 columns: an
//     off-diagonal 256 x 256 block pair (64 tiles, 2 x 4 per wave), and a
//     diagonal double (the two lower 8 x 8-tile triangles of a pair of
//     diagonal blocks, 72 tiles, 9 per wave: rows q and 7 - q of one
//     triangle).  At Dp = 512 that is two workgroups per entity streaming the
//     same rows at nearly the same rate (64 / 72 tiles), on one XCD.
//
// Every tile sees exactly the products of wide_syrk2_kernel, in the same order
// (the same split of the same x~, mfma_x6 per chunk, chunks in order, the same
// two-level accumulation and slab layout), and b the same fp32 sums, so the
// output is bit-identical to the register-staged kernel it replaces
// (tests/test_wide_syrk3_gpu.py).
#include <hip/hip_runtime.h>

#include <type_traits>

#include "common.h"
#include "kernels.h"
#include "wide.h"

namespace frecsys_hip {

namespace {

constexpr int W3ROWF = 512;                   // floats of one staged row (two 256-column blocks)
constexpr int W3ROWB = 4 * W3ROWF;             // 2 KB
constexpr int W3SLOT = kWideChunk * W3ROWB;    // 32 KB: one chunk
constexpr int W3NS = 4;                        // ring slots (chunks c .. c + 3)
constexpr int W3IDS = 8;                       // row-id ring slots (chunks c + 3 .. c + 6, and the prologue's 0 .. 5)
constexpr int W3OFF_IDS = W3NS * W3SLOT;
constexpr int W3OFF_BW = W3OFF_IDS + W3IDS * kWideChunk * 4;
constexpr int W3LDS = W3OFF_BW + W3NS * kWideChunk * 4;

// ---- V kinds: the pre-scaled other side ----
// Row r < n: sa_r X[r] (sa = sqrt(nu_r), the rounded fp32 product, as the
// register-staged kernel forms it); bw[r] = nu_r / sa_r (the rhs weight,
// safer2.h:190-192).  Row n and bw[n]: zero (read past a unit's end).
__global__ void __launch_bounds__(256)
    wide_prescale_kernel(const float* __restrict__ X, int64_t n, int Dp,
                         const float* __restrict__ nu, float* __restrict__ xs,
                         float* __restrict__ bw) {
#pragma clang fp contract(off)
  const int per_row = Dp >> 2;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t r = t / per_row;
  const int c4 = (int)(t % per_row) * 4;
  if (r > n) return;
  float4* out = reinterpret_cast<float4*>(xs + r * Dp + c4);
  if (r == n) {
    *out = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c4 == 0) bw[r] = 0.0f;
    return;
  }
  const float w = nu[r];
  const float sa = sqrtf(w);
  const float4 x = *reinterpret_cast<const float4*>(X + r * Dp + c4);
  *out = make_float4(x.x * sa, x.y * sa, x.z * sa, x.w * sa);
  if (c4 == 0) bw[r] = sa > 0.0f ? w / sa : 0.0f;
}

// ---- LDS-DMA and the waits the compiler does not see ----
// One 16-B (4-B) piece per lane into LDS at dst + 16 lane (4 lane); dst is
// wave-uniform (M0).  Inline asm: hipcc's own LDS-DMA builtin makes it wait
// vmcnt(0) before every ds_read (it cannot tell the ring slots apart), which
// would drain the ring at each chunk; these are counted by hand (vm_wait).
__device__ __forceinline__ void glds16(const void* src, unsigned dst) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(dst)
      : "memory");
}
__device__ __forceinline__ void glds4(const void* src, unsigned dst) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "global_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(dst)
      : "memory");
}
// s_waitcnt vmcnt(n): every vector-memory op of this wave but the n youngest
// has completed (n wave-uniform; the loop issues no other vector loads)
__device__ __forceinline__ void vm_wait(int n) {
  switch (__builtin_amdgcn_readfirstlane(n)) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
    case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    case 11: asm volatile("s_waitcnt vmcnt(11)" ::: "memory"); break;
    case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    case 13: asm volatile("s_waitcnt vmcnt(13)" ::: "memory"); break;
    case 14: asm volatile("s_waitcnt vmcnt(14)" ::: "memory"); break;
    case 15: asm volatile("s_waitcnt vmcnt(15)" ::: "memory"); break;
    case 16: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
    case 17: asm volatile("s_waitcnt vmcnt(17)" ::: "memory"); break;
    case 18: asm volatile("s_waitcnt vmcnt(18)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}
__device__ __forceinline__ void w3_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}

// The fp32 values of the 32 x 16 MFMA operand of LDS column block cb
// (columns 32 cb .. 32 cb + 31 of the staged rows) from the ring slot at LDS
// byte address slot: the lane's column, rows 8 hi .. 8 hi + 7 (lanec = slot
// offset of row 8 hi, column lo).  Conflict-free: the 32 lanes of a
// ds_read_b32 half read 32 consecutive floats of one row.
__device__ __forceinline__ void w3_vals(unsigned slot, unsigned lanec, int cb, float (&x)[8]) {
  const unsigned a0 = slot + lanec + 128u * (unsigned)cb;
#pragma unroll
  for (int e = 0; e < 8; ++e)
    x[e] = *(const __attribute__((address_space(3))) float*)(uintptr_t)(a0 + e * W3ROWB);
}
// ... and its three bf16 pieces (common.h split3: the register-staged
// kernel's split of the same values)
// The split of 8 values, pair by pair: one v_cvt_pk_bf16_f32 per piece and
// pair (round to nearest even, as split3's casts), the piece back to fp32 by a
// shift / mask of the packed word, scalar subtractions (the compiler's SLP
// pairing of these into v_pk_add_f32 costs issue cycles beside MFMAs;
// MI355X_MICROARCH.md, per-instruction constants).  The same pieces as
// common.h split3.  FRECSYS_W3_SPLIT=2: timing ablation, hi piece only.
#ifndef FRECSYS_W3_SPLIT
#define FRECSYS_W3_SPLIT 1
#endif
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned w3_pk(float a, float b) {
  const bf16x2 v = {(__bf16)a, (__bf16)b};
  unsigned u = __builtin_bit_cast(unsigned, v);
  // opaque to the optimiser: else it recomputes the low piece as a second
  // v_cvt_pk_bf16_f32 (a, 0) instead of shifting this word
  asm("" : "+v"(u));
  return u;
}
__device__ __forceinline__ void w3_split(const float (&x)[8], bf16x8 (&f)[3]) {
#if FRECSYS_W3_SPLIT == 2
  unsigned w[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) w[e] = w3_pk(x[2 * e], x[2 * e + 1]);
  f[0] = __builtin_bit_cast(bf16x8, w);
  f[1] = f[0];
  f[2] = f[0];
#elif FRECSYS_W3_SPLIT == 1
#pragma clang fp contract(off)
  unsigned wh[4], wm[4], wl[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float x0 = x[2 * e], x1 = x[2 * e + 1];
    const unsigned H = w3_pk(x0, x1);
    const float r0 = x0 - __uint_as_float(H << 16), r1 = x1 - __uint_as_float(H & 0xffff0000u);
    const unsigned M = w3_pk(r0, r1);
    const float s0 = r0 - __uint_as_float(M << 16), s1 = r1 - __uint_as_float(M & 0xffff0000u);
    wh[e] = H;
    wm[e] = M;
    wl[e] = w3_pk(s0, s1);
  }
  f[0] = __builtin_bit_cast(bf16x8, wh);
  f[1] = __builtin_bit_cast(bf16x8, wm);
  f[2] = __builtin_bit_cast(bf16x8, wl);
#else
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    __bf16 h, m, l;
    split3(x[e], h, m, l);
    f[0][e] = h;
    f[1][e] = m;
    f[2][e] = l;
  }
#endif
}

// rhs part of one operand: bpart += bw_e * x~_e over the lane's 8 rows, in
// row order, each product rounded before its add (the register-staged
// kernel's fp32 sums).  Not VK: bw = 1 (the rows past the unit's end are the
// zero row), and 1 * x~ is x~.
template <bool VK>
__device__ __forceinline__ void w3_bsum(const float (&x)[8], const float (&bw)[8], float& b) {
#pragma clang fp contract(off)
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    if constexpr (VK) b += bw[e] * x[e];
    else b += x[e];
  }
}

// ---- the 4-wave workgroup: one wave per SIMD ----
// A wave's fragments (32-column blocks of the staged rows, each the A operand
// of its row's tiles and the B operand of its column's) are split in a fixed
// order; after split k every tile whose two fragments are now split is
// issued, so the MFMAs start after the first fragment or two and the later
// splits overlap the earlier tiles' MFMAs.  At most 16 tiles per wave: the
// 256 accumulators fit the AGPRs.
//  ROLE 0, off-diagonal pair (64 tiles, 512 staged columns): rows ra .. ra + 3
//    of the row block (fragments A_i = LDS column block 8 + ra + i) x columns
//    cb0 .. cb0 + 3 of the column block (B_j = cb0 + j); order A0 B0 B1 A1 B2
//    A2 B3 A3; 16 tiles.
//  ROLE 1 + q, diagonal block (36 tiles of its lower 8 x 8 triangle, 256
//    staged columns): rows q and 7 - q, every tile (r, j) with j <= r;
//    fragment f = column block f; order q, 7 - q, then the other columns up
//    to 7 - q; 9 tiles.
template <int ROLE>
constexpr int w3_nfrag() {
  return ROLE == 0 ? 8 : 9 - ROLE;
}
template <int ROLE>
constexpr int w3_ntile() {
  return ROLE == 0 ? 16 : 9;
}
// fragment in split position k: ROLE 0: 0..3 = A_0..3, 4..7 = B_0..3;
// diagonal: the column block
template <int ROLE>
constexpr int w3_frag_at(int k) {
  if constexpr (ROLE == 0) {
    constexpr int ord[8] = {0, 4, 5, 1, 6, 2, 7, 3};
    return ord[k];
  } else {
    constexpr int q = ROLE - 1;
    if (k == 0) return q;
    if (k == 1) return 7 - q;
    int n = 2;
    for (int f = 0; f < 7 - q; ++f)
      if (f != q) {
        if (n == k) return f;
        ++n;
      }
    return -1;
  }
}
template <int ROLE>
constexpr int w3_pos(int f) {  // split position of fragment f
  for (int k = 0; k < w3_nfrag<ROLE>(); ++k)
    if (w3_frag_at<ROLE>(k) == f) return k;
  return -1;
}
// tile t (in issue order): its row / column fragment and block-local tile
// coordinates (ROLE 0: i, j in 0..3 relative to ra, cb0)
struct W3Tile {
  int a, b, i, j, step;
};
template <int ROLE>
constexpr W3Tile w3_tile_at(int t) {
  int n = 0;
  for (int k = 0; k < w3_nfrag<ROLE>(); ++k) {
    if constexpr (ROLE == 0) {
      for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
          const int pa = w3_pos<ROLE>(i), pb = w3_pos<ROLE>(4 + j);
          if ((pa > pb ? pa : pb) == k) {
            if (n == t) return W3Tile{i, 4 + j, i, j, k};
            ++n;
          }
        }
    } else {
      constexpr int q = ROLE - 1;
      for (int ri = 0; ri < 2; ++ri) {
        const int r = ri ? 7 - q : q;
        for (int j = 0; j <= r; ++j) {
          const int pa = w3_pos<ROLE>(r), pb = w3_pos<ROLE>(j);
          if ((pa > pb ? pa : pb) == k) {
            if (n == t) return W3Tile{r, j, r, j, k};
            ++n;
          }
        }
      }
    }
  }
  return W3Tile{-1, -1, -1, -1, -1};
}

// MFMAs of the tiles completed at split step k (6 per tile; 0 for k < 0)
template <int ROLE>
constexpr int w3_nmfma(int k) {
  int n = 0;
  for (int t = 0; t < w3_ntile<ROLE>(); ++t)
    if (k >= 0 && w3_tile_at<ROLE>(t).step == k) n += 6;
  return n;
}

template <int N, typename F>
__device__ __forceinline__ void w3_for(F&& f) {
  if constexpr (N > 0) {
    w3_for<N - 1>(f);
    f(std::integral_constant<int, N - 1>{});
  }
}

// Column block (LDS, 32 columns) of fragment f: ROLE 0: A_i = 8 + ra + i,
// B_j = cb0 + j; diagonal: f.
template <int ROLE>
__device__ __forceinline__ int w3_cb(int f, int ra, int cb0) {
  if constexpr (ROLE == 0) return f < 4 ? 8 + ra + f : cb0 + (f - 4);
  else return f;
}

// One pipeline step of the wide SYRK: the MFMAs of chunk c (fragments Fc,
// split in the previous step) interleaved with the reads and splits of chunk
// c + 1's fragments (slot_next -> Fn).  A split is ~44 dependent VALU and
// takes ~270 cycles alone; beside ~12 MFMAs it costs nearly nothing, so the
// splits of one chunk ride under the MFMAs of the one before
// (scripts/micro/mfma_valu_overlap.hip).  pump(g), g = 0 .. NP - 1: the
// step's LDS-DMA issues, placed right after the reads (an inline-asm
// statement ends the compiler's scheduling region).  Diagonal roles: the rhs
// partials of chunk c + 1's two row fragments (split positions 0, 1) from
// their fp32 values.  With SPLIT_ONLY: chunk c + 1's splits alone (prologue).
template <int ROLE, bool VK, int NP, bool SPLIT_ONLY, typename Pump>
__device__ __forceinline__ void w3_step(unsigned slot_next, unsigned lanec, int ra, int cb0,
                                        const bf16x8 (&Fc)[8][3], bf16x8 (&Fn)[8][3],
                                        f32x16 (&acc)[16], const float (&bw)[8], float (&bp)[2],
                                        int skip, Pump&& pump) {
  (void)skip;  // ablation masks (FRECSYS_DEBUG_SKIP): 1 no MFMAs, 2048 no rhs sums
  constexpr int NF = w3_nfrag<ROLE>(), NT = w3_ntile<ROLE>();
  float xb[2][8];  // fragment values, double-buffered by split position
  w3_vals(slot_next, lanec, w3_cb<ROLE>(w3_frag_at<ROLE>(0), ra, cb0), xb[0]);
  w3_for<NF>([&](auto kc) __attribute__((always_inline)) {
    constexpr int k = decltype(kc)::value;
    constexpr int f = w3_frag_at<ROLE>(k);
    float(&x)[8] = xb[k & 1];
#pragma unroll
    for (int g = NP * k / NF; g < NP * (k + 1) / NF; ++g) pump(g);
    if constexpr (k + 1 < NF)
      w3_vals(slot_next, lanec, w3_cb<ROLE>(w3_frag_at<ROLE>(k + 1), ra, cb0), xb[(k + 1) & 1]);
    if constexpr (ROLE != 0 && k < 2) {
      if (!FRECSYS_SKIP(skip, 2048)) w3_bsum<VK>(x, bw, bp[k]);
    }
    w3_split(x, Fn[f]);
    if constexpr (!SPLIT_ONLY) {
      // chunk c's tiles [k NT / NF, (k + 1) NT / NF)
      constexpr int t0 = k * NT / NF, t1 = (k + 1) * NT / NF;
      if (!FRECSYS_SKIP(skip, 1)) {
        w3_for<NT>([&](auto tc) __attribute__((always_inline)) {
          constexpr int t = decltype(tc)::value;
          if constexpr (t >= t0 && t < t1) {
            constexpr W3Tile T = w3_tile_at<ROLE>(t);
            acc[t] = mfma_x6(Fc[T.a], Fc[T.b], acc[t]);
          }
        });
      }
      // the fragment reads first, then MFMA / VALU alternating
      constexpr int NM = 6 * (t1 - t0);
      if constexpr (NM > 0) {
        constexpr int NV = ROLE != 0 && k < 2 ? 56 : 48;
        constexpr int VPER = (NV + NM - 1) / NM;
        if constexpr (k + 1 < NF) __builtin_amdgcn_sched_group_barrier(0x100, 8, k);
        w3_for<NM>([&](auto) __attribute__((always_inline)) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, k);
          __builtin_amdgcn_sched_group_barrier(0x002, VPER, k);
        });
      }
    }
  });
}

// Per-kind finish of one tile of A from its G values (wide_syrk2_kernel's
// epilogue, the same expressions)
template <int FM>
__device__ __forceinline__ void w3_finish(const f32x16& acc, const float (&g)[16], int I, int J,
                                          float* t, int kind, float w, float gscale, float lam,
                                          float hf, float omega, float us, int lo, int hi) {
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int i = acc_row(r, hi);
    const bool dg = 32 * I + i == 32 * J + lo;
    float v = acc[r];
    const float gv = g[r];
    if constexpr (FM == 3) {
      v = assemble(kind, v, gv, dg, w, lam, hf, omega);
    } else {
      float g0 = gscale * gv;
      if constexpr (FM == 0) g0 += dg ? lam : 0.0f;
      v = g0 + v;
      if constexpr (FM == 1) v = v * us + (dg ? lam : 0.0f);
      if constexpr (FM == 2) v = v + (dg ? lam : 0.0f);
    }
    t[i * 32 + lo] = v;
  }
}

template <int MODE, bool VK>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
    wide_syrk3_kernel(SolveArgs a, int Dp, int64_t pos0, float* ws, int64_t n_units) {
  __shared__ __attribute__((aligned(16))) char lds[W3LDS];
  const int tid = threadIdx.x, lane = tid & 63, lo = lane & 31, hi = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int T = Dp >> 5, NT = T * (T + 1) / 2, NB = Dp >> 8;
  const int noff = NB * (NB - 1) / 2;
  int64_t unit;
  int pidx;
  if (!xcd_unit(noff + NB, n_units, unit, pidx)) return;
  // the 256-column blocks staged in LDS columns [0, 256) (L0) and, for an
  // off-diagonal pair, [256, 512) (L1)
  const bool off = pidx < noff;
  int L0, L1;
  if (off) {
    L1 = 1;
    while (L1 * (L1 + 1) / 2 <= pidx) ++L1;
    L0 = pidx - L1 * (L1 - 1) / 2;
  } else {
    L0 = pidx - noff;
    L1 = L0;
  }
  const int kind = a.kind;  // is_v_kind(kind) == VK, checked by the launcher

  SplitWork sw{};
  if (MODE == 2) sw = a.work[unit];
  const QueueRec rec = a.order[MODE == 2 ? (int64_t)sw.pos : pos0 + unit];
  const int64_t e = rec.entity, h = rec.h, p0 = rec.p0;
  if (h == 0) return;  // untouched entity (no barrier passed yet)
  int64_t extra = 0;
  if (VK && a.quirk && h > 128 && (h % 128) != 0) extra = 128 - (h % 128);
  int64_t kbase = 0, klim = h + extra;
  bool fin = false;
  if (MODE == 2) {
    kbase = sw.k0;
    klim = sw.k1;
  } else {
    fin = pos0 + unit < a.n_split;
  }
  const int nchunks = fin ? 0 : (int)((klim - kbase + kWideChunk - 1) / kWideChunk);

  // the rows: X itself, or on the V kinds the pre-scaled copy (a.xsplit:
  // [n_other + 1][Dp], then the rhs weights [n_other + 1]); past a unit's
  // end the zero row (row n_other of the copy, or a.xsplit itself)
  const float* xrows = VK ? reinterpret_cast<const float*>(a.xsplit) : a.X;
  const float* zero = reinterpret_cast<const float*>(a.xsplit) + (VK ? a.n_other * Dp : 0);
  const float* bwt = reinterpret_cast<const float*>(a.xsplit) + (a.n_other + 1) * Dp;
  const unsigned ring = lds_addr(lds), ids = ring + W3OFF_IDS, bws = ring + W3OFF_BW;
  const int* ids_p = reinterpret_cast<const int*>(lds + W3OFF_IDS);
  const float* bws_p = reinterpret_cast<const float*>(lds + W3OFF_BW);

  auto issue_ids = [&](int x) __attribute__((always_inline)) {  // wave 0: chunk x's row ids
    if (lane < kWideChunk) {
      int64_t k = kbase + (int64_t)x * kWideChunk + lane;
      if (k >= klim) k = klim - 1;
      glds4(a.col + p0 + wide_virt_pos(k, h),
            __builtin_amdgcn_readfirstlane(ids + (x % W3IDS) * kWideChunk * 4));
    }
  };
  // the wave's rows 4 wave .. 4 wave + 3 of chunk x: their sources (ids from
  // the ring; wave-uniform, so the bases stay in SGPRs) and LDS address;
  // pump(g) issues half g & 1 (block L0 / L1) of row 4 wave + (g >> 1) -- a
  // diagonal block's workgroup only half 0 (pump(2 g)) -- one 1-KB LDS-DMA,
  // lane l columns 4 l .. 4 l + 3
  const float* rsrc[4] = {zero, zero, zero, zero};
  unsigned rdst = 0;
  const int coff0 = 256 * L0 + 4 * lane, coff1 = 256 * L1 + 4 * lane;
  auto prep_rows = [&](int x) __attribute__((always_inline)) {
    const int4 idq = *reinterpret_cast<const int4*>(ids_p + (x % W3IDS) * kWideChunk + 4 * wave);
    const int idv[4] = {idq.x, idq.y, idq.z, idq.w};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t k = kbase + (int64_t)x * kWideChunk + 4 * wave + r;
      const int id = __builtin_amdgcn_readfirstlane(idv[r]);
      rsrc[r] = k < klim ? xrows + (int64_t)id * Dp : zero;
    }
    rdst = ring + (x % W3NS) * W3SLOT + 4 * wave * W3ROWB;
  };
  auto pump = [&](int g) __attribute__((always_inline)) {
    if (!FRECSYS_SKIP(a.debug_skip, 32))  // no branch in the product build
      glds16(rsrc[g >> 1] + ((g & 1) ? coff1 : coff0),
             __builtin_amdgcn_readfirstlane(rdst + (g >> 1) * W3ROWB + (g & 1) * (W3ROWB / 2)));
  };
  auto issue_bw = [&](int x) __attribute__((always_inline)) {  // wave 3, V kinds: rhs weights
    if (lane < kWideChunk) {
      const int64_t k = kbase + (int64_t)x * kWideChunk + lane;
      const int64_t id = k < klim ? (int64_t)ids_p[(x % W3IDS) * kWideChunk + lane] : a.n_other;
      glds4(bwt + id, __builtin_amdgcn_readfirstlane(bws + (x % W3NS) * kWideChunk * 4));
    }
  };

  // operand-read lane constant (w3_vals): row 8 hi, column lo of a slot
  const unsigned lanec = (unsigned)(8 * hi * W3ROWB + 4 * lo);
  // roles: off-diagonal -- rows ra .. ra + 3 x columns cb0 .. cb0 + 3;
  // diagonal -- rows wave and 7 - wave of the block's triangle
  const int ra = 4 * (wave >> 1), cb0 = 4 * (wave & 1);

  f32x16 acc[16];
#pragma unroll
  for (int s = 0; s < 16; ++s) acc[s] = f32x16{0.f};
  float bp[2] = {0.f, 0.f}, bt[2] = {0.f, 0.f};
  bool flushed = false;
  float* const wslot = MODE == 1 ? ws + unit * ((int64_t)NT * 1024 + Dp) : nullptr;

#ifdef FRECSYS_ABLATION
  // diagnostics (FRECSYS_DUAL_PROF, ablation builds): per-chunk phase cycles
  // of waves 0 and 3 -- 0 the chunk's MFMAs and operand reads, 1 the DMA
  // preparation, 2 the wait for the next chunk and the barrier
  const bool tprof = a.prof && lane == 0 && (wave == 0 || wave == 3);
  unsigned long long tp_t = 0, tp_acc[3] = {0, 0, 0};
  auto tp_mark = [&](int i) __attribute__((always_inline)) {
    if (tprof) {
      const unsigned long long t = clock64();
      if (tp_t) tp_acc[i] += t - tp_t;
      tp_t = t;
    }
  };
#else
  auto tp_mark = [](int) {};
#endif
  auto run = [&](auto role_c) __attribute__((always_inline)) {
    constexpr int ROLE = decltype(role_c)::value;
    constexpr int NS = w3_ntile<ROLE>();
    constexpr int NP = ROLE == 0 ? 8 : 4;  // LDS-DMA issues per chunk and wave
    const int BI = ROLE == 0 ? L1 : L0, BJ = L0;
    auto pump_r = [&](int g) __attribute__((always_inline)) { pump(ROLE == 0 ? g : 2 * g); };
    auto gtile = [&](auto sc, int& I, int& J) __attribute__((always_inline)) {
      constexpr W3Tile t = w3_tile_at<ROLE>(decltype(sc)::value);
      I = 8 * BI + (ROLE == 0 ? ra : 0) + t.i;
      J = 8 * BJ + (ROLE == 0 ? cb0 : 0) + t.j;
    };
    // two-level accumulation: tiles flushed into the workspace slot every
    // kWideFlush chunks (MODE 1 entities longer than 2048 rows)
    auto flush = [&]() __attribute__((always_inline)) {
      w3_for<NS>([&](auto sc) __attribute__((always_inline)) {
        constexpr int s = decltype(sc)::value;
        int I, J;
        gtile(sc, I, J);
        float* t = wslot + (int64_t)tidx(I, J) * 1024;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float* pq = t + acc_row(r, hi) * 32 + lo;
          *pq = flushed ? *pq + acc[s][r] : acc[s][r];
        }
        acc[s] = f32x16{0.f};
        asm volatile("" ::: "memory");
      });
      flushed = true;
    };

    int prev = 0;  // the previous step's DMA issues (left in flight at its wait)
    bf16x8 F[2][8][3];  // split fragments of chunks c (F[c & 1]) and c + 1
    auto bw_of = [&](int x, float(&bw)[8]) __attribute__((always_inline)) {
      // rhs weights of chunk x's lane rows (diagonal roles, V kinds)
      if constexpr (ROLE != 0 && VK) {
#pragma unroll
        for (int ee = 0; ee < 8; ++ee) {
          const int64_t k = kbase + (int64_t)x * kWideChunk + 8 * hi + ee;
          bw[ee] = k < h ? bws_p[(x % W3NS) * kWideChunk + 8 * hi + ee] : 0.0f;
        }
      }
    };
    auto nopump = [](int) {};
    if (nchunks > 0) {
      // prologue: ids of chunks 0..6, rows of chunks 0..3, chunk 0 split
      if (wave == 0)
        for (int x = 0; x < 7 && x < nchunks; ++x) issue_ids(x);
      vm_wait(0);
      w3_barrier();
      int cnt[4] = {0, 0, 0, 0};
      for (int x = 0; x < 4; ++x) {  // past the end: the zero row
        prep_rows(x);
#pragma unroll
        for (int g = 0; g < NP; ++g) pump_r(g);
        cnt[x] = FRECSYS_SKIP(a.debug_skip, 32) ? 0 : NP;
        if (VK && wave == 3) {
          issue_bw(x);
          ++cnt[x];
        }
      }
      vm_wait(cnt[2] + cnt[3]);  // chunks 0 and 1 landed
      w3_barrier();
      prev = cnt[3];
      float bw[8];
      bw_of(0, bw);
      w3_step<ROLE, VK, NP, true>(ring, lanec, ra, cb0, F[1], F[0], acc, bw, bp, a.debug_skip,
                                  nopump);
    }
    // iteration c: chunk c's MFMAs (fragments split in iteration c - 1) with
    // chunk c + 1's reads and splits and chunk c + 4's row DMA beside them
    // (past the unit's end: the zero row, into a slot nobody reads -- issued
    // unconditionally, so that no branch splits the MFMA stream)
    auto iter = [&](int c, auto par) __attribute__((always_inline)) {
      constexpr int P = decltype(par)::value;
      prep_rows(c + 4);
      float bw[8];
      bw_of(c + 1, bw);
      tp_mark(1);
      w3_step<ROLE, VK, NP, false>(ring + ((c + 1) % W3NS) * W3SLOT, lanec, ra, cb0, F[P],
                                   F[1 - P], acc, bw, bp, a.debug_skip, pump_r);
      tp_mark(0);
      int n_iss = FRECSYS_SKIP(a.debug_skip, 32) ? 0 : NP;
      if (VK && wave == 3 && c + 4 < nchunks) {
        issue_bw(c + 4);
        ++n_iss;
      }
      if (wave == 0 && c + 7 < nchunks) {
        issue_ids(c + 7);
        ++n_iss;
      }
      vm_wait(n_iss + prev);  // chunk c + 2 landed; c + 3, c + 4 in flight
      prev = n_iss;
      w3_barrier();
      tp_mark(2);
    };
    // blocks of kWideFlush chunks: the two-level accumulation's flush (MODE 1
    // entities longer than 2048 rows) between blocks, outside the chunk loop
    // (inside it, its registers would spill the loop's); the rhs partial of a
    // block's chunks closes before its last iteration, which splits (and sums)
    // the next block's first chunk
#pragma unroll 1
    for (int c0 = 0; c0 < nchunks; c0 += kWideFlush) {
      const int c1 = c0 + kWideFlush < nchunks ? c0 + kWideFlush : nchunks;
#pragma unroll 1
      for (int c = c0; c < c1; c += 2) {
        if (MODE == 1 && ROLE != 0 && c == c1 - 1 && c1 < nchunks) {
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            bt[q] += bp[q];
            bp[q] = 0.0f;
          }
        }
        iter(c, std::integral_constant<int, 0>{});
        if (c + 1 < c1) {
          if (MODE == 1 && ROLE != 0 && c + 1 == c1 - 1 && c1 < nchunks) {
#pragma unroll
            for (int q = 0; q < 2; ++q) {
              bt[q] += bp[q];
              bp[q] = 0.0f;
            }
          }
          iter(c + 1, std::integral_constant<int, 1>{});
        }
      }
      if (MODE == 1 && c1 < nchunks) flush();  // block-uniform
    }
    // no LDS-DMA may outlive the workgroup (the CU hands its LDS to the next one)
    vm_wait(0);
#ifdef FRECSYS_ABLATION
    if (tprof) {
      const int o = (wave == 3 ? 4 : 0) + (off ? 0 : 8);
      atomicAdd(a.prof + o + 0, tp_acc[0]);
      atomicAdd(a.prof + o + 1, tp_acc[1]);
      atomicAdd(a.prof + o + 2, tp_acc[2]);
      atomicAdd(a.prof + o + 3, (unsigned long long)nchunks);
    }
#endif
    if (flushed) {
      w3_for<NS>([&](auto sc) __attribute__((always_inline)) {
        constexpr int s = decltype(sc)::value;
        int I, J;
        gtile(sc, I, J);
        const float* t = wslot + (int64_t)tidx(I, J) * 1024;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[s][r] += t[acc_row(r, hi) * 32 + lo];
        asm volatile("" ::: "memory");
      });
    }
    // slab layout: tile t's accumulator r of lane l at t * 1024 + r * 64 + l;
    // the diagonal doubles' b partials after the tiles, [block][half][column]
    const size_t slab_floats = (size_t)NT * 1024 + 2 * (size_t)Dp;
    auto bcol = [&](int q) __attribute__((always_inline)) {  // column (in block BI) of b partial q
      return 32 * (q ? 7 - wave : wave) + lo;
    };
    if (MODE == 2) {
      float* sb = a.slabs + (size_t)a.work[unit].slab * slab_floats;
      w3_for<NS>([&](auto sc) __attribute__((always_inline)) {
        constexpr int s = decltype(sc)::value;
        int I, J;
        gtile(sc, I, J);
        float* t = sb + (int64_t)tidx(I, J) * 1024 + lane;
#pragma unroll
        for (int r = 0; r < 16; ++r) t[r * 64] = acc[s][r];
        asm volatile("" ::: "memory");
      });
      if (ROLE != 0) {
        float* bb = sb + (size_t)NT * 1024 + 512 * BI + 256 * hi;
#pragma unroll
        for (int q = 0; q < 2; ++q) bb[bcol(q)] = bp[q];
      }
      return;
    }
    if (fin) {
      // the unsplit sums: slab sums folded left to right (t = s_1, t = t +
      // s_j, ...), b likewise
      const int2 sp = a.split[pos0 + unit];
#pragma unroll 1
      for (int jj = 0; jj < sp.y; ++jj) {
        const float* sb = a.slabs + (size_t)(sp.x + jj) * slab_floats;
        w3_for<NS>([&](auto sc) __attribute__((always_inline)) {
          constexpr int s = decltype(sc)::value;
          int I, J;
          gtile(sc, I, J);
          const float* t = sb + (int64_t)tidx(I, J) * 1024 + lane;
          f32x16 v;
#pragma unroll
          for (int r = 0; r < 16; ++r) v[r] = t[r * 64];
          acc[s] = jj == 0 ? v : acc[s] + v;
          asm volatile("" ::: "memory");
        });
        if (ROLE != 0) {
          const float* bb = sb + (size_t)NT * 1024 + 512 * BI + 256 * hi;
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const float v = bb[bcol(q)];
            if (jj + 1 < sp.y) bt[q] += v;
            else bp[q] = v;
          }
        }
      }
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) bp[q] += bt[q];

    // epilogue: the G part and the per-kind finish of A (as solve.hip)
    const float hf = (float)h;
    const float omega = (is_u_kind(kind) && a.entity_weight) ? a.entity_weight[e] : 1.0f;
    const float lam = entity_lambda(kind, a.reg, a.reg_exp, a.w, a.alpha, h, a.n_other,
                                    a.entity_reg, e, a.lambda_is_reg);
    const float gscale = kind == KIND_IALS ? a.w : (is_u_kind(kind) ? hf * a.w : a.w);
    const float us = omega / hf;
    // the kind is dispatched per tile, after the tile's G loads: with the
    // dispatch outside the tile loop the compiler hoists all tiles' G loads
    // (common to the four variants) above it and spills
    const int fm = is_grad_kind(kind) ? 3 : is_u_kind(kind) ? 1 : VK ? 2 : 0;
    w3_for<NS>([&](auto sc) __attribute__((always_inline)) {
      constexpr int s = decltype(sc)::value;
      int I, J;
      gtile(sc, I, J);
      float* t = wslot + (int64_t)tidx(I, J) * 1024;
      float gv[16];
#pragma unroll
      for (int r = 0; r < 16; ++r)
        gv[r] = a.G[(int64_t)(32 * I + acc_row(r, hi)) * Dp + 32 * J + lo];
      if (fm == 0) w3_finish<0>(acc[s], gv, I, J, t, kind, a.w, gscale, lam, hf, omega, us, lo, hi);
      else if (fm == 1) w3_finish<1>(acc[s], gv, I, J, t, kind, a.w, gscale, lam, hf, omega, us, lo, hi);
      else if (fm == 2) w3_finish<2>(acc[s], gv, I, J, t, kind, a.w, gscale, lam, hf, omega, us, lo, hi);
      else w3_finish<3>(acc[s], gv, I, J, t, kind, a.w, gscale, lam, hf, omega, us, lo, hi);
      asm volatile("" ::: "memory");
    });
    if (ROLE != 0) {  // b of this block: the two row halves of each column
      float* bb = wslot + (int64_t)NT * 1024 + 256 * BI;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        float b = bp[q] + __shfl_xor(bp[q], 32);
        if (is_u_kind(kind)) b *= us;  // rhs *= weight / history_size
        if (hi == 0) bb[bcol(q)] = b;
      }
    }
  };
  if (off) run(std::integral_constant<int, 0>{});
  else if (wave == 0) run(std::integral_constant<int, 1>{});
  else if (wave == 1) run(std::integral_constant<int, 2>{});
  else if (wave == 2) run(std::integral_constant<int, 3>{});
  else run(std::integral_constant<int, 4>{});
}

}  // namespace

hipError_t launch_wide_presplit(int Dp, const SolveArgs& a, char* xs, hipStream_t s) {
  if (!wide_dim(Dp) || !xs) return hipErrorInvalidValue;
  if (!is_v_kind(a.kind))  // the zero row only
    return hipMemsetAsync(xs, 0, sizeof(float) * Dp, s);
  const int64_t threads = (a.n_other + 1) * (Dp / 4);
  float* x = reinterpret_cast<float*>(xs);
  hipLaunchKernelGGL(wide_prescale_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s,
                     a.X, a.n_other, Dp, a.other_weight, x, x + (a.n_other + 1) * Dp);
  return hipGetLastError();
}

hipError_t launch_wide_syrk3(int Dp, const SolveArgs& a, int mode, int64_t pos0, int64_t n,
                             float* ws, hipStream_t s) {
  if (!wide_dim(Dp) || !a.xsplit) return hipErrorInvalidValue;
  if (n <= 0) return hipSuccess;
  const int NB = Dp / 256, P = NB * (NB - 1) / 2 + NB;
  const bool vk = is_v_kind(a.kind);
  const dim3 grid(xcd_grid(n, P)), block(256);
  if (mode == 2) {
    if (vk)
      hipLaunchKernelGGL((wide_syrk3_kernel<2, true>), grid, block, 0, s, a, Dp, (int64_t)0, ws, n);
    else
      hipLaunchKernelGGL((wide_syrk3_kernel<2, false>), grid, block, 0, s, a, Dp, (int64_t)0, ws, n);
  } else {
    if (vk)
      hipLaunchKernelGGL((wide_syrk3_kernel<1, true>), grid, block, 0, s, a, Dp, pos0, ws, n);
    else
      hipLaunchKernelGGL((wide_syrk3_kernel<1, false>), grid, block, 0, s, a, Dp, pos0, ws, n);
  }
  return hipGetLastError();
}

}  // namespace frecsys_hip
