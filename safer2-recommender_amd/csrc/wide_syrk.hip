// wide_syrk.hip -- the d-space SYRK of A = X_h^T D X_h at Dp = 512 / 1024
// (the rank updates of Project / ProjectU / ProjectV at the wide dims:
// ials.h:101-131, safer2.h:133-150, 181-199, erm_mf.h, cvar_mf.h) with every
// staged byte moved by LDS-DMA.
//
// The products are fp32-accurate split-bf16 MFMAs (common.h mfma_x6): each
// fp32 value x~ = sa x (sa = sqrt(nu) on the V kinds, else 1) is three bf16
// pieces.  The pieces depend on the gathered ROW only, not on the entity that
// gathers it, so they are formed once per half-step for the whole other side
// (wide_presplit_kernel: [row][hi | mid | lo][Dp] bf16 + a 128-B tail holding
// the rhs weight), instead of once per (entity, row) in every SYRK workgroup.
// The SYRK workgroups then only move bytes and multiply:
//
//   * LDS-DMA (global_load_lds_dwordx4, a per-lane source address = a row
//     gather) brings each chunk of 16 history rows -- three 1-KB piece rows
//     per row, the two 256-column blocks the workgroup reads -- into a
//     3-slot LDS ring two chunks ahead of its MFMAs.  No VGPR staging, no
//     split VALU, no ds_write; one barrier per chunk.  The row ids arrive the
//     same way (4-byte LDS-DMA, four chunks ahead), so the loop issues no
//     vector load the compiler would wait on.
//   * MFMA operands come out of the ring with ds_read_b64_tr_b16 (the
//     hardware transpose read): the piece rows are stored row-major as they
//     arrive, and a lane reads 4 consecutive k of its column per read.  The
//     16-B chunks of row j are XOR-swizzled by 4 (j mod 4) on the DMA's source
//     address, which makes every transposed read conflict-free.
//   * Two kinds of workgroup per unit, both reading whole 512-column piece
//     rows: an off-diagonal 256 x 256 block pair (64 tiles, 2 x 4 per wave),
//     and a diagonal double (the two lower 8 x 8-tile triangles of a pair of
//     diagonal blocks, 72 tiles, 9 per wave: rows q and 7 - q of one
//     triangle).  At Dp = 512 that is two workgroups per entity streaming the
//     same rows at nearly the same rate (64 / 72 tiles), on one XCD.
//
// Every tile sees exactly the products of wide_syrk2_kernel, in the same order
// (mfma_x6 per chunk, chunks in order, the same two-level accumulation and
// slab layout), and b the same fp32 sums (x~ = hi + mid + lo exactly), so the
// output is bit-identical to the register-staged kernel it replaces
// (tests/test_wide_syrk3_gpu.py).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "common.h"
#include "kernels.h"
#include "wide.h"

namespace frecsys_hip {

namespace {

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int W3ROW = 1024;                  // one staged piece row: 512 bf16
constexpr int W3PIECE = kWideChunk * W3ROW;  // 16 KB: one piece of a chunk
constexpr int W3SLOT = 3 * W3PIECE;          // 48 KB: a chunk's three pieces
constexpr int W3NS = 3;                      // ring slots
constexpr int W3IDS = 4;                     // row-id ring slots
constexpr int W3OFF_IDS = W3NS * W3SLOT;
constexpr int W3OFF_TAIL = W3OFF_IDS + W3IDS * kWideChunk * 4;
constexpr int W3LDS = W3OFF_TAIL + W3NS * kWideChunk * 16;

// ---- pre-split table ----
// Grid-stride over the (n + 1) * Dp / 4 column quads: the grid is capped
// (launch_wide_presplit), so any row count launches (a one-thread-per-quad
// grid passes 2^32 work-items past ~16.7M rows at Dp = 1024).
__global__ void __launch_bounds__(256)
    wide_presplit_kernel(const float* __restrict__ X, int64_t n, int Dp,
                         const float* __restrict__ nu, char* __restrict__ xs, int64_t rb) {
#pragma clang fp contract(off)
  const int per_row = Dp >> 2;
  const int64_t total = (n + 1) * per_row;
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < total; t += stride) {
    const int64_t r = t / per_row;
    const int c4 = (int)(t % per_row) * 4;
    char* row = xs + r * rb;
    if (r == n) {  // the zero row
#pragma unroll
      for (int p = 0; p < 3; ++p)
        *reinterpret_cast<uint2*>(row + 2 * ((int64_t)p * Dp + c4)) = make_uint2(0u, 0u);
      if (c4 == 0) *reinterpret_cast<float4*>(row + 6 * (int64_t)Dp) = make_float4(0.f, 0.f, 0.f, 0.f);
      continue;
    }
    float sa = 1.0f, bw = 1.0f;
    if (nu) {  // rows pre-scaled by sqrt(nu); rhs weight nu / sqrt(nu) (safer2.h:190-192)
      const float w = nu[r];
      sa = sqrtf(w);
      bw = sa > 0.0f ? w / sa : 0.0f;
    }
    const float4 x4 = *reinterpret_cast<const float4*>(X + r * Dp + c4);
    const float xv[4] = {x4.x * sa, x4.y * sa, x4.z * sa, x4.w * sa};
    __bf16 pc[3][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) split3(xv[j], pc[0][j], pc[1][j], pc[2][j]);
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      uint2 u;
      __builtin_memcpy(&u, pc[p], 8);
      *reinterpret_cast<uint2*>(row + 2 * ((int64_t)p * Dp + c4)) = u;
    }
    if (c4 == 0) *reinterpret_cast<float4*>(row + 6 * (int64_t)Dp) = make_float4(bw, 0.f, 0.f, 0.f);
  }
}

// LDS-DMA helpers (glds16, glds4, vm_wait, w3_barrier, lds_addr): common.h

// The three pieces of the 32 x 16 MFMA operand of LDS column block cb
// (columns 32 cb .. 32 cb + 31 of the staged rows) from the ring slot at LDS
// byte address slot: two ds_read_b64_tr_b16 per piece (k 0-3, 4-7 of the
// lane's half).  lanec: the lane's row / chunk offset (see the kernel), q =
// (lane >> 2) & 3 its row within each 4-row read (the swizzle key).
__device__ __forceinline__ void w3_frag(unsigned slot, unsigned lanec, int q, int cb,
                                        bf16x8 (&f)[3]) {
  const unsigned a0 = slot + lanec + 64u * (unsigned)(cb ^ q);
#pragma unroll
  for (int p = 0; p < 3; ++p) {
    const s16x4 x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(uintptr_t)(a0 + p * W3PIECE));
    const s16x4 x1 =
        __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(uintptr_t)(a0 + p * W3PIECE + 4 * W3ROW));
    const s16x8 v = __builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7);
    f[p] = __builtin_bit_cast(bf16x8, v);
  }
}

// rhs part of one operand: bpart += bw_e * x~_e over the lane's 8 rows, in
// row order, each product rounded before its add (the register-staged
// kernel's fp32 sums; x~ = (hi + mid) + lo exactly).  Not VK: bw = 1 (the
// rows past the unit's end are the zero row), and 1 * x~ is x~.
template <bool VK>
__device__ __forceinline__ void w3_bsum(const bf16x8 (&f)[3], const float (&bw)[8], float& b) {
#pragma clang fp contract(off)
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float x = ((float)f[0][e] + (float)f[1][e]) + (float)f[2][e];
    if constexpr (VK) b += bw[e] * x;
    else b += x;
  }
}

// Tile coordinates (block-local tile row / column) of accumulator slot s:
// ROLE 0 = off-diagonal pair (rows ra, ra + 1 of the pair's row block x
// columns cb0 .. cb0 + 3 of its column block), ROLE 1 + q = diagonal
// triangle rows 7 - q (slots 0 .. 7 - q) and q (slots 8 - q .. 8).
template <int ROLE>
__device__ __forceinline__ void w3_tile(int s, int ra, int cb0, int& i, int& j) {
  if constexpr (ROLE == 0) {
    i = ra + (s >> 2);
    j = cb0 + (s & 3);
  } else {
    constexpr int q = ROLE - 1;
    if (s <= 7 - q) {
      i = 7 - q;
      j = s;
    } else {
      i = q;
      j = s - (8 - q);
    }
  }
}
template <int ROLE>
constexpr int w3_slots() {
  return ROLE == 0 ? 8 : 9;
}

// The MFMAs of one chunk.  ROLE 0: A fragments of LDS column blocks
// 8 + ra, 9 + ra (the row block), B of cb0 .. cb0 + 3 (the column block);
// ROLE 1 + q: the triangle of LDS column blocks 8 tr .. 8 tr + 7, A of rows q
// and 7 - q, B of columns 0 .. 7 - q (the A fragments serve as B at columns q
// and 7 - q).  Every tile: one mfma_x6 (A = its row, B = its column).
// pump(g), g = 0..5: the chunk's six LDS-DMA issues for a later chunk, spread
// over the tile groups so that the DMA's issue cost hides under the MFMAs.
template <int ROLE, bool BOWN, bool VK, typename Pump>
__device__ __forceinline__ void w3_chunk(unsigned slot, unsigned lanec, int q, int ra, int cb0,
                                         int tr, f32x16 (&acc)[9], const float (&bw)[8],
                                         float& blo, float& bhi, int skip, Pump&& pump) {
  (void)skip;  // ablation masks (FRECSYS_DEBUG_SKIP): 1 no MFMAs, 2048 no rhs sums
  if constexpr (ROLE == 0) {
    bf16x8 A0[3], A1[3], B[3], Bn[3];
    w3_frag(slot, lanec, q, 8 + ra, A0);
    w3_frag(slot, lanec, q, 9 + ra, A1);
    w3_frag(slot, lanec, q, cb0, B);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (j < 3) w3_frag(slot, lanec, q, cb0 + j + 1, Bn);
      if (!FRECSYS_SKIP(skip, 1)) {
        acc[j] = mfma_x6(A0, B, acc[j]);
        acc[4 + j] = mfma_x6(A1, B, acc[4 + j]);
      }
      if (j < 3) {
        pump(2 * j);
        pump(2 * j + 1);
#pragma unroll
        for (int p = 0; p < 3; ++p) B[p] = Bn[p];
      }
    }
  } else {
    constexpr int Q = ROLE - 1, G = 8 - Q;  // tile groups (B columns 0 .. 7 - Q)
    const int base = 8 * tr;
    bf16x8 Alo[3], Ahi[3], B[3], Bn[3];
    w3_frag(slot, lanec, q, base + Q, Alo);
    w3_frag(slot, lanec, q, base + 7 - Q, Ahi);
    // B fragments read: columns 0 .. 7 - Q except Q and 7 - Q
    auto need = [](int j) { return j != Q && j != 7 - Q; };
    int first = 0;
    while (first <= 7 - Q && !need(first)) ++first;
    if (first <= 7 - Q) w3_frag(slot, lanec, q, base + first, B);
#pragma unroll
    for (int j = 0; j < G; ++j) {
      int nx = j + 1;
      while (nx <= 7 - Q && !need(nx)) ++nx;
      if (need(j) && nx <= 7 - Q) w3_frag(slot, lanec, q, base + nx, Bn);
      const bf16x8(&Bj)[3] = j == Q ? Alo : (j == 7 - Q ? Ahi : B);
      if (!FRECSYS_SKIP(skip, 1)) {
        acc[j] = mfma_x6(Ahi, Bj, acc[j]);
        if (j <= Q) acc[8 - Q + j] = mfma_x6(Alo, Bj, acc[8 - Q + j]);
      }
#pragma unroll
      for (int g = 6 * j / G; g < 6 * (j + 1) / G; ++g) pump(g);
      if (need(j) && nx <= 7 - Q) {
#pragma unroll
        for (int p = 0; p < 3; ++p) B[p] = Bn[p];
      }
    }
    if (BOWN && !FRECSYS_SKIP(skip, 2048)) {
      w3_bsum<VK>(Alo, bw, blo);
      w3_bsum<VK>(Ahi, bw, bhi);
    }
  }
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
__global__ void __launch_bounds__(512)
    wide_syrk3_kernel(SolveArgs a, int Dp, int64_t pos0, float* ws, int64_t n_units) {
  __shared__ __attribute__((aligned(16))) char lds[W3LDS];
  const int tid = threadIdx.x, lane = tid & 63, lo = lane & 31, hi = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int T = Dp >> 5, NT = T * (T + 1) / 2, NB = Dp >> 8;
  const int noff = NB * (NB - 1) / 2;
  int64_t unit;
  int pidx;
  if (!xcd_unit(noff + NB / 2, n_units, unit, pidx)) return;
  // the two 256-column blocks in LDS columns [0, 256) (L0) and [256, 512) (L1)
  const bool off = pidx < noff;
  int L0, L1;
  if (off) {
    L1 = 1;
    while (L1 * (L1 + 1) / 2 <= pidx) ++L1;
    L0 = pidx - L1 * (L1 - 1) / 2;
  } else {
    L0 = 2 * (pidx - noff);
    L1 = L0 + 1;
  }
  const int kind = a.kind;
  constexpr bool vk = VK;  // is_v_kind(kind), checked by the launcher

  SplitWork sw{};
  if (MODE == 2) sw = a.work[unit];
  const QueueRec rec = a.order[MODE == 2 ? (int64_t)sw.pos : pos0 + unit];
  const int64_t e = rec.entity, h = rec.h, p0 = rec.p0;
  if (h == 0) return;  // untouched entity (no barrier passed yet)
  int64_t extra = 0;
  if (vk && a.quirk && h > 128 && (h % 128) != 0) extra = 128 - (h % 128);
  int64_t kbase = 0, klim = h + extra;
  bool fin = false;
  if (MODE == 2) {
    kbase = sw.k0;
    klim = sw.k1;
  } else {
    fin = pos0 + unit < a.n_split;
  }
  const int nchunks = fin ? 0 : (int)((klim - kbase + kWideChunk - 1) / kWideChunk);

  const char* xs = a.xsplit;
  const int64_t rb = wide_xsplit_row_bytes(Dp);
  const int64_t zrow = a.n_other;
  const unsigned ring = lds_addr(lds), ids = ring + W3OFF_IDS, tails = ring + W3OFF_TAIL;
  const int* ids_p = reinterpret_cast<const int*>(lds + W3OFF_IDS);
  const float* tails_p = reinterpret_cast<const float*>(lds + W3OFF_TAIL);

  // the DMA lane map: lane l fills 16-B chunk l of a staged row j from the
  // row's logical chunk l ^ 4 (j mod 4), i.e. columns 8 lc .. 8 lc + 7 of
  // block L[lc >> 5]; this wave fills rows 2 wave, 2 wave + 1
  int64_t colb[2];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int lc = lane ^ (4 * ((2 * wave + r) & 3));
    colb[r] = 2 * (int64_t)(256 * (lc < 32 ? L0 : L1) + 8 * (lc & 31));
  }
  auto issue_ids = [&](int x) __attribute__((always_inline)) {  // wave 0: chunk x's row ids
    if (lane < kWideChunk) {
      int64_t k = kbase + (int64_t)x * kWideChunk + lane;
      if (k >= klim) k = klim - 1;
      glds4(a.col + p0 + wide_virt_pos(k, h),
            __builtin_amdgcn_readfirstlane(ids + (x % W3IDS) * kWideChunk * 4));
    }
  };
  // the wave's two rows of chunk x: their sources (ids from the ring) and the
  // LDS address of row 2 wave of x's slot; pump(g) issues piece g % 3 of row
  // 2 wave + g / 3 (one 1-KB LDS-DMA), the chunk's six spread over its MFMAs
  const char* rsrc[2] = {xs, xs};
  unsigned rdst = 0;
  bool rlive = false;
  auto prep_rows = [&](int x) __attribute__((always_inline)) {
    const int2 idp = *reinterpret_cast<const int2*>(ids_p + (x % W3IDS) * kWideChunk + 2 * wave);
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int64_t k = kbase + (int64_t)x * kWideChunk + 2 * wave + r;
      const int64_t id = k < klim ? (int64_t)(r ? idp.y : idp.x) : zrow;
      rsrc[r] = xs + id * rb + colb[r];
    }
    rdst = ring + (x % W3NS) * W3SLOT + 2 * wave * W3ROW;
  };
  auto pump = [&](int g) __attribute__((always_inline)) {
    if (rlive)
      glds16(rsrc[g / 3] + 2 * (int64_t)(g % 3) * Dp,
             __builtin_amdgcn_readfirstlane(rdst + (g % 3) * W3PIECE + (g / 3) * W3ROW));
  };
  auto issue_tail = [&](int x) __attribute__((always_inline)) {  // wave 7, V kinds: rhs weights
    if (lane < kWideChunk) {
      const int64_t k = kbase + (int64_t)x * kWideChunk + lane;
      const int64_t id = k < klim ? (int64_t)ids_p[(x % W3IDS) * kWideChunk + lane] : zrow;
      glds16(xs + id * rb + 6 * (int64_t)Dp,
             __builtin_amdgcn_readfirstlane(tails + (x % W3NS) * kWideChunk * 16));
    }
  };

  // operand-read lane constants (w3_frag)
  const int q = (lane >> 2) & 3, pp = lane & 3, g = lane >> 4;
  const unsigned lanec = (unsigned)((8 * hi + q) * W3ROW + 8 * (pp & 1) + 16 * (2 * (g & 1) + (pp >> 1)));
  // roles
  const int ra = 2 * (wave >> 1), cb0 = 4 * (wave & 1);  // off-diagonal
  const int tr = wave >> 2, qd = wave & 3;               // diagonal

  f32x16 acc[9];
#pragma unroll
  for (int s = 0; s < 9; ++s) acc[s] = f32x16{0.f};
  float blo = 0.0f, bhi = 0.0f, btlo = 0.0f, bthi = 0.0f;
  bool flushed = false;
  float* const wslot = MODE == 1 ? ws + unit * ((int64_t)NT * 1024 + Dp) : nullptr;

#ifdef FRECSYS_ABLATION
  // diagnostics (FRECSYS_DUAL_PROF, ablation builds): per-chunk phase cycles
  // of waves 0 and 7 -- 0 the chunk's MFMAs and operand reads, 1 the DMA
  // issue, 2 the wait for the next chunk and the barrier
  const bool tprof = a.prof && lane == 0 && (wave == 0 || wave == 7);
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
    constexpr int NS = w3_slots<ROLE>();
    const int BI = ROLE == 0 ? L1 : (tr ? L1 : L0), BJ = ROLE == 0 ? L0 : BI;
    auto gtile = [&](int s, int& I, int& J) __attribute__((always_inline)) {
      int i, j;
      w3_tile<ROLE>(s, ra, cb0, i, j);
      I = 8 * BI + i;
      J = 8 * BJ + j;
    };
    // two-level accumulation: tiles flushed into the workspace slot every
    // kWideFlush chunks (MODE 1 entities longer than 2048 rows)
    auto flush = [&]() __attribute__((always_inline)) {
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        int I, J;
        gtile(s, I, J);
        float* t = wslot + (int64_t)tidx(I, J) * 1024;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float* pq = t + acc_row(r, hi) * 32 + lo;
          *pq = flushed ? *pq + acc[s][r] : acc[s][r];
        }
        acc[s] = f32x16{0.f};
        asm volatile("" ::: "memory");
      }
      flushed = true;
    };

    if (nchunks > 0) {
      // prologue: ids of chunks 0..3, then rows of chunks 0, 1
      if (wave == 0)
        for (int x = 0; x < 4 && x < nchunks; ++x) issue_ids(x);
      vm_wait(0);
      w3_barrier();
      int n1 = 0;
      for (int x = 0; x < 2 && x < nchunks; ++x) {
        prep_rows(x);
        rlive = true;
#pragma unroll
        for (int g = 0; g < 6; ++g) pump(g);
        if (vk && wave == 7) issue_tail(x);
        if (x == 1) n1 = 6 + ((vk && wave == 7) ? 1 : 0);
      }
      vm_wait(n1);
      w3_barrier();
    }
#pragma unroll 1
    for (int c = 0; c < nchunks; ++c) {
      // chunk c's MFMAs, with chunk c + 2's row DMA spread over them
      rlive = c + 2 < nchunks && !FRECSYS_SKIP(a.debug_skip, 32);
      if (rlive) prep_rows(c + 2);
      // rhs weights of the lane's 8 rows (diagonal doubles, V kinds)
      float bw[8];
      if constexpr (ROLE != 0 && VK) {
#pragma unroll
        for (int ee = 0; ee < 8; ++ee) {
          const int64_t k = kbase + (int64_t)c * kWideChunk + 8 * hi + ee;
          bw[ee] = k < h ? tails_p[((c % W3NS) * kWideChunk + 8 * hi + ee) * 4] : 0.0f;
        }
      }
      tp_mark(1);
      w3_chunk<ROLE, ROLE != 0, VK>(ring + (c % W3NS) * W3SLOT, lanec, q, ra, cb0, tr, acc, bw,
                                    blo, bhi, a.debug_skip, pump);
      tp_mark(0);
      int n_iss = rlive ? 6 : 0;
      if (rlive && vk && wave == 7) {
        issue_tail(c + 2);
        ++n_iss;
      }
      if (wave == 0 && c + 4 < nchunks) {
        issue_ids(c + 4);
        ++n_iss;
      }
      if (MODE == 1 && (c + 1) % kWideFlush == 0 && c + 1 < nchunks) {  // block-uniform
        if (ROLE != 0) {
          btlo += blo;
          bthi += bhi;
          blo = 0.0f;
          bhi = 0.0f;
        }
        flush();
      }
      vm_wait(n_iss);
      w3_barrier();
      tp_mark(2);
    }
#ifdef FRECSYS_ABLATION
    if (tprof) {
      const int o = (wave == 7 ? 4 : 0) + (off ? 0 : 8);
      atomicAdd(a.prof + o + 0, tp_acc[0]);
      atomicAdd(a.prof + o + 1, tp_acc[1]);
      atomicAdd(a.prof + o + 2, tp_acc[2]);
      atomicAdd(a.prof + o + 3, (unsigned long long)nchunks);
    }
#endif
    if (flushed) {
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        int I, J;
        gtile(s, I, J);
        const float* t = wslot + (int64_t)tidx(I, J) * 1024;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[s][r] += t[acc_row(r, hi) * 32 + lo];
        asm volatile("" ::: "memory");
      }
    }
    // slab layout: tile t's accumulator r of lane l at t * 1024 + r * 64 + l;
    // the diagonal doubles' b partials after the tiles, [block][half][column]
    const size_t slab_floats = (size_t)NT * 1024 + 2 * (size_t)Dp;
    const int qlo = ROLE == 0 ? 0 : ROLE - 1;
    const int clo = 32 * qlo + lo, chi = 32 * (7 - qlo) + lo;  // columns in block BI
    if (MODE == 2) {
      float* sb = a.slabs + (size_t)a.work[unit].slab * slab_floats;
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        int I, J;
        gtile(s, I, J);
        float* t = sb + (int64_t)tidx(I, J) * 1024 + lane;
#pragma unroll
        for (int r = 0; r < 16; ++r) t[r * 64] = acc[s][r];
        asm volatile("" ::: "memory");
      }
      if (ROLE != 0) {
        float* bb = sb + (size_t)NT * 1024 + 512 * BI + 256 * hi;
        bb[clo] = blo;
        bb[chi] = bhi;
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
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          int I, J;
          gtile(s, I, J);
          const float* t = sb + (int64_t)tidx(I, J) * 1024 + lane;
          f32x16 v;
#pragma unroll
          for (int r = 0; r < 16; ++r) v[r] = t[r * 64];
          acc[s] = jj == 0 ? v : acc[s] + v;
          asm volatile("" ::: "memory");
        }
        if (ROLE != 0) {
          const float* bb = sb + (size_t)NT * 1024 + 512 * BI + 256 * hi;
          const float vlo = bb[clo], vhi = bb[chi];
          if (jj + 1 < sp.y) {
            btlo += vlo;
            bthi += vhi;
          } else {
            blo = vlo;
            bhi = vhi;
          }
        }
      }
    }
    blo += btlo;
    bhi += bthi;

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
    const int fm = is_grad_kind(kind) ? 3 : is_u_kind(kind) ? 1 : vk ? 2 : 0;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      int I, J;
      gtile(s, I, J);
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
    }
    if (ROLE != 0) {  // b of this block: the two row halves of each column
      float b0 = blo + __shfl_xor(blo, 32);
      float b1 = bhi + __shfl_xor(bhi, 32);
      if (hi == 0) {
        if (is_u_kind(kind)) {  // rhs *= weight / history_size
          b0 *= us;
          b1 *= us;
        }
        float* bb = wslot + (int64_t)NT * 1024 + 256 * BI;
        bb[clo] = b0;
        bb[chi] = b1;
      }
    }
  };
  if (off) run(std::integral_constant<int, 0>{});
  else if (qd == 0) run(std::integral_constant<int, 1>{});
  else if (qd == 1) run(std::integral_constant<int, 2>{});
  else if (qd == 2) run(std::integral_constant<int, 3>{});
  else run(std::integral_constant<int, 4>{});
}

}  // namespace

hipError_t launch_wide_presplit(int Dp, const SolveArgs& a, char* xs, hipStream_t s) {
  if (!wide_dim(Dp) || !xs) return hipErrorInvalidValue;
  const int64_t threads = (a.n_other + 1) * (Dp / 4);
  const float* nu = is_v_kind(a.kind) ? a.other_weight : nullptr;
  // 256 CUs x 8 workgroups x 32 quads each per pass: far past the chip's
  // residency, and the grid-stride loop takes any row count
  const int64_t blocks = std::min<int64_t>((threads + 255) / 256, (int64_t)1 << 16);
  hipLaunchKernelGGL(wide_presplit_kernel, dim3((unsigned)blocks), dim3(256), 0, s,
                     a.X, a.n_other, Dp, nu, xs, wide_xsplit_row_bytes(Dp));
  return hipGetLastError();
}

hipError_t launch_wide_syrk3(int Dp, const SolveArgs& a, int mode, int64_t pos0, int64_t n,
                             float* ws, hipStream_t s) {
  if (!wide_dim(Dp) || !a.xsplit) return hipErrorInvalidValue;
  if (n <= 0) return hipSuccess;
  const int NB = Dp / 256, P = NB * (NB - 1) / 2 + NB / 2;
  const bool vk = is_v_kind(a.kind);
  const dim3 grid(xcd_grid(n, P)), block(512);
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
