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
//   3. solve: right-looking blocked Cholesky on the LDS tiles -- a 32x32
//      diagonal factor (one wave, register rows + readlane broadcasts), a
//      lane-per-row TRSM of the panel (the right-hand side rides along as
//      one extra row, so y = L^-1 b comes out of the factorisation), MFMA
//      trailing updates; then L^T x = y by one wave.
//   CVaR-MF kinds skip 3 and take one gradient step with the full matrix
//   whose strict upper triangle lacks the observed term (cvar_mf.h:133).
//
// Small kernel (Dp = 8, 16): one wave per entity, VALU assembly, the dense
// solve by one lane (the reference's own tests run at dim 8).
#include <hip/hip_runtime.h>

#include "common.h"
#include "kernels.h"

namespace frecsys_hip {

namespace {

constexpr int kRing = 4;

template <int T>
struct TiledCfg {
  static constexpr int Dp = 32 * T;
  static constexpr int NT = T * (T + 1) / 2;
  static constexpr int NW = (T <= 2) ? 4 : 8;       // waves per workgroup
  static constexpr int NTHR = NW * 64;
  static constexpr int MT = (NT + NW - 1) / NW;     // tiles per wave (max)
  static constexpr int R = (T <= 2) ? 16 : 32;      // rows per staged chunk
  static constexpr int NSLOT = R * Dp / 4;          // float4 per chunk
  static constexpr int NQ = (NSLOT + NTHR - 1) / NTHR;
  // LDS carve (floats); every offset a multiple of 4 floats (16 B).
  static constexpr int TILES = NT * 1024;
  static constexpr int STAGE = 2 * R * Dp;          // aliases TILES
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
};

// Virtual history position k -> offset within the entity's CSR row: k < h
// are the real rows; with the tail quirk rows h .. h+extra-1 re-read the
// positions [h-128, h-r) (safer2.h:200-204).
__device__ __forceinline__ int64_t virt_pos(int64_t k, int64_t h) {
  return k < h ? k : (h - 128 + (k - h));
}

// 32x32 diagonal factor by one wave (lane r and r+32 own row r; only lanes
// < 32 write).  Left-looking over columns: at step k every lane forms
// t = a[k] - sum_{m<k} a[m] L[k][m] (for lane k that is the pivot); row k of
// L is read back as LDS broadcasts from the unswizzled copy `ld`, which each
// lane fills with its own L[r][k] as soon as it is known (LDS operations of
// one wave complete in issue order).  Writes the factor (upper zeroed) back
// into the swizzled tile and leaves the row-major copy for the TRSM.
__device__ __forceinline__ bool diag_factor(float* tile, float* ld, int lane) {
  const int r = lane & 31;
  const bool wr = lane < 32;
  float a[32];
#pragma unroll
  for (int c = 0; c < 32; ++c) a[c] = tile[sw(r, c)];
  bool ok = true;
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    float t = a[k];
#pragma unroll 4
    for (int m = 0; m < k; ++m) t -= a[m] * ld[k * 32 + m];
    if (r == k) {
      ok = t > 0.0f;
      a[k] = sqrtf(t);
      if (wr) ld[k * 32 + k] = a[k];
    }
    __builtin_amdgcn_wave_barrier();
    const float d = ld[k * 32 + k];
    if (r > k) {
      a[k] = t / d;
      if (wr) ld[r * 32 + k] = a[k];
    }
  }
  if (wr) {
#pragma unroll
    for (int c = 0; c < 32; ++c) {
      const float v = (c <= r) ? a[c] : 0.0f;
      tile[sw(r, c)] = v;
      ld[r * 32 + c] = v;
    }
  }
  // the pivot check lives on lane r == k; fold it over the wave
  return __all(ok) != 0;
}

// Forward substitution x := x L^-T for one row of 32 (L row-major, lower).
__device__ __forceinline__ void trsm_row(float (&x)[32], const float* L) {
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    float t = x[k];
#pragma unroll 4
    for (int m = 0; m < k; ++m) t -= x[m] * L[k * 32 + m];
    x[k] = t / L[k * 32 + k];
  }
}

template <int T>
__global__ void __launch_bounds__(TiledCfg<T>::NTHR)
    solve_tiled_kernel(SolveArgs a) {
  using C = TiledCfg<T>;
  constexpr int Dp = C::Dp, NT = C::NT, NW = C::NW, NTHR = C::NTHR, MT = C::MT;
  constexpr int R = C::R, NQ = C::NQ, NSLOT = C::NSLOT;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* tiles = smem;
  float* stage = smem;
  float* bvec = smem + C::OFF_B;
  float* xvec = smem + C::OFF_X;
  float* ldc = smem + C::OFF_LD;
  float* ring_sa = smem + C::OFF_SA;
  float* ring_bw = smem + C::OFF_BW;
  int* ring_id = reinterpret_cast<int*>(smem + C::OFF_ID);
  int* flag = reinterpret_cast<int*>(smem + C::OFF_FLAG);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lo = lane & 31, hi = lane >> 5;
  const int64_t e = a.row_lo + blockIdx.x;
  const int64_t p0 = a.row_ptr[e];
  const int64_t h = a.row_ptr[e + 1] - p0;
  if (h == 0) return;  // not in by_user / by_item: untouched
  const int kind = a.kind;
  const bool vk = is_v_kind(kind);
  int64_t extra = 0;
  if (vk && a.quirk && h > 128 && (h % 128) != 0) extra = 128 - (h % 128);
  const int64_t ntot = h + extra;
  const int nchunks = (int)((ntot + R - 1) / R);

  // ---- ring of history ids + scales, one chunk ahead of the data ----
  auto ring_load = [&](int c, int& id, float& sa, float& bw) {
    const int64_t k = (int64_t)c * R + tid;
    id = -1;
    sa = 0.0f;
    bw = 0.0f;
    if (k < ntot) {
      id = a.col[p0 + virt_pos(k, h)];
      if (vk) {
        const float nu = a.other_weight[id];
        sa = sqrtf(nu);              // factor col = sqrt(w) * cp_v, safer2.h:192
        bw = (k < h) ? nu : 0.0f;    // rhs += w * cp_v, safer2.h:190
      } else {
        sa = 1.0f;
        bw = 1.0f;
      }
    }
  };
  auto ring_store = [&](int c, int id, float sa, float bw) {
    const int s = (c % kRing) * R + tid;
    ring_id[s] = id;
    ring_sa[s] = sa;
    ring_bw[s] = bw;
  };
  float4 regs[NQ];
  auto load_data = [&](int c) {
    const int slot = c % kRing;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int sidx = tid + q * NTHR;
      regs[q] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (NSLOT % NTHR == 0 || sidx < NSLOT) {
        const int r = sidx / (Dp / 4), c4 = sidx % (Dp / 4);
        const int id = ring_id[slot * R + r];
        if (id >= 0) regs[q] = *reinterpret_cast<const float4*>(a.X + (int64_t)id * Dp + 4 * c4);
      }
    }
  };
  auto store_stage = [&](int buf) {
    float* st = stage + buf * R * Dp;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int sidx = tid + q * NTHR;
      if (NSLOT % NTHR == 0 || sidx < NSLOT) *reinterpret_cast<float4*>(st + 4 * sidx) = regs[q];
    }
  };

  if (tid == 0) flag[0] = 0;
  if (tid < R) {
    int id;
    float sa, bw;
    ring_load(0, id, sa, bw);
    ring_store(0, id, sa, bw);
    if (nchunks > 1) {
      ring_load(1, id, sa, bw);
      ring_store(1, id, sa, bw);
    }
  }
  if (is_grad_kind(kind) && tid < Dp) xvec[tid] = a.E[e * Dp + tid];
  __syncthreads();
  load_data(0);
  store_stage(0);
  __syncthreads();

  // ---- my tiles ----
  f32x16 acc[MT];
  int aoff[MT], boff[MT];
  bool valid[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    acc[m] = f32x16{0.f};
    const int t = wave + m * NW;
    valid[m] = t < NT;
    int I = 0;
    while ((I + 1) * (I + 2) / 2 <= t) ++I;
    const int J = t - I * (I + 1) / 2;
    aoff[m] = 32 * I + lo;
    boff[m] = 32 * J + lo;
  }
  float bacc = 0.0f;

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
#pragma unroll 4
    for (int s = 0; s < R / 2; ++s) {
      const float* rowp = st + (2 * s + hi) * Dp;
      const float sa = vk ? ring_sa[slot * R + 2 * s + hi] : 1.0f;
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        if (valid[m]) {
          float fa = rowp[aoff[m]];
          float fb = rowp[boff[m]];
          if (vk) {
            fa *= sa;
            fb *= sa;
          }
          acc[m] = mfma32(fa, fb, acc[m]);
        }
      }
    }
    if (tid < Dp) {
#pragma unroll 4
      for (int r = 0; r < R; ++r) bacc += ring_bw[slot * R + r] * st[r * Dp + tid];
    }
    if (more) store_stage(buf ^ 1);
    if (ring_more) ring_store(c + 2, nid, nsa, nbw);
    __syncthreads();
  }

  // ---- epilogue: A = f(S, G) into the swizzled LDS tiles ----
  const float hf = (float)h;
  const float omega = (is_u_kind(kind) && a.entity_weight) ? a.entity_weight[e] : 1.0f;
  const float lam = entity_lambda(kind, a.reg, a.reg_exp, a.w, a.alpha, h, a.n_other,
                                  a.entity_reg, e);
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    if (valid[m]) {
      const int I = (aoff[m] - lo) >> 5, J = (boff[m] - lo) >> 5;
      float* tile = tiles + tidx(I, J) * 1024;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int i = acc_row(q, hi);
        const int gi = 32 * I + i, gj = 32 * J + lo;
        const float g = a.G[(int64_t)gi * Dp + gj];
        tile[sw(i, lo)] = assemble(kind, acc[m][q], g, gi == gj, a.w, lam, hf, omega);
      }
    }
  }
  if (tid < Dp) {
    float b = bacc;
    if (is_u_kind(kind)) b *= (omega / hf);  // rhs *= weight / history_size
    bvec[tid] = b;
  }
  __syncthreads();

  // ---- CVaR-MF: one gradient step with the full (stale-upper) matrix ----
  if (is_grad_kind(kind)) {
    if (tid < Dp) {
      const int i = tid, I = i >> 5, ri = i & 31;
      float y = 0.0f;
      for (int j = 0; j < Dp; ++j) {
        float aij;
        if (j <= i)
          aij = tiles[tidx(I, j >> 5) * 1024 + sw(ri, j & 31)];
        else
          aij = cvar_upper(kind, a.G[(int64_t)i * Dp + j], a.w, omega);
        y += aij * xvec[j];
      }
      a.out[e * Dp + i] = xvec[i] - a.eta * (y - bvec[i]);
    }
    return;
  }

  // ---- blocked right-looking Cholesky, rhs as an extra panel row ----
  for (int p = 0; p < T; ++p) {
    float* Tpp = tiles + tidx(p, p) * 1024;
    if (wave == 0) {
      const bool ok = diag_factor(Tpp, ldc, lane);
      if (!ok && lane == 0) flag[0] = 1;
    }
    __syncthreads();
    const int nrow = 32 * (T - 1 - p) + 1;
    if (tid < nrow) {
      float x[32];
      const bool isb = (tid == nrow - 1);
      const int I = p + 1 + (tid >> 5), r = tid & 31;
      float* tl = tiles + tidx(isb ? p : I, p) * 1024;
#pragma unroll
      for (int c = 0; c < 32; ++c) x[c] = isb ? bvec[32 * p + c] : tl[sw(r, c)];
      trsm_row(x, ldc);
#pragma unroll
      for (int c = 0; c < 32; ++c) {
        if (isb) bvec[32 * p + c] = x[c];
        else tl[sw(r, c)] = x[c];
      }
    }
    __syncthreads();
    if (p < T - 1) {
      const int nb = 32 * (T - 1 - p);
      if (tid < nb) {  // b_J -= L_Jp y_p
        const int J = p + 1 + (tid >> 5), r = tid & 31;
        const float* L = tiles + tidx(J, p) * 1024;
        float t = 0.0f;
#pragma unroll
        for (int k = 0; k < 32; ++k) t += L[sw(r, k)] * bvec[32 * p + k];
        bvec[32 * J + r] -= t;
      }
      const int ntr = (T - 1 - p) * (T - p) / 2;
      for (int tt = wave; tt < ntr; tt += NW) {  // A_IJ -= L_Ip L_Jp^T
        int Ir = 0;
        while ((Ir + 1) * (Ir + 2) / 2 <= tt) ++Ir;
        const int Jr = tt - Ir * (Ir + 1) / 2;
        const int I = p + 1 + Ir, J = p + 1 + Jr;
        const float* Lip = tiles + tidx(I, p) * 1024;
        const float* Ljp = tiles + tidx(J, p) * 1024;
        f32x16 u = f32x16{0.f};
#pragma unroll
        for (int s = 0; s < 16; ++s)
          u = mfma32(Lip[sw(lo, 2 * s + hi)], Ljp[sw(lo, 2 * s + hi)], u);
        float* Aij = tiles + tidx(I, J) * 1024;
#pragma unroll
        for (int q = 0; q < 16; ++q) Aij[sw(acc_row(q, hi), lo)] -= u[q];
      }
    }
    __syncthreads();
  }

  // ---- back substitution L^T x = y (wave 0, lane k owns x_k) ----
  if (wave == 0) {
    const int k = lo;
    for (int p = T - 1; p >= 0; --p) {
      float r = bvec[32 * p + k];
      for (int q = p + 1; q < T; ++q) {
        const float* L = tiles + tidx(q, p) * 1024;
#pragma unroll 8
        for (int m = 0; m < 32; ++m) r -= L[sw(m, k)] * xvec[32 * q + m];
      }
      const float* Lpp = tiles + tidx(p, p) * 1024;
      float* xp = xvec + 32 * p;
#pragma unroll 4
      for (int kk = 31; kk >= 0; --kk) {
        if (k == kk && hi == 0) xp[kk] = r / Lpp[sw(kk, kk)];
        __builtin_amdgcn_wave_barrier();
        const float xk = xp[kk];
        if (k < kk) r -= Lpp[sw(kk, k)] * xk;
      }
    }
  }
  __syncthreads();
  if (tid < Dp) a.out[e * Dp + tid] = xvec[tid];
  if (tid == 0 && flag[0]) atomicMin(a.fail, (unsigned long long)(e + 1));
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
                                  a.entity_reg, e);
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

template <int T>
hipError_t launch_tiled(const SolveArgs& a, hipStream_t s) {
  using C = TiledCfg<T>;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t err = hipFuncSetAttribute((const void*)solve_tiled_kernel<T>,
                                         hipFuncAttributeMaxDynamicSharedMemorySize,
                                         (int)C::BYTES);
    if (err != hipSuccess) return err;
    attr_set = true;
  }
  hipLaunchKernelGGL(solve_tiled_kernel<T>, dim3((unsigned)a.n_rows), dim3(C::NTHR), C::BYTES, s,
                     a);
  return hipGetLastError();
}

template <int Dp>
hipError_t launch_small(const SolveArgs& a, hipStream_t s) {
  const unsigned nb = (unsigned)((a.n_rows + 3) / 4);
  hipLaunchKernelGGL(solve_small_kernel<Dp>, dim3(nb), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace

int padded_dim(int dim) {
  if (dim <= 0) return 0;
  if (dim <= 8) return 8;
  if (dim <= 16) return 16;
  if (dim <= 256) return ((dim + 31) / 32) * 32;
  return 0;
}

hipError_t launch_solve(int Dp, const SolveArgs& a, hipStream_t s) {
  if (a.n_rows <= 0) return hipSuccess;
  switch (Dp) {
    case 8: return launch_small<8>(a, s);
    case 16: return launch_small<16>(a, s);
    case 32: return launch_tiled<1>(a, s);
    case 64: return launch_tiled<2>(a, s);
    case 96: return launch_tiled<3>(a, s);
    case 128: return launch_tiled<4>(a, s);
    case 160: return launch_tiled<5>(a, s);
    case 192: return launch_tiled<6>(a, s);
    case 224: return launch_tiled<7>(a, s);
    case 256: return launch_tiled<8>(a, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace frecsys_hip
