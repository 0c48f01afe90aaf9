// dual.hip -- history-space solve for short-history entities on gfx950.
//
// Same result as the d-space solve (solve.hip; reference Project /
// ProjectU / ProjectV, ials.h:88-144, safer2.h:104-221) for entities whose
// history (plus tail-quirk rows) h_eff is at most 32 * kDualMaxTiles, at a
// fraction of the work when h_eff < d.  Write the normal matrix as
//   A = M + Xt^T Xt,  M = mu*G + lam*I,  b = Xt^T s
// (Xt: history rows times c_j = sqrt of their weight in A; s_j = c_j for
// real rows, 0 for the rows the ProjectV tail quirk adds to A only).
// Push-through: x = M^-1 Xt^T (I + Xt M^-1 Xt^T)^-1 s.  In the basis of
// G = Q T Q^T (spectral.hip) M = Q (mu*T + lam*I) Q^T, and with the LDL^T
// factorisation mu*T + lam*I = L D L^T (L unit lower bidiagonal):
//   Z = Y L^-T  (Y = Xt Q: gathered rows of the pre-rotated other side),
//   S = I + Z D^-1 Z^T              h_p x h_p, MFMA SYRK over k = 0..Dp-1
//   z = S^-1 s                       blocked Cholesky in LDS (chol.h)
//   x' = L^-T D^-1 L^-1 (Y^T z)     two bidiagonal sweeps
// and x = Q x' is applied to all rows of the launch by rot_gemm afterwards.
//
// Three kernels per half-step (plus the basis change, spectral.hip):
//   dual_ldl_kernel    one thread per entity: LDL^T of its tridiagonal
//                      mu*T + lam*I into a [3][Dp] table row (the serial
//                      chains run entity-parallel instead of per workgroup);
//   dual_solve_kernel  one workgroup per entity (below), writes Y^T (c.*z);
//   dual_sweep_kernel  one thread per entity: x' = L^-T D^-1 L^-1 (Y^T c.*z).
// dual_solve_kernel, per workgroup (one entity, NW waves):
//   * the entity's l_k and D^-1/2 come from its table row;
//   * per slab (32 columns of the h_p rows; row j's slab loaded by thread j
//     into registers one slab ahead -- with FRECSYS_SYRK_F32=1 staged in LDS
//     with a padded row stride instead): each row's lane runs the bidiagonal
//     recurrence z_j[k] = y_j[k] - l_k z_j[k-1] across the slab (carry in a
//     register) and writes D^-1/2-scaled values k-major; the waves then
//     accumulate their S tiles while the next slab's loads are in flight --
//     by default on the bf16 matrix cores with fp32-accurate 3-piece split
//     operands (common.h mfma_x6), FRECSYS_SYRK_F32=1: v_mfma_f32_32x32x2_f32;
//   * S tiles go to LDS (aliasing the slab buffers), chol_solve_df, then
//     Y^T (c.*z) re-reads the (cache-resident) rows with float4 loads.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <type_traits>

#include "chol.h"
#include "common.h"
#include "kernels.h"

namespace frecsys_hip {

namespace {

constexpr int kMaxDp = 1024;

// BF = true: S accumulates on the bf16 matrix cores with 3-piece split
// operands (common.h mfma_x6, fp32-accurate): the recurrence lane of row j
// writes its 32 scaled slab values as pieces, 16-B granule (piece p, k group
// g of 16, k-half hh, row j) = the bf16x8 fragment lane (j & 31, hh) of
// v_mfma_f32_32x32x16_bf16 reads (dgran below).
template <int HP>
__device__ __forceinline__ int dgran(int p, int g, int hh, int j) {
  return ((p * 2 + g) * 2 + hh) * HP + j;
}

// BF: register-direct slabs -- thread j loads row j's 32-column slab itself
// (float4 x 8, the next slab's loads issued as the current one is consumed)
// instead of the workgroup staging it in LDS (the fp32 path): no staging
// stores or buffer, no LDS reads in the recurrence.  Bit-identical to the
// staged form; measured (ML-20M d = 256, serialised) 5.50 -> 5.30 ms of
// bucket kernels per epoch.
template <int TH, bool BF>
struct DualCfg {
  static constexpr int HP = 32 * TH;                // padded history rows
  static constexpr int NT = TH * (TH + 1) / 2;      // lower tiles of S
  static constexpr int NW = (TH <= 4) ? 4 : 8;      // more, smaller workgroups per CU
  static constexpr int NTHR = NW * 64;
  static constexpr int MT = (NT + NW - 1) / NW;
  static constexpr int SROW = 33;                   // slab row stride
  static constexpr int STG = HP * SROW;
  static constexpr int ZS = (BF ? 48 : 32) * HP;   // k-major scaled Z slab (BF: pieces)
  static constexpr int TILES = NT * 1024;
  static constexpr int NSTAGE = BF ? 0 : ((TH <= 4) ? 1 : 2);  // LDS stages for the slab prefetch
  static constexpr int NSTG1 = NSTAGE > 0 ? NSTAGE : 1;
  static constexpr int LOOP = ((NSTAGE * STG + ZS + 3) / 4) * 4;
  static constexpr int REGION0 = TILES > LOOP ? TILES : LOOP;
  static constexpr int OFF_C = REGION0;             // c_j
  static constexpr int OFF_ID = OFF_C + HP;         // row ids
  static constexpr int OFF_B = OFF_ID + HP;         // s, then y
  static constexpr int OFF_X = OFF_B + HP;          // z
  static constexpr int PART = NTHR > NW * 32 ? NTHR : NW * 32;
  static constexpr int OFF_PART = OFF_X + HP;
  static constexpr int OFF_FLAG = OFF_PART + PART;
  static constexpr int OFF_L = OFF_FLAG + 4;        // l_k [Dp], then D^-1/2 [Dp]
  static constexpr int NQ = (HP * 8 + NTHR - 1) / NTHR;  // float4 per thread per slab
  // waves per SIMD the register allocation must allow (TH = 3: 4 workgroups
  // of 4 waves per CU, TH = 4: 3 of 4, TH = 5: 2 of 8 -- their LDS allows
  // it; the bigger buckets are LDS-bound)
  static constexpr int WPE = (TH == 3 || TH == 5) ? 4 : (TH == 4 ? 3 : 1);
  static constexpr size_t bytes(int Dp) { return (size_t)(OFF_L + 2 * Dp) * 4; }
  static_assert(bytes(kMaxDp) <= 163840, "LDS budget");
};

__device__ __forceinline__ int64_t virt_pos_d(int64_t k, int64_t h) {
  return k < h ? k : (h - 128 + (k - h));
}

// mu, lambda and omega of one entity (see the file comment): iALS
// lambda from RegularizationValue (ials.h:310-315), ProjectU
// omega = entity weight (safer2.h:146-147), ProjectV item_reg_.
__device__ __forceinline__ void dual_scalars(const DualArgs& a, int64_t e, int64_t h, float& mu,
                                             float& lam, float& omega) {
  const int kind = a.kind;
  const bool uk = is_u_kind(kind);
  omega = (uk && a.entity_weight) ? a.entity_weight[e] : 1.0f;
  lam = entity_lambda(kind, a.reg, a.reg_exp, a.w, a.alpha, h, a.n_other, a.entity_reg, e,
                      a.lambda_is_reg);
  mu = uk ? omega * a.w : a.w;
}

__global__ void __launch_bounds__(256) dual_ldl_kernel(DualArgs a) {
  __shared__ float td[kMaxDp], to[kMaxDp];
  const int Dp = a.Dp, tid = threadIdx.x;
  if (a.unit_m) {
    // Cholesky basis (spectral.hip chol_basis_kernel): the rows are already
    // in the basis where M = I, so the table is the unit one; a failed
    // factorisation of M fails every entity of the launch
    const int64_t p = (int64_t)blockIdx.x * 256 + tid;
    if (p >= a.n_rows) return;
    const int64_t pp = a.pos0 + p;
    for (int k = 0; k < Dp; ++k) {
      a.table[blk_t(pp, 0, k, Dp)] = 0.0f;
      a.table[blk_t(pp, 1, k, Dp)] = 1.0f;
      a.table[blk_t(pp, 2, k, Dp)] = 1.0f;
    }
    if (!(a.basis_status[0] > 0.5f)) atomicMin(a.fail, (unsigned long long)(a.order[p].entity + 1));
    return;
  }
  for (int k = tid; k < Dp; k += 256) {
    td[k] = a.tdiag[k];
    to[k] = a.toff[k];
  }
  lds_barrier();
  const int64_t p = (int64_t)blockIdx.x * 256 + tid;
  if (p >= a.n_rows) return;
  const QueueRec rec = a.order[p];
  float mu, lam, omega;
  dual_scalars(a, rec.entity, rec.h, mu, lam, omega);
  // l_k = b_k / d_{k-1}, d_k = a_k - l_k b_k (a = mu*diag + lam, b = mu*sub);
  // position-blocked table: consecutive lanes write consecutive floats
  const int64_t pp = a.pos0 + p;
  float r = 0.0f;
  bool ok = true;
  for (int k = 0; k < Dp; ++k) {
    const float b = k > 0 ? mu * to[k - 1] : 0.0f;
    const float l = b * r;
    const float dk = (mu * td[k] + lam) - l * b;
    ok = ok && (dk > 0.0f);
    r = __builtin_amdgcn_rcpf(dk);
    a.table[blk_t(pp, 0, k, Dp)] = l;
    a.table[blk_t(pp, 1, k, Dp)] = __builtin_amdgcn_rsqf(dk);
    a.table[blk_t(pp, 2, k, Dp)] = r;
  }
  if (!ok) atomicMin(a.fail, (unsigned long long)(rec.entity + 1));
}

// x' = L^-T D^-1 L^-1 v, in place on the entity's out_rot row.  Only the
// u / x chain is serial: each 32-step chunk's v, l_k and D^-1 (independent of
// it) are loaded into registers before the chunk's recurrence runs, so a
// thread keeps 96 loads in flight instead of waiting out one memory round
// trip per few steps (the sweep is latency-bound whenever the launch is
// small: 14K entities at N = 8).  Same operations in the same order.
constexpr int SWEEP_CH = 32;
__global__ void __launch_bounds__(256) dual_sweep_kernel(DualArgs a) {
  const int Dp = a.Dp;
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (p >= a.n_rows) return;
  const int64_t pp = a.pos0 + p;
  float u = 0.0f;
  for (int k0 = 0; k0 < Dp; k0 += SWEEP_CH) {  // L u = v, then D^-1
    float vv[SWEEP_CH], ll[SWEEP_CH], dd[SWEEP_CH];
#pragma unroll
    for (int j = 0; j < SWEEP_CH; ++j) {
      vv[j] = a.out_rot[blk_v(pp, k0 + j, Dp)];
      ll[j] = a.table[blk_t(pp, 0, k0 + j, Dp)];
      dd[j] = a.table[blk_t(pp, 2, k0 + j, Dp)];
    }
#pragma unroll
    for (int j = 0; j < SWEEP_CH; ++j) {
      u = vv[j] - ll[j] * u;
      a.out_rot[blk_v(pp, k0 + j, Dp)] = u * dd[j];
    }
  }
  float x = 0.0f;
  for (int k1 = Dp; k1 > 0; k1 -= SWEEP_CH) {  // L^T x = D^-1 u
    float vv[SWEEP_CH], ll[SWEEP_CH];
#pragma unroll
    for (int j = 0; j < SWEEP_CH; ++j) {
      const int k = k1 - 1 - j;
      vv[j] = a.out_rot[blk_v(pp, k, Dp)];
      ll[j] = k + 1 < Dp ? a.table[blk_t(pp, 0, k + 1, Dp)] : 0.0f;
    }
#pragma unroll
    for (int j = 0; j < SWEEP_CH; ++j) {
      x = vv[j] - ll[j] * x;
      a.out_rot[blk_v(pp, k1 - 1 - j, Dp)] = x;
    }
  }
}

// Smallest bucket whose Cholesky runs the blocked diagonal factor and the
// split-bf16 tile products (chol.h BLK).
constexpr int kDualBlkTH = 3;

template <int TH, bool BF>
__global__ void __launch_bounds__((DualCfg<TH, BF>::NTHR))
    __attribute__((amdgpu_waves_per_eu(DualCfg<TH, BF>::WPE, 8))) dual_solve_kernel(DualArgs a) {
  using C = DualCfg<TH, BF>;
  constexpr bool RDS = BF;  // register-direct slabs
  constexpr int HP = C::HP, NT = C::NT, NW = C::NW, NTHR = C::NTHR, MT = C::MT;
  constexpr int SROW = C::SROW, NQ = C::NQ;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* tiles = smem;
  float* stage = smem;
  float* zs = smem + C::NSTAGE * C::STG;
  float* lsub = smem + C::OFF_L;
  float* dsq = lsub + a.Dp;
  float* cvec = smem + C::OFF_C;
  int* ids = reinterpret_cast<int*>(smem + C::OFF_ID);
  float* bvec = smem + C::OFF_B;
  float* xvec = smem + C::OFF_X;
  float* part = smem + C::OFF_PART;
  int* flag = reinterpret_cast<int*>(smem + C::OFF_FLAG);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform branches
  const int lo = lane & 31, hi = lane >> 5;
  const int kind = a.kind;
  const bool vk = is_v_kind(kind), uk = is_u_kind(kind);
  const int Dp = a.Dp, NC = Dp >> 5;

  const QueueRec rec = a.order[blockIdx.x];
  const int64_t e = rec.entity;
  const int64_t h = rec.h;
  const int64_t p0 = rec.p0;
  int64_t extra = 0;
  if (vk && a.quirk && h > 128 && (h % 128) != 0) extra = 128 - (h % 128);
  const int ntot = (int)(h + extra);  // <= HP (host bucketing)

  const float hf = (float)h;
  float mu, lam, omega;
  dual_scalars(a, e, h, mu, lam, omega);
  (void)mu;
  (void)lam;

  int my_id = -1;  // RDS: the thread's own history row
  if (tid < HP) {
    int id = -1;
    float cj = 0.0f;
    if (tid < ntot) {
      id = a.col[p0 + virt_pos_d(tid, h)];
      // weights of the row in A (= in b): iALS 1 (ials.h:122-126), ProjectU
      // omega/h (safer2.h:143-147), ProjectV nu (safer2.h:185-192)
      cj = vk ? sqrtf(a.other_weight[id]) : (uk ? sqrtf(omega / hf) : 1.0f);
    }
    ids[tid] = id;
    cvec[tid] = cj;
    bvec[tid] = tid < h ? cj : 0.0f;
    my_id = id;
  }
  if (tid == 0) flag[0] = 0;
  unsigned long long t_prev = a.prof ? clock64() : 0;
  auto mark = [&](int ph) {
    if (a.prof && tid == 0) {
      const unsigned long long t = clock64();
      atomicAdd(a.prof + ph, t - t_prev);
      t_prev = t;
    }
  };
  {  // l_k and D^-1/2 from the entity's table row
    const int64_t pp = a.pos0 + blockIdx.x;
    for (int k = tid; k < Dp; k += NTHR) {
      lsub[k] = FRECSYS_SKIP(a.debug_skip, 256) ? 0.5f : a.table[blk_t(pp, 0, k, Dp)];
      dsq[k] = FRECSYS_SKIP(a.debug_skip, 256) ? 0.5f : a.table[blk_t(pp, 1, k, Dp)];
    }
  }
  lds_barrier();

  // two register sets and two LDS stages: slab c+2's loads are issued when
  // slab c starts and stored at the end of slab c+1 (two slabs of cover)
  float4 ra[NQ], rb[NQ];
  // the padding rows (id < 0) load row 0 and are zeroed where they are
  // stored: a conditional load with a zero default made the waitcnt pass
  // wait (vmcnt) for the fresh slab at the loop head and mid-slab
  auto load_slab = [&](int c, float4 (&regs)[NQ]) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int s = tid + q * NTHR;
      if ((HP * 8) % NTHR == 0 || s < HP * 8) {
        const int r = s >> 3, c4 = s & 7;
        const int id = max(ids[r], 0);
        regs[q] = *reinterpret_cast<const float4*>(a.Xrot + (int64_t)id * Dp + 32 * c + 4 * c4);
      }
    }
  };
  auto store_slab = [&](const float4 (&regs)[NQ], int buf) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int s = tid + q * NTHR;
      if ((HP * 8) % NTHR == 0 || s < HP * 8) {
        const int r = s >> 3, c4 = s & 7;
        const bool ok = ids[r] >= 0 && !FRECSYS_SKIP(a.debug_skip, 32);
        float* d = stage + (buf % C::NSTG1) * C::STG + r * SROW + 4 * c4;
        d[0] = ok ? regs[q].x : 0.0f;
        d[1] = ok ? regs[q].y : 0.0f;
        d[2] = ok ? regs[q].z : 0.0f;
        d[3] = ok ? regs[q].w : 0.0f;
      }
    }
  };

  // RDS: row slab in registers; padding rows read row 0 (c_j = 0 zeroes
  // their contribution), so every load is unconditional
  const float* myrow = a.Xrot + (int64_t)max(my_id, 0) * Dp;
  float4 yq[RDS ? 8 : 1];
  if constexpr (RDS) {
    if (tid < HP) {
#pragma unroll
      for (int q = 0; q < 8; ++q) yq[q] = *reinterpret_cast<const float4*>(myrow + 4 * q);
    }
  } else {
    load_slab(0, ra);
    if (NC > 1) load_slab(1, rb);
    store_slab(ra, 0);
  }
  lds_barrier();
  mark(0);

  // ---- S = Z D^-1 Z^T accumulated over the 32-column slabs ----
  f32x16 acc[MT];
  int aoff[MT], boff[MT];
  bool valid[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int t = wave + m * NW;
    valid[m] = t < NT;
    int I = 0;
    while ((I + 1) * (I + 2) / 2 <= t) ++I;
    const int J = t - I * (I + 1) / 2;
    aoff[m] = 32 * I + lo;
    boff[m] = 32 * J + lo;
    acc[m] = f32x16{0.f};
  }
  float carry = 0.0f;
  const float cj = tid < HP ? cvec[tid] : 0.0f;
  // slab c: in LDS stage c&1; slab c+1 in the other register set
  auto slab_step = [&](int c, float4 (&mine)[NQ], float4 (&next)[NQ]) {
    if (!RDS && c + 2 < NC) load_slab(c + 2, mine);
    if (RDS && tid < HP && !FRECSYS_SKIP(a.debug_skip, 128)) {
      // the same recurrence on the registers; each float4 pair, once used,
      // takes the next slab's loads
      bf16x8* zb = reinterpret_cast<bf16x8*>(zs);
      float z = carry;
#pragma unroll
      for (int gh = 0; gh < 4; ++gh) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const float4 y4 = yq[2 * gh + (u >> 2)];
          const float yv = (u & 3) == 0 ? y4.x : (u & 3) == 1 ? y4.y : (u & 3) == 2 ? y4.z : y4.w;
          const int k = 32 * c + 8 * gh + u;
          z = yv - lsub[k] * z;
          v[u] = (cj * z) * dsq[k];
        }
        if (c + 1 < NC) {
          yq[2 * gh] = *reinterpret_cast<const float4*>(myrow + 32 * (c + 1) + 8 * gh);
          yq[2 * gh + 1] = *reinterpret_cast<const float4*>(myrow + 32 * (c + 1) + 8 * gh + 4);
        }
        bf16x8 f[3];
        split3x8(v, f);
#pragma unroll
        for (int p = 0; p < 3; ++p) zb[dgran<HP>(p, gh >> 1, gh & 1, tid)] = f[p];
      }
      carry = z;
    }
    if (!RDS && tid < HP && !FRECSYS_SKIP(a.debug_skip, 128)) {
      const float* yrow = stage + ((c & 1) % C::NSTG1) * C::STG + tid * SROW;
      float y[BF ? 1 : 32];
      if constexpr (!BF) {
#pragma unroll
        for (int kk = 0; kk < 32; ++kk) y[kk] = yrow[kk];
      }
      float z = carry;
      if constexpr (BF) {
        bf16x8* zb = reinterpret_cast<bf16x8*>(zs);
#pragma unroll
        for (int gh = 0; gh < 4; ++gh) {  // (k group, k-half) = 8 consecutive k
          float v[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const int kk = 8 * gh + u, k = 32 * c + kk;
            z = yrow[kk] - lsub[k] * z;
            v[u] = (cj * z) * dsq[k];
          }
          bf16x8 f[3];
          split3x8(v, f);
#pragma unroll
          for (int p = 0; p < 3; ++p) zb[dgran<HP>(p, gh >> 1, gh & 1, tid)] = f[p];
        }
      } else {
#pragma unroll
        for (int kk = 0; kk < 32; ++kk) {
          const int k = 32 * c + kk;
          z = y[kk] - lsub[k] * z;
          zs[kk * HP + tid] = (cj * z) * dsq[k];
        }
      }
      carry = z;
    }
    lds_barrier();
    if (!FRECSYS_SKIP(a.debug_skip, 1)) {
      if constexpr (BF) {
        const bf16x8* zb = reinterpret_cast<const bf16x8*>(zs);
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          if (valid[m]) {  // wave-uniform
#pragma unroll
            for (int g = 0; g < 2; ++g) {
              bf16x8 av[3], bv[3];
#pragma unroll
              for (int p = 0; p < 3; ++p) {
                av[p] = zb[dgran<HP>(p, g, hi, aoff[m])];
                bv[p] = zb[dgran<HP>(p, g, hi, boff[m])];
              }
              acc[m] = mfma_x6(av, bv, acc[m]);
            }
          }
        }
      } else {
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          if (valid[m]) {  // wave-uniform
#pragma unroll
            for (int s = 0; s < 16; ++s) {
              const float* zr = zs + (2 * s + hi) * HP;
              acc[m] = mfma32(zr[aoff[m]], zr[boff[m]], acc[m]);
            }
          }
        }
      }
    }
    if (!RDS && c + 1 < NC) store_slab(next, (c + 1) & 1);
    lds_barrier();
  };
  for (int c = 0; c < NC; c += 2) {
    slab_step(c, ra, rb);
    if (c + 1 < NC) slab_step(c + 1, rb, ra);
  }

  // ---- S = I + acc into the swizzled LDS tiles (aliasing the slabs) ----
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    if (valid[m]) {
      const int I = (aoff[m] - lo) >> 5, J = (boff[m] - lo) >> 5;
      float* tile = tiles + tidx(I, J) * 1024;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int i = acc_row(q, hi);
        const bool dg = (32 * I + i) == (32 * J + lo);
        tile[sw(i, lo)] = acc[m][q] + (dg ? 1.0f : 0.0f);
      }
    }
  }
  lds_barrier();
  mark(1);
  // the MFMA-blocked diagonal factor where the register budget allows it
  // (every bucket since the granule tile layout: TH = 4, 5 keep their
  // occupancy without spills; TH = 3 at 128 registers spills 8, measured
  // faster all the same)
  chol_solve_df<TH, NW, (TH >= kDualBlkTH)>(tiles, bvec, xvec, part, flag, tid, a.debug_skip,
                                            a.prof);
  mark(2);

  // ---- v = Y^T (c.*z): the rows again, float4 per lane, 8 rows in flight ----
  {
    const int D4 = Dp >> 2, R = NTHR / D4;  // column quads x row groups
    const int c4 = tid % D4, g = tid / D4;
    float* red = tiles;  // the S tiles are dead after the solve
    float4 acc4 = make_float4(0.f, 0.f, 0.f, 0.f);
    if (g < R && !FRECSYS_SKIP(a.debug_skip, 64)) {
      for (int j0 = g; j0 < ntot; j0 += 8 * R) {
        float4 rv[8];
        float wv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int j = j0 + u * R;
          rv[u] = make_float4(0.f, 0.f, 0.f, 0.f);
          wv[u] = 0.0f;
          if (j < ntot) {
            wv[u] = cvec[j] * xvec[j];
            rv[u] = *reinterpret_cast<const float4*>(a.Xrot + (int64_t)ids[j] * Dp + 4 * c4);
          }
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          acc4.x += wv[u] * rv[u].x;
          acc4.y += wv[u] * rv[u].y;
          acc4.z += wv[u] * rv[u].z;
          acc4.w += wv[u] * rv[u].w;
        }
      }
      *reinterpret_cast<float4*>(red + g * Dp + 4 * c4) = acc4;
    }
    lds_barrier();
    for (int i = tid; i < Dp; i += NTHR) {
      float v = 0.0f;
      for (int gg = 0; gg < R; ++gg) v += red[gg * Dp + i];
      a.out_rot[blk_v(a.pos0 + blockIdx.x, i, Dp)] = v;
    }
  }
  mark(3);
  if (a.prof && tid == 0) atomicAdd(a.prof + 4, 1ull);
  if (tid == 0 && flag[0]) atomicMin(a.fail, (unsigned long long)(e + 1));
}


// ---------------------------------------------------------------------
// Short histories (h_eff <= 64): one wave per entity, four independent
// entities per workgroup, no workgroup barrier anywhere.  Lane j owns
// history row j: the wave fetches the rows' 32-column slab (coalesced, one
// slab ahead) and hands lane j its row through LDS, lane j runs the
// bidiagonal recurrence with l_k and D^-1/2 as
// wave-uniform scalars from the entity's table row, and writes the scaled
// values k-major to its wave's LDS slab; the same wave then accumulates
// the S tiles with MFMA, factors S (chol_solve_wave) and forms Y^T (c.*z)
// with coalesced whole-row loads.
// ---------------------------------------------------------------------
__device__ __forceinline__ void wave_sync() { wave_lds_sync(); }

// The Cholesky solve for one wave (T <= 2): x = S^-1 b, S's lower tiles in
// LDS (swizzled), diagonal tiles become L_pp^-1; the blocked diagonal
// factor and split-bf16 tile products (chol.h).
template <int T>
__device__ __forceinline__ void chol_solve_wave(float* tiles, float* bvec, float* xvec,
                                                int* flag, int lane, int debug_skip) {
  const int lo = lane & 31, hi = lane >> 5;
  float y[T];
#pragma unroll
  for (int p = 0; p < T; ++p) {
    float* Tpp = tiles + tidx(p, p) * 1024;
    if (!FRECSYS_SKIP(debug_skip, 2) && !diag_factor_inv<true>(Tpp, lane) && lane == 0)
      flag[0] = 1;
    wave_sync();
    // y_p = L_pp^-1 b_p  (lane lo, both halves compute, half 0 keeps it)
    float yp = 0.0f;
#pragma unroll
    for (int g = 0; g < 8; ++g) {  // row lo by granules (common.h row_gran), k ascending
      const f32x4v x4 = row_gran(Tpp, lo, g);
#pragma unroll
      for (int t = 0; t < 4; ++t) yp += x4[t] * bvec[32 * p + 4 * g + t];
    }
    y[p] = yp;
    if (hi == 0) xvec[32 * p + lo] = yp;  // y staged for the panel update
    if (p + 1 < T) {
      float* A10 = tiles + tidx(p + 1, p) * 1024;
      const f32x16 u = tile_pqT_x6(A10, Tpp, lo, hi);  // L_10 = A_10 L_00^-T
      wave_sync();
#pragma unroll
      for (int q = 0; q < 16; ++q) A10[sw(acc_row(q, hi), lo)] = u[q];
      wave_sync();
      // b_1 -= L_10 y_0 ; A_11 -= L_10 L_10^T
      float t = 0.0f;
#pragma unroll
      for (int g = 0; g < 8; ++g) {
        const f32x4v x4 = row_gran(A10, lo, g);
#pragma unroll
        for (int u = 0; u < 4; ++u) t += x4[u] * xvec[32 * p + 4 * g + u];
      }
      const f32x16 w = tile_pqT_x6<true>(A10, A10, lo, hi);
      float* A11 = tiles + tidx(p + 1, p + 1) * 1024;
      wave_sync();
      if (hi == 0) bvec[32 * (p + 1) + lo] -= t;
#pragma unroll
      for (int q = 0; q < 16; ++q) A11[sw(acc_row(q, hi), lo)] -= w[q];
      wave_sync();
    }
  }
  // back substitution
  float x1 = 0.0f;
  if (T == 2) {
    const float* T11 = tiles + tidx(1, 1) * 1024;
    float x = 0.0f;
#pragma unroll
    for (int i = 0; i < 32; ++i) x += T11[sw(i, lo)] * rdlane(y[1], i);
    x1 = x;
    if (hi == 0) xvec[32 + lo] = x;
    wave_sync();
  }
  float r = y[0];
  if (T == 2) {  // r_0 = y_0 - L_10^T x_1
    const float* L10 = tiles + tidx(1, 0) * 1024;
    float t = 0.0f;
#pragma unroll 8
    for (int m = 0; m < 32; ++m) t += L10[sw(m, lo)] * xvec[32 + m];
    r -= t;
  }
  const float* T00 = tiles;
  float x = 0.0f;
#pragma unroll
  for (int i = 0; i < 32; ++i) x += T00[sw(i, lo)] * rdlane(r, i);
  wave_sync();
  if (hi == 0) xvec[lo] = x;
  (void)x1;
  wave_sync();
}

// LDS per wave does not grow with Dp: the entity's l_k and D^-1/2 pass
// through a 64-float window one slab at a time (loaded a slab ahead with the
// rows), and c_j stays in its row's lane.  Staging the whole table row (2 Dp
// floats) held the launch to 1 workgroup per CU at Dp = 1024 (one wave per
// SIMD) and 2 at Dp = 256 / 512; now TH = 2 fits 3 (its register limit) and
// TH = 1 fits 4 at every Dp.
template <int TH, bool BF>
struct WaveCfg {
  static constexpr int HP = 32 * TH;
  static constexpr int NT = TH * (TH + 1) / 2;
  static constexpr int ZS = (BF ? 48 : 32) * HP;
  static constexpr int REG0 = NT * 1024 > ZS ? NT * 1024 : ZS;
  static constexpr int REG = REG0 > HP * 36 ? REG0 : HP * 36;  // + the coalesced slab staging
  static constexpr int OFF_ID = REG, OFF_B = OFF_ID + HP, OFF_X = OFF_B + HP;
  static constexpr int OFF_FLAG = OFF_X + HP;
  static constexpr int OFF_T = OFF_FLAG + 4;  // the slab's l_k [32], then D^-1/2 [32]
  static constexpr int pw(int) { return OFF_T + 64; }  // floats per wave
  static constexpr size_t bytes(int Dp) { return (size_t)4 * pw(Dp) * 4; }
  static_assert(TH <= 2, "one history row per lane");
  static_assert(3 * ((bytes(0) + 511) / 512) * 512 <= 163840, "three workgroups per CU");
};

template <int TH, bool BF>
__global__ void __launch_bounds__(256) dual_wave_kernel(DualArgs a) {
  using C = WaveCfg<TH, BF>;
  constexpr int HP = C::HP, NT = C::NT;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lo = lane & 31, hi = lane >> 5;
  const int64_t pos = (int64_t)blockIdx.x * 4 + wave;
  if (pos >= a.n_rows) return;  // whole wave; no workgroup barriers below
  float* base = smem + wave * C::pw(a.Dp);
  float* zs = base;
  float* tiles = base;
  int* ids = reinterpret_cast<int*>(base + C::OFF_ID);
  float* bvec = base + C::OFF_B;
  float* xvec = base + C::OFF_X;
  int* flag = reinterpret_cast<int*>(base + C::OFF_FLAG);

  const int kind = a.kind;
  const bool vk = is_v_kind(kind), uk = is_u_kind(kind);
  const int Dp = a.Dp, NC = Dp >> 5;
  const QueueRec rec = a.order[pos];
  const int64_t e = rec.entity, h = rec.h, p0 = rec.p0;
  int64_t extra = 0;
  if (vk && a.quirk && h > 128 && (h % 128) != 0) extra = 128 - (h % 128);
  const int ntot = (int)(h + extra);
  float mu, lam, omega;
  dual_scalars(a, e, h, mu, lam, omega);
  (void)mu;
  (void)lam;
  const float hf = (float)h;

  // my history row
  const int j = lane;
  int id = -1;
  float cj = 0.0f;
  if (j < ntot) {
    id = a.col[p0 + virt_pos_d(j, h)];
    cj = vk ? sqrtf(a.other_weight[id]) : (uk ? sqrtf(omega / hf) : 1.0f);
  }
  if (j < HP) {
    ids[j] = id;
    bvec[j] = j < h ? cj : 0.0f;
  }
  if (lane == 0) flag[0] = 0;
  // the slab's l_k (lanes 0-31) and D^-1/2 (lanes 32-63) of the entity's
  // table row, loaded with the slab's rows and written to the wave's window
  // when the slab starts: the recurrence then waits on LDS only (lgkmcnt)
  float* trow = base + C::OFF_T;
  const int64_t tpp = a.pos0 + pos;
  auto tload = [&](int c) { return a.table[blk_t(tpp, lane >> 5, 32 * c + lo, Dp)]; };
  const float* xrow = a.Xrot + (int64_t)(id < 0 ? 0 : id) * Dp;

  float4 yr[8], yn[8];
#ifndef FRECSYS_WAVE_COAL
#define FRECSYS_WAVE_COAL 1
#endif
  // COAL (default): the slab's rows are fetched 8 lanes per row (8 rows x
  // 128 B per instruction, 8 cache lines) and turned to one row per lane
  // through the wave's zs area (rows padded to 36 floats: conflict-free both
  // ways), instead of each lane fetching its own row's 128 B (64 lines per
  // instruction).  Bit-identical; config 5 1230 -> 1207 ms per epoch, MSD
  // and ML-20M unchanged (profiles/r06/wave_coal/).
  constexpr bool COAL = FRECSYS_WAVE_COAL != 0;
  constexpr int NQ = COAL ? HP / 8 : 8;  // prefetch registers per lane
  // COAL: row 8 q + lane / 8's offset (32-bit while rows x Dp < 2^32, as the
  // wave's own rows: the wave kernels run at Dp <= 1024 on tables < 4G floats)
  uint32_t coff[COAL ? NQ : 1];
  if constexpr (COAL) {
#pragma unroll
    for (int q = 0; q < NQ; ++q)
      coff[q] = (uint32_t)max(ids[8 * q + (lane >> 3)], 0) * (uint32_t)Dp + 4u * (lane & 7);
  }
  // unconditional loads (row 0 stands in for padding rows, whose c_j = 0):
  // no branches around the loads, so the prefetch stays in flight
  auto load = [&](int c, float4* dst) {
    if constexpr (COAL) {
#pragma unroll
      for (int q = 0; q < NQ; ++q)
        dst[q] = *reinterpret_cast<const float4*>(a.Xrot + (size_t)(coff[q] + 32u * c));
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) dst[q] = *reinterpret_cast<const float4*>(xrow + 32 * c + 4 * q);
    }
  };
  float tn = tload(0);
  load(0, yn);
  wave_sync();
  f32x16 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f32x16{0.f};
  float carry = 0.0f;
  for (int c = 0; c < NC; ++c) {
    // slab c arrives (the one wait per slab), slab c+1 goes in flight, and
    // everything below runs on registers / LDS only
    if constexpr (COAL) {
      // the previous slab's zs reads finished at its closing wave_sync
#pragma unroll
      for (int q = 0; q < NQ; ++q)  // (component stores: a float4 struct copy stays in scratch)
        *reinterpret_cast<f32x4v*>(zs + (8 * q + (lane >> 3)) * 36 + 4 * (lane & 7)) =
            f32x4v{yn[q].x, yn[q].y, yn[q].z, yn[q].w};
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) yr[q] = yn[q];
    }
    trow[lane] = tn;  // the previous slab's window reads finished at its wave_sync
    if (c + 1 < NC) {
      tn = tload(c + 1);
      load(c + 1, yn);
    }
    wave_sync();
    if constexpr (COAL) {
      if (j < HP) {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const f32x4v t = *reinterpret_cast<const f32x4v*>(zs + j * 36 + 4 * q);
          yr[q] = make_float4(t[0], t[1], t[2], t[3]);
        }
      }
      wave_sync();  // the recurrence overwrites zs with the pieces
    }
    if (j < HP) {
      float z = carry;
      if constexpr (BF) {
        bf16x8* zb = reinterpret_cast<bf16x8*>(zs);
#pragma unroll
        for (int gh = 0; gh < 4; ++gh) {  // 8 consecutive k: float4 pairs 2gh, 2gh+1
          float v[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const float4 y4 = yr[2 * gh + (u >> 2)];
            const float yv = (u & 3) == 0 ? y4.x : (u & 3) == 1 ? y4.y : (u & 3) == 2 ? y4.z : y4.w;
            const int k = 8 * gh + u;
            z = yv - trow[k] * z;
            v[u] = (cj * z) * trow[32 + k];
          }
          bf16x8 f[3];
          split3x8(v, f);
#pragma unroll
          for (int p = 0; p < 3; ++p) zb[dgran<HP>(p, gh >> 1, gh & 1, j)] = f[p];
        }
      } else {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const float yv[4] = {yr[q].x, yr[q].y, yr[q].z, yr[q].w};
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int kk = 4 * q + u;
            z = yv[u] - trow[kk] * z;
            zs[kk * HP + j] = (cj * z) * trow[32 + kk];
          }
        }
      }
      carry = z;
    }
    wave_sync();
    if constexpr (BF) {
      // each row block's pieces once, reused by every tile it takes part in
      const bf16x8* zb = reinterpret_cast<const bf16x8*>(zs);
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        bf16x8 fr[TH][3];
#pragma unroll
        for (int b = 0; b < TH; ++b)
#pragma unroll
          for (int p = 0; p < 3; ++p) fr[b][p] = zb[dgran<HP>(p, g, hi, 32 * b + lo)];
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          int I = 0;
          while ((I + 1) * (I + 2) / 2 <= t) ++I;
          const int J = t - I * (I + 1) / 2;
          acc[t] = mfma_x6(fr[I], fr[J], acc[t]);
        }
      }
    } else {
#pragma unroll
      for (int s2 = 0; s2 < 16; ++s2) {
        const float* zr = zs + (2 * s2 + hi) * HP;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          int I = 0;
          while ((I + 1) * (I + 2) / 2 <= t) ++I;
          const int J = t - I * (I + 1) / 2;
          acc[t] = mfma32(zr[32 * I + lo], zr[32 * J + lo], acc[t]);
        }
      }
    }
    wave_sync();
  }
  // S = I + acc
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    int I = 0;
    while ((I + 1) * (I + 2) / 2 <= t) ++I;
    const int J = t - I * (I + 1) / 2;
    float* tile = tiles + t * 1024;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int i = acc_row(q, hi);
      tile[sw(i, lo)] = acc[t][q] + ((32 * I + i) == (32 * J + lo) ? 1.0f : 0.0f);
    }
  }
  wave_sync();
  chol_solve_wave<TH>(tiles, bvec, xvec, flag, lane, a.debug_skip);

  // v = Y^T (c.*z): lane owns columns 4*lane + 256*cg .. +3
  constexpr int YZ = 8;  // row loads in flight (16 measured the same)
  for (int cg = 0; 256 * cg < Dp; ++cg) {
  const int c4 = 4 * lane + 256 * cg;
  float4 v4 = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c4 < Dp && !FRECSYS_SKIP(a.debug_skip, 64)) {
    for (int j0 = 0; j0 < ntot; j0 += YZ) {
      float4 rv[YZ];
      float wv[YZ];
#pragma unroll
      for (int u = 0; u < YZ; ++u) {
        const int jj = j0 + u;
        wv[u] = 0.0f;
        rv[u] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (jj < ntot) {  // c_j from row jj's lane (jj wave-uniform)
          wv[u] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cj), jj)) * xvec[jj];
          rv[u] = *reinterpret_cast<const float4*>(a.Xrot + (int64_t)ids[jj] * Dp + c4);
        }
      }
#pragma unroll
      for (int u = 0; u < YZ; ++u) {
        v4.x += wv[u] * rv[u].x;
        v4.y += wv[u] * rv[u].y;
        v4.z += wv[u] * rv[u].z;
        v4.w += wv[u] * rv[u].w;
      }
    }
  }
  if (c4 < Dp) {
    const int64_t pp = a.pos0 + pos;
    a.out_rot[blk_v(pp, c4 + 0, Dp)] = v4.x;
    a.out_rot[blk_v(pp, c4 + 1, Dp)] = v4.y;
    a.out_rot[blk_v(pp, c4 + 2, Dp)] = v4.z;
    a.out_rot[blk_v(pp, c4 + 3, Dp)] = v4.w;
  }
  }
  if (lane == 0 && flag[0]) atomicMin(a.fail, (unsigned long long)(e + 1));
}


// ---------------------------------------------------------------------
// Wide bucket: 256 < h_eff <= 512 at Dp = 512 / 1024.  S (up to 512 x 512)
// no longer fits a CU's LDS, so the bucket runs the same algebra as
// dual_solve_kernel through HBM workspaces, a batch of entities at a time:
//   dual_wide_z_kernel    one workgroup (512 threads, thread j = row j) per
//                         entity: the recurrence z_j[k] = y_j[k] - l_k
//                         z_j[k-1] scaled by c_j D_k^-1/2, written as the
//                         3-piece bf16 split fragments of the MFMA operand
//                         (zs: [Dp/16][piece][k-half][512] x bf16x8), and
//                         s (c_j for real rows) as the rhs of the slot;
//   dual_wide_s_kernel    S = I + Z D^-1 Z^T on the bf16 matrix cores
//                         (mfma_x6, fp32-accurate) straight from those
//                         fragments: a workgroup per (entity, 128 x 128
//                         block pair), each wave a 64 x 64 quarter (2 x 2
//                         tiles, fragments shared), into the Cholesky slot
//                         (row-major 32 x 32 tiles, tidx order);
//   wide_chol_kernel<16>  (wide.hip) z = S^-1 s;
//   dual_wide_v_kernel    Y^T (c.*z) into out_rot, as dual_solve_kernel's
//                         epilogue, for dual_sweep_kernel + the back rotation.
// Padding rows (j >= h_eff) have c_j = 0: zero fragments, identity rows of S,
// s_j = 0, so z_j = 0.
// ---------------------------------------------------------------------
constexpr int kWideHP = 512;

__device__ __forceinline__ int64_t wz_gran(int kb, int p, int hh, int j) {
  return (((int64_t)kb * 3 + p) * 2 + hh) * kWideHP + j;
}

__global__ void __launch_bounds__(512) dual_wide_z_kernel(DualArgs a, bf16x8* zs_all,
                                                          float* slots, int64_t slot_floats) {
  __shared__ float lsub[kMaxDp], dsq[kMaxDp];
  const int tid = threadIdx.x, Dp = a.Dp;
  const QueueRec rec = a.order[blockIdx.x];
  const int64_t e = rec.entity, h = rec.h, p0 = rec.p0;
  const bool vk = is_v_kind(a.kind), uk = is_u_kind(a.kind);
  int64_t extra = 0;
  if (vk && a.quirk && h > 128 && (h % 128) != 0) extra = 128 - (h % 128);
  const int ntot = (int)(h + extra);  // <= kWideHP (host bucketing)
  float mu, lam, omega;
  dual_scalars(a, e, h, mu, lam, omega);
  int id = 0;
  float cj = 0.0f;
  if (tid < ntot) {
    id = a.col[p0 + virt_pos_d(tid, h)];
    cj = vk ? sqrtf(a.other_weight[id]) : (uk ? sqrtf(omega / (float)h) : 1.0f);
  }
  float* slot = slots + (int64_t)blockIdx.x * slot_floats;
  slot[slot_floats - kWideHP + tid] = tid < h ? cj : 0.0f;  // s, the rhs of S z = s
  const int64_t pp = a.pos0 + blockIdx.x;
  for (int k = tid; k < Dp; k += 512) {
    lsub[k] = a.table[blk_t(pp, 0, k, Dp)];
    dsq[k] = a.table[blk_t(pp, 1, k, Dp)];
  }
  __syncthreads();
  bf16x8* zs = zs_all + (int64_t)blockIdx.x * (Dp / 16) * 3 * 2 * kWideHP;
  // rows past the entity's last tile are never read (dual_wide_s_kernel)
  if (tid >= 32 * ((ntot + 31) / 32)) return;
  const float* row = a.Xrot + (int64_t)id * Dp;
  // the row's 16-column steps through a 4-deep register ring: the loads of
  // steps kb+1 .. kb+3 are in flight under step kb's recurrence (the loop
  // unrolled by 4 so every ring slot is a fixed set of registers; Dp / 16 is
  // a multiple of 4)
  constexpr int R = 4;
  const int NK = Dp / 16;
  float4 ring[R][4];
  auto ld = [&](int kb, float4(&dst)[4]) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < 4; ++q) dst[q] = *reinterpret_cast<const float4*>(row + 16 * kb + 4 * q);
  };
#pragma unroll
  for (int j = 0; j < R - 1; ++j) ld(j, ring[j]);
  float z = 0.0f;
#pragma unroll 1
  for (int kb0 = 0; kb0 < NK; kb0 += R) {
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const int kb = kb0 + j;
      if (kb + R - 1 < NK) ld(kb + R - 1, ring[(j + R - 1) % R]);
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const float4 y4 = ring[j][2 * hh + (u >> 2)];
          const float yv = (u & 3) == 0 ? y4.x : (u & 3) == 1 ? y4.y : (u & 3) == 2 ? y4.z : y4.w;
          const int k = 16 * kb + 8 * hh + u;
          z = yv - lsub[k] * z;
          v[u] = (cj * z) * dsq[k];
        }
        bf16x8 f[3];
        split3x8(v, f);
#pragma unroll
        for (int p = 0; p < 3; ++p) zs[wz_gran(kb, p, hh, tid)] = f[p];
      }
    }
  }
}

// grid: (entity of the batch) x 10 block pairs (BI >= BJ of 4 x 4 blocks of
// 128); 256 threads, wave w: tiles rows 4 BI + 2 (w >> 1) + {0, 1}, columns
// 4 BJ + 2 (w & 1) + {0, 1} (upper tiles of a diagonal pair skipped).
__global__ void __launch_bounds__(256) dual_wide_s_kernel(const bf16x8* zs_all, int Dp,
                                                          const QueueRec* order, int quirk_v,
                                                          float* slots, int64_t slot_floats) {
  const int tid = threadIdx.x, lane = tid & 63, lo = lane & 31, hi = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t b = blockIdx.x / 10;
  int pr = blockIdx.x % 10, BI = 0;
  while ((BI + 1) * (BI + 2) / 2 <= pr) ++BI;
  const int BJ = pr - BI * (BI + 1) / 2;
  const int I0 = 4 * BI + 2 * (wave >> 1), J0 = 4 * BJ + 2 * (wave & 1);
  float* slot = slots + b * slot_floats;
  // tiles past the entity's rows: S = I there, no products
  const QueueRec rec = order[b];
  int64_t extra = 0;
  if (quirk_v && rec.h > 128 && (rec.h % 128) != 0) extra = 128 - (rec.h % 128);
  const int te = (int)((rec.h + extra + 31) / 32);  // tiles holding rows
  const bf16x8* zs = zs_all + b * (Dp / 16) * 3 * 2 * kWideHP;
  f32x16 acc[2][2];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int v = 0; v < 2; ++v) acc[u][v] = f32x16{0.f};
  const bool live = I0 < te && J0 < te && !(BI == BJ && J0 > I0 + 1);
  if (live) {
    bf16x8 fa[2][3], fb[2][3];
    auto load = [&](int kb, bf16x8(&A)[2][3], bf16x8(&B)[2][3]) __attribute__((always_inline)) {
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int p = 0; p < 3; ++p) {
          A[u][p] = zs[wz_gran(kb, p, hi, 32 * (I0 + u) + lo)];
          B[u][p] = zs[wz_gran(kb, p, hi, 32 * (J0 + u) + lo)];
        }
    };
    load(0, fa, fb);
#pragma unroll 1
    for (int kb = 0; kb < Dp / 16; ++kb) {
      bf16x8 na[2][3], nb[2][3];
      if (kb + 1 < Dp / 16) load(kb + 1, na, nb);
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int v = 0; v < 2; ++v)
          if (!(BI == BJ && J0 + v > I0 + u)) acc[u][v] = mfma_x6(fa[u], fb[v], acc[u][v]);
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int p = 0; p < 3; ++p) {
          fa[u][p] = na[u][p];
          fb[u][p] = nb[u][p];
        }
    }
  }
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int v = 0; v < 2; ++v) {
      const int I = I0 + u, J = J0 + v;
      if (J > I) continue;
      float* tile = slot + (int64_t)tidx(I, J) * 1024;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int r = acc_row(q, hi);
        tile[r * 32 + lo] = acc[u][v][q] + ((I == J && r == lo) ? 1.0f : 0.0f);
      }
    }
}

// S of the wide bucket from LDS-DMA stages: two workgroups (8 waves) per
// entity -- the off-diagonal 256 x 256 block (rows 256..511 x columns 0..255,
// 64 tiles, wave w: rows 2 (w >> 1), +1 x columns 4 (w & 1) .. +3) and the two
// diagonal triangles (72 tiles, wave w: triangle w >> 2, its rows q and 7 - q,
// q = w & 3: 9 tiles) -- each reading every k16 step's fragments of all 16
// row tiles (48 KB: 16 tiles x 3 pieces x 1 KB, the z kernel's fragment
// layout) once into a 3-stage ring two steps ahead, instead of every wave of
// dual_wide_s_kernel's 10 workgroups loading its own 12 KB from L2 (4 waves x
// 12 KB for 24 MFMAs each: L2-bound, MFMA busy 0.29).  The tiles holding rows
// (I < te) get the same products in the same k order as dual_wide_s_kernel
// (bit-identical); the others are written as identity tiles (never read:
// the Cholesky factors the te live tiles only).
constexpr int WS_STG = 3, WS_STAGE = 16 * 3 * 1024;  // 48 KB
constexpr size_t WS_LDS = (size_t)WS_STG * WS_STAGE;  // 144 KB: one workgroup per CU

template <int ROLE>
__global__ void __launch_bounds__(512) dual_wide_s_lds_kernel(const bf16x8* zs_all, int Dp,
                                                              const QueueRec* order, int quirk_v,
                                                              float* slots, int64_t slot_floats,
                                                              int64_t n) {
  extern __shared__ __attribute__((aligned(16))) char ws_lds[];
  const int tid = threadIdx.x, lane = tid & 63, lo = lane & 31, hi = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // one launch per role (ROLE 0: the off-diagonal block, 1: the triangles)
  constexpr int role = ROLE;
  const int64_t b = blockIdx.x;
  if (b >= n) return;
  (void)tid;
  float* slot = slots + b * slot_floats;
  const QueueRec rec = order[b];
  int64_t extra = 0;
  if (quirk_v && rec.h > 128 && (rec.h % 128) != 0) extra = 128 - (rec.h % 128);
  const int te = (int)((rec.h + extra + 31) / 32);  // tiles holding rows
  const bf16x8* zs = zs_all + b * (Dp / 16) * 3 * 2 * kWideHP;
  const unsigned ring = lds_addr(ws_lds);
  const int NS = Dp / 16;
  // this wave's 6 fragment DMAs per step: f = 6 w + i -> (tile f / 3, piece f % 3)
  auto issue = [&](int kb) __attribute__((always_inline)) {
    const unsigned st = ring + (unsigned)((kb % WS_STG) * WS_STAGE);
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      const int f = 6 * wave + i, t = f / 3, p = f % 3;
      glds16(zs + wz_gran(kb, p, hi, 32 * t + lo), st + (unsigned)(f * 1024));
    }
  };
  // tile coordinates of accumulator slot m (global 32-row tiles)
  auto tile_of = [&](int m, int& I, int& J) __attribute__((always_inline)) {
    if constexpr (role == 0) {
      I = 8 + 2 * (wave >> 1) + (m >> 2);
      J = 4 * (wave & 1) + (m & 3);
    } else {
      const int tr = wave >> 2, q = wave & 3;
      if (m <= 7 - q) {
        I = 8 * tr + 7 - q;
        J = 8 * tr + m;
      } else {
        I = 8 * tr + q;
        J = 8 * tr + 8 - m;
      }
    }
  };
  constexpr int nm = role == 0 ? 8 : 9;
  f32x16 acc[nm];
#pragma unroll
  for (int m = 0; m < nm; ++m) acc[m] = f32x16{0.f};
  issue(0);
  if (NS > 1) issue(1);
#pragma unroll 1
  for (int kb = 0; kb < NS; ++kb) {
    vm_wait(kb + 1 < NS ? 6 : 0);
    w3_barrier();
    if (kb + 2 < NS) issue(kb + 2);
    const char* st = ws_lds + (kb % WS_STG) * WS_STAGE;
    auto frag = [&](int t, bf16x8(&f)[3]) __attribute__((always_inline)) {
#pragma unroll
      for (int p = 0; p < 3; ++p)
        f[p] = *reinterpret_cast<const bf16x8*>(st + ((t * 3 + p) * 64 + lane) * 16);
    };
    if constexpr (role == 0) {
      bf16x8 A0[3], A1[3];
      const int i0 = 8 + 2 * (wave >> 1);
      frag(i0, A0);
      frag(i0 + 1, A1);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        bf16x8 B[3];
        frag(4 * (wave & 1) + c, B);
        if (i0 < te) acc[c] = mfma_x6(A0, B, acc[c]);
        if (i0 + 1 < te) acc[4 + c] = mfma_x6(A1, B, acc[4 + c]);
      }
    } else {
      // rows 7 - q and q of triangle tr; slot j <- tile (7 - q, j), slot
      // 8 - j <- tile (q, j): every accumulator index static, q wave-uniform
      const int tr = wave >> 2, q = wave & 3;
      bf16x8 Ahi[3], Alo[3];
      frag(8 * tr + 7 - q, Ahi);
      frag(8 * tr + q, Alo);
      const bool lhi = 8 * tr + 7 - q < te, llo = 8 * tr + q < te;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (j <= 7 - q) {  // wave-uniform
          bf16x8 B[3];
          frag(8 * tr + j, B);
          if (lhi) acc[j] = mfma_x6(Ahi, B, acc[j]);
          if (j <= q && llo) acc[8 - j] = mfma_x6(Alo, B, acc[8 - j]);
        }
      }
    }
  }
#pragma unroll
  for (int m = 0; m < nm; ++m) {
    int I, J;
    tile_of(m, I, J);
    float* tile = slot + (int64_t)tidx(I, J) * 1024;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int r = acc_row(q, hi);
      tile[r * 32 + lo] = (I < te ? acc[m][q] : 0.0f) + ((I == J && r == lo) ? 1.0f : 0.0f);
    }
  }
}

// v = Y^T (c.*z) of one entity (z: the Cholesky output row of its slot)
__global__ void __launch_bounds__(256) dual_wide_v_kernel(DualArgs a, const float* zb) {
  __shared__ float red[1024];
  const int tid = threadIdx.x, Dp = a.Dp;
  const QueueRec rec = a.order[blockIdx.x];
  const int64_t e = rec.entity, h = rec.h, p0 = rec.p0;
  const bool vk = is_v_kind(a.kind), uk = is_u_kind(a.kind);
  int64_t extra = 0;
  if (vk && a.quirk && h > 128 && (h % 128) != 0) extra = 128 - (h % 128);
  const int ntot = (int)(h + extra);
  float mu, lam, omega;
  dual_scalars(a, e, h, mu, lam, omega);
  const float cu = uk ? sqrtf(omega / (float)h) : 1.0f;
  const float* z = zb + (int64_t)blockIdx.x * kWideHP;
  const int D4 = Dp >> 2, R = 256 / D4;
  const int c4 = tid % D4, g = tid / D4;
  float4 acc4 = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int j0 = g; j0 < ntot; j0 += 8 * R) {
    float4 rv[8];
    float wv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int j = j0 + u * R;
      rv[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      wv[u] = 0.0f;
      if (j < ntot) {
        const int id = a.col[p0 + virt_pos_d(j, h)];
        const float cj = vk ? sqrtf(a.other_weight[id]) : cu;
        wv[u] = cj * z[j];
        rv[u] = *reinterpret_cast<const float4*>(a.Xrot + (int64_t)id * Dp + 4 * c4);
      }
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      acc4.x += wv[u] * rv[u].x;
      acc4.y += wv[u] * rv[u].y;
      acc4.z += wv[u] * rv[u].z;
      acc4.w += wv[u] * rv[u].w;
    }
  }
  *reinterpret_cast<float4*>(red + g * Dp + 4 * c4) = acc4;
  __syncthreads();
  for (int i = tid; i < Dp; i += 256) {
    float v = 0.0f;
    for (int gg = 0; gg < R; ++gg) v += red[gg * Dp + i];
    a.out_rot[blk_v(a.pos0 + blockIdx.x, i, Dp)] = v;
  }
}

template <int TH, bool BF>
hipError_t launch_wave_v(const DualArgs& a, hipStream_t s) {
  using C = WaveCfg<TH, BF>;
  const unsigned nb = (unsigned)((a.n_rows + 3) / 4);
  hipLaunchKernelGGL((dual_wave_kernel<TH, BF>), dim3(nb), dim3(256), C::bytes(a.Dp), s, a);
  return hipGetLastError();
}

template <int TH>
hipError_t launch_wave_t(const DualArgs& a, hipStream_t s) {
  return syrk_split_bf16() ? launch_wave_v<TH, true>(a, s) : launch_wave_v<TH, false>(a, s);
}

template <int TH, bool BF>
hipError_t launch_dual_v(const DualArgs& a, hipStream_t s) {
  using C = DualCfg<TH, BF>;
  static bool attr = false;
  if (!attr) {
    hipError_t err = hipFuncSetAttribute((const void*)dual_solve_kernel<TH, BF>,
                                         hipFuncAttributeMaxDynamicSharedMemorySize,
                                         (int)C::bytes(kMaxDp));
    if (err != hipSuccess) return err;
    attr = true;
  }
  hipLaunchKernelGGL((dual_solve_kernel<TH, BF>), dim3((unsigned)a.n_rows), dim3(C::NTHR),
                     C::bytes(a.Dp), s, a);
  return hipGetLastError();
}

template <int TH>
hipError_t launch_dual_t(const DualArgs& a, hipStream_t s) {
  return syrk_split_bf16() ? launch_dual_v<TH, true>(a, s) : launch_dual_v<TH, false>(a, s);
}

}  // namespace

hipError_t launch_dual_ldl(const DualArgs& a, hipStream_t s) {
  if (a.n_rows <= 0) return hipSuccess;
  if (a.Dp < 64 || a.Dp > kMaxDp || (a.Dp & 31)) return hipErrorInvalidValue;
  const unsigned nb = (unsigned)((a.n_rows + 255) / 256);
  hipLaunchKernelGGL(dual_ldl_kernel, dim3(nb), dim3(256), 0, s, a);
  return hipGetLastError();
}

size_t dual_wide_zs_bytes(int Dp) { return (size_t)(Dp / 16) * 3 * 2 * kWideHP * sizeof(bf16x8); }
size_t dual_wide_slot_floats() { return (size_t)16 * 17 / 2 * 1024 + kWideHP; }

hipError_t launch_dual_wide(const DualArgs& a, void* zs, float* slots, float* zbuf,
                            unsigned long long* fail, hipStream_t s) {
  if (a.n_rows <= 0) return hipSuccess;
  if (a.Dp != 512 && a.Dp != 1024) return hipErrorInvalidValue;
  const int64_t sf = (int64_t)dual_wide_slot_floats();
  bf16x8* z = reinterpret_cast<bf16x8*>(zs);
  hipLaunchKernelGGL(dual_wide_z_kernel, dim3((unsigned)a.n_rows), dim3(512), 0, s, a, z, slots, sf);
#ifndef FRECSYS_WIDE_S_LDS_DEFAULT
#define FRECSYS_WIDE_S_LDS_DEFAULT 1
#endif
  const char* sl = getenv("FRECSYS_WIDE_S_LDS");  // 0: dual_wide_s_kernel (A/B, bitwise tests)
  if (a.Dp == 1024 && (sl ? atoi(sl) != 0 : FRECSYS_WIDE_S_LDS_DEFAULT != 0)) {
    static bool attr = false;
    if (!attr) {
      for (const void* f : {(const void*)dual_wide_s_lds_kernel<0>, (const void*)dual_wide_s_lds_kernel<1>}) {
        hipError_t err = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)WS_LDS);
        if (err != hipSuccess) return err;
      }
      attr = true;
    }
    const int qv = (int)(is_v_kind(a.kind) && a.quirk);
    hipLaunchKernelGGL(dual_wide_s_lds_kernel<1>, dim3((unsigned)a.n_rows), dim3(512), WS_LDS, s,
                       (const bf16x8*)z, a.Dp, a.order, qv, slots, sf, (int64_t)a.n_rows);
    hipLaunchKernelGGL(dual_wide_s_lds_kernel<0>, dim3((unsigned)a.n_rows), dim3(512), WS_LDS, s,
                       (const bf16x8*)z, a.Dp, a.order, qv, slots, sf, (int64_t)a.n_rows);
  } else {
    hipLaunchKernelGGL(dual_wide_s_kernel, dim3((unsigned)(a.n_rows * 10)), dim3(256), 0, s,
                       (const bf16x8*)z, a.Dp, a.order,
                       (int)(is_v_kind(a.kind) && a.quirk), slots, sf);
  }
  hipError_t e = launch_wide_chol_slots(a.order, a.n_rows, slots, zbuf, fail,
                                        (int)(is_v_kind(a.kind) && a.quirk), s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(dual_wide_v_kernel, dim3((unsigned)a.n_rows), dim3(256), 0, s, a,
                     (const float*)zbuf);
  return hipGetLastError();
}

hipError_t launch_dual_sweep(const DualArgs& a, hipStream_t s) {
  if (a.n_rows <= 0) return hipSuccess;
  const unsigned nb = (unsigned)((a.n_rows + 255) / 256);
  hipLaunchKernelGGL(dual_sweep_kernel, dim3(nb), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_dual(int tiles, const DualArgs& a, hipStream_t s) {
  if (a.n_rows <= 0) return hipSuccess;
  if (a.Dp < 64 || a.Dp > kMaxDp || (a.Dp & 31)) return hipErrorInvalidValue;
  switch (tiles) {
    case 1: return FRECSYS_SKIP(a.debug_skip, 512) ? launch_dual_t<1>(a, s) : launch_wave_t<1>(a, s);
    case 2: return FRECSYS_SKIP(a.debug_skip, 512) ? launch_dual_t<2>(a, s) : launch_wave_t<2>(a, s);
    case 3: return launch_dual_t<3>(a, s);
    case 4: return launch_dual_t<4>(a, s);
    case 5: return launch_dual_t<5>(a, s);
    case 6: return launch_dual_t<6>(a, s);
    case 7: return launch_dual_t<7>(a, s);
    case 8: return launch_dual_t<8>(a, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace frecsys_hip
