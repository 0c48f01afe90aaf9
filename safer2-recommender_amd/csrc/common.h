// common.h -- device helpers shared by the gfx950 kernels.  Internal header.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

// Ablation masks (FRECSYS_DEBUG_SKIP) skip whole phases of the solve kernels
// for profiling.  They exist only in builds made with -DFRECSYS_ABLATION;
// in the shipped library every FRECSYS_SKIP(...) is the constant 0 and the
// skipped branches are compiled out.
#ifdef FRECSYS_ABLATION
#define FRECSYS_SKIP(mask, bit) ((mask) & (bit))
#else
#define FRECSYS_SKIP(mask, bit) 0
#endif

namespace frecsys_hip {

typedef float f32x16 __attribute__((ext_vector_type(16)));

enum {
  KIND_IALS = 0,
  KIND_WEIGHTED_U = 1,
  KIND_WEIGHTED_V = 2,
  KIND_CVAR_GRAD_U = 3,
  KIND_CVAR_GRAD_V = 4,
};

__host__ __device__ __forceinline__ bool is_v_kind(int k) {
  return k == KIND_WEIGHTED_V || k == KIND_CVAR_GRAD_V;
}
__host__ __device__ __forceinline__ bool is_u_kind(int k) {
  return k == KIND_WEIGHTED_U || k == KIND_CVAR_GRAD_U;
}
__host__ __device__ __forceinline__ bool is_grad_kind(int k) {
  return k == KIND_CVAR_GRAD_U || k == KIND_CVAR_GRAD_V;
}

// Tile (I, J), I >= J, of a T x T lower block layout.
__host__ __device__ constexpr int tidx(int I, int J) { return I * (I + 1) / 2 + J; }

// 32x32 fp32 tile in LDS, XOR-swizzled so that both row accesses (fixed r,
// lanes over c) and column accesses (fixed c, lanes over r) hit 32 distinct
// banks: element (r, c) at r*32 + (c ^ r).
__device__ __forceinline__ int sw(int r, int c) { return r * 32 + (c ^ r); }

// Row of a 32x32x2 f32 MFMA accumulator register q for a lane half `hi`
// (column = lane & 31).  gfx950 C/D layout.
__device__ __forceinline__ int acc_row(int q, int hi) {
  return (q & 3) + 8 * (q >> 2) + 4 * hi;
}

// Workgroup barrier for kernels whose waves exchange data through LDS only.
// __syncthreads() also drains every outstanding global load of the wave
// (s_waitcnt vmcnt(0)), which would land the one-chunk-ahead prefetches of
// the gather loops on the critical path at each barrier; this waits for LDS
// traffic only.  Register results of in-flight loads are waited on at
// their first use as usual.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Same-wave LDS ordering point (no global-memory drain).
__device__ __forceinline__ void wave_lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// ---- fp32 products on the bf16 matrix cores ----
// x = hi + mid + lo with three bf16 pieces (8 significant bits each; every
// subtraction is exact, the remainder is below 2^-26 |x|).  The six products
// hi*hi, hi*mid, mid*hi, mid*mid, hi*lo, lo*hi carry every term down to
// 2^-24 relative; the dropped mid*lo, lo*mid, lo*lo are <= 2^-25 |x y|.  So
// the accumulated sum is as accurate as an fp32 FMA chain, at 6 bf16 MFMAs
// (32 cycles each) per 16 products per output instead of 8 f32 MFMAs (64
// cycles each): 2.7x the product rate of v_mfma_f32_32x32x2_f32.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void split3(float x, __bf16& h, __bf16& m, __bf16& l) {
  h = (__bf16)x;
  float r = x - (float)h;
  m = (__bf16)r;
  r -= (float)m;
  l = (__bf16)r;
}

__device__ __forceinline__ f32x16 mfma_bf16(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// c += A B over 16 k for the split operands a[piece], b[piece]
// (piece 0 = hi, 1 = mid, 2 = lo): small terms first.
__device__ __forceinline__ f32x16 mfma_x6(const bf16x8 (&a)[3], const bf16x8 (&b)[3], f32x16 c) {
  c = mfma_bf16(a[2], b[0], c);
  c = mfma_bf16(a[0], b[2], c);
  c = mfma_bf16(a[1], b[1], c);
  c = mfma_bf16(a[1], b[0], c);
  c = mfma_bf16(a[0], b[1], c);
  c = mfma_bf16(a[0], b[0], c);
  return c;
}

// The same six products ordered so that each one after the first needs one
// more fragment than the one before it: the operand reads stagger behind
// the MFMAs instead of all being waited on up front (c already holds the
// running sum, so the order does not change the rounding).  Holds all six
// fragments at once: for kernels with registers to spare (solve.hip).
__device__ __forceinline__ f32x16 mfma_x6s(const bf16x8 (&a)[3], const bf16x8 (&b)[3], f32x16 c) {
  c = mfma_bf16(a[0], b[0], c);
  c = mfma_bf16(a[0], b[1], c);
  c = mfma_bf16(a[1], b[0], c);
  c = mfma_bf16(a[0], b[2], c);
  c = mfma_bf16(a[1], b[1], c);
  c = mfma_bf16(a[2], b[0], c);
  return c;
}

// Pieces of 8 consecutive-k values as three bf16x8 fragments.
__device__ __forceinline__ void split3x8(const float (&x)[8], bf16x8 (&f)[3]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    __bf16 h, m, l;
    split3(x[j], h, m, l);
    f[0][j] = h;
    f[1][j] = m;
    f[2][j] = l;
  }
}

// Lambda (regularisation) of one entity, per kind.
//  iALS: RegularizationValue, ials.h:310-315
//  U kinds: UserRegularizationValue, safer2.h:418-421
//  V kinds: ItemRegularizationValue, safer2.h:426-432
__device__ __forceinline__ float entity_lambda(int kind, float reg, float reg_exp, float w,
                                               float alpha, int64_t h, int64_t n_other,
                                               const float* entity_reg, int64_t e,
                                               int lambda_is_reg = 0) {
  if (lambda_is_reg) return reg;
  if (kind == KIND_IALS) return reg * powf((float)h + w * (float)n_other, reg_exp);
  if (is_u_kind(kind)) return reg * (1.0f + w * (float)n_other);
  return reg * (entity_reg[e] + alpha * w * (float)n_other);
}

// Assembled A(i, j) (i >= j part) from the accumulated observed sum s and
// the Gramian entry g, mirroring each reference's operation order:
//  iALS  (ials.h:101-105, 123):  (w*G + reg*I) + S
//  U     (safer2.h:143-150):     ((S / h) + w*G) * omega + reg*I
//  V     (safer2.h:178, 196, 206-208): (w*G + S) + reg*I
__device__ __forceinline__ float assemble(int kind, float s, float g, bool diag, float w,
                                          float lam, float hf, float omega) {
  if (kind == KIND_IALS) return (w * g + (diag ? lam : 0.0f)) + s;
  if (is_u_kind(kind)) return ((s / hf) + w * g) * omega + (diag ? lam : 0.0f);
  return (w * g + s) + (diag ? lam : 0.0f);
}

// Strict-upper entry of the full matrix read by CVaR-MF's `matrix * e`
// (cvar_mf.h:133, 179): the rank updates never wrote it.
__device__ __forceinline__ float cvar_upper(int kind, float g, float w, float omega) {
  if (kind == KIND_CVAR_GRAD_U) return (w * g) * omega;
  return w * g;
}

}  // namespace frecsys_hip
