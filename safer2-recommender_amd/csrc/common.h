// common.h -- device helpers shared by the gfx950 kernels.  Internal header.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

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
