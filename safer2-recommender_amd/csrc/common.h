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

// 32x32 fp32 tile in LDS: 16-B granules XOR-swizzled per row pair --
// element (r, c) at r*32 + 4 ((c/4) ^ (r/2 % 8)) + c % 4 -- so that a lane
// reading 4 consecutive columns of ITS row (lanes over rows: the MFMA operand
// reads, the diagonal factor's row loads) issues one conflict-free
// ds_read_b128 (row_gran: the 16 lanes of each b128 lane group cover 16
// distinct bank quads), and scalar accesses with lanes over the columns of
// one row (the accumulator-layout stores) stay conflict-free.  (The element
// swizzle r*32 + (c ^ r) it replaced, no vector row reads, was slower.)
__device__ __forceinline__ int sw(int r, int c) {
  return r * 32 + ((((c >> 2) ^ (r >> 1)) & 7) << 2) + (c & 3);
}
typedef float f32x4v __attribute__((ext_vector_type(4)));
// Columns 4G .. 4G+3 of row r of a swizzled tile.
__device__ __forceinline__ f32x4v row_gran(const float* tile, int r, int G) {
  return *reinterpret_cast<const f32x4v*>(tile + r * 32 + (((G ^ (r >> 1)) & 7) << 2));
}

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
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    case 24: asm volatile("s_waitcnt vmcnt(24)" ::: "memory"); break;
    case 48: asm volatile("s_waitcnt vmcnt(48)" ::: "memory"); break;
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


// ---- tagged words: a value and the step that produced it in one 64-bit
// word, stored and polled with agent-scope atomics (no fence, no barrier
// counter: a reader takes the word once its tag matches).  Cross-workgroup
// exchange of the persistent tridiagonalisation (wide.hip) and of the
// reflectors it publishes to the Q-row workers (qrows_worker below).
__device__ __forceinline__ void tstore(unsigned long long* p, unsigned tag, float v) {
  __hip_atomic_store(p, ((unsigned long long)tag << 32) | __float_as_uint(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
// Bounded wait (~2^24 polls): on timeout *err (if given) is set, *tcount
// (if given: the context's cumulative timeout counter, frecsys_counter
// "tagged_timeouts") incremented and 0 / NaN (nan_on_timeout) returned, so a
// caller never spins forever.
__device__ __forceinline__ float tpoll(const unsigned long long* p, unsigned tag, int* err,
                                       bool nan_on_timeout = false,
                                       unsigned* tcount = nullptr) {
  unsigned spins = 0;
  while (true) {
    const unsigned long long v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((unsigned)(v >> 32) == tag) return __uint_as_float((unsigned)v);
    if (++spins > (1u << 24)) {
      if (err) atomicExch(err, 1);
      if (tcount) atomicAdd(tcount, 1u);
      return nan_on_timeout ? __builtin_nanf("") : 0.0f;
    }
    if (err && (spins & 255) == 0 &&
        __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
      return nan_on_timeout ? __builtin_nanf("") : 0.0f;
    __builtin_amdgcn_s_sleep(1);
  }
}

// Rows of Q = H_0 H_1 ... H_{nsteps-1} by forward accumulation, consuming the
// reflectors as a tridiagonalisation publishes them: row r of Q starts as
// e_r and takes q_r <- q_r - tau_k (q_r . v_k) v_k^T per step (rows are
// independent).  One workgroup of NT threads owns rows 32*wid .. +31, NT/32
// threads per row, columns c = cs + (NT/32) j in registers.  Reflector k:
// vt[k * n + r] (r > k, tag k+1; entries r <= k are zero), tau_k: tt[k]
// (tag k+1).  vsh: LDS [2][NMAX], tau2: LDS [2] (double-buffered, one
// barrier per step).  A timed-out poll leaves NaN in the rows (the history-
// space pivots then fail and the call reruns in d-space).  At the end the
// rows go to Q (row-major); the workgroup then reads its 32 rows back (its
// own stores, visible after the barrier) into its granules of the split
// images of Q and Q^T that the rotations read (split_basis_kernel's layout;
// n a multiple of 32): row groups 2 wid, 2 wid + 1 of Q's image, column
// block wid of Q^T's.  (Staging them in LDS instead would size every
// workgroup of the reduction's launch for it: 64 / 128 KB at 512 / 1024.)
template <int NMAX, int NT>
__device__ __forceinline__ void qrows_worker(int wid, int n, int nsteps,
                                             const unsigned long long* vt,
                                             const unsigned long long* tt, float* Q,
                                             bf16x8* img_q, bf16x8* img_qt, float* vsh,
                                             float* tau2, unsigned* tcount) {
  constexpr int TPR = NT / 32, NC = NMAX / TPR;
  const int tid = threadIdx.x, rr = tid / TPR, cs = tid % TPR;
  const int row = 32 * wid + rr;
  float q[NC];
#pragma unroll
  for (int j = 0; j < NC; ++j) q[j] = (cs + TPR * j == row) ? 1.0f : 0.0f;
  for (int k = 0; k < nsteps; ++k) {
    float* v = vsh + (k & 1) * NMAX;
    for (int r = tid; r < NMAX; r += NT)
      v[r] = (r > k && r < n) ? tpoll(vt + (size_t)k * n + r, k + 1, nullptr, true, tcount) : 0.0f;
    if (tid == 0) tau2[k & 1] = tpoll(tt + k, k + 1, nullptr, true, tcount);
    __syncthreads();
    const float tau = tau2[k & 1];
    if (tau != 0.0f) {  // workgroup-uniform
      float d = 0.0f;
#pragma unroll
      for (int j = 0; j < NC; ++j) d += q[j] * v[cs + TPR * j];
#pragma unroll
      for (int o = 1; o < TPR; o <<= 1) d += __shfl_xor(d, o);
      d *= tau;
#pragma unroll
      for (int j = 0; j < NC; ++j) q[j] -= d * v[cs + TPR * j];
    }
  }
#pragma unroll
  for (int j = 0; j < NC; ++j) {
    const int c = cs + TPR * j;
    if (row < n && c < n) Q[(size_t)row * n + c] = q[j];
  }
  __syncthreads();
  if (!img_q || 32 * wid >= n) return;
  const float* qb = Q + (size_t)32 * wid * n;  // my 32 rows
  const int nct = n / 32, ns = n / 16;
  for (int g = tid; g < 2 * nct * 64; g += NT) {  // Q: rows 16 s + 8 hi .. +7 of column 32 C + lo
    const int lane = g & 63, lo = lane & 31, hi = lane >> 5;
    const int sc = g >> 6, C = sc % nct, s = 2 * wid + sc / nct;
    float x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = qb[(size_t)(16 * (s - 2 * wid) + 8 * hi + j) * n + 32 * C + lo];
    bf16x8 f[3];
    split3x8(x, f);
#pragma unroll
    for (int p = 0; p < 3; ++p) img_q[((size_t)(s * nct + C) * 3 + p) * 64 + lane] = f[p];
  }
  for (int g = tid; g < ns * 64; g += NT) {  // Q^T: B[k][col] = Q[col][k], col = 32 wid + lo
    const int lane = g & 63, lo = lane & 31, hi = lane >> 5;
    const int s = g >> 6;
    float x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = qb[(size_t)lo * n + 16 * s + 8 * hi + j];
    bf16x8 f[3];
    split3x8(x, f);
#pragma unroll
    for (int p = 0; p < 3; ++p) img_qt[((size_t)(s * nct + wid) * 3 + p) * 64 + lane] = f[p];
  }
}
}  // namespace frecsys_hip
