/*
 * cpu_baseline.c -- the timed CPU baseline of bench.py ("kind": "port"):
 * the reference's per-entity Project / ProjectU / ProjectV (ials.h:88-144,
 * safer2.h:104-221) restated the way its Eigen build executes them --
 * cache-blocked, vectorised SYRK of 128-row batches (Eigen's
 * SelfAdjointView::rankUpdate is a blocked GEMM kernel) and a blocked
 * right-looking LLT (Eigen's llt_inplace::blocked) -- so the GPU/CPU ratio
 * is against a competitive CPU path, not the unblocked parity restatement of
 * frecsys_oracle.c.
 *
 * TEST INFRASTRUCTURE ONLY, like the rest of oracle/: nothing in the product
 * links, loads or calls it; bench.py's cpu_baseline leg times it and
 * tests/test_oracle.py checks it against oracle_step (rounding-level
 * differences only: the summation order is the blocked one).
 *
 * Compiled -O3 -march=native: the 16x16 micro-kernel below is written so
 * that gcc keeps the accumulator block in vector registers and turns its
 * inner loop into broadcast-FMAs (AVX-512: one zmm per accumulator row).
 */
#include <math.h>
#include <pthread.h>
#ifdef __AVX512F__
#include <immintrin.h>
#endif
#include <stdatomic.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define KB 128 /* rows per rank update (ials.h:108-123: batches of 128) */
#define MB 16  /* micro-kernel block */
#define NB 32  /* LLT panel width */

/* C (MB x MB, ldc) += sum_k A[k][0..MB) B[k][0..MB)^T-style outer products:
 * C[i][j] += sum_k a[k * lda + i] * b[k * ldb + j] (a, b k-major). */
static inline void mk_acc(float* restrict C, int ldc, const float* restrict a, int lda,
                          const float* restrict b, int ldb, int kn, float sign) {
#ifdef __AVX512F__
  /* one zmm accumulator per row of the block, broadcast-FMA per k */
  __m512 acc[MB];
  for (int i = 0; i < MB; ++i) acc[i] = _mm512_setzero_ps();
  for (int k = 0; k < kn; ++k) {
    const float* ak = a + (size_t)k * lda;
    const __m512 bk = _mm512_loadu_ps(b + (size_t)k * ldb);
#pragma GCC unroll 16
    for (int i = 0; i < MB; ++i) acc[i] = _mm512_fmadd_ps(_mm512_set1_ps(ak[i]), bk, acc[i]);
  }
  const __m512 sg = _mm512_set1_ps(sign);
  for (int i = 0; i < MB; ++i) {
    float* ci = C + (size_t)i * ldc;
    _mm512_storeu_ps(ci, _mm512_fmadd_ps(sg, acc[i], _mm512_loadu_ps(ci)));
  }
#else
  float acc[MB][MB];
  memset(acc, 0, sizeof(acc));
  for (int k = 0; k < kn; ++k) {
    const float* ak = a + (size_t)k * lda;
    const float* bk = b + (size_t)k * ldb;
    for (int i = 0; i < MB; ++i) {
      const float av = ak[i];
      for (int j = 0; j < MB; ++j) acc[i][j] += av * bk[j];
    }
  }
  for (int i = 0; i < MB; ++i)
    for (int j = 0; j < MB; ++j) C[(size_t)i * ldc + j] += sign * acc[i][j];
#endif
}

/* A (lower, n x n padded to np, ld np) += sign * P^T P over kn rows of the
 * k-major P [kn][np] (only blocks on or below the diagonal, from row block
 * r0 on). */
static void syrk_lower(float* A, int np, const float* P, int kn, int r0, float sign) {
  for (int i0 = r0; i0 < np; i0 += MB)
    for (int j0 = r0; j0 <= i0; j0 += MB)
      mk_acc(A + (size_t)i0 * np + j0, np, P + i0, np, P + j0, np, kn, sign);
}

typedef struct {
  const int64_t* row_ptr;
  const int32_t* col;
  const float* X;
  const float* G;
  int64_t n_other;
  int dim, np, kind, quirk;
  float reg, reg_exp, w, alpha;
  const float* entity_weight;
  const float* entity_reg;
  const float* other_weight;
  float* out;
  atomic_llong next;
  atomic_llong fail;
  int64_t n_rows;
} cb_ctx;

/* One entity: A, b as the reference builds them, then the blocked LLT
 * solve.  Scratch: A [np*np], P [KB*np] (then the k-major panel), b, x. */
static int cb_entity(cb_ctx* c, int64_t r, float* A, float* P, float* b) {
  const int d = c->dim, np = c->np;
  const int64_t p0 = c->row_ptr[r], h = c->row_ptr[r + 1] - p0;
  if (h == 0) return 0;
  int64_t extra = 0;
  const int vk = c->kind == 2;
  if (vk && c->quirk && h > 128 && (h % 128) != 0) extra = 128 - (h % 128);
  const int64_t ntot = h + extra;
  float lam, omega = 1.0f;
  if (c->kind == 0)
    lam = c->reg * powf((float)h + c->w * (float)c->n_other, c->reg_exp);
  else if (c->kind == 1)
    lam = c->reg * (1.0f + c->w * (float)c->n_other);
  else
    lam = c->reg * (c->entity_reg[r] + c->alpha * c->w * (float)c->n_other);
  if (c->kind == 1 && c->entity_weight) omega = c->entity_weight[r];
  memset(A, 0, sizeof(float) * (size_t)np * np);
  memset(b, 0, sizeof(float) * (size_t)np);
  /* the G part first for iALS / V (ials.h:101-105, safer2.h:178); U kinds
   * scale the observed sum first (safer2.h:143-150) */
  if (c->kind != 1)
    for (int i = 0; i < d; ++i)
      for (int j = 0; j <= i; ++j) A[(size_t)i * np + j] = c->w * c->G[(size_t)i * d + j];
  for (int64_t k0 = 0; k0 < ntot; k0 += KB) {
    const int kn = (int)(ntot - k0 < KB ? ntot - k0 : KB);
    for (int k = 0; k < kn; ++k) {
      const int64_t kk = k0 + k;
      const int64_t pos = kk < h ? kk : h - 128 + (kk - h); /* tail quirk (App. A.1) */
      const int32_t id = c->col[p0 + pos];
      const float* x = c->X + (size_t)id * d;
      float* pk = P + (size_t)k * np;
      float sa = 1.0f, bw = 1.0f;
      if (vk) {
        const float nu = c->other_weight[id];
        sa = sqrtf(nu);
        bw = (kk < h && sa > 0.0f) ? nu / sa : 0.0f;
      }
      for (int j = 0; j < d; ++j) pk[j] = x[j] * sa;
      for (int j = d; j < np; ++j) pk[j] = 0.0f;
      if (kk < h)
        for (int j = 0; j < d; ++j) b[j] += bw * pk[j];
    }
    syrk_lower(A, np, P, kn, 0, 1.0f);
  }
  if (c->kind == 1) {
    const float ih = 1.0f / (float)h;
    for (int i = 0; i < d; ++i) {
      for (int j = 0; j <= i; ++j) {
        float v = A[(size_t)i * np + j] * ih + c->w * c->G[(size_t)i * d + j];
        A[(size_t)i * np + j] = v * omega;
      }
      b[i] *= omega * ih;
    }
  }
  for (int i = 0; i < d; ++i) A[(size_t)i * np + i] += lam;
  for (int i = d; i < np; ++i) A[(size_t)i * np + i] = 1.0f; /* padding: identity */
  /* blocked right-looking LLT (lower) */
  for (int p = 0; p < np; p += NB) {
    const int pe = p + NB;
    /* diagonal block, unblocked */
    for (int j = p; j < pe; ++j) {
      float s = A[(size_t)j * np + j];
      for (int k = p; k < j; ++k) s -= A[(size_t)j * np + k] * A[(size_t)j * np + k];
      if (!(s > 0.0f)) return -1;
      const float ljj = sqrtf(s), inv = 1.0f / ljj;
      A[(size_t)j * np + j] = ljj;
      for (int i = j + 1; i < pe; ++i) {
        float t = A[(size_t)i * np + j];
        for (int k = p; k < j; ++k) t -= A[(size_t)i * np + k] * A[(size_t)j * np + k];
        A[(size_t)i * np + j] = t * inv;
      }
    }
    if (pe >= np) break;
    /* panel rows below: L_ip = A_ip L_pp^-T with the explicit L_pp^-1 (a
     * GEMM on the micro-kernel, as Eigen's blocked TRSM kernels run) */
    float* Li = b + np;  /* [NB][NB]: row j = column j of L_pp^-1 */
    memset(Li, 0, sizeof(float) * NB * NB);
    for (int j = 0; j < NB; ++j) {  /* column j of L_pp^-1: L x = e_j */
      for (int i = j; i < NB; ++i) {
        float t = i == j ? 1.0f : 0.0f;
        const float* li = A + (size_t)(p + i) * np + p;
        for (int k = j; k < i; ++k) t -= li[k] * Li[j * NB + k];
        Li[j * NB + i] = t / li[i];
      }
    }
    for (int k = 0; k < NB; ++k)
      for (int i = pe; i < np; ++i) P[(size_t)k * np + i] = A[(size_t)i * np + p + k];
    for (int i = pe; i < np; ++i) memset(A + (size_t)i * np + p, 0, sizeof(float) * NB);
    /* L_ip[i][j] = sum_k A_ip[i][k] L^-1[j][k]: a = P (k-major A_ip^T),
     * b[k][j] = L^-1[j][k] = element j of column k = Li[k][j] */
    for (int i0 = pe; i0 < np; i0 += MB)
      for (int j0 = 0; j0 < NB; j0 += MB)
        mk_acc(A + (size_t)i0 * np + p + j0, np, P + i0, np, Li + j0, NB, NB, 1.0f);
    /* k-major copy of the panel, then the trailing update by the micro-kernel */
    for (int k = 0; k < NB; ++k)
      for (int i = pe; i < np; ++i) P[(size_t)k * np + i] = A[(size_t)i * np + p + k];
    syrk_lower(A, np, P, NB, pe, -1.0f);
  }
  /* L y = b, L^T x = y */
  for (int i = 0; i < np; ++i) {
    float t = i < d ? b[i] : 0.0f;
    const float* li = A + (size_t)i * np;
    for (int k = 0; k < i; ++k) t -= li[k] * b[k];
    b[i] = t / li[i];
  }
  for (int i = np - 1; i >= 0; --i) {
    float t = b[i];
    for (int k = i + 1; k < np; ++k) t -= A[(size_t)k * np + i] * b[k];
    b[i] = t / A[(size_t)i * np + i];
  }
  memcpy(c->out + (size_t)r * d, b, sizeof(float) * (size_t)d);
  return 0;
}

static void* cb_worker(void* arg) {
  cb_ctx* c = (cb_ctx*)arg;
  const int np = c->np;
  float* A = (float*)aligned_alloc(64, sizeof(float) * (size_t)np * np);
  float* P = (float*)aligned_alloc(64, sizeof(float) * (size_t)KB * np);
  float* b = (float*)aligned_alloc(64, sizeof(float) * ((size_t)np + 2 * NB * NB) + 64);
  for (;;) {
    const int64_t r = atomic_fetch_add(&c->next, 1);
    if (r >= c->n_rows) break;
    if (cb_entity(c, r, A, P, b)) {
      long long cur = atomic_load(&c->fail);
      while ((cur == 0 || cur > r + 1) &&
             !atomic_compare_exchange_weak(&c->fail, &cur, (long long)(r + 1))) {
      }
    }
  }
  free(A);
  free(P);
  free(b);
  return NULL;
}

/* Rows [0, n_rows) of a half-step of kind 0 (iALS), 1 (ProjectU) or 2
 * (ProjectV with the tail quirk when quirk != 0); out [n_rows][dim].
 * Returns 0, or 1 + the first row whose LLT failed. */
int64_t cpu_baseline_step(int64_t n_rows, const int64_t* row_ptr, const int32_t* col,
                          const float* X, int64_t n_other, int dim, const float* G, int kind,
                          float reg, float reg_exp, float w, float alpha, int quirk,
                          const float* entity_weight, const float* entity_reg,
                          const float* other_weight, float* out, int nthreads) {
  cb_ctx c;
  memset(&c, 0, sizeof(c));
  c.row_ptr = row_ptr;
  c.col = col;
  c.X = X;
  c.G = G;
  c.n_other = n_other;
  c.dim = dim;
  c.np = (dim + MB - 1) / MB * MB;
  if (c.np % NB) c.np = (c.np + NB - 1) / NB * NB;
  c.kind = kind;
  c.quirk = quirk;
  c.reg = reg;
  c.reg_exp = reg_exp;
  c.w = w;
  c.alpha = alpha;
  c.entity_weight = entity_weight;
  c.entity_reg = entity_reg;
  c.other_weight = other_weight;
  c.out = out;
  c.n_rows = n_rows;
  atomic_init(&c.next, 0);
  atomic_init(&c.fail, 0);
  int t = nthreads > 0 ? nthreads : 1;
  if (t > n_rows) t = (int)(n_rows > 0 ? n_rows : 1);
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)t);
  for (int i = 0; i < t; ++i) pthread_create(&th[i], NULL, cb_worker, &c);
  for (int i = 0; i < t; ++i) pthread_join(th[i], NULL);
  free(th);
  return (int64_t)atomic_load(&c.fail);
}
