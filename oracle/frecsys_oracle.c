/*
 * frecsys_oracle.c -- CPU restatement of the reference's closed-form solve
 * loop.  TEST INFRASTRUCTURE ONLY: see frecsys_oracle.h for what may use it
 * and for the parity status.  Every function cites the reference lines it
 * restates (paths relative to the reference root).
 *
 * Arithmetic is float32 like the reference's Eigen `float` types, in the
 * reference's operation order where that order is visible in its source
 * (scaling order in Project*, batch-of-128 rank updates, float/double
 * promotions in the SAFER2 scalar math).  Inner-product summation order
 * inside Eigen's GEMM/SYRK/LLT kernels is not visible and is restated as
 * plain sequential loops; that changes results only at fp32 rounding level.
 */
#define _GNU_SOURCE
#include "frecsys_oracle.h"

#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#define KMAXBATCH 128 /* kMaxBatchSize, ials.h:107, safer2.h:117/177 */

static int resolve_threads(int n) {
  if (n > 0) return n;
  const char* e = getenv("OMP_NUM_THREADS");
  if (e && atoi(e) > 0) return atoi(e);
  long c = sysconf(_SC_NPROCESSORS_ONLN); /* hardware_concurrency() */
  return c > 0 ? (int)c : 1;
}

/* ------------------------------------------------------------------ */
/* std::mt19937 (libstdc++), restated.                                 */
/* ------------------------------------------------------------------ */
void oracle_mt_seed(oracle_mt19937* g, uint32_t seed) {
  g->mt[0] = seed;
  for (int i = 1; i < 624; ++i)
    g->mt[i] = 1812433253u * (g->mt[i - 1] ^ (g->mt[i - 1] >> 30)) + (uint32_t)i;
  g->idx = 624;
}

static void mt_twist(oracle_mt19937* g) {
  for (int i = 0; i < 624; ++i) {
    uint32_t y = (g->mt[i] & 0x80000000u) | (g->mt[(i + 1) % 624] & 0x7fffffffu);
    uint32_t v = g->mt[(i + 397) % 624] ^ (y >> 1);
    if (y & 1u) v ^= 0x9908b0dfu;
    g->mt[i] = v;
  }
  g->idx = 0;
}

uint32_t oracle_mt_next(oracle_mt19937* g) {
  if (g->idx >= 624) mt_twist(g);
  uint32_t y = g->mt[g->idx++];
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}

/* std::generate_canonical<float, 24>(mt19937): one draw, float(u)/2^32,
 * clamped below 1 (libstdc++ bits/random.tcc). */
static float canonical_float(oracle_mt19937* g) {
  float s = (float)oracle_mt_next(g);
  float r = s / 4294967296.0f;
  if (r >= 1.0f) r = nextafterf(1.0f, 0.0f);
  return r;
}

typedef struct {
  int saved_available;
  float saved;
} normal_state;

/* std::normal_distribution<float>::operator() (Marsaglia polar method,
 * libstdc++ bits/random.tcc).  Contraction into FMA is disabled so that
 * x*x + y*y rounds exactly like the un-fused libstdc++ code. */
__attribute__((optimize("fp-contract=off"))) static float normal_float(
    oracle_mt19937* g, normal_state* st, float mean, float stddev) {
  float ret;
  if (st->saved_available) {
    st->saved_available = 0;
    ret = st->saved;
  } else {
    float x, y, r2;
    do {
      x = (float)((double)(2.0f * canonical_float(g)) - 1.0);
      y = (float)((double)(2.0f * canonical_float(g)) - 1.0);
      r2 = x * x + y * y;
    } while (r2 > 1.0 || r2 == 0.0);
    const float mult = sqrtf(-2 * logf(r2) / r2);
    st->saved = x * mult;
    st->saved_available = 1;
    ret = y * mult;
  }
  ret = ret * stddev + mean;
  return ret;
}

/* Model ctor init: ials.h:47-51 (safer2.h:50-54, erm_mf.h:46-50,
 * cvar_mf.h:45-49) calling init_matrix (recommender.h:61-67), which builds
 * a NEW normal_distribution for each matrix (the polar method's saved
 * second value does not carry from U to V). */
void oracle_init_embeddings(uint32_t seed, float stdev, int dim, float* U,
                            int64_t nu, float* V, int64_t ni) {
  oracle_mt19937 g;
  oracle_mt_seed(&g, seed);
  float adjusted = (float)((double)stdev / sqrt((double)dim));
  normal_state st = {0, 0.f};
  for (int64_t i = 0; i < nu * dim; ++i) U[i] = normal_float(&g, &st, 0.f, adjusted);
  normal_state st2 = {0, 0.f};
  for (int64_t i = 0; i < ni * dim; ++i) V[i] = normal_float(&g, &st2, 0.f, adjusted);
}

/* ------------------------------------------------------------------ */
/* Small thread pool helper: run fn(ctx, item) for item in [0, n).     */
/* ------------------------------------------------------------------ */
typedef void (*item_fn)(void* ctx, int64_t item, float* scratch);
typedef struct {
  item_fn fn;
  void* ctx;
  int64_t n;
  atomic_llong next;
  size_t scratch_floats;
} pool_job;

static void* pool_worker(void* arg) {
  pool_job* j = (pool_job*)arg;
  float* scratch = j->scratch_floats ? (float*)malloc(j->scratch_floats * sizeof(float)) : NULL;
  for (;;) {
    int64_t i = atomic_fetch_add(&j->next, 1);
    if (i >= j->n) break;
    j->fn(j->ctx, i, scratch);
  }
  free(scratch);
  return NULL;
}

static void run_pool(item_fn fn, void* ctx, int64_t n, int nthreads, size_t scratch_floats) {
  pool_job j;
  j.fn = fn;
  j.ctx = ctx;
  j.n = n;
  atomic_init(&j.next, 0);
  j.scratch_floats = scratch_floats;
  int t = resolve_threads(nthreads);
  if (t > n) t = (int)(n > 0 ? n : 1);
  if (t <= 1) {
    pool_worker(&j);
    return;
  }
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * t);
  for (int i = 0; i < t; ++i) pthread_create(&th[i], NULL, pool_worker, &j);
  for (int i = 0; i < t; ++i) pthread_join(th[i], NULL);
  free(th);
}

/* ------------------------------------------------------------------ */
/* Gramian.  ials.h:321 `item_embedding.transpose() * item_embedding`;  */
/* weighted form safer2.h:504-509: W = U .* omega (row scale), G=U^T W. */
/* Partials over fixed row blocks summed in block order (deterministic */
/* for any thread count).                                              */
/* ------------------------------------------------------------------ */
typedef struct {
  const float* X;
  int64_t n;
  int dim;
  const float* w;
  int64_t block;
  float* partials;
} gram_ctx;

static void gram_block(void* vctx, int64_t b, float* scratch) {
  (void)scratch;
  gram_ctx* c = (gram_ctx*)vctx;
  const int d = c->dim;
  float* P = c->partials + (size_t)b * d * d;
  memset(P, 0, sizeof(float) * d * d);
  int64_t r0 = b * c->block, r1 = r0 + c->block;
  if (r1 > c->n) r1 = c->n;
  float* wx = (float*)malloc(sizeof(float) * d);
  for (int64_t r = r0; r < r1; ++r) {
    const float* x = c->X + (size_t)r * d;
    for (int j = 0; j < d; ++j) wx[j] = c->w ? x[j] * c->w[r] : x[j];
    for (int i = 0; i < d; ++i) {
      const float a = x[i];
      float* Pi = P + (size_t)i * d;
      for (int j = 0; j < d; ++j) Pi[j] += a * wx[j];
    }
  }
  free(wx);
}

void oracle_gramian(const float* X, int64_t n, int dim, const float* w, float* G,
                    int nthreads) {
  int64_t block = 4096;
  if (n / 64 > block) block = (n + 63) / 64;
  int64_t nb = (n + block - 1) / block;
  memset(G, 0, sizeof(float) * dim * dim);
  if (nb == 0) return;
  gram_ctx c = {X, n, dim, w, block, (float*)malloc(sizeof(float) * dim * dim * nb)};
  run_pool(gram_block, &c, nb, nthreads, 0);
  for (int64_t b = 0; b < nb; ++b) {
    const float* P = c.partials + (size_t)b * dim * dim;
    for (int i = 0; i < dim * dim; ++i) G[i] += P[i];
  }
  free(c.partials);
}

/* ------------------------------------------------------------------ */
/* Dense helpers: lower rank update, Cholesky (Eigen LLT<Lower>), solve */
/* ------------------------------------------------------------------ */

/* T(lower incl. diagonal) = sum over rows of s_r^2 x_r x_r^T; written
 * only in the lower triangle like SelfAdjointView<Lower>::rankUpdate. */
static void batch_syrk_lower(float* T, int d, const float* X, const int32_t* rows,
                             int64_t count, const float* scale_or_null) {
  for (int i = 0; i < d; ++i) memset(T + (size_t)i * d, 0, sizeof(float) * (i + 1));
  for (int64_t c = 0; c < count; ++c) {
    const float* x = X + (size_t)rows[c] * d;
    float s = scale_or_null ? scale_or_null[c] : 1.0f;
    for (int i = 0; i < d; ++i) {
      const float a = s * x[i];
      float* Ti = T + (size_t)i * d;
      for (int j = 0; j <= i; ++j) Ti[j] += a * (s * x[j]);
    }
  }
}

static void add_lower(float* A, const float* T, int d) {
  for (int i = 0; i < d; ++i)
    for (int j = 0; j <= i; ++j) A[(size_t)i * d + j] += T[(size_t)i * d + j];
}

/* LLT<MatrixXf, Lower> (ials.h:140): reads the lower triangle only.
 * The formulas are those of Eigen 3.4's llt_inplace::unblocked
 * (Eigen/src/Cholesky/LLT.h): L(i,j) = (A(i,j) - sum_k<j L(i,k)L(j,k)) /
 * L(j,j), L(j,j) = sqrt(A(j,j) - sum_k<j L(j,k)^2), each sum formed here
 * sequentially in ascending k, no FMA contraction (-std=c11).  This is NOT
 * Eigen's summation order: LLT::compute calls llt_inplace::blocked, which
 * runs the unblocked kernel only below size 32 and otherwise factors panels
 * of clamp((d/8)/16*16, 8, 128) columns with a TRSM and a rankUpdate of the
 * trailing block, and its squaredNorm / GEMV reductions are packet-
 * vectorised (an order that depends on the SIMD width of the reference's
 * build).  The two orders agree to fp32 rounding, far inside the 1e-4 bar;
 * element-wise parity with Eigen itself stays unpinned (Eigen is absent,
 * SURVEY 8(c)).  Run right-looking -- column j's products are subtracted
 * from the trailing lower triangle as soon as column j is final -- which
 * performs the same subtractions in the same order per element as the
 * ascending-k dot-product form (bit-identical results) with a unit-stride
 * inner loop the compiler vectorises.  L overwrites lower. */
static int cholesky_lower(float* A, int d) {
  float* c = (float*)malloc(sizeof(float) * (size_t)(d > 0 ? d : 1));
  int rc = 0;
  for (int j = 0; j < d; ++j) {
    float* Lj = A + (size_t)j * d;
    const float s = Lj[j];
    if (!(s > 0.0f)) {
      rc = -1;
      break;
    }
    const float ljj = sqrtf(s);
    Lj[j] = ljj;
    for (int i = j + 1; i < d; ++i) {
      float* Li = A + (size_t)i * d;
      Li[j] = Li[j] / ljj;
      c[i] = Li[j];
    }
    for (int i = j + 1; i < d; ++i) {
      float* Li = A + (size_t)i * d;
      const float lij = c[i];
      for (int k = j + 1; k <= i; ++k) Li[k] -= lij * c[k];
    }
  }
  free(c);
  return rc;
}

/* cholesky.solve(rhs): L y = b, L^T x = y. */
static void cholesky_solve(const float* L, int d, const float* b, float* x) {
  for (int i = 0; i < d; ++i) {
    const float* Li = L + (size_t)i * d;
    float t = b[i];
    for (int k = 0; k < i; ++k) t -= Li[k] * x[k];
    x[i] = t / Li[i];
  }
  for (int i = d - 1; i >= 0; --i) {
    float t = x[i];
    for (int k = i + 1; k < d; ++k) t -= L[(size_t)k * d + i] * x[k];
    x[i] = t / L[(size_t)i * d + i];
  }
}

/* Full dense y = M e (Eigen `matrix * user_emb`, cvar_mf.h:133). */
static void matvec_full(const float* M, int d, const float* e, float* y) {
  for (int i = 0; i < d; ++i) {
    const float* Mi = M + (size_t)i * d;
    float t = 0.f;
    for (int j = 0; j < d; ++j) t += Mi[j] * e[j];
    y[i] = t;
  }
}

/* Rank-updates in batches of <= 128 columns, as ials.h:107-131: each batch
 * product is formed then added.  With quirk != 0 the trailing partial batch
 * is the reference's stale full batch (safer2.h:200-204): history positions
 * [h-128, h) -- see DESIGN.md, Appendix "tail quirk". */
static void batched_rank_update(float* A, float* T, int d, const int32_t* hist, int64_t h,
                                const float* X, const float* nu_or_null, int quirk,
                                float* sc) {
  const int64_t bs = h < KMAXBATCH ? h : KMAXBATCH;
  const int64_t nfull = h / bs;
  const int64_t rem = h - nfull * bs;
  for (int64_t b = 0; b < nfull; ++b) {
    const int32_t* rows = hist + b * bs;
    if (nu_or_null)
      for (int64_t c = 0; c < bs; ++c) sc[c] = sqrtf(nu_or_null[rows[c]]);
    batch_syrk_lower(T, d, X, rows, bs, nu_or_null ? sc : NULL);
    add_lower(A, T, d);
  }
  if (rem != 0) {
    int64_t start = nfull * bs, count = rem;
    if (quirk) {
      start = h - bs;
      count = bs;
    }
    const int32_t* rows = hist + start;
    if (nu_or_null)
      for (int64_t c = 0; c < count; ++c) sc[c] = sqrtf(nu_or_null[rows[c]]);
    batch_syrk_lower(T, d, X, rows, count, nu_or_null ? sc : NULL);
    add_lower(A, T, d);
  }
}

/* scratch layout used by the projections: A[d*d], T[d*d], b[d], y[d],
 * sc[128] */
static size_t project_scratch(int d) { return (size_t)2 * d * d + 2 * d + KMAXBATCH; }

/* iALS Project, ials.h:88-144. */
static int project_ials_s(const int32_t* hist, int64_t h, const float* X, int d,
                          const float* G, float reg, float w, float* out, float* s) {
  float *A = s, *T = s + (size_t)d * d, *b = T + (size_t)d * d, *sc = b + 2 * d;
  for (int i = 0; i < d * d; ++i) A[i] = w * G[i];           /* :101 */
  for (int i = 0; i < d; ++i) A[(size_t)i * d + i] += reg;   /* :103-105 */
  memset(b, 0, sizeof(float) * d);
  for (int64_t c = 0; c < h; ++c) {                          /* :114-126 */
    const float* x = X + (size_t)hist[c] * d;
    for (int i = 0; i < d; ++i) b[i] += x[i];
  }
  batched_rank_update(A, T, d, hist, h, X, NULL, 0, sc);     /* :122-131 */
  if (cholesky_lower(A, d)) return -1;                       /* :140-141 */
  cholesky_solve(A, d, b, out);                              /* :142 */
  return 0;
}

/* ProjectU assembly, safer2.h:116-150 (== erm_mf.h:103-137,
 * cvar_mf.h:100-131, cvar_mf.h:194-225). Leaves A (full) and b. */
static void assemble_u(const int32_t* hist, int64_t h, const float* X, int d, const float* G,
                       float reg, float w, float weight, float* A, float* T, float* b,
                       float* sc) {
  memset(A, 0, sizeof(float) * d * d);                       /* :116 */
  memset(b, 0, sizeof(float) * d);
  for (int64_t c = 0; c < h; ++c) {                          /* :124-137 */
    const float* x = X + (size_t)hist[c] * d;
    for (int i = 0; i < d; ++i) b[i] += x[i];
  }
  batched_rank_update(A, T, d, hist, h, X, NULL, 0, sc);
  const float hf = (float)h;
  for (int i = 0; i < d * d; ++i) A[i] /= hf;                /* :143 */
  for (int i = 0; i < d * d; ++i) A[i] += w * G[i];          /* :145 */
  for (int i = 0; i < d * d; ++i) A[i] *= weight;            /* :146 */
  const float rs = weight / hf;                              /* :147 */
  for (int i = 0; i < d; ++i) b[i] *= rs;
  for (int i = 0; i < d; ++i) A[(size_t)i * d + i] += reg;   /* :148-150 */
}

/* ProjectV assembly, safer2.h:177-208 (== erm_mf.h:164-195,
 * cvar_mf.h:146-177). */
static void assemble_v(const int32_t* hist, int64_t h, const float* X, int d, const float* G,
                       float reg, float w, const float* nu, int quirk, float* A, float* T,
                       float* b, float* sc) {
  for (int i = 0; i < d * d; ++i) A[i] = w * G[i];           /* :178 */
  memset(b, 0, sizeof(float) * d);
  for (int64_t c = 0; c < h; ++c) {                          /* :185-190 */
    const float* x = X + (size_t)hist[c] * d;
    const float wt = nu[hist[c]];
    for (int i = 0; i < d; ++i) b[i] += wt * x[i];
  }
  batched_rank_update(A, T, d, hist, h, X, nu, quirk, sc);   /* :192-204 */
  for (int i = 0; i < d; ++i) A[(size_t)i * d + i] += reg;   /* :206-208 */
}

static int project_u_s(const int32_t* hist, int64_t h, const float* X, int d, const float* G,
                       float reg, float w, float weight, float* out, float* s) {
  float *A = s, *T = s + (size_t)d * d, *b = T + (size_t)d * d, *sc = b + 2 * d;
  assemble_u(hist, h, X, d, G, reg, w, weight, A, T, b, sc);
  if (cholesky_lower(A, d)) return -1;                       /* :159-161 */
  cholesky_solve(A, d, b, out);
  return 0;
}

static int project_v_s(const int32_t* hist, int64_t h, const float* X, int d, const float* G,
                       float reg, float w, const float* nu, int quirk, float* out, float* s) {
  float *A = s, *T = s + (size_t)d * d, *b = T + (size_t)d * d, *sc = b + 2 * d;
  assemble_v(hist, h, X, d, G, reg, w, nu, quirk, A, T, b, sc);
  if (cholesky_lower(A, d)) return -1;                       /* :217-219 */
  cholesky_solve(A, d, b, out);
  return 0;
}

/* e - eta (A e - b) with the full A (cvar_mf.h:133, :179). */
static void grad_step(const float* A, int d, const float* e, const float* b, float eta,
                      float* y, float* out) {
  matvec_full(A, d, e, y);
  for (int i = 0; i < d; ++i) out[i] = e[i] - eta * (y[i] - b[i]);
}

static void cvar_u_s(const int32_t* hist, int64_t h, const float* e, const float* X, int d,
                     const float* G, float reg, float w, float eta, float weight, float* out,
                     float* s) {
  float *A = s, *T = s + (size_t)d * d, *b = T + (size_t)d * d, *y = b + d, *sc = b + 2 * d;
  assemble_u(hist, h, X, d, G, reg, w, weight, A, T, b, sc);
  grad_step(A, d, e, b, eta, y, out);
}

static void cvar_v_s(const int32_t* hist, int64_t h, const float* e, const float* X, int d,
                     const float* G, float reg, float w, const float* nu, float eta, int quirk,
                     float* out, float* s) {
  float *A = s, *T = s + (size_t)d * d, *b = T + (size_t)d * d, *y = b + d, *sc = b + 2 * d;
  assemble_v(hist, h, X, d, G, reg, w, nu, quirk, A, T, b, sc);
  grad_step(A, d, e, b, eta, y, out);
}

int oracle_project_ials(const int32_t* hist, int64_t h, const float* X, int dim, const float* G,
                        float reg, float w, float* out) {
  float* s = (float*)malloc(project_scratch(dim) * sizeof(float));
  int r = project_ials_s(hist, h, X, dim, G, reg, w, out, s);
  free(s);
  return r;
}
int oracle_project_u(const int32_t* hist, int64_t h, const float* X, int dim, const float* G,
                     float reg, float w, float weight, float* out) {
  float* s = (float*)malloc(project_scratch(dim) * sizeof(float));
  int r = project_u_s(hist, h, X, dim, G, reg, w, weight, out, s);
  free(s);
  return r;
}
int oracle_project_v(const int32_t* hist, int64_t h, const float* X, int dim, const float* G,
                     float reg, float w, const float* nu, int quirk, float* out) {
  float* s = (float*)malloc(project_scratch(dim) * sizeof(float));
  int r = project_v_s(hist, h, X, dim, G, reg, w, nu, quirk, out, s);
  free(s);
  return r;
}
void oracle_cvar_project_u(const int32_t* hist, int64_t h, const float* e, const float* X,
                           int dim, const float* G, float reg, float w, float stepsize,
                           float weight, float* out) {
  float* s = (float*)malloc(project_scratch(dim) * sizeof(float));
  cvar_u_s(hist, h, e, X, dim, G, reg, w, stepsize, weight, out, s);
  free(s);
}
void oracle_cvar_project_v(const int32_t* hist, int64_t h, const float* e, const float* X,
                           int dim, const float* G, float reg, float w, const float* nu,
                           float stepsize, int quirk, float* out) {
  float* s = (float*)malloc(project_scratch(dim) * sizeof(float));
  cvar_v_s(hist, h, e, X, dim, G, reg, w, nu, stepsize, quirk, out, s);
  free(s);
}

/* ------------------------------------------------------------------ */
/* Side steps.  ials.h:317-365 (iALS Step), safer2.h:437-490 (StepU),  */
/* safer2.h:493-555 (StepV), cvar_mf.h:427-538 (gradient steps).       */
/* ------------------------------------------------------------------ */
typedef struct {
  const int64_t* row_ptr;
  const int32_t* col;
  const float* X;
  int64_t n_other;
  int dim;
  const float* G;
  const oracle_solve_params* p;
  const float* E;
  float* Out;
  atomic_llong first_fail;
} step_ctx;

static void step_row(void* vctx, int64_t r, float* s) {
  step_ctx* c = (step_ctx*)vctx;
  const int64_t h = c->row_ptr[r + 1] - c->row_ptr[r];
  if (h == 0) return; /* not in by_user/by_item: untouched */
  const int32_t* hist = c->col + c->row_ptr[r];
  const int d = c->dim;
  const oracle_solve_params* p = c->p;
  float* out = c->Out + (size_t)r * d;
  int rc = 0;
  float reg;
  switch (p->kind) {
    case 0: /* RegularizationValue, ials.h:310-315 */
      reg = p->reg * powf((float)h + p->w * (float)c->n_other, p->reg_exp);
      rc = project_ials_s(hist, h, c->X, d, c->G, reg, p->w, out, s);
      break;
    case 1: /* UserRegularizationValue, safer2.h:418-421 */
      reg = p->reg * (1 + p->w * (float)c->n_other);
      rc = project_u_s(hist, h, c->X, d, c->G, reg, p->w,
                       p->entity_weight ? p->entity_weight[r] : 1.0f, out, s);
      break;
    case 2: /* ItemRegularizationValue, safer2.h:426-432 */
      reg = p->reg * (p->entity_reg[r] + p->alpha * p->w * (float)c->n_other);
      rc = project_v_s(hist, h, c->X, d, c->G, reg, p->w, p->other_weight, p->quirk, out, s);
      break;
    case 3:
      reg = p->reg * (1 + p->w * (float)c->n_other);
      cvar_u_s(hist, h, c->E + (size_t)r * d, c->X, d, c->G, reg, p->w, p->stepsize,
               p->entity_weight ? p->entity_weight[r] : 1.0f, out, s);
      break;
    case 4:
      reg = p->reg * (p->entity_reg[r] + p->alpha * p->w * (float)c->n_other);
      cvar_v_s(hist, h, c->E + (size_t)r * d, c->X, d, c->G, reg, p->w, p->other_weight,
               p->stepsize, p->quirk, out, s);
      break;
  }
  if (rc) {
    long long cur = atomic_load(&c->first_fail);
    while ((cur == 0 || cur > r + 1) &&
           !atomic_compare_exchange_weak(&c->first_fail, &cur, (long long)(r + 1))) {
    }
  }
}

int64_t oracle_step(int64_t n_rows, const int64_t* row_ptr, const int32_t* col, const float* X,
                    int64_t n_other, int dim, const float* G, const oracle_solve_params* p,
                    const float* E, float* Out, int nthreads) {
  step_ctx c;
  c.row_ptr = row_ptr;
  c.col = col;
  c.X = X;
  c.n_other = n_other;
  c.dim = dim;
  c.G = G;
  c.p = p;
  c.E = E;
  c.Out = Out;
  atomic_init(&c.first_fail, 0);
  run_pool(step_row, &c, n_rows, nthreads, project_scratch(dim));
  return (int64_t)atomic_load(&c.first_fail);
}

/* ------------------------------------------------------------------ */
/* iALS++ (ialspp.h): PredictDataset (:480-520), Step (:351-424) with   */
/* ProjectBlock (:85-145) on one column block [start, end).            */
/* ------------------------------------------------------------------ */
typedef struct {
  const int64_t* row_ptr;
  const int32_t* col;
  const int32_t* rix;
  const float* X;
  const float* E;
  float* Eout;
  float* pred;
  const float* Gl;   /* b x b   local Gramian  (:360-361) */
  const float* Glg;  /* b x dim local-global   (:362-363) */
  int64_t n_other;
  int dim, start, b, kind;
  float reg, reg_exp, w, alpha;
  const float *entity_weight, *entity_reg, *other_weight;
  double* resid; /* per row */
  atomic_llong first_fail;
} pp_ctx;

static void pp_predict_row(void* vctx, int64_t r, float* s) {
  pp_ctx* c = (pp_ctx*)vctx;
  (void)s;
  const float* u = c->E + (size_t)r * c->dim;
  for (int64_t k = c->row_ptr[r]; k < c->row_ptr[r + 1]; ++k) {
    const float* x = c->X + (size_t)c->col[k] * c->dim;
    float t = 0.f;
    for (int j = 0; j < c->dim; ++j) t += x[j] * u[j];
    c->pred[c->rix[k]] = t;
  }
}

void oracle_pp_predict(int64_t n_rows, const int64_t* row_ptr, const int32_t* col,
                       const int32_t* rix, const float* X, int dim, const float* E, float* pred,
                       int nthreads) {
  pp_ctx c;
  memset(&c, 0, sizeof(c));
  c.row_ptr = row_ptr;
  c.col = col;
  c.rix = rix;
  c.X = X;
  c.E = E;
  c.pred = pred;
  c.dim = dim;
  run_pool(pp_predict_row, &c, n_rows, nthreads, 1);
}

static void pp_step_row(void* vctx, int64_t r, float* s) {
  pp_ctx* c = (pp_ctx*)vctx;
  const int64_t h = c->row_ptr[r + 1] - c->row_ptr[r];
  if (h == 0) return;
  const int b = c->b, d = c->dim, st = c->start;
  float *A = s, *T = s + (size_t)b * b, *rhs = T + (size_t)b * b, *nv = rhs + b;
  const float* u = c->E + (size_t)r * d;
  const int32_t* hist = c->col + c->row_ptr[r];
  /* kind 0: iALS++ ProjectBlock (ialspp.h:85-145), reg =
   * RegularizationValue(h, num_items) (:377, :313-318);
   * kind 1: SAFER2++ ProjectU (safer2pp.h:97-160), reg =
   * UserRegularizationValue, weight = dual weight;
   * kind 2: SAFER2++ ProjectV (safer2pp.h:162-216), reg =
   * ItemRegularizationValue, per-row weight nu_u = omega_u / |H_u|, the
   * Gramians weighted by omega (StepV, safer2pp.h:530-541). */
  float reg, wt = 1.0f;
  if (c->kind == 0) {
    reg = c->reg * powf((float)h + c->w * (float)c->n_other, c->reg_exp);
  } else if (c->kind == 1) {
    reg = c->reg * (1 + c->w * (float)c->n_other);
    wt = c->entity_weight ? c->entity_weight[r] : 1.0f;
  } else {
    reg = c->reg * (c->entity_reg[r] + c->alpha * c->w * (float)c->n_other);
  }
  if (c->kind == 1) {
    memset(A, 0, sizeof(float) * (size_t)b * b);
  } else {
    for (int i = 0; i < b * b; ++i) A[i] = c->w * c->Gl[i];          /* :95 / :173 */
    for (int i = 0; i < b; ++i) A[(size_t)i * b + i] += reg;         /* :97-99 */
  }
  memset(rhs, 0, sizeof(float) * b);
  for (int64_t k = 0; k < h; ++k) {                                  /* :107-121 */
    const int32_t o = hist[k];
    const float* x = c->X + (size_t)o * d + st;
    const float nu = c->kind == 2 ? c->other_weight[o] : 1.0f;
    const float res = c->pred[c->rix[c->row_ptr[r] + k]] - 1.0f;
    for (int i = 0; i < b; ++i) rhs[i] += c->kind == 2 ? x[i] * res * nu : x[i] * res;
  }
  /* rank updates in 128-column batches (:102-131), lower only */
  for (int64_t k0 = 0; k0 < h; k0 += KMAXBATCH) {
    const int64_t cnt = h - k0 < KMAXBATCH ? h - k0 : KMAXBATCH;
    for (int i = 0; i < b; ++i) memset(T + (size_t)i * b, 0, sizeof(float) * (i + 1));
    for (int64_t k = k0; k < k0 + cnt; ++k) {
      const float* x = c->X + (size_t)hist[k] * d + st;
      const float sq = c->kind == 2 ? sqrtf(c->other_weight[hist[k]]) : 1.0f;
      for (int i = 0; i < b; ++i)
        for (int j = 0; j <= i; ++j) T[(size_t)i * b + j] += (x[i] * sq) * (x[j] * sq);
    }
    add_lower(A, T, b);
  }
  if (c->kind == 1) { /* safer2pp.h:136-150 */
    for (int i = 0; i < b; ++i)
      for (int j = 0; j <= i; ++j) {
        float v = A[(size_t)i * b + j] / (float)h;
        v += c->w * c->Gl[(size_t)i * b + j];
        A[(size_t)i * b + j] = v * wt;
      }
    for (int i = 0; i < b; ++i) rhs[i] *= wt / (float)h;
  }
  for (int i = 0; i < b; ++i) {                                      /* :134-137 */
    float t = 0.f;
    for (int j = 0; j < d; ++j) t += c->Glg[(size_t)i * d + j] * u[j];
    rhs[i] += c->kind == 1 ? c->w * t * wt : c->w * t;
    rhs[i] += reg * u[st + i];
  }
  if (c->kind == 1)
    for (int i = 0; i < b; ++i) A[(size_t)i * b + i] += reg;
  if (cholesky_lower(A, b)) {                                        /* :139-140 */
    long long cur = atomic_load(&c->first_fail);
    while ((cur == 0 || cur > r + 1) &&
           !atomic_compare_exchange_weak(&c->first_fail, &cur, (long long)(r + 1))) {
    }
    return;
  }
  cholesky_solve(A, b, rhs, nv);
  double res2 = 0.0;
  float* out = c->Eout + (size_t)r * d + st;
  for (int i = 0; i < b; ++i) {
    const float nw = u[st + i] - nv[i];                              /* :141 */
    nv[i] = nw - u[st + i];                                          /* delta (:398-399) */
    out[i] = nw;
    res2 += (double)nv[i] * nv[i];
  }
  for (int64_t k = 0; k < h; ++k) {                                  /* :400-404 */
    const float* x = c->X + (size_t)hist[k] * d + st;
    float t = 0.f;
    for (int i = 0; i < b; ++i) t += nv[i] * x[i];
    c->pred[c->rix[c->row_ptr[r] + k]] += t;
  }
  c->resid[r] = res2;
}

int64_t oracle_pp_step(int64_t n_rows, const int64_t* row_ptr, const int32_t* col,
                       const int32_t* rix, const float* X, int64_t n_other, int dim, float* E,
                       float* pred, int start, int end, const oracle_solve_params* p,
                       const float* gram_w, double* residual, int nthreads) {
  const int b = end - start;
  pp_ctx c;
  memset(&c, 0, sizeof(c));
  float* Gl = (float*)calloc((size_t)b * b, sizeof(float));
  float* Glg = (float*)calloc((size_t)b * dim, sizeof(float));
  float* Ecopy = (float*)malloc(sizeof(float) * (size_t)(n_rows > 0 ? n_rows : 1) * dim);
  double* res = (double*)calloc((size_t)(n_rows > 0 ? n_rows : 1), sizeof(double));
  /* local_gramian = Xb^T Xb, local_global = Xb^T X (:356-363); weighted
   * by gram_w (the dual weights) for the SAFER2++ V step */
  for (int64_t o = 0; o < n_other; ++o) {
    const float* x = X + (size_t)o * dim;
    const float gw = gram_w ? gram_w[o] : 1.0f;
    for (int i = 0; i < b; ++i) {
      const float a = gram_w ? x[start + i] * gw : x[start + i];
      for (int j = 0; j < b; ++j) Gl[(size_t)i * b + j] += a * x[start + j];
      for (int j = 0; j < dim; ++j) Glg[(size_t)i * dim + j] += a * x[j];
    }
  }
  memcpy(Ecopy, E, sizeof(float) * (size_t)n_rows * dim);
  c.row_ptr = row_ptr;
  c.col = col;
  c.rix = rix;
  c.X = X;
  c.E = Ecopy;
  c.Eout = E;
  c.pred = pred;
  c.Gl = Gl;
  c.Glg = Glg;
  c.n_other = n_other;
  c.dim = dim;
  c.start = start;
  c.b = b;
  c.kind = p->kind;
  c.reg = p->reg;
  c.reg_exp = p->reg_exp;
  c.w = p->w;
  c.alpha = p->alpha;
  c.entity_weight = p->entity_weight;
  c.entity_reg = p->entity_reg;
  c.other_weight = p->other_weight;
  c.resid = res;
  atomic_init(&c.first_fail, 0);
  run_pool(pp_step_row, &c, n_rows, nthreads, (size_t)2 * b * b + 2 * b);
  double tot = 0.0;
  for (int64_t r = 0; r < n_rows; ++r) tot += res[r];
  if (residual) *residual = tot;
  free(Gl);
  free(Glg);
  free(Ecopy);
  free(res);
  return (int64_t)atomic_load(&c.first_fail);
}

/* ------------------------------------------------------------------ */
/* User loss: ComputeLoss ials.h:70-86 / safer2.h:85-101 via           */
/* ComputeUserLoss ials.h:367-408 / safer2.h:558-596.                  */
/* ------------------------------------------------------------------ */
typedef struct {
  const int64_t* row_ptr;
  const int32_t* col;
  const float *U, *V, *G;
  int dim;
  float beta;
  int half;
  float* out;
} loss_ctx;

static void loss_row(void* vctx, int64_t u, float* s) {
  loss_ctx* c = (loss_ctx*)vctx;
  const int64_t h = c->row_ptr[u + 1] - c->row_ptr[u];
  if (h == 0) return;
  const int d = c->dim;
  const float* e = c->U + (size_t)u * d;
  float loss = 0;
  for (int64_t k = c->row_ptr[u]; k < c->row_ptr[u + 1]; ++k) {
    const float* x = c->V + (size_t)c->col[k] * d;
    float dot = 0.f;
    for (int i = 0; i < d; ++i) dot += x[i] * e[i];
    const float t = dot - 1;
    loss = (float)((double)loss + (double)t * (double)t); /* pow(.,2.0) */
  }
  loss /= (float)h;
  /* ireg = u^T G u evaluated as (u^T G) u */
  for (int j = 0; j < d; ++j) {
    float t = 0.f;
    for (int i = 0; i < d; ++i) t += e[i] * c->G[(size_t)i * d + j];
    s[j] = t;
  }
  float ireg = 0.f;
  for (int j = 0; j < d; ++j) ireg += s[j] * e[j];
  loss += c->beta * ireg;
  if (c->half) loss = (float)((double)loss / 2.0);
  c->out[u] = loss;
}

void oracle_user_loss(int64_t n_users, const int64_t* row_ptr, const int32_t* col,
                      const float* U, const float* V, int dim, const float* G, float beta,
                      int half, float* out, int nthreads) {
  loss_ctx c = {row_ptr, col, U, V, G, dim, beta, half, out};
  run_pool(loss_row, &c, n_users, nthreads, (size_t)dim);
}

/* ------------------------------------------------------------------ */
/* SAFER2 smoothed quantile (safer2.h:598-742) and weights (:745-794). */
/* Mixed float/double promotions follow the source expressions.        */
/* ------------------------------------------------------------------ */
static float gaussian_kernel(float u, float h) { /* :599-602 */
  return (float)(pow(2 * M_PI, -0.5) * exp(-pow((double)(u / h) * M_SQRT1_2, 2)) / h);
}
static float gaussian_kernel_cdf(float u, float h) { /* :604-607 */
  return (float)(0.5 * erfc(-(double)(u / h) * M_SQRT1_2));
}
static float gaussian_loss(float u, float h, float alpha) { /* :609-615 */
  float ell = h * gaussian_kernel(u, h) + (u / h) * (1 - 2 * gaussian_kernel_cdf(-u, h));
  return (float)((double)((h / 2) * ell) + ((double)(1 - alpha) - 0.5) * (double)u);
}
static float epanechnikov_kernel(float u, float h) { /* :618-622 */
  float uh = u / h;
  return (float)((3.0 / 4.0) * (1 - pow((double)uh, 2)) * (int)(fabsf(uh) < 1) / h);
}
static float epanechnikov_kernel_cdf(float u, float h) { /* :624-634 */
  float uh = u / h;
  int in_supp = (int)(fabsf(uh) <= 1);
  int pos = (int)(uh > 1);
  double cdf = ((pow((double)h, -3) / 4.0) *
                ((3 * (double)u * pow((double)h, 2) - pow((double)u, 3)) + 2 * pow((double)h, 3)) *
                in_supp) +
               (double)((1 - in_supp) * pos);
  return (float)cdf;
}
static float epanechnikov_loss(float u, float h, float alpha) { /* :636-647 */
  float uh = u / h;
  int in_supp = (int)(fabsf(uh) <= 1);
  int pos = (int)(uh > 1);
  float ell = (float)(((3.0 / 4.0) * pow((double)uh, 2) - (1.0 / 8.0) * pow((double)uh, 4) +
                       (3.0 / 8.0)) *
                          in_supp +
                      (double)(fabsf(uh) * pos));
  return (float)((1.0 / 2.0) * h * ell + ((double)(1 - alpha) - 0.5) * (double)u);
}

float oracle_safer2_weight(float loss, float xi, float bandwidth, int epan) {
  float r = loss - xi; /* :770 */
  if (epan) return 1 - epanechnikov_kernel_cdf(-r, bandwidth);
  return 1 - gaussian_kernel_cdf(-r, bandwidth);
}

/* EvaluateQuantile, safer2.h:652-689.  r = user_loss.array() - xi in float;
 * each r.unaryExpr(lambda).mean() is Eigen's reduction of an expression
 * without packet access (Redux.h DefaultTraversal): sequential float sum
 * from the first element, divided by float(n). */
static void evaluate_quantile(float xi, const float* loss, int64_t n, float alpha, float bw,
                              int epan, float* value, float* grad, float* H) {
  float sc = 0, sk = 0, sl = 0;
  for (int64_t i = 0; i < n; ++i) {
    const float u = loss[i] - xi;
    float c, k, l;
    if (epan) {
      c = epanechnikov_kernel_cdf(-u, bw);
      k = epanechnikov_kernel(-u, bw);
      l = epanechnikov_loss(u, bw, alpha);
    } else {
      c = gaussian_kernel_cdf(-u, bw);
      k = gaussian_kernel(-u, bw);
      l = gaussian_loss(u, bw, alpha);
    }
    if (i == 0) {
      sc = c;
      sk = k;
      sl = l;
    } else {
      sc += c;
      sk += k;
      sl += l;
    }
  }
  const float fn = (float)n;
  *grad = (-(1 - alpha) + sc / fn) / alpha;
  *H = (sk / fn) / alpha;
  *value = (sl / fn) / alpha;
}

/* ComputeXiDirection, safer2.h:692-712 (Armijo uses grad at the trial
 * point, as in the source). */
static float xi_direction(float xi, const float* loss, int64_t n, float alpha, float bw,
                          int epan) {
  float f0, g0, H;
  evaluate_quantile(xi, loss, n, alpha, bw, epan, &f0, &g0, &H);
  const float d = g0 / H;
  const float c = 1e-4f;
  float gamma = 1.0f;
  float x = xi + gamma * (-d);
  for (int k = 0; k < 32; k++) {
    float fx, gx, Hx;
    evaluate_quantile(x, loss, n, alpha, bw, epan, &fx, &gx, &Hx);
    if (fx > f0 + c * gamma * gx * (-d)) {
      gamma *= 0.5f;
      x = xi + gamma * (-d);
    } else {
      break;
    }
  }
  return -gamma * d;
}

/* ComputeXi, safer2.h:716-742 (use_snr = false path). */
float oracle_safer2_xi(const float* loss, int64_t n, float prev_xi, int iterations, float alpha,
                       float bandwidth, int epan) {
  float xi = prev_xi;
  for (int t = 0; t < iterations; ++t) xi = xi + xi_direction(xi, loss, n, alpha, bandwidth, epan);
  return xi;
}

/* std::uniform_int_distribution<int>(0, range - 1)(mt19937) of libstdc++
 * (GCC 11, bits/uniform_int_dist.h): the generator yields exactly 32 bits,
 * so the draw is Lemire's nearly-divisionless reduction _S_nd with 64-bit
 * products.  Checked against libstdc++ itself in tests/test_oracle.py. */
uint32_t oracle_uniform_int(oracle_mt19937* g, uint32_t range) {
  uint64_t product = (uint64_t)oracle_mt_next(g) * (uint64_t)range;
  uint32_t low = (uint32_t)product;
  if (low < range) {
    const uint32_t threshold = (uint32_t)(-range) % range;
    while (low < threshold) {
      product = (uint64_t)oracle_mt_next(g) * (uint64_t)range;
      low = (uint32_t)product;
    }
  }
  return (uint32_t)(product >> 32);
}

/* ComputeXi, safer2.h:716-742, use_snr = true: every iteration draws
 * int(N * sampling_ratio) user indices uniformly with replacement
 * (:727-734) and takes the Newton/Armijo step on that sample (:735).  The
 * reference seeds a fresh mt19937 from std::random_device per iteration;
 * the build's --seed replaces that with one seeded generator (SURVEY
 * App. A.7) that persists across calls, restated here as *g. */
float oracle_safer2_xi_snr(const float* loss, int64_t n, float prev_xi, int iterations,
                           float alpha, float bandwidth, int epan, float sampling_ratio,
                           oracle_mt19937* g) {
  float xi = prev_xi;
  const int ns = (int)((float)n * sampling_ratio);
  float* sample = (float*)malloc(sizeof(float) * (ns > 0 ? ns : 1));
  for (int t = 0; t < iterations; ++t) {
    for (int j = 0; j < ns; ++j) sample[j] = loss[oracle_uniform_int(g, (uint32_t)n)];
    xi = xi + xi_direction(xi, sample, ns, alpha, bandwidth, epan);
  }
  free(sample);
  return xi;
}

static int cmp_float_asc(const void* a, const void* b) {
  float x = *(const float*)a, y = *(const float*)b;
  return (x > y) - (x < y);
}

/* CVaR-MF ComputeXi, cvar_mf.h:582-595: -nth_element(-loss)[N*alpha]. */
float oracle_cvar_xi(const float* loss, int64_t n, float alpha) {
  float* v = (float*)malloc(sizeof(float) * n);
  for (int64_t i = 0; i < n; ++i) v[i] = -loss[i];
  qsort(v, n, sizeof(float), cmp_float_asc);
  size_t k = (size_t)((float)n * alpha);
  float xi = -v[k];
  free(v);
  return xi;
}

/* ------------------------------------------------------------------ */
/* Whole models.                                                       */
/* ------------------------------------------------------------------ */
struct oracle_model {
  oracle_model_params p;
  float *U, *V, *Uprev;
  float *item_gramian, *G2;
  float *user_loss, *dual_weight, *hsize, *item_reg, *nu;
  float prev_xi;
  oracle_mt19937 snr;
  const int64_t *u_ptr, *i_ptr;
  const int32_t *u_col, *i_col;
};

oracle_model* oracle_model_create(const oracle_model_params* p, uint32_t seed) {
  oracle_model* m = (oracle_model*)calloc(1, sizeof(oracle_model));
  m->p = *p;
  const int d = p->dim;
  m->U = (float*)malloc(sizeof(float) * p->n_users * d);
  m->Uprev = (float*)malloc(sizeof(float) * p->n_users * d);
  m->V = (float*)malloc(sizeof(float) * p->n_items * d);
  m->item_gramian = (float*)malloc(sizeof(float) * d * d);
  m->G2 = (float*)malloc(sizeof(float) * d * d);
  m->user_loss = (float*)calloc(p->n_users, sizeof(float));
  m->dual_weight = (float*)malloc(sizeof(float) * p->n_users);
  m->hsize = (float*)calloc(p->n_users, sizeof(float));
  m->nu = (float*)calloc(p->n_users, sizeof(float));
  m->item_reg = (float*)calloc(p->n_items, sizeof(float));
  oracle_init_embeddings(seed, p->stdev, d, m->U, p->n_users, m->V, p->n_items);
  for (int64_t u = 0; u < p->n_users; ++u) m->dual_weight[u] = p->alpha; /* safer2.h:56 */
  oracle_gramian(m->V, p->n_items, d, NULL, m->item_gramian, p->nthreads); /* :55 */
  m->prev_xi = 0.0f;
  oracle_mt_seed(&m->snr, seed + 7919u);
  return m;
}

void oracle_model_destroy(oracle_model* m) {
  if (!m) return;
  free(m->U);
  free(m->Uprev);
  free(m->V);
  free(m->item_gramian);
  free(m->G2);
  free(m->user_loss);
  free(m->dual_weight);
  free(m->hsize);
  free(m->nu);
  free(m->item_reg);
  free(m);
}

void oracle_model_set_data(oracle_model* m, const int64_t* u_ptr, const int32_t* u_col,
                           const int64_t* i_ptr, const int32_t* i_col) {
  m->u_ptr = u_ptr;
  m->u_col = u_col;
  m->i_ptr = i_ptr;
  m->i_col = i_col;
}

void oracle_model_set_embeddings(oracle_model* m, const float* U, const float* V) {
  const int d = m->p.dim;
  memcpy(m->U, U, sizeof(float) * m->p.n_users * d);
  memcpy(m->V, V, sizeof(float) * m->p.n_items * d);
  oracle_gramian(m->V, m->p.n_items, d, NULL, m->item_gramian, m->p.nthreads);
}

void oracle_model_get_embeddings(const oracle_model* m, float* U, float* V) {
  const int d = m->p.dim;
  if (U) memcpy(U, m->U, sizeof(float) * m->p.n_users * d);
  if (V) memcpy(V, m->V, sizeof(float) * m->p.n_items * d);
}

void oracle_model_get_state(const oracle_model* m, float* user_loss, float* dual_weight,
                            float* xi) {
  if (user_loss) memcpy(user_loss, m->user_loss, sizeof(float) * m->p.n_users);
  if (dual_weight) memcpy(dual_weight, m->dual_weight, sizeof(float) * m->p.n_users);
  if (xi) *xi = m->prev_xi;
}

/* VectorXf::mean() of the reference (Eigen 3.4 Redux.h,
 * LinearVectorizedTraversal, AVX-512 packets of 16 floats under
 * -march=native): two packet accumulators, the predux<Packet16f> tree, the
 * trailing scalars, then / float(n).  Same restatement as the product's
 * include/frecsys/types.h detail::eigen_packet_sum. */
static float eigen_packet_sum(const float* x, int64_t n) {
  enum { P = 16 };
  if (n <= 0) return 0.0f;
  const int64_t aligned = n / P * P, aligned2 = n / (2 * P) * (2 * P);
  if (aligned == 0) {
    float r = x[0];
    for (int64_t i = 1; i < n; ++i) r += x[i];
    return r;
  }
  float p0[P], p1[P];
  for (int k = 0; k < P; ++k) p0[k] = x[k];
  if (aligned > P) {
    for (int k = 0; k < P; ++k) p1[k] = x[P + k];
    for (int64_t i = 2 * P; i < aligned2; i += 2 * P)
      for (int k = 0; k < P; ++k) {
        p0[k] += x[i + k];
        p1[k] += x[i + P + k];
      }
    for (int k = 0; k < P; ++k) p0[k] += p1[k];
    if (aligned > aligned2)
      for (int k = 0; k < P; ++k) p0[k] += x[aligned2 + k];
  }
  float s8[8], s4[4];
  for (int k = 0; k < 8; ++k) s8[k] = p0[k] + p0[k + 8];
  for (int k = 0; k < 4; ++k) s4[k] = s8[k] + s8[k + 4];
  const float t0 = s4[0] + s4[2], t1 = s4[1] + s4[3];
  float r = t0 + t1;
  for (int64_t i = aligned; i < n; ++i) r += x[i];
  return r;
}

float oracle_mean(const float* x, int64_t n) {
  return n > 0 ? eigen_packet_sum(x, n) / (float)n : 0.0f;
}

/* SAFER2 ComputeXi of the model: exact Newton, or SNR on the model's
 * seeded sample stream (the product seeds it with seed + 7919). */
static float model_xi(oracle_model* m, float prev) {
  const oracle_model_params* p = &m->p;
  if (p->use_snr)
    return oracle_safer2_xi_snr(m->user_loss, p->n_users, prev, p->xi_iterations, p->alpha,
                                p->bandwidth, p->use_epanechnikov, p->sampling_ratio, &m->snr);
  return oracle_safer2_xi(m->user_loss, p->n_users, prev, p->xi_iterations, p->alpha,
                          p->bandwidth, p->use_epanechnikov);
}

/* Initialize: safer2.h:819-838, erm_mf.h:573-587, cvar_mf.h:710-726. */
void oracle_model_initialize(oracle_model* m) {
  const oracle_model_params* p = &m->p;
  if (p->model == 0) return;
  oracle_user_loss(p->n_users, m->u_ptr, m->u_col, m->U, m->V, p->dim, m->item_gramian, p->w, 1,
                   m->user_loss, p->nthreads);
  if (p->model == 3) {
    float prev = oracle_mean(m->user_loss, p->n_users);
    m->prev_xi = model_xi(m, prev);
  }
  for (int64_t u = 0; u < p->n_users; ++u) m->hsize[u] = (float)(m->u_ptr[u + 1] - m->u_ptr[u]);
  for (int64_t v = 0; v < p->n_items; ++v) {
    for (int64_t k = m->i_ptr[v]; k < m->i_ptr[v + 1]; ++k)
      m->item_reg[v] = (float)((double)m->item_reg[v] + 1.0 / (double)m->hsize[m->i_col[k]]);
  }
}

/* StepV: safer2.h:493-555 (ERM erm_mf.h:452-513, CVaR cvar_mf.h:473-538). */
static int64_t model_step_v(oracle_model* m, const float* Ufor, int grad) {
  const oracle_model_params* p = &m->p;
  for (int64_t u = 0; u < p->n_users; ++u) m->nu[u] = m->dual_weight[u] / m->hsize[u];
  oracle_gramian(Ufor, p->n_users, p->dim, m->dual_weight, m->G2, p->nthreads);
  oracle_solve_params sp = {grad ? 4 : 2, p->reg,  p->reg_exp,  p->w,   p->alpha,
                            p->stepsize,  p->quirk, NULL,       m->item_reg, m->nu};
  return oracle_step(p->n_items, m->i_ptr, m->i_col, Ufor, p->n_users, p->dim, m->G2, &sp, m->V,
                     m->V, p->nthreads);
}

int64_t oracle_model_train(oracle_model* m) {
  const oracle_model_params* p = &m->p;
  const int d = p->dim;
  int64_t rc = 0;
  if (p->model == 0) { /* IALSRecommender::Train, ials.h:187-224 */
    oracle_solve_params sp = {0, p->reg, p->reg_exp, p->w, p->alpha, p->stepsize, 0, NULL, NULL, NULL};
    oracle_gramian(m->V, p->n_items, d, NULL, m->G2, p->nthreads);
    rc = oracle_step(p->n_users, m->u_ptr, m->u_col, m->V, p->n_items, d, m->G2, &sp, NULL, m->U,
                     p->nthreads);
    if (rc) return rc;
    oracle_gramian(m->U, p->n_users, d, NULL, m->G2, p->nthreads);
    rc = oracle_step(p->n_items, m->i_ptr, m->i_col, m->U, p->n_users, d, m->G2, &sp, NULL, m->V,
                     p->nthreads);
    if (rc) return -rc;
    oracle_gramian(m->V, p->n_items, d, NULL, m->item_gramian, p->nthreads); /* :371 */
    oracle_user_loss(p->n_users, m->u_ptr, m->u_col, m->U, m->V, d, m->item_gramian, p->w, 0,
                     m->user_loss, p->nthreads);
    return 0;
  }
  if (p->model == 2) { /* CVaRMFRecommender::Train, cvar_mf.h:276-330 */
    for (int64_t u = 0; u < p->n_users; ++u)
      if (m->u_ptr[u + 1] > m->u_ptr[u])
        m->dual_weight[u] = (float)((m->user_loss[u] - m->prev_xi) >= 0); /* :623 */
    memcpy(m->Uprev, m->U, sizeof(float) * p->n_users * d);
    oracle_solve_params sp = {3, p->reg, p->reg_exp, p->w, p->alpha, p->stepsize, p->quirk,
                              m->dual_weight, NULL, NULL};
    oracle_step(p->n_users, m->u_ptr, m->u_col, m->V, p->n_items, d, m->item_gramian, &sp, m->U,
                m->U, p->nthreads);
    model_step_v(m, m->Uprev, 1);
    oracle_gramian(m->V, p->n_items, d, NULL, m->item_gramian, p->nthreads);
    oracle_user_loss(p->n_users, m->u_ptr, m->u_col, m->U, m->V, d, m->item_gramian, p->w, 1,
                     m->user_loss, p->nthreads);
    m->prev_xi = oracle_cvar_xi(m->user_loss, p->n_users, p->alpha);
    return 0;
  }
  /* ERM-MF (erm_mf.h:257-301) and SAFER2 (safer2.h:266-334). */
  const int iters = p->model == 3 ? p->pd_iterations : 1;
  for (int t = 0; t < iters; ++t) {
    if (p->model == 3) {
      for (int64_t u = 0; u < p->n_users; ++u)
        if (m->u_ptr[u + 1] > m->u_ptr[u])
          m->dual_weight[u] =
              oracle_safer2_weight(m->user_loss[u], m->prev_xi, p->bandwidth, p->use_epanechnikov);
    }
    oracle_solve_params sp = {1, p->reg, p->reg_exp, p->w, p->alpha, p->stepsize, p->quirk,
                              m->dual_weight, NULL, NULL};
    rc = oracle_step(p->n_users, m->u_ptr, m->u_col, m->V, p->n_items, d, m->item_gramian, &sp,
                     NULL, m->U, p->nthreads);
    if (rc) return rc;
    rc = model_step_v(m, m->U, 0);
    if (rc) return -rc;
    oracle_gramian(m->V, p->n_items, d, NULL, m->item_gramian, p->nthreads);
    oracle_user_loss(p->n_users, m->u_ptr, m->u_col, m->U, m->V, d, m->item_gramian, p->w, 1,
                     m->user_loss, p->nthreads);
  }
  if (p->model == 3) m->prev_xi = model_xi(m, m->prev_xi);
  return 0;
}

/* Fold-in: ials.h:148-185 (fresh V^T V), safer2.h:225-263 and
 * erm_mf.h:214-255 (StepU, weight 1, cached gramian), cvar_mf.h:233-274
 * (StepU_eval: LLT solve, weight 1). */
int64_t oracle_model_fold_in(const oracle_model* m, int64_t n_eval, const int64_t* ptr,
                             const int32_t* col, float* Ueval) {
  const oracle_model_params* p = &m->p;
  const int d = p->dim;
  memset(Ueval, 0, sizeof(float) * n_eval * d);
  if (p->model == 0) {
    float* G = (float*)malloc(sizeof(float) * d * d);
    oracle_gramian(m->V, p->n_items, d, NULL, G, p->nthreads);
    oracle_solve_params sp = {0, p->reg, p->reg_exp, p->w, p->alpha, p->stepsize, 0, NULL, NULL, NULL};
    int64_t rc = oracle_step(n_eval, ptr, col, m->V, p->n_items, d, G, &sp, NULL, Ueval, p->nthreads);
    free(G);
    return rc;
  }
  oracle_solve_params sp = {1, p->reg, p->reg_exp, p->w, p->alpha, p->stepsize, 0, NULL, NULL, NULL};
  return oracle_step(n_eval, ptr, col, m->V, p->n_items, d, m->item_gramian, &sp, NULL, Ueval,
                     p->nthreads);
}

/* ------------------------------------------------------------------ */
/* EvaluateUser, recommender.h:132-199.                                */
/* ------------------------------------------------------------------ */
typedef struct {
  const float *Ueval, *V;
  int64_t n_items;
  int dim;
  const int64_t *ex_ptr, *gt_ptr;
  const int32_t *ex_col, *gt_col;
  const int* k_list;
  int nk;
  float *recall, *ndcg;
} eval_ctx;

typedef struct {
  float s;
  int32_t i;
} scored;

static int cmp_scored_desc(const void* a, const void* b) {
  const scored *x = (const scored*)a, *y = (const scored*)b;
  if (x->s > y->s) return -1;
  if (x->s < y->s) return 1;
  return (x->i > y->i) - (x->i < y->i);
}

static void eval_row(void* vctx, int64_t r, float* s) {
  (void)s;
  eval_ctx* c = (eval_ctx*)vctx;
  const int d = c->dim;
  const int64_t ni = c->n_items;
  scored* sc = (scored*)malloc(sizeof(scored) * ni);
  const float* u = c->Ueval + (size_t)r * d;
  for (int64_t i = 0; i < ni; ++i) {
    const float* v = c->V + (size_t)i * d;
    float t = 0.f;
    for (int k = 0; k < d; ++k) t += v[k] * u[k];
    sc[i].s = t;
    sc[i].i = (int32_t)i;
  }
  for (int64_t k = c->ex_ptr[r]; k < c->ex_ptr[r + 1]; ++k) sc[c->ex_col[k]].s = -FLT_MAX;
  int maxk = 0;
  for (int k = 0; k < c->nk; ++k)
    if (c->k_list[k] > maxk) maxk = c->k_list[k];
  qsort(sc, ni, sizeof(scored), cmp_scored_desc);
  const int64_t g0 = c->gt_ptr[r], g1 = c->gt_ptr[r + 1];
  /* gt set membership via a mark array */
  unsigned char* mark = (unsigned char*)calloc(ni, 1);
  int64_t ngt = 0;
  for (int64_t k = g0; k < g1; ++k)
    if (!mark[c->gt_col[k]]) {
      mark[c->gt_col[k]] = 1;
      ++ngt;
    }
  for (int q = 0; q < c->nk; ++q) {
    const int k = c->k_list[q];
    double hits = 0.0, dcg = 0.0, norm = 0.0;
    for (int i = 0; i < k && i < ni; ++i)
      if (mark[sc[i].i]) {
        hits += 1.0;
        dcg += 1.0 / log2(i + 2.0);
      }
    const int m = (int)(k < ngt ? k : ngt);
    for (int i = 0; i < m; ++i) norm += 1.0 / log2(i + 2.0);
    const float mn = (float)k < (float)ngt ? (float)k : (float)ngt;
    c->recall[r * c->nk + q] = (float)(hits / mn);
    c->ndcg[r * c->nk + q] = (float)(dcg / norm);
  }
  free(mark);
  free(sc);
}

void oracle_evaluate(int64_t n_eval, const float* Ueval, const float* V, int64_t n_items, int dim,
                     const int64_t* ex_ptr, const int32_t* ex_col, const int64_t* gt_ptr,
                     const int32_t* gt_col, const int* k_list, int nk, float* recall, float* ndcg,
                     int nthreads) {
  eval_ctx c = {Ueval, V, n_items, dim, ex_ptr, gt_ptr, ex_col, gt_col, k_list, nk, recall, ndcg};
  run_pool(eval_row, &c, n_eval, nthreads, 0);
}
