/*
 * frecsys_oracle.h -- CPU restatement of the reference's closed-form solve
 * loop (riktor/safer2-recommender, "frecsys").
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (the HIP library, the
 * frecsys:: C++ headers, run_model) links, loads or calls this code.  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it, and
 * only as the checker / the timed CPU baseline ("kind": "port").
 *
 * Parity status (see DESIGN.md "Oracle"): the reference cannot be built in
 * this image (Eigen 3.4.0 / glog / fmt / gtest absent, bazel absent, no
 * network), and it ships no golden vectors.  Element-wise parity against the
 * reference binary is therefore UNPINNED.  The restatement is pinned by
 *   (1) the reference's own known-answer tests on its own fixture
 *       (tests/ml-1m): NDCG@20 >= 0.2 after training (ials_test.cc:45,
 *       erm_mf_test.cc:45, cvar_mf_test.cc:46, safer2_test.cc:99) and the
 *       SAFER2 mean dual weight alpha +- 0.02 (safer2_test.cc:135);
 *   (2) an independent float64 numpy restatement (tests/test_oracle.py);
 *   (3) libstdc++'s own std::mt19937 / std::normal_distribution<float>
 *       for the seeded initialisation (tests/test_oracle.py).
 *
 * Layout contract (same as the product's C-ABI): interactions are CSR per
 * side (int64 row_ptr[n+1], int32 col[nnz]) with each row's entries in file
 * order (dataset.h:83-92); embeddings are row-major float32 [n][dim]
 * (types.h:23-27).  Gramians are full dim x dim row-major.
 */
#ifndef FRECSYS_ORACLE_H_
#define FRECSYS_ORACLE_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- libstdc++ RNG restatement (recommender.h:61-67, ials.h:47-51) ---- */
typedef struct {
  uint32_t mt[624];
  int idx;
} oracle_mt19937;

void oracle_mt_seed(oracle_mt19937* g, uint32_t seed);
uint32_t oracle_mt_next(oracle_mt19937* g);

/* Fill U (nu x dim) then V (ni x dim) exactly like the model ctors:
 * one mt19937 seeded with `seed`, a fresh normal_distribution<float>(0, s)
 * per matrix, s = stdev / sqrt(dim).  (ials.h:47-51, safer2.h:50-54) */
void oracle_init_embeddings(uint32_t seed, float stdev, int dim, float* U,
                            int64_t nu, float* V, int64_t ni);

/* ---- Gramian (ials.h:321; safer2.h:55, 294-295, 504-509) ----
 * G = X^T diag(w) X over rows [0, n); w == NULL means unweighted. */
void oracle_gramian(const float* X, int64_t n, int dim, const float* w,
                    float* G, int nthreads);

/* ---- per-entity projections; return 0, or -1 if not SPD ---- */
/* iALS Project (ials.h:88-144) */
int oracle_project_ials(const int32_t* hist, int64_t h, const float* X,
                        int dim, const float* G, float reg, float w,
                        float* out);
/* ERM-MF / SAFER2 ProjectU, CVaR-MF ProjectU_eval
 * (safer2.h:104-163, erm_mf.h:91-151, cvar_mf.h:182-229) */
int oracle_project_u(const int32_t* hist, int64_t h, const float* X,
                     int dim, const float* G, float reg, float w,
                     float weight, float* out);
/* ERM-MF / SAFER2 ProjectV with the tail quirk (safer2.h:166-221,
 * erm_mf.h:153-210); nu[] indexed by the other-side id. */
int oracle_project_v(const int32_t* hist, int64_t h, const float* X,
                     int dim, const float* G, float reg, float w,
                     const float* nu, int quirk, float* out);
/* CVaR-MF gradient steps (cvar_mf.h:88-134, 136-180) */
void oracle_cvar_project_u(const int32_t* hist, int64_t h, const float* e,
                           const float* X, int dim, const float* G,
                           float reg, float w, float stepsize, float weight,
                           float* out);
void oracle_cvar_project_v(const int32_t* hist, int64_t h, const float* e,
                           const float* X, int dim, const float* G,
                           float reg, float w, const float* nu, float stepsize,
                           int quirk, float* out);

/* ---- side-level steps (ials.h:317-365 and model Step* drivers) ----
 * kind: 0 IALS, 1 WEIGHTED_U, 2 WEIGHTED_V, 3 CVAR_GRAD_U, 4 CVAR_GRAD_V.
 * Rows with no history are left untouched (they are not in the reference's
 * by_user / by_item maps).  Out may alias the current embeddings E for the
 * CVaR kinds only through the `E` argument (E is read, Out written).
 * entity_weight: omega per solved row (NULL -> 1);  entity_reg: per-row
 * base term item_reg_[v];  other_weight: nu per other-side row.
 * Returns 0 or (1 + row) of the first non-SPD row. */
typedef struct {
  int kind;
  float reg, reg_exp, w, alpha, stepsize;
  int quirk;
  const float* entity_weight;
  const float* entity_reg;
  const float* other_weight;
} oracle_solve_params;

int64_t oracle_step(int64_t n_rows, const int64_t* row_ptr,
                    const int32_t* col, const float* X, int64_t n_other,
                    int dim, const float* G, const oracle_solve_params* p,
                    const float* E, float* Out, int nthreads);

/* ---- user loss (ials.h:70-86 with half=0; safer2.h:85-101 half=1) ----
 * Rows with no history get loss 0 (never written in the reference). */
/* iALS++ (ialspp.h): PredictDataset (pred[rix[k]] = X[col[k]] . E[row]) and one
 * block Step + ProjectBlock of a side on columns [start, end); E updated in
 * place, pred updated with each row's delta.  Returns first failing row + 1. */
void oracle_pp_predict(int64_t n_rows, const int64_t* row_ptr, const int32_t* col,
                       const int32_t* rix, const float* X, int dim, const float* E, float* pred,
                       int nthreads);
/* p->kind: 0 iALS++ ProjectBlock, 1 SAFER2++ ProjectU (entity_weight),
 * 2 SAFER2++ ProjectV (entity_reg, other_weight = nu); gram_w weights the
 * local Gramians (SAFER2++ V step: the dual weights) or NULL. */
int64_t oracle_pp_step(int64_t n_rows, const int64_t* row_ptr, const int32_t* col,
                       const int32_t* rix, const float* X, int64_t n_other, int dim, float* E,
                       float* pred, int start, int end, const oracle_solve_params* p,
                       const float* gram_w, double* residual, int nthreads);
void oracle_user_loss(int64_t n_users, const int64_t* row_ptr,
                      const int32_t* col, const float* U, const float* V,
                      int dim, const float* G, float beta, int half,
                      float* out, int nthreads);

/* ---- SAFER2 dual / quantile machinery (safer2.h:598-794) ---- */
float oracle_safer2_weight(float loss, float xi, float bandwidth, int epan);
float oracle_safer2_xi(const float* loss, int64_t n, float prev_xi,
                       int iterations, float alpha, float bandwidth, int epan);
/* use_snr: N*sampling_ratio indices per iteration from *g (see .c). */
float oracle_safer2_xi_snr(const float* loss, int64_t n, float prev_xi, int iterations,
                           float alpha, float bandwidth, int epan, float sampling_ratio,
                           oracle_mt19937* g);
/* libstdc++ uniform_int_distribution<int>(0, range-1) over mt19937. */
uint32_t oracle_uniform_int(oracle_mt19937* g, uint32_t range);
/* Eigen VectorXf::mean() restated (AVX-512 packet redux). */
float oracle_mean(const float* x, int64_t n);
/* CVaR-MF exact quantile (cvar_mf.h:582-595) */
float oracle_cvar_xi(const float* loss, int64_t n, float alpha);

/* ---- whole models (Train() sequences) ----
 * model: 0 ials, 1 erm_mf, 2 cvar_mf, 3 safer2. */
typedef struct oracle_model oracle_model;
typedef struct {
  int model;
  int dim;
  int64_t n_users, n_items;
  float reg, reg_exp, w, stdev, alpha, bandwidth, stepsize;
  int xi_iterations, pd_iterations, use_epanechnikov;
  int quirk;
  int nthreads;
  int use_snr;          /* SAFER2 sub-sampled Newton (safer2.h:724-737) */
  float sampling_ratio;
} oracle_model_params;

oracle_model* oracle_model_create(const oracle_model_params* p,
                                  uint32_t seed);
void oracle_model_destroy(oracle_model* m);
/* Attach the training data (both orientations). Kept by pointer. */
void oracle_model_set_data(oracle_model* m, const int64_t* u_ptr,
                           const int32_t* u_col, const int64_t* i_ptr,
                           const int32_t* i_col);
void oracle_model_set_embeddings(oracle_model* m, const float* U,
                                 const float* V);
void oracle_model_get_embeddings(const oracle_model* m, float* U, float* V);
/* Initialize() of erm_mf / cvar_mf / safer2; no-op for ials. */
void oracle_model_initialize(oracle_model* m);
int64_t oracle_model_train(oracle_model* m);
/* state readers: user_loss (n_users), dual_weight (n_users), xi */
void oracle_model_get_state(const oracle_model* m, float* user_loss,
                            float* dual_weight, float* xi);
/* Fold-in (EvaluateDataset's Step) over an eval CSR of n_eval rows;
 * writes n_eval x dim. */
int64_t oracle_model_fold_in(const oracle_model* m, int64_t n_eval,
                             const int64_t* ptr, const int32_t* col,
                             float* Ueval);

/* ---- top-K evaluation (recommender.h:132-199) ----
 * For each eval row r: scores = V u_r, history excluded; writes
 * recall[r*nk+k], ndcg[r*nk+k]. */
void oracle_evaluate(int64_t n_eval, const float* Ueval, const float* V,
                     int64_t n_items, int dim, const int64_t* ex_ptr,
                     const int32_t* ex_col, const int64_t* gt_ptr,
                     const int32_t* gt_col, const int* k_list, int nk,
                     float* recall, float* ndcg, int nthreads);

#ifdef __cplusplus
}
#endif
#endif
