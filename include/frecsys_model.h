/*
 * frecsys_model.h -- C-ABI of libfrecsys_model.so: the reference's model
 * surface (the abstract frecsys::Recommender, recommender.h:40-59, and the
 * model constructors ials.h:39-42, ialspp.h, safer2.h:37-43, safer2pp.h,
 * erm_mf.h:37-40, cvar_mf.h:36-38) for callers that cannot link C++
 * (ctypes / cgo / JNI), driving the same C++ classes as run_model.
 *
 *   frecsys_model_create      -- run_model's Dataset(train) + get_model()
 *                                (run_model.cc:43-123, 233-241): the model is
 *                                sized max_user + 1 / max_item + 1 of the
 *                                tuples, seeded init of U then V
 *   frecsys_model_initialize  -- the Initialize(train) calls of
 *                                run_model.cc:246-257 (SAFER2, SAFER2++,
 *                                ERM-MF, CVaR-MF; no-op for iALS / iALS++)
 *   frecsys_model_train       -- `recommender->Train(train)` of the epoch
 *                                loop (run_model.cc:258-266), `epochs` times
 *   frecsys_model_context     -- the device context (include/frecsys_hip.h)
 *                                the model runs on: embeddings, timers
 *
 * Conditions the reference treats as fatal (a failed LLT, ials.h:141; NaN
 * losses, ials.h:291-296) end the process as they do there.  The tuples
 * passed to frecsys_model_create are copied; nothing is retained.
 */
#ifndef FRECSYS_MODEL_H_
#define FRECSYS_MODEL_H_

#include <stdint.h>

#include "frecsys_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct frecsys_model frecsys_model;

/* The run_model flags (run_model.cc:129-230), one field each. */
typedef struct {
  const char* model_name; /* ials | ialspp | safer2 | safer2pp | erm_mf | cvar_mf */
  int32_t dim;
  float l2_reg;
  float l2_reg_exp;
  float uobs_weight;
  float stdev;
  float alpha;
  float bandwidth;
  float stepsize;
  float sampling_ratio;
  int32_t block_size;
  int32_t xi_iterations;
  int32_t pd_iterations;
  int32_t use_epanechnikov;
  int32_t use_snr;
  int32_t print_train_stats;
  int32_t print_residual_stats;
  int32_t print_var_stats;
  int64_t seed;           /* -1: std::random_device, as the reference */
  int32_t device;         /* HIP ordinal; -1: LOCAL_RANK or the current device */
  int32_t parity_quirks;  /* SURVEY App. A.1 */
  int32_t world;          /* 0: WORLD_SIZE (1 if unset) */
  int32_t rank;           /* -1: RANK */
  const uint8_t* comm_id; /* world > 1: the 128-byte RCCL id of rank 0
                             (frecsys_comm_unique_id); NULL: FRECSYS_COMM_FILE */
} frecsys_model_config;

/* The run_model defaults (model_name NULL: must be set by the caller). */
void frecsys_model_config_default(frecsys_model_config* cfg);
/* users[k], items[k]: the k-th training tuple (file order). */
int frecsys_model_create(const frecsys_model_config* cfg, const int32_t* users,
                         const int32_t* items, int64_t n_tuples, frecsys_model** out);
int frecsys_model_initialize(frecsys_model* m);
int frecsys_model_train(frecsys_model* m, int32_t epochs);
frecsys_ctx* frecsys_model_context(frecsys_model* m);
/* GetMeanWeight() of SAFER2 / SAFER2++ (safer2.h:815-817); alpha for ERM-MF. */
float frecsys_model_mean_weight(const frecsys_model* m);
/* The dual state of ERM-MF / CVaR-MF / SAFER2 (-MF++): weights[n_users] =
 * the omega the last Train() (or Initialize()) left -- the weights its
 * half-steps used (safer2.h:272-290) --, losses[n_users] = user_loss_ of the
 * last ComputeUserLoss, item_reg[n_items] = item_reg_ (safer2.h:831-837),
 * xi = the current xi (SAFER2 / SAFER2++; NaN otherwise).  Any pointer may be
 * NULL; iALS has none of these (FRECSYS_ERR_INVALID for weights/item_reg). */
int frecsys_model_dual_state(const frecsys_model* m, float* weights, float* losses,
                             float* item_reg, float* xi);
void frecsys_model_destroy(frecsys_model* m);
const char* frecsys_model_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* FRECSYS_MODEL_H_ */
