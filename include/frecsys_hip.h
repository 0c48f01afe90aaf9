/*
 * frecsys_hip.h -- C-ABI of libfrecsys_hip.so, the MI355X (gfx950) solve
 * loop behind iALS / ERM-MF / CVaR-MF / SAFER2.
 *
 * Plain C types only (no torch / HIP / RCCL types).  Every call is
 * synchronous on return (the reference's Step* functions block until all
 * threads join, ials.h:359-361) and returns FRECSYS_OK (0) or an error code;
 * frecsys_last_error() gives the message.  The library owns every device
 * buffer (embeddings, Gramians, CSR, workspaces); they stay resident in HBM
 * across epochs.  Host pointers passed in are never retained after a call.
 *
 * Which reference interface each entry point replaces (reference paths are
 * relative to riktor/safer2-recommender):
 *
 *   frecsys_ctx_create / destroy  -- the model ctor's allocation of
 *       user_embedding_ / item_embedding_ / item_gramian_
 *       (ials.h:39-45, safer2.h:37-48, erm_mf.h:36-44, cvar_mf.h:36-43)
 *   frecsys_load_csr              -- Dataset::by_user()/by_item()
 *       (dataset.h:27-32, 83-92): the per-entity SpVector histories, as CSR
 *       rows kept in file order
 *   frecsys_set/get_embeddings    -- init_matrix writes (recommender.h:61-67)
 *       and item_embedding() reads (ials.h:410-412)
 *   frecsys_init_embeddings       -- std::mt19937 + normal_distribution<float>
 *       init of U then V (ials.h:47-51, recommender.h:61-67), seeded
 *   frecsys_gramian               -- `X.transpose() * X` (ials.h:321,
 *       ials.h:371, safer2.h:55, safer2.h:294-295) and the weighted
 *       `U^T (U .* omega)` (safer2.h:504-509, erm_mf.h:462-467,
 *       cvar_mf.h:484-489)
 *   frecsys_solve_side            -- Step / StepU / StepV / StepU_eval with
 *       their static per-entity Project / ProjectU / ProjectV /
 *       ProjectU_eval (ials.h:88-144 + 317-365; safer2.h:104-221 + 437-555;
 *       erm_mf.h:91-210 + 397-513; cvar_mf.h:88-229 + 427-538 + 645-692)
 *   frecsys_user_loss             -- ComputeUserLoss / ComputeLoss
 *       (ials.h:70-86 + 367-408; safer2.h:85-101 + 558-596)
 *   frecsys_comm_* / frecsys_partition -- new: the reference has no
 *       multi-device path; these shard the entity loop of the Step* drivers
 *       (safer2.h:447-487) across one process per GPU (RCCL over xGMI).
 */
#ifndef FRECSYS_HIP_H_
#define FRECSYS_HIP_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ---- */
#define FRECSYS_OK 0
#define FRECSYS_ERR_INVALID 1     /* bad argument / state */
#define FRECSYS_ERR_HIP 2         /* HIP runtime error */
#define FRECSYS_ERR_RCCL 3        /* RCCL error */
#define FRECSYS_ERR_NOT_SPD 4     /* LLT failed (reference: assert, ials.h:141);
                                     entity id via frecsys_last_error_entity */
#define FRECSYS_ERR_NAN 5         /* NaN detected (reference: LOG(ERROR) + exit) */
#define FRECSYS_ERR_UNSUPPORTED 6 /* e.g. dim beyond the kernels built */
#define FRECSYS_ERR_NO_DEVICE 7   /* no HIP device visible */

/* ---- sides ---- */
#define FRECSYS_SIDE_USER 0 /* train by_user: rows = users, cols = items */
#define FRECSYS_SIDE_ITEM 1 /* train by_item: rows = items, cols = users */
#define FRECSYS_SIDE_EVAL 2 /* fold-in users (EvaluateDataset, ials.h:148-174);
                               rows = compacted eval users, cols = items */

/* ---- per-entity solve kinds ---- */
#define FRECSYS_KIND_IALS 0        /* ials.h:88-144 */
#define FRECSYS_KIND_WEIGHTED_U 1  /* safer2.h:104-163, erm_mf.h:91-151,
                                      cvar_mf.h:182-229 (ProjectU_eval) */
#define FRECSYS_KIND_WEIGHTED_V 2  /* safer2.h:166-221, erm_mf.h:153-210 */
#define FRECSYS_KIND_CVAR_GRAD_U 3 /* cvar_mf.h:88-134 */
#define FRECSYS_KIND_CVAR_GRAD_V 4 /* cvar_mf.h:136-180 */

typedef struct frecsys_ctx frecsys_ctx;

typedef struct {
  int32_t dim;           /* embedding dimension (reference --dim) */
  int32_t device;        /* HIP device ordinal; -1 = current device */
  int32_t parity_quirks; /* 1: reproduce reference quirks */
  int32_t reserved;
  int64_t n_users;       /* max_user + 1 (run_model.cc:240) */
  int64_t n_items;       /* max_item + 1 */
} frecsys_config;

typedef struct {
  int32_t kind;            /* FRECSYS_KIND_* */
  float reg;               /* l2_reg */
  float reg_exp;           /* l2_reg_exp (iALS only, ials.h:312-314) */
  float unobserved_weight; /* uobs_weight */
  float alpha;             /* alpha (ItemRegularizationValue, safer2.h:430) */
  float stepsize;          /* CVaR-MF eta (cvar_mf.h:133) */
  int32_t from_snapshot;   /* 1: X = snapshot of the other side (CVaR StepV
                              uses the pre-step U, cvar_mf.h:282,294) */
  int32_t lambda_is_reg;   /* 1: use `reg` itself as every entity's lambda
                              (the static Project* API receives the final
                              lambda, ials.h:88-90) */
  const float* entity_weight; /* host [rows of side]: omega_u (WEIGHTED_U,
                                 CVAR_GRAD_U); NULL -> 1 */
  const float* entity_reg;    /* host [rows of side]: item_reg_[v]
                                 (WEIGHTED_V, CVAR_GRAD_V) */
  const float* other_weight;  /* host [rows of other side]: nu_u =
                                 omega_u / |H_u| (WEIGHTED_V, CVAR_GRAD_V) */
} frecsys_solve_params;

/* ---- context ---- */
int frecsys_device_count(int32_t* n);
int frecsys_ctx_create(const frecsys_config* cfg, frecsys_ctx** out);
void frecsys_ctx_destroy(frecsys_ctx* ctx);
/* Message of the last error on ctx (ctx may be NULL: last global error). */
const char* frecsys_last_error(const frecsys_ctx* ctx);
/* Entity (row of the side) of the last FRECSYS_ERR_NOT_SPD, or -1. */
int64_t frecsys_last_error_entity(const frecsys_ctx* ctx);
/* Padded leading dimension used on device (dim rounded up). */
int32_t frecsys_padded_dim(int32_t dim);

/* ---- multi-GPU (one process per GPU) ---- */
/* Host-only: contiguous nnz-balanced split of rows into nparts ranges,
 * bounds[0]=0 .. bounds[nparts]=n_rows (safe to call without a GPU). */
int frecsys_partition(int64_t n_rows, const int64_t* row_ptr, int32_t nparts,
                      int64_t* bounds);
/* Host-only: the partition-independent Gramian plan of n_rows rows at
 * `dim` (frecsys_gramian): rows per leaf, leaves, groups (group g = leaves
 * [g*n_leaves/n_groups, (g+1)*n_leaves/n_groups)) and the groups
 * [own_lo, own_hi) rank `rank` of `world` computes.  Any output may be NULL. */
int frecsys_gram_plan(int32_t dim, int64_t n_rows, int32_t world, int32_t rank,
                      int64_t* rows_per_leaf, int64_t* n_leaves, int32_t* n_groups,
                      int32_t* own_lo, int32_t* own_hi);
/* RCCL unique id (128 bytes) -- call on rank 0, broadcast to the others. */
int frecsys_comm_unique_id(uint8_t id[128]);
/* Join rank `rank` of `world`.  id != NULL: RCCL communicator; the library
 * all-reduces the Gramians and all-gathers factor rows / losses itself.
 * id == NULL (world > 1): external exchange -- no communicator; every call
 * works on this rank's shard only (frecsys_gramian returns the partial Gramian
 * over the rank's rows, solve_side / user_loss write only its rows) and the
 * caller performs the exchange (frecsys_set_gramian, set_embeddings), e.g.
 * over its own MPI / gloo transport or, in tests, several contexts of one
 * process sharing a device. */
int frecsys_comm_init(frecsys_ctx* ctx, int32_t world, int32_t rank,
                      const uint8_t id[128]);
/* World size and rank the context joined, and the rank count of its RCCL
 * communicator (ncclCommCount; 0 without one). */
int frecsys_comm_world(const frecsys_ctx* ctx, int32_t* world, int32_t* rank,
                       int32_t* comm_ranks);
/* Row range [lo, hi) of `side` owned by this rank (after load_csr). */
int frecsys_shard_range(const frecsys_ctx* ctx, int32_t side, int64_t* lo,
                        int64_t* hi);

/* ---- data ---- */
int frecsys_load_csr(frecsys_ctx* ctx, int32_t side, int64_t n_rows,
                     const int64_t* row_ptr, const int32_t* col);
int frecsys_set_embeddings(frecsys_ctx* ctx, int32_t side, const float* host,
                           int64_t ld);
int frecsys_get_embeddings(frecsys_ctx* ctx, int32_t side, float* host,
                           int64_t ld);
/* Seeded init of U then V, identical to std::mt19937{seed} +
 * std::normal_distribution<float>(0, stdev/sqrt(dim)) per matrix. */
int frecsys_init_embeddings(frecsys_ctx* ctx, uint32_t seed, float stdev);
/* Copy the current embeddings of side into its snapshot slot. */
int frecsys_snapshot(frecsys_ctx* ctx, int32_t side);

/* ---- compute ---- */
/* G[side] = X^T diag(w) X over all rows of side's embeddings (or of its
 * snapshot).  Partition-independent: the rows are cut into fixed leaves and
 * the leaves into n_groups fixed groups (frecsys_gram_groups; the cut depends
 * only on the row count); each rank computes the slabs of its own groups,
 * the slabs are all-gathered over RCCL and every rank sums them in group
 * order, so G is bitwise the same at every world size.  Without a
 * communicator at world > 1 (external exchange) G is the sum of this rank's
 * groups only; the caller exchanges the group slabs (frecsys_get_gram_groups
 * / frecsys_set_gram_groups) or partial Gramians (frecsys_set_gramian).
 * weights: host [rows of side] or NULL.  host_out (dim x dim, row-major) may
 * be NULL. */
int frecsys_gramian(frecsys_ctx* ctx, int32_t side, const float* weights,
                    int32_t from_snapshot, float* host_out);
/* Read G[side] as the context holds it (dim x dim, leading dim ld). */
int frecsys_get_gramian(frecsys_ctx* ctx, int32_t side, float* host, int64_t ld);
/* The Gramian plan of `side`: group count, the groups [own_lo, own_hi) this
 * rank computes, floats per group slab (any pointer may be NULL). */
int frecsys_gram_groups(const frecsys_ctx* ctx, int32_t side, int32_t* n_groups,
                        int32_t* own_lo, int32_t* own_hi, int64_t* floats_per_group);
/* All group slabs of the last Gramian of `side` formed here (host
 * [n_groups * floats_per_group]; at world > 1 without a communicator, the
 * other ranks' slabs are zero). */
int frecsys_get_gram_groups(frecsys_ctx* ctx, int32_t side, float* host);
/* G[side] = the group-order sum of the given slabs (every group's slab, as
 * gathered from the owners): the external-exchange completion of
 * frecsys_gramian. */
int frecsys_set_gram_groups(frecsys_ctx* ctx, int32_t side, const float* host);
/* Overwrite G[side] with a host dim x dim matrix (row-major, leading dim
 * ld) -- the static Project* entry points take an arbitrary Gramian. */
int frecsys_set_gramian(frecsys_ctx* ctx, int32_t side, const float* host,
                        int64_t ld);
/* Solve every row of `side` owned by this rank against the other side's
 * embeddings and G[other side]; rows with an empty history are left
 * untouched.  USER/ITEM results are then all-gathered across ranks.  EVAL
 * solves against ITEM and writes the EVAL embeddings. */
int frecsys_solve_side(frecsys_ctx* ctx, int32_t side,
                       const frecsys_solve_params* params);
/* Per-user loss over `side` (USER or EVAL) rows against ITEM embeddings and
 * G[ITEM]: (1/h) sum (x.u - 1)^2 + beta u^T G u, halved if half != 0.
 * Rows with empty history get 0.  host_out [rows] may be NULL (result kept
 * on device); for USER it is gathered across ranks first. */
int frecsys_user_loss(frecsys_ctx* ctx, int32_t side, float beta, int32_t half,
                      float* host_out);
/* ---- iALS++ subspace solver (ialspp.h) ----
 * Rating index of every CSR entry of side USER or ITEM (the tuple's position
 * in the training file: the second member of the by_user / by_item pairs),
 * [nnz of side]; allocates the prediction vector of the training tuples.
 * EVAL rows use their CSR position as rating index. */
int frecsys_pp_set_rating_index(frecsys_ctx* ctx, int32_t side, const int32_t* rix);
/* PredictDataset (ialspp.h:480-520) over the rows of side USER (training
 * prediction vector) or EVAL (fold-in prediction vector):
 * pred[rating index] = item . user. */
int frecsys_pp_predict(frecsys_ctx* ctx, int32_t side);
/* One block Step of every row of `side` (USER, ITEM or EVAL) on columns
 * [start, end), end - start <= 128, against the other side's embeddings and
 * G[other]: params->kind IALS = iALS++ Step + ProjectBlock
 * (ialspp.h:351-424, 85-145; reg, reg_exp, unobserved_weight),
 * WEIGHTED_U / WEIGHTED_V = SAFER2++ StepU + ProjectU / StepV + ProjectV
 * (safer2pp.h:449-653, 97-216; entity_weight / entity_reg + other_weight +
 * alpha as for frecsys_solve_side, G[other] the omega-weighted Gramian for
 * WEIGHTED_V).  Updates the block of the rows and their predictions.
 * At world > 1 (USER / ITEM) each rank solves its own shard of the rows
 * (frecsys_shard_range).  With an in-call exchange -- RCCL, or the caller's
 * transport (frecsys_set_transport): one code path, only the transport call
 * differs -- the rows are then all-gathered, every rank replays the other
 * ranks' prediction updates from them, takes the same NOT_SPD verdict (a
 * min over ranks) and sums every rank's per-row residuals in the
 * single-rank order, so the embeddings, the prediction vector and the
 * residual are bitwise the single-rank ones.  Every rank must make the same
 * sequence of calls.  Without either (external exchange, no transport) the
 * caller copies the other ranks' rows in (frecsys_set_embeddings) and calls
 * frecsys_pp_sync -- also after a step that returned FRECSYS_ERR_NOT_SPD,
 * whose updates were applied; until it does, a further frecsys_pp_step or
 * frecsys_pp_predict on the context fails with FRECSYS_ERR_INVALID
 * ("pp_sync pending").  A step that fails for another reason leaves nothing
 * pending; its rows are then undefined (rerun frecsys_pp_predict).
 * residual (may be NULL): sum of squared block deltas (over every rank's
 * rows with an in-call exchange, this rank's rows otherwise). */
int frecsys_pp_step(frecsys_ctx* ctx, int32_t side, int32_t start, int32_t end,
                    const frecsys_solve_params* params, double* residual);
/* External-exchange completion of a sharded frecsys_pp_step on `side`: after
 * the other ranks' rows were set, apply their block updates to this rank's
 * prediction vector.  No reference counterpart (the sharded path is new). */
int frecsys_pp_sync(frecsys_ctx* ctx, int32_t side);
/* The prediction vector of the training tuples (side USER) or of the EVAL
 * rows (side EVAL), [nnz of the side] floats, indexed by rating index. */
int frecsys_pp_get_predictions(frecsys_ctx* ctx, int32_t side, float* host);
/* Caller-provided transport for the exchanges a sharded call makes inside
 * itself when the context has no RCCL communicator (frecsys_comm_init with
 * id NULL): the same points in the same order as the RCCL calls (today:
 * frecsys_pp_step).  Each callback returns 0 on success; every rank calls
 * them in the same order.
 *   allgather_rows: `rows` is a host copy of a whole per-row table of `side`
 *     (n_rows x ld floats, row-major); on entry rows [lo, hi) hold this
 *     rank's values, on return every row must hold its owner rank's values
 *     (an all-gather with the uneven counts of frecsys_shard_range);
 *   allreduce_min_u64: *value becomes the minimum over the ranks.
 * t == NULL removes the transport.  No reference counterpart. */
typedef struct frecsys_transport {
  void* user;
  int (*allgather_rows)(void* user, int32_t side, float* rows, int64_t n_rows, int64_t ld,
                        int64_t lo, int64_t hi);
  int (*allreduce_min_u64)(void* user, uint64_t* value);
} frecsys_transport;
int frecsys_set_transport(frecsys_ctx* ctx, const frecsys_transport* t);
/* Fold-in evaluation ranking (replaces the scoring + top-K of
 * EvaluateDatasetInternal / EvaluateUser, recommender.h:78-199): for every
 * row r of the EVAL side, scores s = V u_r over all items (fp32), the items
 * of row r's own EVAL history set to lowest() (the reference's `exclude`,
 * its fold-in history), then the k best items by descending score, ties by
 * ascending item id (the reference leaves tie order unspecified), into
 * topk[r*k .. r*k+k) (host int32).  1 <= k <= 1024, k <= items. */
int frecsys_eval_topk(frecsys_ctx* ctx, int32_t k, int32_t* topk);
/* Train-loss diagnostics (ComputeLosses / PrintLosses, ials.h:226-305,
 * safer2.h:337-413), all rows of both sides on every rank: observed = sum
 * over every USER-side interaction of (v.u - 1)^2 (per-user fp32 sums,
 * total in double), unobserved = sum_ij (U^T U)_ij (V^T V)_ij (unweighted
 * Gramians, double), and the squared row norms of U and V (host [n_users]
 * and [n_items]).  Any output pointer may be NULL.  The Gramian slots used
 * by the solves are left untouched. */
int frecsys_train_stats(frecsys_ctx* ctx, double* observed, double* unobserved,
                        float* user_norm2, float* item_norm2);
/* Sum over every row of `side` of ||X_r - snapshot_r||^2 (double), against
 * the snapshot frecsys_snapshot took: the residual norms of
 * --print_residual_stats, squared (StepU's sum of squared row changes,
 * safer2.h:475-478 / erm_mf.h:434-437; StepV's (V - V_prev).norm(),
 * safer2.h:550-553 / erm_mf.h:508-511 / cvar_mf.h:533-536). */
int frecsys_snapshot_residual(frecsys_ctx* ctx, int32_t side, double* sq);
/* Cumulative event counters of the context (never reset):
 *   "hspace_reruns"   solves of a side rerun on the d-space path after a
 *                     history-space pivot failure (a silent slow path);
 *   "tagged_timeouts" device polls of the tagged-word exchange of the
 *                     tridiagonalisation that timed out (each one poisons
 *                     the basis and forces a rerun);
 *   "ws_shrinks"      wide workspaces (d = 257..1024) cut below their
 *                     budget by a failed device allocation: a halved batch,
 *                     fewer long-history slabs, or the register-staged SYRK
 *                     instead of the pre-split table -- results unchanged.
 * No reference counterpart (diagnostics of the MI355X path). */
int frecsys_counter(frecsys_ctx* ctx, const char* what, int64_t* value);
/* Block until all queued device work is done (all calls already do). */
int frecsys_synchronize(frecsys_ctx* ctx);
/* Free the wide-dim workspaces (batch workspace of A tiles, long-history
 * slabs, pre-split table, history-space wide bucket); the next solve sizes
 * them again within FRECSYS_WIDE_WS_MB and a quarter of the then free device
 * memory each.  For a caller that needs the device memory between phases
 * (evaluation, another model).  No reference counterpart: the reference's
 * per-thread Eigen temporaries are freed per entity. */
int frecsys_release_workspaces(frecsys_ctx* ctx);

/* ---- profiling hooks (bench.py) ----
 * Kernel time accumulated with HIP events recorded on the library's
 * streams around each launch of kernel class `what` ("solve_user",
 * "solve_item", "solve_eval", "gramian", "user_loss", "allgather",
 * "allreduce"; per solve also "<solve>.dspace" (d x d solve of the long
 * histories), "<solve>.split" (partial SYRKs of the longest of them),
 * "<solve>.basis" (tridiagonalisation of G + rotation of the other side),
 * "<solve>.hspace" (history-space solve), "<solve>.rotate")
 * since the last frecsys_timing_reset. */
int frecsys_timing(const frecsys_ctx* ctx, const char* what, double* total_ms,
                   int64_t* launches);
int frecsys_timing_reset(frecsys_ctx* ctx);
/* The algorithmic work the library launched under timer key `what` since
 * the last frecsys_timing_reset (SURVEY 8(d) definitions at the logical
 * dim d, per entity of h assembly rows): "<solve>.dspace" h d (d+1) +
 * d^3/3 + 2 d^2 flops (the SYRK of split entities is "<solve>.split"'s),
 * gather bytes h d 4 + h 4 + 8 + d 4; "<solve>.hspace" h^2 d + h^3/3 +
 * 4 h d flops, bytes 2 h d 4 + h 4 + 8 + 4 d 4; "gramian" 2 N d^2 flops over
 * the rows this rank formed, N d 4 bytes; "user_loss" 2 nnz d + 2 N d^2
 * flops, nnz d 4 + nnz 4 + (N+1) 8 + N 4 bytes.  `launches` counts the
 * timed calls, as frecsys_timing does.  Any output may be NULL. */
int frecsys_work(const frecsys_ctx* ctx, const char* what, double* flops, double* bytes,
                 int64_t* entities, int64_t* launches);
/* Longest assembly history (h_eff) the history-space path takes on this
 * context (0: that path is off); longer histories run the d-space solve. */
int32_t frecsys_history_space_max_h(const frecsys_ctx* ctx);
/* The same for one solved side (FRECSYS_SIDE_USER / _ITEM: the rows solved by
 * frecsys_solve_side(side)); the sides differ where a default or
 * FRECSYS_DUAL_MAX_H_USER / _ITEM sets them apart (Dp = 512: users 320,
 * items 256).  0 for another side or with the path off. */
int32_t frecsys_history_space_max_h_side(const frecsys_ctx* ctx, int32_t side);

/* ---- diagnostics (tests) ----
 * The basis the history-space solve uses for G[side]: G = Q T Q^T with Q
 * orthogonal (Dp x Dp, row-major) and T tridiagonal (diag[Dp],
 * sub[Dp]: T(k+1, k), sub[Dp-1] = 0); Dp = frecsys_padded_dim(dim).  No
 * reference counterpart. */
int frecsys_debug_basis(frecsys_ctx* ctx, int32_t side, float* q, float* diag, float* sub);
/* The two diagonal-block factorisations of the blocked Cholesky (the
 * 32x32 pivot blocks of every solve): for each of n_tiles row-major 32x32
 * SPD tiles a[t], linv[t] = L^-1 with L L^T = a[t] (lower; upper part 0),
 * by the MFMA-blocked factor (blocked != 0) or the lane recurrence;
 * ok[t] = 0 on a non-positive pivot.  No reference counterpart (Eigen's
 * LLT inner kernel, ials.h:140). */
int frecsys_debug_diag_factor(frecsys_ctx* ctx, int32_t blocked, int32_t n_tiles, const float* a,
                              float* linv, int32_t* ok);

#ifdef __cplusplus
}
#endif
#endif /* FRECSYS_HIP_H_ */
