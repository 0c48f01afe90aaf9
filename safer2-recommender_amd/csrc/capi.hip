// capi.hip -- host side of libfrecsys_hip.so: the C-ABI declared in
// include/frecsys_hip.h.  Owns the device state of one process (one GPU):
// embeddings (row-major, padded leading dim), Gramians, CSR of each side,
// workspaces, the RCCL communicator, and the HIP stream everything runs on.
//
// Sharding (one process per GPU): every rank keeps full replicas of U and V
// (they fit HBM at every configured size) and owns a contiguous nnz-balanced
// range of users and of items.  A half-step is
//   partial G over own rows -> ncclAllReduce -> solve own rows ->
//   grouped ncclBroadcast of every rank's rows (an all-gather with uneven
//   counts, in place).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <functional>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../../include/frecsys_hip.h"
#include "kernels.h"
#include "wide.h"

using namespace frecsys_hip;

namespace {

std::string g_last_error;
unsigned long long* g_dual_prof = nullptr;  // FRECSYS_DUAL_PROF diagnostics

struct Timer {
  double total_ms = 0.0;
  int64_t launches = 0;
};

// Algorithmic work the library launched under a timer key (SURVEY 8(d)
// definitions, logical dim d; frecsys_work), accumulated per launch.
struct Work {
  double flops = 0.0, bytes = 0.0;
  int64_t entities = 0, launches = 0;
};

}  // namespace

struct frecsys_ctx {
  int dim = 0, Dp = 0, device = 0, quirks = 1;
  int64_t n[3] = {0, 0, 0};
  hipStream_t stream = nullptr;
  float* emb[3] = {nullptr, nullptr, nullptr};
  float* snap[2] = {nullptr, nullptr};
  float* gram[2] = {nullptr, nullptr};
  int64_t* rp[3] = {nullptr, nullptr, nullptr};
  int32_t* col[3] = {nullptr, nullptr, nullptr};
  int64_t nnz[3] = {0, 0, 0};
  std::vector<int64_t> host_rp[2];
  std::vector<int64_t> bounds[2];
  // per-entity vectors (device)
  float* d_entity_weight = nullptr;
  size_t cap_entity_weight = 0;
  float* d_entity_reg = nullptr;
  size_t cap_entity_reg = 0;
  float* d_other_weight = nullptr;
  size_t cap_other_weight = 0;
  float* d_gram_w = nullptr;
  size_t cap_gram_w = 0;
  float* d_partials = nullptr;   // Gramian leaf workspace
  size_t cap_partials = 0;
  float* d_gslabs[3] = {nullptr, nullptr, nullptr};  // Gramian group slabs per side (2: train stats)
  size_t cap_gslabs[3] = {0, 0, 0};
  GramPlan gplan[2];             // plan of the last Gramian formed per side
  int gram_own[2][2] = {{0, 0}, {0, 0}};  // ... and the groups this rank computed
  float* d_loss = nullptr;
  size_t cap_loss = 0;
  float* d_quad = nullptr;
  size_t cap_quad = 0;
  unsigned long long* d_fail = nullptr;
  unsigned int* d_counter = nullptr;
  // cumulative event counters (frecsys_counter): [0] tagged-word polls that
  // timed out on the device (common.h tpoll); history-space reruns on host
  unsigned int* d_events = nullptr;
  int64_t hspace_reruns = 0;
  // per side: the rank's entities in decreasing-history order (LPT queue)
  QueueRec* d_order[3] = {nullptr, nullptr, nullptr};
  int64_t order_n[3] = {0, 0, 0};
  bool order_stale[3] = {true, true, true};
  std::vector<int64_t> host_rp_eval;
  ncclComm_t comm = nullptr;
  int world = 1, rank = 0;
  std::string err;
  int64_t err_entity = -1;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  std::map<std::string, Timer> timers;
  std::map<std::string, Work> work;
  std::map<float**, std::pair<float*, size_t>> pinned;  // upload() staging per destination
  // history-space (dual) path: a second stream for the concurrent d-space
  // solve of the long histories, the basis of each side's Gramian, the
  // rotated copy of each side, and the solved rows in the rotated basis
  hipStream_t stream2 = nullptr;
  hipStream_t stream3 = nullptr;  // second lane of history-space buckets
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  hipEvent_t ev_fork3 = nullptr, ev_join3 = nullptr;
  float* q[2] = {nullptr, nullptr};      // Dp x Dp
  float* tri[2] = {nullptr, nullptr};    // [2 * Dp]: diagonal, subdiagonal
  float* refl[2] = {nullptr, nullptr};   // Dp x Dp reflectors + [Dp] tau
  float* xrot[2] = {nullptr, nullptr};   // n_s x Dp
  void* qsplit[2][2] = {{nullptr, nullptr}, {nullptr, nullptr}};  // split images of Q, Q^T
  void* gsplit = nullptr;  // split image of G[ITEM] for the wide user loss
  float* out_rot[3] = {nullptr, nullptr, nullptr};
  size_t cap_xrot[2] = {0, 0};
  size_t cap_out_rot[3] = {0, 0, 0};
  float* dual_table = nullptr;  // [entities][3][Dp] LDL^T factors
  size_t cap_dual_table = 0;
  // wide dims (Dp = 512 / 1024): tridiagonalisation work, d-space workspace
  float* tri_work = nullptr;
  size_t cap_tri_work = 0;
  int32_t* d_rix[2] = {nullptr, nullptr};  // iALS++: rating index per CSR entry
  float* d_pred[2] = {nullptr, nullptr};   // iALS++: training / EVAL prediction vectors
  size_t cap_pred[2] = {0, 0};
  float* d_resid = nullptr;
  size_t cap_resid = 0;
  // sharded iALS++ / SAFER2++ block steps: the block columns of the side's
  // rows before the step ([n][bw]), for the prediction refresh of the rows
  // other ranks solve (frecsys_pp_step with RCCL; frecsys_pp_sync without)
  float* d_pp_old = nullptr;
  size_t cap_pp_old = 0;
  int pp_old_side = -1, pp_old_start = 0, pp_old_bw = 0;
  // external-exchange transport (frecsys_set_transport): the in-call
  // exchanges of a sharded call without a communicator
  frecsys_transport transport{};
  bool has_transport = false;
  std::vector<int32_t> pp_order_all[2];  // every row of the side by decreasing h (stable)
  float* d_resid_e = nullptr;            // per-entity residuals [n] of a sharded pp_step
  size_t cap_resid_e = 0;
  float* d_rows = nullptr;       // train stats: per-row values
  size_t cap_rows = 0;
  float* d_gstat = nullptr;      // train stats: U^T U, V^T V
  size_t cap_gstat = 0;
  double* d_dot = nullptr;
  size_t cap_dot = 0;
  float* d_scores = nullptr;     // evaluation: [batch][items] scores
  size_t cap_scores = 0;
  int32_t* d_topk = nullptr;     // [eval rows][k]
  size_t cap_topk = 0;
  float* wide_ws = nullptr;      // [wide batch][wide_slot_floats(Dp)]
  size_t cap_wide_ws = 0;
  // the pre-split copy of the other side for the wide d-space SYRK
  // (wide_syrk.hip; FRECSYS_WIDE_PRESPLIT=0: the register-staged SYRK)
  char* wide_xs = nullptr;
  size_t cap_wide_xs = 0;
  // the history-space wide bucket (dual.hip, 256 < h_eff <= 512): split Z
  // fragments, Cholesky slots of S, z
  char* dw_zs = nullptr;
  size_t cap_dw_zs = 0;
  float* dw_slots = nullptr;
  size_t cap_dw_slots = 0;
  float* dw_z = nullptr;
  size_t cap_dw_z = 0;
  bool wide_presplit = true;
  // FRECSYS_WIDE_WS_MB: the budget of EACH of the wide workspaces (the batch
  // workspace of A tiles, the long-history slabs, the history-space wide
  // bucket), each allocated only as large as its batch needs (8 GB instead of
  // 4 measured 0.6 % faster at MSD and config 5, 16 GB another 1.5 % at
  // config 5 -- fewer, fuller batches).  Each is also capped at a quarter of
  // the device memory free when it is sized (ws_budget), and a failed
  // allocation halves its batch instead of failing the call (ensure_batch);
  // the pre-split table of the other side ((n_other + 1) (6 Dp + 128) B:
  // 12.6 GB for config 5's 2M users) falls back to the register-staged SYRK
  // (bit-identical) when it does not fit.  At the default, the three
  // workspaces and the table take <= 61 GB of 288 at config 5.
  int64_t wide_ws_mb = 16384;
  bool ws_free_cap = true;   // FRECSYS_WS_FREE_CAP=0: no free-memory cap (tests of the OOM path)
  int64_t ws_shrinks = 0;    // allocations cut by a failed hipMalloc (frecsys_counter "ws_shrinks")
  // long-history split of the d-space solve
  int split_rows = 4096;         // rows per partial SYRK (FRECSYS_SPLIT_ROWS, 0 = off; swept 512..4096 at ML-20M d=256: 4096 best)
  std::vector<int2> h_split;
  std::vector<SplitWork> h_work;
  int2* d_split = nullptr;
  size_t cap_split = 0;
  SplitWork* d_work = nullptr;
  size_t cap_work = 0;
  float* d_slabs = nullptr;
  size_t cap_slabs = 0;
  std::vector<int32_t> order_h[3];       // history lengths in queue order
  std::vector<QueueRec> h_order[3];      // host copy of each side's queue (source of its upload)
  int dual_on = 1;
  // Content versions (every write of a side's embeddings or Gramian takes a
  // fresh number): a Gramian recomputed from unchanged embeddings is reused
  // (the computation is deterministic, the result would be identical), and
  // a basis / rotated copy is rebuilt only when its inputs changed.  When a
  // Gramian is formed for a side whose consumer last took the history-space
  // path, its basis is built right away on stream5 (e.g. during the user
  // loss and the host's xi / omega math between epochs) instead of on the
  // next solve's critical path.
  uint64_t ver_counter = 0;
  uint64_t emb_ver[3] = {0, 0, 0};
  uint64_t gram_ver[2] = {0, 0};
  uint64_t gram_src[2] = {0, 0};    // emb_ver the Gramian was formed from (0: not reusable)
  uint64_t basis_gram[2] = {0, 0};  // gram_ver the basis (T, Q, Q pieces) belongs to
  uint64_t xrot_emb[2] = {0, 0};    // emb_ver of the rotated copy (0: stale / snapshot)
  uint64_t xrot_gram[2] = {0, 0};   // ... and the basis it was rotated into
  uint64_t xrot_sub[2] = {0, 0};    // ... and the row subset it covers (0: every row)
  // Row subsets of the forward rotation: the rows of the other side that a
  // consumer side's history-space entities read (its shard's queue positions
  // [key0, key1)).  At N ranks a shard's short histories touch a fraction of
  // the other side, so the replicated rotation shrinks with N.  Built once
  // per (queue, split point) -- the histories do not change between epochs.
  QueueRec* d_hrows[3] = {nullptr, nullptr, nullptr};
  size_t cap_hrows[3] = {0, 0, 0};
  int64_t n_hrows[3] = {-1, -1, -1};  // rows in the subset; -1: none (every row)
  int64_t hrows_key[3][2] = {{-1, -1}, {-1, -1}, {-1, -1}};
  // Prefix sums over each side's queue of h_eff, h_eff^2, h_eff^3 and the
  // non-empty count (two variants: with / without the ProjectV tail rows):
  // the frecsys_work accounting of any queue range in O(1) instead of a host
  // loop over the entities on every solve.  Rebuilt with the queue.
  struct WorkPrefix {
    bool valid = false;
    std::vector<double> h1, h2, h3;
    std::vector<int64_t> nz;
  };
  WorkPrefix wprefix[3][2];
  uint64_t hrows_gen[3] = {0, 0, 0};  // subset id (0: every row)
  uint8_t* d_mark = nullptr;
  size_t cap_mark = 0;
  bool dual_used[3] = {false, false, false};  // the side's last solve took history space
  int eager_on = 1;                 // FRECSYS_EAGER=0: no early basis builds (A/B)
  // Basis kind per side: 0 = tridiagonal (G = Q T Q^T, any mu / lambda per
  // entity), 1 = Cholesky of the one M = mu*G + lam*I every entity of the
  // consumer's launch shares (q[] then holds L^-T, tri[][0] its status).
  // want_*: what the consumer's last history-space solve used (early builds).
  int basis_mode[2] = {0, 0};
  float basis_mu[2] = {0.f, 0.f}, basis_lam[2] = {0.f, 0.f};
  int want_mode[2] = {0, 0};
  float want_mu[2] = {0.f, 0.f}, want_lam[2] = {0.f, 0.f};
  int chol_basis_on = 1;            // FRECSYS_CHOL_BASIS=0: always tridiagonal (A/B, tests)
  float* chol_work = nullptr;
  size_t cap_chol_work = 0;
  hipStream_t stream5 = nullptr;  // early basis builds: an alias of stream3
  hipEvent_t ev_pre5 = nullptr;
  hipEvent_t ev_eager[2] = {nullptr, nullptr};
  bool eager_pending[2] = {false, false};
  int dual_max_h = 256;  // longest h_eff on the history-space path (set per Dp at create)
  int dual_max_h_side[3] = {256, 256, 256};  // per solved side (FRECSYS_DUAL_MAX_H_USER / _ITEM)
  int dual_serial = 0;  // FRECSYS_DUAL_SERIAL=1: no stream overlap (profiling)
  int debug_skip = 0;   // FRECSYS_DEBUG_SKIP ablation mask (-DFRECSYS_ABLATION builds only)
  // per-kernel event pairs, resolved after the call's final synchronisation
  struct Pending {
    std::string name;
    hipEvent_t a, b;
  };
  std::vector<Pending> pending;
  std::vector<hipEvent_t> event_pool;
};

namespace {

int fail(frecsys_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  g_last_error = msg;
  return code;
}

#define HIP_TRY(c, expr)                                                            \
  do {                                                                              \
    hipError_t _e = (expr);                                                         \
    if (_e != hipSuccess)                                                           \
      return fail((c), FRECSYS_ERR_HIP,                                             \
                  std::string(#expr) + ": " + hipGetErrorString(_e));               \
  } while (0)

#define NCCL_TRY(c, expr)                                                           \
  do {                                                                              \
    ncclResult_t _r = (expr);                                                       \
    if (_r != ncclSuccess)                                                          \
      return fail((c), FRECSYS_ERR_RCCL,                                            \
                  std::string(#expr) + ": " + ncclGetErrorString(_r));              \
  } while (0)

void add_work(frecsys_ctx* c, const std::string& key, double flops, double bytes,
              int64_t entities) {
  Work& w = c->work[key];
  w.flops += flops;
  w.bytes += bytes;
  w.entities += entities;
  w.launches += 1;
}

// SURVEY 8(d) per entity of h assembly rows at dim d: d-space SYRK
// h d (d+1) and LLT d^3/3 + 2 d^2 flops; gather bytes h d 4 (rows) + h 4
// (ids) + 8 (row offset) + d 4 (the solution written).
// (SYRK and gather are linear in h: summed from the queue prefix sums,
// heff_sums below.)
double dspace_solve_flops(double d) { return d * d * d / 3.0 + 2.0 * d * d; }

template <typename T>
int ensure(frecsys_ctx* c, T** p, size_t* cap, size_t count) {
  if (*cap >= count && *p) return FRECSYS_OK;
  if (*p) HIP_TRY(c, hipFree(*p));
  *p = nullptr;
  *cap = 0;
  HIP_TRY(c, hipMalloc((void**)p, sizeof(T) * std::max<size_t>(count, 1)));
  *cap = count;
  return FRECSYS_OK;
}

// ensure() that reports an out-of-memory hipMalloc instead of failing: *oom
// is set, *p left null and HIP's sticky last error cleared (the next launch
// check would otherwise see it).
template <typename T>
int try_ensure(frecsys_ctx* c, T** p, size_t* cap, size_t count, bool* oom) {
  *oom = false;
  if (*cap >= count && *p) return FRECSYS_OK;
  if (*p) HIP_TRY(c, hipFree(*p));
  *p = nullptr;
  *cap = 0;
  const hipError_t e = hipMalloc((void**)p, sizeof(T) * std::max<size_t>(count, 1));
  if (e == hipSuccess) {
    *cap = count;
    return FRECSYS_OK;
  }
  *p = nullptr;
  (void)hipGetLastError();
  if (e != hipErrorOutOfMemory)
    return fail(c, FRECSYS_ERR_HIP, std::string("hipMalloc: ") + hipGetErrorString(e));
  *oom = true;
  return FRECSYS_OK;
}

// Bytes one wide workspace may take now: FRECSYS_WIDE_WS_MB, capped at a
// quarter of the device memory that is free (plus what the workspace
// already holds), so several contexts or other tenants of the device leave
// each other room.
size_t ws_budget(frecsys_ctx* c, size_t held) {
  size_t b = (size_t)c->wide_ws_mb << 20;
  size_t fr = 0, tot = 0;
  if (c->ws_free_cap) {
    if (hipMemGetInfo(&fr, &tot) == hipSuccess)
      b = std::min(b, (fr + held) / 4);
    else
      (void)hipGetLastError();
  }
  return b;
}

// A workspace of *batch slots of `per` elements: a failed hipMalloc halves
// the batch (counted in ws_shrinks) until one slot does not fit either.
// Entities are independent, so the batch size never changes a result.
template <typename T>
int ensure_batch(frecsys_ctx* c, T** p, size_t* cap, size_t per, int64_t* batch) {
  while (true) {
    bool oom = false;
    int rc = try_ensure(c, p, cap, per * (size_t)*batch, &oom);
    if (rc || !oom) return rc;
    if (*batch <= 1)
      return fail(c, FRECSYS_ERR_HIP, "hipMalloc: out of memory for one workspace slot");
    *batch = (*batch + 1) / 2;
    ++c->ws_shrinks;
  }
}

bool valid_side(int side) { return side >= 0 && side <= 2; }

// Contiguous nnz-balanced split: rank r gets rows whose prefix nnz falls in
// [r*nnz/P, (r+1)*nnz/P).
void partition_rows(int64_t n_rows, const int64_t* row_ptr, int parts, int64_t* bounds) {
  const int64_t nnz = row_ptr[n_rows] - row_ptr[0];
  bounds[0] = 0;
  for (int r = 1; r < parts; ++r) {
    const int64_t target = row_ptr[0] + (nnz * r) / parts;
    const int64_t* it = std::lower_bound(row_ptr, row_ptr + n_rows + 1, target);
    int64_t b = it - row_ptr;
    if (b < bounds[r - 1]) b = bounds[r - 1];
    if (b > n_rows) b = n_rows;
    bounds[r] = b;
  }
  bounds[parts] = n_rows;
}

void refresh_bounds(frecsys_ctx* c, int side) {
  if (side > 1) return;
  c->bounds[side].assign(c->world + 1, 0);
  if (!c->host_rp[side].empty()) {
    partition_rows(c->n[side], c->host_rp[side].data(), c->world, c->bounds[side].data());
  } else {
    for (int r = 0; r <= c->world; ++r) c->bounds[side][r] = c->n[side] * r / c->world;
  }
}

void shard(const frecsys_ctx* c, int side, int64_t* lo, int64_t* hi) {
  if (side > 1 || c->world == 1 || c->bounds[side].empty()) {
    *lo = 0;
    *hi = c->n[side];
    return;
  }
  *lo = c->bounds[side][c->rank];
  *hi = c->bounds[side][c->rank + 1];
}

// Entities of the rank's shard of `side`, longest history first (stable),
// uploaded as the work queue of the tiled solve kernel (one 16-B record per
// entity: id, history length, CSR offset).
int build_order(frecsys_ctx* c, int side) {
  if (!c->order_stale[side] && c->d_order[side]) return FRECSYS_OK;
  int64_t lo, hi;
  shard(c, side, &lo, &hi);
  const std::vector<int64_t>& rp = side == 2 ? c->host_rp_eval : c->host_rp[side];
  std::vector<int32_t> ord((size_t)(hi - lo));
  for (int64_t i = lo; i < hi; ++i) ord[i - lo] = (int32_t)i;
  std::stable_sort(ord.begin(), ord.end(), [&](int32_t x, int32_t y) {
    return (rp[x + 1] - rp[x]) > (rp[y + 1] - rp[y]);
  });
  std::vector<QueueRec>& recs = c->h_order[side];  // lives until the next rebuild (async copy)
  recs.resize(ord.size());
  for (size_t i = 0; i < ord.size(); ++i) {
    const int32_t e = ord[i];
    recs[i].entity = e;
    recs[i].h = (int32_t)(rp[e + 1] - rp[e]);
    recs[i].p0 = rp[e];
  }
  if (c->d_order[side]) {
    hipError_t err = hipFree(c->d_order[side]);
    (void)err;
  }
  c->d_order[side] = nullptr;
  if (hipMalloc((void**)&c->d_order[side], sizeof(QueueRec) * std::max<size_t>(recs.size(), 1)) !=
      hipSuccess)
    return fail(c, FRECSYS_ERR_HIP, "hipMalloc failed (order)");
  if (!recs.empty() && hipMemcpyAsync(c->d_order[side], recs.data(),
                                      sizeof(QueueRec) * recs.size(), hipMemcpyHostToDevice,
                                      c->stream) != hipSuccess)
    return fail(c, FRECSYS_ERR_HIP, "hipMemcpy failed (order)");
  c->order_n[side] = (int64_t)recs.size();
  c->order_h[side].resize(recs.size());
  for (size_t i = 0; i < recs.size(); ++i) c->order_h[side][i] = recs[i].h;
  c->order_stale[side] = false;
  c->wprefix[side][0].valid = c->wprefix[side][1].valid = false;
  c->hrows_key[side][0] = c->hrows_key[side][1] = -1;  // subsets follow the queue
  return FRECSYS_OK;
}

// Sums of h_eff, h_eff^2, h_eff^3 and of the non-empty entities over queue
// positions [lo, hi) of `side` (vq: the V kinds' tail-quirk h_eff).
struct HeffSums {
  double h1 = 0, h2 = 0, h3 = 0;
  int64_t nz = 0;
};
HeffSums heff_sums(frecsys_ctx* c, int side, bool vq, int64_t lo, int64_t hi) {
  frecsys_ctx::WorkPrefix& p = c->wprefix[side][vq ? 1 : 0];
  const std::vector<int32_t>& hs = c->order_h[side];
  if (!p.valid || p.h1.size() != hs.size() + 1) {
    const size_t n = hs.size();
    p.h1.assign(n + 1, 0.0);
    p.h2.assign(n + 1, 0.0);
    p.h3.assign(n + 1, 0.0);
    p.nz.assign(n + 1, 0);
    for (size_t i = 0; i < n; ++i) {
      const int64_t h0 = hs[i];
      const double h = (double)((vq && c->quirks && h0 > 128 && (h0 % 128) != 0)
                                    ? h0 + 128 - (h0 % 128) : h0);
      p.h1[i + 1] = p.h1[i] + h;
      p.h2[i + 1] = p.h2[i] + h * h;
      p.h3[i + 1] = p.h3[i] + h * h * h;
      p.nz[i + 1] = p.nz[i] + (h > 0 ? 1 : 0);
    }
    p.valid = true;
  }
  HeffSums s;
  if (hi <= lo) return s;
  s.h1 = p.h1[hi] - p.h1[lo];
  s.h2 = p.h2[hi] - p.h2[lo];
  s.h3 = p.h3[hi] - p.h3[lo];
  s.nz = p.nz[hi] - p.nz[lo];
  return s;
}

// Long-history split of the d-space queue prefix [0, n): entities with
// more than 2*C assembly rows get their SYRK cut into C-row slabs done by
// separate workgroups (launch_split_syrk / wide_syrk2_kernel<2>) before the
// solve; at most max_slabs slabs of slab_floats each (longest entities first;
// shrink: fewer when their allocation fails -- only where the split does not
// change the sums' order, the wide dims).
int plan_split(frecsys_ctx* c, const std::vector<int32_t>& hs, int64_t n,
               const std::function<int64_t(int64_t)>& heff, SolveArgs* a, int64_t C,
               size_t slab_floats, int64_t max_slabs, hipStream_t s, bool shrink = false) {
  a->split = nullptr;
  a->n_split = 0;
  a->slabs = nullptr;
  a->work = nullptr;
  a->n_work = 0;
  if (c->split_rows <= 0 || C <= 0 || c->Dp < 32) return FRECSYS_OK;
  int32_t slab = 0;
  while (true) {
    c->h_split.clear();
    c->h_work.clear();
    slab = 0;
    for (int64_t i = 0; i < n && heff(hs[i]) > 2 * C; ++i) {
      const int64_t ne = heff(hs[i]);
      if (slab + (ne + C - 1) / C > max_slabs) break;
      const int32_t first = slab;
      for (int64_t k = 0; k < ne; k += C)
        c->h_work.push_back(SplitWork{(int32_t)i, (int32_t)k, (int32_t)std::min(ne, k + C), slab++});
      c->h_split.push_back(int2{first, slab - first});
    }
    if (c->h_split.empty()) return FRECSYS_OK;
    if (!shrink) {
      int rc = ensure(c, &c->d_slabs, &c->cap_slabs, (size_t)slab * slab_floats);
      if (rc) return rc;
      break;
    }
    // the wide dims (split and unsplit SYRKs are bit-identical there): fewer
    // slabs when the allocation fails
    bool oom = false;
    int rc = try_ensure(c, &c->d_slabs, &c->cap_slabs, (size_t)slab * slab_floats, &oom);
    if (rc) return rc;
    if (!oom) break;
    ++c->ws_shrinks;
    max_slabs = slab / 2;
  }
  int rc = ensure(c, &c->d_split, &c->cap_split, c->h_split.size());
  if (rc) return rc;
  rc = ensure(c, &c->d_work, &c->cap_work, c->h_work.size());
  if (rc) return rc;
  // on the solve's own stream: a blocking hipMemcpy went through a queue that
  // could be FIFO-behind the basis chain, holding the d-space launch back
  // (h_split / h_work live in the context until the next call, after the
  // stream has been synchronised)
  HIP_TRY(c, hipMemcpyAsync(c->d_split, c->h_split.data(), sizeof(int2) * c->h_split.size(),
                            hipMemcpyHostToDevice, s));
  HIP_TRY(c, hipMemcpyAsync(c->d_work, c->h_work.data(), sizeof(SplitWork) * c->h_work.size(),
                            hipMemcpyHostToDevice, s));
  a->split = c->d_split;
  a->n_split = (int64_t)c->h_split.size();
  a->slabs = c->d_slabs;
  a->work = c->d_work;
  a->n_work = (int64_t)c->h_work.size();
  return FRECSYS_OK;
}

// Stream s waits (on the device) for the early basis builds still running
// on stream5 (mask bit per side).
int join_eager(frecsys_ctx* c, int mask, hipStream_t s) {
  for (int t = 0; t < 2; ++t)
    if ((mask >> t & 1) && c->eager_pending[t]) {
      HIP_TRY(c, hipStreamWaitEvent(s, c->ev_eager[t], 0));
      c->eager_pending[t] = false;
    }
  return FRECSYS_OK;
}
void emb_written(frecsys_ctx* c, int side) { c->emb_ver[side] = ++c->ver_counter; }

// Basis of the other side's Gramian, G = Q T Q^T, and the other side
// rotated into it (X Q): the inputs of the history-space solve.  Rebuilt
// only when the Gramian (basis) or the rows (rotation) changed since.
int prepare_basis(frecsys_ctx* c, int other, const float* X, hipStream_t s, int mode = 0,
                  float mu = 0.f, float lam = 0.f, const QueueRec* rows = nullptr,
                  int64_t nrows = 0, uint64_t sub = 0) {
  const int Dp = c->Dp;
  size_t cap = 0;
  if (!c->q[other]) {
    int rc = ensure(c, &c->q[other], &cap, (size_t)Dp * Dp);
    if (rc) return rc;
    cap = 0;
    rc = ensure(c, &c->tri[other], &cap, (size_t)2 * Dp);
    if (rc) return rc;
    cap = 0;
    rc = ensure(c, &c->refl[other], &cap, (size_t)Dp * Dp + Dp);
    if (rc) return rc;
  }
  if (mode == 0) mu = lam = 0.f;
  const bool same_kind = c->basis_mode[other] == mode && c->basis_mu[other] == mu &&
                         c->basis_lam[other] == lam;
  const bool need_basis = c->basis_gram[other] == 0 ||
                          c->basis_gram[other] != c->gram_ver[other] || !same_kind;
  const uint64_t xkey = X == c->emb[other] ? c->emb_ver[other] : 0;
  if (!rows) sub = 0;
  const bool need_rot = need_basis || xkey == 0 || c->xrot_emb[other] != xkey ||
                        c->xrot_gram[other] != c->gram_ver[other] ||
                        (c->xrot_sub[other] != 0 && c->xrot_sub[other] != sub);
  const int64_t nrot = rows ? nrows : c->n[other];
  if (s != c->stream5) {
    // an early build of this basis (or one sharing tri_work) may still run
    int rc = join_eager(c, 3, s);
    if (rc) return rc;
  }
  if (!need_rot) return FRECSYS_OK;
  int rc = ensure(c, &c->xrot[other], &c->cap_xrot[other],
                  (size_t)std::max<int64_t>(c->n[other], 1) * Dp);
  if (rc) return rc;
  c->xrot_emb[other] = xkey;
  c->xrot_gram[other] = c->gram_ver[other];
  c->xrot_sub[other] = sub;
  if (!need_basis) {
    HIP_TRY(c, launch_rotate(X, rows, 0, nrot, c->qsplit[other][0], c->xrot[other], Dp,
                             s));
    return FRECSYS_OK;
  }
  c->basis_gram[other] = c->gram_ver[other];
  {  // Cholesky + triangular inverse n^3/3 + n^3/3; Householder reduction 4n^3/3 + Q 4n^3/3
    const double n = Dp;
    add_work(c, mode == 1 ? "basis_chol" : "basis_tridiag",
             mode == 1 ? 2.0 * n * n * n / 3.0 : 8.0 * n * n * n / 3.0, 2.0 * n * n * 4.0, 1);
  }
  c->basis_mode[other] = mode;
  c->basis_mu[other] = mu;
  c->basis_lam[other] = lam;
  for (int t = 0; t < 2; ++t)  // bf16-piece images of the forward and back rotations
    if (!c->qsplit[other][t]) HIP_TRY(c, hipMalloc(&c->qsplit[other][t], basis_split_bytes(Dp)));
  if (mode == 1) {
    // q = L^-T: forward X L^-T (image of q), back x' L^-1 (image of q^T)
    rc = ensure(c, &c->chol_work, &c->cap_chol_work, chol_basis_work_floats(Dp));
    if (rc) return rc;
    HIP_TRY(c, launch_chol_basis(c->gram[other], Dp, mu, lam, c->chol_work, c->q[other],
                                 c->tri[other], s));
    HIP_TRY(c, launch_split_basis(c->q[other], Dp, 0, c->qsplit[other][0], s));
    HIP_TRY(c, launch_split_basis(c->q[other], Dp, 1, c->qsplit[other][1], s));
    HIP_TRY(c, launch_rotate(X, rows, 0, nrot, c->qsplit[other][0], c->xrot[other], Dp,
                             s));
    return FRECSYS_OK;
  }
  float* tau = c->refl[other] + (size_t)Dp * Dp;
  const bool qpipe = tridiag_forms_q(Dp);
  if (wide_dim(Dp) || qpipe) {
    rc = ensure(c, &c->tri_work, &c->cap_tri_work, tridiag_work_floats(Dp));
    if (rc) return rc;
  }
  if (qpipe) {
    // Q rows and their split images formed inside the reduction's launch
    HIP_TRY(c, launch_tridiag(c->gram[other], Dp, c->tri[other], c->tri[other] + Dp,
                              c->refl[other], tau, s, c->tri_work, c->q[other],
                              c->qsplit[other][0], c->qsplit[other][1], c->d_events));
    HIP_TRY(c, launch_rotate(X, rows, 0, nrot, c->qsplit[other][0], c->xrot[other], Dp,
                             s));
    return FRECSYS_OK;
  }
  HIP_TRY(c, launch_tridiag(c->gram[other], Dp, c->tri[other], c->tri[other] + Dp, c->refl[other],
                            tau, s, c->tri_work, nullptr, nullptr, nullptr, c->d_events));
  HIP_TRY(c, launch_form_q(c->refl[other], tau, Dp, c->q[other], s, c->qsplit[other][0],
                           c->qsplit[other][1]));
  HIP_TRY(c, launch_rotate(X, rows, 0, nrot, c->qsplit[other][0], c->xrot[other], Dp, s));
  return FRECSYS_OK;
}

// The rows of `other` that side's history-space entities (its queue
// positions [q0, q1)) read: a row list when it is well below the whole
// table, else none (rotate every row).  Marked on the device, compacted on
// the host once per queue and split point (one synchronisation then).
int hspace_rows(frecsys_ctx* c, int side, int other, int64_t q0, int64_t q1,
                const QueueRec** rows, int64_t* nrows, uint64_t* sub) {
  *rows = nullptr;
  *nrows = 0;
  *sub = 0;
  if (q1 <= q0) return FRECSYS_OK;
  if (c->hrows_key[side][0] != q0 || c->hrows_key[side][1] != q1) {
    // an early build may still be rotating with the old list (stream5): the
    // synchronisation below then covers it before the list is rewritten
    int rc = join_eager(c, 3, c->stream);
    if (rc) return rc;
    const int64_t no = c->n[other];
    rc = ensure(c, &c->d_mark, &c->cap_mark, (size_t)no);
    if (rc) return rc;
    HIP_TRY(c, hipMemsetAsync(c->d_mark, 0, (size_t)no, c->stream));
    HIP_TRY(c, launch_mark_rows(c->d_order[side] + q0, q1 - q0, c->col[side], c->d_mark,
                                c->stream));
    std::vector<uint8_t> mark((size_t)no);
    HIP_TRY(c, hipMemcpyAsync(mark.data(), c->d_mark, (size_t)no, hipMemcpyDeviceToHost,
                              c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    std::vector<QueueRec> list;
    for (int64_t r = 0; r < no; ++r)
      if (mark[r]) list.push_back(QueueRec{(int32_t)r, 0, 0});
    c->hrows_key[side][0] = q0;
    c->hrows_key[side][1] = q1;
    c->hrows_gen[side] = ++c->ver_counter;
    if ((double)list.size() > 0.7 * (double)no) {
      c->n_hrows[side] = -1;  // most of the table: one plain pass over it
    } else {
      rc = ensure(c, &c->d_hrows[side], &c->cap_hrows[side], std::max<size_t>(list.size(), 1));
      if (rc) return rc;
      if (!list.empty())
        HIP_TRY(c, hipMemcpy(c->d_hrows[side], list.data(), sizeof(QueueRec) * list.size(),
                             hipMemcpyHostToDevice));
      c->n_hrows[side] = (int64_t)list.size();
    }
  }
  if (c->n_hrows[side] >= 0) {
    *rows = c->d_hrows[side];
    *nrows = c->n_hrows[side];
    *sub = c->hrows_gen[side];
  }
  return FRECSYS_OK;
}

// A Gramian of side g was just formed on c->stream: build its basis on
// stream5 now if the side that consumes it took the history-space path last
// time and will want it again.
int maybe_start_eager(frecsys_ctx* c, int g) {
  const int consumer = 1 - g;
  if (!c->eager_on || c->dual_serial || !c->dual_on || c->Dp < 64 || c->dual_max_h <= 0 ||
      !c->dual_used[consumer] || c->eager_pending[g])
    return FRECSYS_OK;
  // the consumer's last row subset (its next solve checks it still applies)
  const bool subset = c->n_hrows[consumer] >= 0 && c->hrows_key[consumer][0] >= 0;
  const QueueRec* rows = subset ? c->d_hrows[consumer] : nullptr;
  const uint64_t sub = subset ? c->hrows_gen[consumer] : 0;
  if (c->basis_gram[g] == c->gram_ver[g] && c->xrot_emb[g] == c->emb_ver[g] &&
      c->xrot_gram[g] == c->gram_ver[g] && c->basis_mode[g] == c->want_mode[g] &&
      c->basis_mu[g] == c->want_mu[g] && c->basis_lam[g] == c->want_lam[g] &&
      (c->xrot_sub[g] == 0 || c->xrot_sub[g] == sub))
    return FRECSYS_OK;  // already current
  HIP_TRY(c, hipEventRecord(c->ev_pre5, c->stream));
  HIP_TRY(c, hipStreamWaitEvent(c->stream5, c->ev_pre5, 0));
  int rc = prepare_basis(c, g, c->emb[g], c->stream5, c->want_mode[g], c->want_mu[g],
                         c->want_lam[g], rows, subset ? c->n_hrows[consumer] : 0, sub);
  if (rc) return rc;
  HIP_TRY(c, hipEventRecord(c->ev_eager[g], c->stream5));
  c->eager_pending[g] = true;
  return FRECSYS_OK;
}

// Row-range all-gather of a [rows x ld] float matrix (uneven per-rank
// counts): every rank broadcasts its own range in place.
int allgather_rows(frecsys_ctx* c, float* base, int side, int64_t ld) {
  if (!c->comm) return FRECSYS_OK;  // world 1 without RCCL, or external exchange: the caller's
  NCCL_TRY(c, ncclGroupStart());
  for (int r = 0; r < c->world; ++r) {
    const int64_t lo = c->bounds[side][r], hi = c->bounds[side][r + 1];
    const size_t cnt = (size_t)(hi - lo) * ld;
    if (cnt == 0) continue;
    float* p = base + lo * ld;
    NCCL_TRY(c, ncclBroadcast(p, p, cnt, ncclFloat, r, c->comm, c->stream));
  }
  NCCL_TRY(c, ncclGroupEnd());
  return FRECSYS_OK;
}

// The exchanges a sharded call makes inside itself, one code path for both
// transports: RCCL (a communicator) or the caller's callbacks
// (frecsys_set_transport).  Without either (world 1, or external exchange
// with no transport) a call does not exchange; the caller completes it.
bool in_call_exchange(const frecsys_ctx* c) { return c->world > 1 && (c->comm || c->has_transport); }

// All-gather of a per-row device table of `side` (ld floats per row).
int xchg_rows(frecsys_ctx* c, float* base, int side, int64_t ld) {
  if (c->comm) return allgather_rows(c, base, side, ld);
  if (!c->has_transport) return FRECSYS_OK;
  const int64_t n = c->n[side];
  std::vector<float> h((size_t)std::max<int64_t>(n * ld, 1));
  if (n) HIP_TRY(c, hipMemcpyAsync(h.data(), base, sizeof(float) * n * ld, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  int64_t lo, hi;
  shard(c, side, &lo, &hi);
  if (c->transport.allgather_rows(c->transport.user, side, h.data(), n, ld, lo, hi) != 0)
    return fail(c, FRECSYS_ERR_RCCL, "transport: allgather_rows failed");
  if (n) HIP_TRY(c, hipMemcpyAsync(base, h.data(), sizeof(float) * n * ld, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return FRECSYS_OK;
}

// In-place minimum over ranks of one device u64.
int xchg_min_u64(frecsys_ctx* c, unsigned long long* dval) {
  if (c->comm) {
    NCCL_TRY(c, ncclAllReduce(dval, dval, 1, ncclUint64, ncclMin, c->comm, c->stream));
    return FRECSYS_OK;
  }
  if (!c->has_transport) return FRECSYS_OK;
  uint64_t v = 0;
  HIP_TRY(c, hipMemcpyAsync(&v, dval, sizeof(v), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  if (c->transport.allreduce_min_u64(c->transport.user, &v) != 0)
    return fail(c, FRECSYS_ERR_RCCL, "transport: allreduce_min_u64 failed");
  HIP_TRY(c, hipMemcpyAsync(dval, &v, sizeof(v), hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return FRECSYS_OK;
}

// Host -> device upload of a per-entity vector through a pinned staging
// buffer of its own (one per destination): a DMA the stream orders like a
// kernel, instead of a pageable-memory copy that the runtime stages itself
// (observed waiting for work queued on other streams).  Every call that
// uploads synchronises its stream before returning, so a staging buffer is
// never rewritten while its copy is in flight.
int upload(frecsys_ctx* c, float** dptr, size_t* cap, const float* host, size_t n) {
  int rc = ensure(c, dptr, cap, n);
  if (rc) return rc;
  auto& pin = c->pinned[dptr];
  if (pin.second < n) {
    if (pin.first) HIP_TRY(c, hipHostFree(pin.first));
    pin.first = nullptr;
    pin.second = 0;
    HIP_TRY(c, hipHostMalloc((void**)&pin.first, sizeof(float) * std::max<size_t>(n, 1),
                             hipHostMallocDefault));
    pin.second = n;
  }
  if (n) std::memcpy(pin.first, host, sizeof(float) * n);
  HIP_TRY(c, hipMemcpyAsync(*dptr, pin.first, sizeof(float) * n, hipMemcpyHostToDevice, c->stream));
  return FRECSYS_OK;
}

struct ScopedTimer {
  frecsys_ctx* c;
  const char* name;
  ScopedTimer(frecsys_ctx* c_, const char* n_) : c(c_), name(n_) {
    (void)hipEventRecord(c->ev0, c->stream);
  }
  // Stops the timer: synchronises on the end event and accumulates.
  void stop() {
    (void)hipEventRecord(c->ev1, c->stream);
    (void)hipEventSynchronize(c->ev1);
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, c->ev0, c->ev1) == hipSuccess) {
      Timer& t = c->timers[name];
      t.total_ms += ms;
      t.launches += 1;
    }
  }
};

// Event pair around one launch on any stream; resolved by flush_ktimers
// after the stream has been synchronised.
hipEvent_t pool_event(frecsys_ctx* c) {
  if (!c->event_pool.empty()) {
    hipEvent_t e = c->event_pool.back();
    c->event_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  (void)hipEventCreate(&e);
  return e;
}
size_t ktimer_begin(frecsys_ctx* c, const std::string& name, hipStream_t s) {
  frecsys_ctx::Pending p{name, pool_event(c), pool_event(c)};
  (void)hipEventRecord(p.a, s);
  c->pending.push_back(p);
  return c->pending.size() - 1;
}
void ktimer_end(frecsys_ctx* c, size_t i, hipStream_t s) {
  (void)hipEventRecord(c->pending[i].b, s);
}
void flush_ktimers(frecsys_ctx* c) {
  for (auto& p : c->pending) {
    float ms = 0.f;
    if (hipEventSynchronize(p.b) == hipSuccess &&
        hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
      Timer& t = c->timers[p.name];
      t.total_ms += ms;
      t.launches += 1;
    }
    c->event_pool.push_back(p.a);
    c->event_pool.push_back(p.b);
  }
  c->pending.clear();
}

// Group slabs of [r's groups] broadcast from their owners (an all-gather
// with uneven counts, in place).
int allgather_groups(frecsys_ctx* c, float* gslabs, const GramPlan& pl) {
  if (!c->comm || pl.ngroup == 0) return FRECSYS_OK;
  NCCL_TRY(c, ncclGroupStart());
  for (int r = 0; r < c->world; ++r) {
    int lo, hi;
    gram_owned_groups(pl, c->world, r, &lo, &hi);
    if (hi <= lo) continue;
    float* p = gslabs + (size_t)lo * pl.slab_floats;
    NCCL_TRY(c, ncclBroadcast(p, p, (size_t)(hi - lo) * pl.slab_floats, ncclFloat, r, c->comm,
                              c->stream));
  }
  NCCL_TRY(c, ncclGroupEnd());
  return FRECSYS_OK;
}

// G = X^T diag(w) X over all rows of X (n rows) by the partition-
// independent plan (kernels.h GramPlan): this rank computes its own groups,
// the group slabs are all-gathered (with a communicator) and every rank sums
// them in group order.  Without a communicator at world > 1 (external
// exchange) the other ranks' slabs are zero: G is this rank's partial sum.
// `all_groups`: compute every group here (diagnostics on one rank).
int form_gramian(frecsys_ctx* c, int slot, const float* X, int64_t n, const float* dw, float* G,
                 bool all_groups) {
  const GramPlan pl = gram_plan(c->Dp, n);
  int g_lo = 0, g_hi = pl.ngroup;
  if (!all_groups) gram_owned_groups(pl, c->world, c->rank, &g_lo, &g_hi);
  int rc = ensure(c, &c->d_partials, &c->cap_partials, gram_leaf_floats(pl, g_lo, g_hi));
  if (rc) return rc;
  rc = ensure(c, &c->d_gslabs[slot], &c->cap_gslabs[slot],
              std::max<size_t>((size_t)pl.ngroup * pl.slab_floats, 1));
  if (rc) return rc;
  if (!all_groups && c->world > 1 && !c->comm && pl.ngroup > 0)
    HIP_TRY(c, hipMemsetAsync(c->d_gslabs[slot], 0, sizeof(float) * pl.ngroup * pl.slab_floats,
                              c->stream));
  GramArgs g{};
  g.X = X;
  g.w = dw;
  g.partials = c->d_partials;
  g.gslabs = c->d_gslabs[slot];
  g.plan = pl;
  g.g_lo = g_lo;
  g.g_hi = g_hi;
  HIP_TRY(c, launch_gramian(c->Dp, g, c->stream));
  if (slot < 2 && g_hi > g_lo) {  // 2 N d^2 over the rows of the groups formed here
    const int64_t r0 = gram_group_leaf(pl, g_lo) * pl.rpl;
    const int64_t r1 = std::min<int64_t>(n, gram_group_leaf(pl, g_hi) * pl.rpl);
    const double rows = (double)(r1 - r0), dd = c->dim;
    add_work(c, "gramian", 2.0 * rows * dd * dd, rows * dd * 4.0, r1 - r0);
  }
  if (!all_groups && c->comm) {
    const size_t k = ktimer_begin(c, "gram_exchange", c->stream);
    rc = allgather_groups(c, c->d_gslabs[slot], pl);
    if (rc) return rc;
    ktimer_end(c, k, c->stream);
  }
  HIP_TRY(c, launch_gram_final(c->Dp, pl, c->d_gslabs[slot], G, c->stream));
  if (slot < 2) {
    c->gplan[slot] = pl;
    c->gram_own[slot][0] = g_lo;
    c->gram_own[slot][1] = g_hi;
  }
  return FRECSYS_OK;
}

// Restatement of libstdc++ std::normal_distribution<float>::operator()
// (Marsaglia polar; bits/random.tcc) over std::generate_canonical<float,24>
// of std::mt19937, with FMA contraction off so x*x + y*y rounds like the
// un-fused library code.  Drives the seeded init of init_matrix
// (recommender.h:61-67).
#pragma clang fp contract(off)
struct NormalF {
  bool saved_available = false;
  float saved = 0.f;
  static float canonical(std::mt19937& g) {
    float s = (float)g();
    float r = s / 4294967296.0f;
    if (r >= 1.0f) r = std::nextafter(1.0f, 0.0f);
    return r;
  }
  float operator()(std::mt19937& g, float mean, float stddev) {
    float ret;
    if (saved_available) {
      saved_available = false;
      ret = saved;
    } else {
      float x, y, r2;
      do {
        x = (float)((double)(2.0f * canonical(g)) - 1.0);
        y = (float)((double)(2.0f * canonical(g)) - 1.0);
        r2 = x * x + y * y;
      } while (r2 > 1.0 || r2 == 0.0);
      const float mult = std::sqrt(-2 * std::log(r2) / r2);
      saved = x * mult;
      saved_available = true;
      ret = y * mult;
    }
    return ret * stddev + mean;
  }
};

// n draws of a fresh NormalF (a new distribution per matrix,
// recommender.h:61-67) from g, bit-identical to calling it n times, in two
// passes: the polar method's accept / reject decisions need only the
// uniforms (a cheap sequential scan that advances g exactly as NormalF
// does), and the log / sqrt of each accepted pair are independent, so they
// run on threads.  2M x 1024 + 500K x 1024 draws: the serial loop's ~1 min
// becomes a few seconds.
void fill_normal(std::mt19937& g, float mean, float stddev, float* out, size_t n) {
  const size_t pairs = (n + 1) / 2;
  std::vector<float> px(pairs), py(pairs), pr(pairs);
  for (size_t p = 0; p < pairs; ++p) {
    float x, y, r2;
    do {
      x = (float)((double)(2.0f * NormalF::canonical(g)) - 1.0);
      y = (float)((double)(2.0f * NormalF::canonical(g)) - 1.0);
      r2 = x * x + y * y;
    } while (r2 > 1.0 || r2 == 0.0);
    px[p] = x;
    py[p] = y;
    pr[p] = r2;
  }
  auto work = [&](size_t lo, size_t hi) {
    for (size_t p = lo; p < hi; ++p) {
      const float r2 = pr[p];
      const float mult = std::sqrt(-2 * std::log(r2) / r2);
      const float first = py[p] * mult;   // returned first ...
      const float second = px[p] * mult;  // ... then the saved value
      out[2 * p] = first * stddev + mean;
      if (2 * p + 1 < n) out[2 * p + 1] = second * stddev + mean;
    }
  };
  const size_t nt = std::min<size_t>(16, std::max(1u, std::thread::hardware_concurrency()));
  if (pairs < (size_t)1 << 16 || nt == 1) {
    work(0, pairs);
    return;
  }
  std::vector<std::thread> th;
  for (size_t t = 0; t < nt; ++t)
    th.emplace_back(work, pairs * t / nt, pairs * (t + 1) / nt);
  for (auto& t : th) t.join();
}
#pragma clang fp contract(on)

}  // namespace

extern "C" {

int32_t frecsys_padded_dim(int32_t dim) { return padded_dim(dim); }

int frecsys_device_count(int32_t* n) {
  int cnt = 0;
  hipError_t e = hipGetDeviceCount(&cnt);
  if (e != hipSuccess) {
    *n = 0;
    return fail(nullptr, FRECSYS_ERR_NO_DEVICE, hipGetErrorString(e));
  }
  *n = cnt;
  return FRECSYS_OK;
}

const char* frecsys_last_error(const frecsys_ctx* ctx) {
  return ctx ? ctx->err.c_str() : g_last_error.c_str();
}

int64_t frecsys_last_error_entity(const frecsys_ctx* ctx) { return ctx ? ctx->err_entity : -1; }

int frecsys_partition(int64_t n_rows, const int64_t* row_ptr, int32_t nparts, int64_t* bounds) {
  if (n_rows < 0 || nparts <= 0 || !row_ptr || !bounds)
    return fail(nullptr, FRECSYS_ERR_INVALID, "frecsys_partition: bad arguments");
  partition_rows(n_rows, row_ptr, nparts, bounds);
  return FRECSYS_OK;
}

int frecsys_gram_plan(int32_t dim, int64_t n_rows, int32_t world, int32_t rank,
                      int64_t* rows_per_leaf, int64_t* n_leaves, int32_t* n_groups,
                      int32_t* own_lo, int32_t* own_hi) {
  const int Dp = padded_dim(dim);
  if (Dp == 0 || n_rows < 0 || world <= 0 || rank < 0 || rank >= world)
    return fail(nullptr, FRECSYS_ERR_INVALID, "frecsys_gram_plan: bad arguments");
  const GramPlan pl = gram_plan(Dp, n_rows);
  int lo, hi;
  gram_owned_groups(pl, world, rank, &lo, &hi);
  if (rows_per_leaf) *rows_per_leaf = pl.rpl;
  if (n_leaves) *n_leaves = pl.nleaf;
  if (n_groups) *n_groups = pl.ngroup;
  if (own_lo) *own_lo = lo;
  if (own_hi) *own_hi = hi;
  return FRECSYS_OK;
}

int frecsys_ctx_create(const frecsys_config* cfg, frecsys_ctx** out) {
  if (!cfg || !out) return fail(nullptr, FRECSYS_ERR_INVALID, "null argument");
  *out = nullptr;
  const int Dp = padded_dim(cfg->dim);
  if (Dp == 0)
    return fail(nullptr, FRECSYS_ERR_UNSUPPORTED,
                "dim " + std::to_string(cfg->dim) + " not supported (1..1024 built)");
  if (cfg->n_users < 0 || cfg->n_items < 0)
    return fail(nullptr, FRECSYS_ERR_INVALID, "negative entity counts");
  int cnt = 0;
  if (hipGetDeviceCount(&cnt) != hipSuccess || cnt == 0)
    return fail(nullptr, FRECSYS_ERR_NO_DEVICE, "no HIP device visible");
  auto* c = new frecsys_ctx();
  c->dim = cfg->dim;
  c->Dp = Dp;
  c->quirks = cfg->parity_quirks;
  c->n[0] = cfg->n_users;
  c->n[1] = cfg->n_items;
  if (cfg->device >= 0) {
    c->device = cfg->device;
  } else {
    (void)hipGetDevice(&c->device);
  }
  auto bail = [&](int rc) {
    g_last_error = c->err;
    frecsys_ctx_destroy(c);
    return rc;
  };
  if (hipSetDevice(c->device) != hipSuccess)
    return bail(fail(c, FRECSYS_ERR_NO_DEVICE, "hipSetDevice failed"));
  {  // the history-space chain (basis -> buckets) runs on the high-priority stream
    int lo_pri = 0, hi_pri = 0;
    (void)hipDeviceGetStreamPriorityRange(&lo_pri, &hi_pri);
    if (hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, hi_pri) != hipSuccess)
      return bail(fail(c, FRECSYS_ERR_HIP, "hipStreamCreate failed"));
  }
  if (hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess)
    return bail(fail(c, FRECSYS_ERR_HIP, "hipEventCreate failed"));
  // the second bucket lane / early builds at normal priority (high priority
  // measured no better)
  const int s3_pri = 0;
  if (hipStreamCreateWithFlags(&c->stream2, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithPriority(&c->stream3, hipStreamNonBlocking, s3_pri) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_fork3, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_join3, hipEventDisableTiming) != hipSuccess)
    return bail(fail(c, FRECSYS_ERR_HIP, "hipStreamCreate failed (stream2/3)"));
  // the early basis builds share stream3 with the second bucket lane: with
  // GPU_MAX_HW_QUEUES = 4 a fifth stream shared a hardware queue with the
  // d-space stream, whose solve then waited (in FIFO order) for the whole
  // basis chain queued before it -- 0.5 ms per ML-20M epoch.  stream3 is idle
  // when a Gramian triggers an early build, and the buckets it runs later
  // need that basis anyway.
  c->stream5 = c->stream3;
  if (hipEventCreateWithFlags(&c->ev_pre5, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_eager[0], hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_eager[1], hipEventDisableTiming) != hipSuccess)
    return bail(fail(c, FRECSYS_ERR_HIP, "hipEventCreate failed (early builds)"));
  if (const char* v = getenv("FRECSYS_DUAL")) c->dual_on = atoi(v);
  if (const char* v = getenv("FRECSYS_EAGER")) c->eager_on = atoi(v);
  if (const char* v = getenv("FRECSYS_CHOL_BASIS")) c->chol_basis_on = atoi(v);
  // d-space / history-space crossover: by flops h = d, but at Dp <= 256 the
  // d-space kernel overtakes the TH = 8 bucket (225 < h <= 256) in time (epoch
  // 15.6 -> 15.1 ms at the ML-20M shape, threshold sweep in DESIGN.md 3.2).
  // Dp = 1024: the wide bucket (256 < h_eff <= 512, dual.hip) as well (config
  // 5 epoch 1470 -> 1274 ms); Dp = 512: 256 (the wide bucket at 384 / 512
  // measured 124 / 129 ms against 115 at MSD).
  c->dual_max_h = Dp <= 256 ? 224 : Dp == 1024 ? 512 : 256;
  if (const char* v = getenv("FRECSYS_DUAL_MAX_H")) c->dual_max_h = atoi(v);
  if (const char* v = getenv("FRECSYS_DUAL_SERIAL")) c->dual_serial = atoi(v);
  if (const char* v = getenv("FRECSYS_SPLIT_ROWS")) c->split_rows = atoi(v);
  if (const char* v = getenv("FRECSYS_DEBUG_SKIP")) {
#ifdef FRECSYS_ABLATION
    c->debug_skip = atoi(v);
#else
    // a release build has no ablation masks: refuse rather than silently
    // run the full work under a variable that claims to skip some
    if (atoi(v) != 0)
      return bail(fail(c, FRECSYS_ERR_INVALID,
                       "FRECSYS_DEBUG_SKIP needs a -DFRECSYS_ABLATION build of libfrecsys_hip.so"));
#endif
  }
  if (const char* v = getenv("FRECSYS_WIDE_WS_MB")) c->wide_ws_mb = std::max(1, atoi(v));
  if (const char* v = getenv("FRECSYS_WIDE_PRESPLIT")) c->wide_presplit = atoi(v) != 0;
  if (const char* v = getenv("FRECSYS_WS_FREE_CAP")) c->ws_free_cap = atoi(v) != 0;
  // the wide dims add the wide bucket (256 < h_eff <= 512, dual.hip)
  const int max_h_cap = Dp >= 512 ? kDualWideMaxH : 32 * kDualMaxTiles;
  c->dual_max_h = std::min(c->dual_max_h, max_h_cap);
  for (int t = 0; t < 3; ++t) c->dual_max_h_side[t] = c->dual_max_h;
  // Dp = 512, user side: 320.  That half-step is bound by its d-space stream
  // (MSD: 45 ms beside 29 of history space), and the wide bucket takes the
  // users with 256 < h_eff <= 320 off it: MSD 115.3 -> 114.1 ms (items: no
  // gain; DESIGN.md 3.8, profiles/r06/dual_max_h/)
  if (Dp == 512 && !getenv("FRECSYS_DUAL_MAX_H"))
    c->dual_max_h_side[FRECSYS_SIDE_USER] = std::min(320, max_h_cap);
  if (const char* v = getenv("FRECSYS_DUAL_MAX_H_USER"))
    c->dual_max_h_side[0] = std::min(atoi(v), max_h_cap);
  if (const char* v = getenv("FRECSYS_DUAL_MAX_H_ITEM"))
    c->dual_max_h_side[1] = std::min(atoi(v), max_h_cap);
  for (int s = 0; s < 2; ++s) {
    const size_t rows = (size_t)std::max<int64_t>(c->n[s], 1);
    if (hipMalloc((void**)&c->emb[s], sizeof(float) * rows * Dp) != hipSuccess ||
        hipMalloc((void**)&c->gram[s], sizeof(float) * Dp * Dp) != hipSuccess)
      return bail(fail(c, FRECSYS_ERR_HIP, "hipMalloc failed (embeddings)"));
    (void)hipMemsetAsync(c->emb[s], 0, sizeof(float) * rows * Dp, c->stream);
    (void)hipMemsetAsync(c->gram[s], 0, sizeof(float) * Dp * Dp, c->stream);
  }
  if (hipMalloc((void**)&c->d_fail, sizeof(unsigned long long)) != hipSuccess ||
      hipMalloc((void**)&c->d_counter, sizeof(unsigned int)) != hipSuccess ||
      hipMalloc((void**)&c->d_events, 4 * sizeof(unsigned int)) != hipSuccess)
    return bail(fail(c, FRECSYS_ERR_HIP, "hipMalloc failed"));
  (void)hipMemsetAsync(c->d_events, 0, 4 * sizeof(unsigned int), c->stream);
  c->bounds[0] = {0, c->n[0]};
  c->bounds[1] = {0, c->n[1]};
  if (hipStreamSynchronize(c->stream) != hipSuccess)
    return bail(fail(c, FRECSYS_ERR_HIP, "stream sync failed"));
  *out = c;
  return FRECSYS_OK;
}

void frecsys_ctx_destroy(frecsys_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream5) (void)hipStreamSynchronize(c->stream5);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->comm) ncclCommDestroy(c->comm);
  for (int s = 0; s < 3; ++s) {
    if (c->emb[s]) (void)hipFree(c->emb[s]);
    if (c->rp[s]) (void)hipFree(c->rp[s]);
    if (c->col[s]) (void)hipFree(c->col[s]);
  }
  for (int s = 0; s < 2; ++s) {
    if (c->snap[s]) (void)hipFree(c->snap[s]);
    if (c->gram[s]) (void)hipFree(c->gram[s]);
  }
  for (float* p : {c->d_entity_weight, c->d_entity_reg, c->d_other_weight, c->d_gram_w,
                   c->d_partials, c->d_loss, c->d_quad, c->d_gslabs[0], c->d_gslabs[1],
                   c->d_gslabs[2]})
    if (p) (void)hipFree(p);
  if (c->d_fail) (void)hipFree(c->d_fail);
  if (c->d_counter) (void)hipFree(c->d_counter);
  if (c->d_events) (void)hipFree(c->d_events);
  for (int s = 0; s < 3; ++s)
    if (c->d_order[s]) (void)hipFree(c->d_order[s]);
  for (int s = 0; s < 2; ++s) {
    for (float* p : {c->q[s], c->tri[s], c->refl[s], c->xrot[s]})
      if (p) (void)hipFree(p);
    for (void* p : c->qsplit[s])
      if (p) (void)hipFree(p);
  }
  if (c->gsplit) (void)hipFree(c->gsplit);
  for (int s = 0; s < 3; ++s)
    if (c->out_rot[s]) (void)hipFree(c->out_rot[s]);
  for (int s = 0; s < 3; ++s)
    if (c->d_hrows[s]) (void)hipFree(c->d_hrows[s]);
  if (c->d_mark) (void)hipFree(c->d_mark);
  if (c->dual_table) (void)hipFree(c->dual_table);
  if (c->tri_work) (void)hipFree(c->tri_work);
  if (c->chol_work) (void)hipFree(c->chol_work);
  if (c->wide_ws) (void)hipFree(c->wide_ws);
  if (c->wide_xs) (void)hipFree(c->wide_xs);
  if (c->dw_zs) (void)hipFree(c->dw_zs);
  if (c->dw_slots) (void)hipFree(c->dw_slots);
  if (c->dw_z) (void)hipFree(c->dw_z);
  if (c->d_scores) (void)hipFree(c->d_scores);
  if (c->d_rows) (void)hipFree(c->d_rows);
  for (int s = 0; s < 2; ++s) {
    if (c->d_rix[s]) (void)hipFree(c->d_rix[s]);
    if (c->d_pred[s]) (void)hipFree(c->d_pred[s]);
  }
  if (c->d_resid) (void)hipFree(c->d_resid);
  if (c->d_resid_e) (void)hipFree(c->d_resid_e);
  if (c->d_gstat) (void)hipFree(c->d_gstat);
  if (c->d_dot) (void)hipFree(c->d_dot);
  if (c->d_topk) (void)hipFree(c->d_topk);
  if (c->d_split) (void)hipFree(c->d_split);
  if (c->d_work) (void)hipFree(c->d_work);
  if (c->d_slabs) (void)hipFree(c->d_slabs);
  for (auto& kv : c->pinned)
    if (kv.second.first) (void)hipHostFree(kv.second.first);
  for (auto& p : c->pending) c->event_pool.insert(c->event_pool.end(), {p.a, p.b});
  for (hipEvent_t e : c->event_pool) (void)hipEventDestroy(e);
  if (c->ev_fork3) (void)hipEventDestroy(c->ev_fork3);
  if (c->ev_join3) (void)hipEventDestroy(c->ev_join3);
  if (c->stream3) {
    (void)hipStreamSynchronize(c->stream3);
    (void)hipStreamDestroy(c->stream3);
  }
  if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
  if (c->ev_join) (void)hipEventDestroy(c->ev_join);
  if (c->stream2) {
    (void)hipStreamSynchronize(c->stream2);
    (void)hipStreamDestroy(c->stream2);
  }
  for (hipEvent_t e : {c->ev_pre5, c->ev_eager[0], c->ev_eager[1]})
    if (e) (void)hipEventDestroy(e);
  c->stream5 = nullptr;  // = stream3, destroyed above
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

int frecsys_comm_unique_id(uint8_t id[128]) {
  ncclUniqueId uid;
  ncclResult_t r = ncclGetUniqueId(&uid);
  if (r != ncclSuccess) return fail(nullptr, FRECSYS_ERR_RCCL, ncclGetErrorString(r));
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
  std::memcpy(id, &uid, 128);
  return FRECSYS_OK;
}

int frecsys_comm_init(frecsys_ctx* c, int32_t world, int32_t rank, const uint8_t id[128]) {
  if (!c || world <= 0 || rank < 0 || rank >= world)
    return fail(c, FRECSYS_ERR_INVALID, "frecsys_comm_init: bad rank/world");
  HIP_TRY(c, hipSetDevice(c->device));
  if (c->comm) {
    ncclCommDestroy(c->comm);
    c->comm = nullptr;
  }
  int rc = join_eager(c, 3, c->stream);
  if (rc) return rc;
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  c->gram_src[0] = c->gram_src[1] = 0;  // partials now sum over other shards
  c->world = world;
  c->rank = rank;
  if (id) {  // a communicator at every world size (world 1: the exchange path still runs)
    ncclUniqueId uid;
    std::memcpy(&uid, id, 128);
    NCCL_TRY(c, ncclCommInitRank(&c->comm, world, uid, rank));
  }
  refresh_bounds(c, 0);
  refresh_bounds(c, 1);
  c->order_stale[0] = c->order_stale[1] = true;
  return FRECSYS_OK;
}

int frecsys_shard_range(const frecsys_ctx* c, int32_t side, int64_t* lo, int64_t* hi) {
  if (!c || !valid_side(side) || !lo || !hi) return FRECSYS_ERR_INVALID;
  shard(c, side, lo, hi);
  return FRECSYS_OK;
}

int frecsys_load_csr(frecsys_ctx* c, int32_t side, int64_t n_rows, const int64_t* row_ptr,
                     const int32_t* col) {
  if (!c || !valid_side(side) || !row_ptr || n_rows < 0)
    return fail(c, FRECSYS_ERR_INVALID, "frecsys_load_csr: bad arguments");
  if (side < 2 && n_rows != c->n[side])
    return fail(c, FRECSYS_ERR_INVALID,
                "frecsys_load_csr: row count " + std::to_string(n_rows) + " != " +
                    std::to_string(c->n[side]));
  const int64_t nnz = row_ptr[n_rows] - row_ptr[0];
  if (row_ptr[0] != 0 || nnz < 0)
    return fail(c, FRECSYS_ERR_INVALID, "frecsys_load_csr: row_ptr must start at 0");
  if (side < 2) c->pp_order_all[side].clear();  // the residual order of a sharded pp_step
  const int other = side == 1 ? 0 : 1;
  const int64_t n_other = c->n[other];
  for (int64_t i = 0; i < n_rows; ++i)
    if (row_ptr[i + 1] < row_ptr[i])
      return fail(c, FRECSYS_ERR_INVALID, "frecsys_load_csr: row_ptr not monotone");
  for (int64_t k = 0; k < nnz; ++k)
    if (col[k] < 0 || col[k] >= n_other)  // assert(cp < item_embeddings.rows()), ials.h:116
      return fail(c, FRECSYS_ERR_INVALID,
                  "frecsys_load_csr: column id " + std::to_string(col[k]) + " out of range");
  HIP_TRY(c, hipSetDevice(c->device));
  {
    int rc = join_eager(c, 3, c->stream);
    if (rc) return rc;
    HIP_TRY(c, hipStreamSynchronize(c->stream));
  }
  c->gram_src[0] = c->gram_src[1] = 0;
  if (side == 2) emb_written(c, 2);
  if (c->rp[side]) HIP_TRY(c, hipFree(c->rp[side]));
  if (c->col[side]) HIP_TRY(c, hipFree(c->col[side]));
  c->rp[side] = nullptr;
  c->col[side] = nullptr;
  HIP_TRY(c, hipMalloc((void**)&c->rp[side], sizeof(int64_t) * (n_rows + 1)));
  HIP_TRY(c, hipMalloc((void**)&c->col[side], sizeof(int32_t) * std::max<int64_t>(nnz, 1)));
  HIP_TRY(c, hipMemcpyAsync(c->rp[side], row_ptr, sizeof(int64_t) * (n_rows + 1),
                            hipMemcpyHostToDevice, c->stream));
  if (nnz)
    HIP_TRY(c, hipMemcpyAsync(c->col[side], col, sizeof(int32_t) * nnz, hipMemcpyHostToDevice,
                              c->stream));
  c->nnz[side] = nnz;
  c->order_stale[side] = true;
  if (side == 2) {
    c->host_rp_eval.assign(row_ptr, row_ptr + n_rows + 1);
    c->n[2] = n_rows;
    if (c->emb[2]) HIP_TRY(c, hipFree(c->emb[2]));
    c->emb[2] = nullptr;
    HIP_TRY(c, hipMalloc((void**)&c->emb[2],
                         sizeof(float) * std::max<int64_t>(n_rows, 1) * c->Dp));
    HIP_TRY(c, hipMemsetAsync(c->emb[2], 0, sizeof(float) * std::max<int64_t>(n_rows, 1) * c->Dp,
                              c->stream));
  } else {
    c->host_rp[side].assign(row_ptr, row_ptr + n_rows + 1);
    refresh_bounds(c, side);
  }
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return FRECSYS_OK;
}

int frecsys_set_embeddings(frecsys_ctx* c, int32_t side, const float* host, int64_t ld) {
  if (!c || !valid_side(side) || !host || ld < c->dim)
    return fail(c, FRECSYS_ERR_INVALID, "frecsys_set_embeddings: bad arguments");
  if (!c->emb[side]) return fail(c, FRECSYS_ERR_INVALID, "side has no embeddings yet");
  HIP_TRY(c, hipSetDevice(c->device));
  int rc = join_eager(c, 3, c->stream);
  if (rc) return rc;
  emb_written(c, side);
  const int64_t rows = c->n[side];
  HIP_TRY(c, hipMemsetAsync(c->emb[side], 0, sizeof(float) * std::max<int64_t>(rows, 1) * c->Dp,
                            c->stream));
  if (rows)
    HIP_TRY(c, hipMemcpy2DAsync(c->emb[side], sizeof(float) * c->Dp, host, sizeof(float) * ld,
                                sizeof(float) * c->dim, rows, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return FRECSYS_OK;
}

int frecsys_get_embeddings(frecsys_ctx* c, int32_t side, float* host, int64_t ld) {
  if (!c || !valid_side(side) || !host || ld < c->dim)
    return fail(c, FRECSYS_ERR_INVALID, "frecsys_get_embeddings: bad arguments");
  if (!c->emb[side]) return fail(c, FRECSYS_ERR_INVALID, "side has no embeddings yet");
  HIP_TRY(c, hipSetDevice(c->device));
  const int64_t rows = c->n[side];
  if (rows)
    HIP_TRY(c, hipMemcpy2DAsync(host, sizeof(float) * ld, c->emb[side], sizeof(float) * c->Dp,
                                sizeof(float) * c->dim, rows, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return FRECSYS_OK;
}

int frecsys_init_embeddings(frecsys_ctx* c, uint32_t seed, float stdev) {
  if (!c) return fail(c, FRECSYS_ERR_INVALID, "null ctx");
  // ials.h:47-51: adjusted_stdev = stdev / sqrt(embedding_dim); one
  // generator, a new distribution per matrix (recommender.h:61-67).
  std::mt19937 gen{seed};
  const float adjusted = (float)((double)stdev / std::sqrt((double)c->dim));
  for (int s = 0; s < 2; ++s) {
    std::vector<float> h((size_t)c->n[s] * c->dim);
    fill_normal(gen, 0.0f, adjusted, h.data(), h.size());
    if (c->n[s]) {
      int rc = frecsys_set_embeddings(c, s, h.data(), c->dim);
      if (rc) return rc;
    }
  }
  return FRECSYS_OK;
}

int frecsys_snapshot(frecsys_ctx* c, int32_t side) {
  if (!c || side < 0 || side > 1) return fail(c, FRECSYS_ERR_INVALID, "snapshot: bad side");
  HIP_TRY(c, hipSetDevice(c->device));
  const size_t bytes = sizeof(float) * std::max<int64_t>(c->n[side], 1) * c->Dp;
  if (!c->snap[side]) HIP_TRY(c, hipMalloc((void**)&c->snap[side], bytes));
  HIP_TRY(c, hipMemcpyAsync(c->snap[side], c->emb[side], bytes, hipMemcpyDeviceToDevice,
                            c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return FRECSYS_OK;
}

int frecsys_gramian(frecsys_ctx* c, int32_t side, const float* weights, int32_t from_snapshot,
                    float* host_out) {
  if (!c || side < 0 || side > 1) return fail(c, FRECSYS_ERR_INVALID, "gramian: bad side");
  if (from_snapshot && !c->snap[side])
    return fail(c, FRECSYS_ERR_INVALID, "gramian: no snapshot taken");
  HIP_TRY(c, hipSetDevice(c->device));
  int rc;
  const bool plain = !weights && !from_snapshot;
  if (plain && c->gram_src[side] != 0 && c->gram_src[side] == c->emb_ver[side]) {
    // the embeddings are unchanged since this Gramian was formed: the same
    // deterministic computation would write the same bits (on every rank)
    if (host_out)
      HIP_TRY(c, hipMemcpy2DAsync(host_out, sizeof(float) * c->dim, c->gram[side],
                                  sizeof(float) * c->Dp, sizeof(float) * c->dim, c->dim,
                                  hipMemcpyDeviceToHost, c->stream));
    rc = maybe_start_eager(c, side);
    if (rc) return rc;
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    return FRECSYS_OK;
  }
  rc = join_eager(c, 1 << side, c->stream);  // an early basis build still reading this G
  if (rc) return rc;
  const float* dw = nullptr;
  if (weights) {
    rc = upload(c, &c->d_gram_w, &c->cap_gram_w, weights, (size_t)c->n[side]);
    if (rc) return rc;
    dw = c->d_gram_w;
  }
  {
    ScopedTimer t(c, "gramian");
    rc = form_gramian(c, side, from_snapshot ? c->snap[side] : c->emb[side], c->n[side], dw,
                      c->gram[side], false);
    if (rc) return rc;
    t.stop();
  }
  c->gram_ver[side] = ++c->ver_counter;
  c->gram_src[side] = plain ? c->emb_ver[side] : 0;
  if (host_out)
    HIP_TRY(c, hipMemcpy2DAsync(host_out, sizeof(float) * c->dim, c->gram[side],
                                sizeof(float) * c->Dp, sizeof(float) * c->dim, c->dim,
                                hipMemcpyDeviceToHost, c->stream));
  rc = maybe_start_eager(c, side);
  if (rc) return rc;
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  flush_ktimers(c);
  return FRECSYS_OK;
}

int frecsys_get_gramian(frecsys_ctx* c, int32_t side, float* host, int64_t ld) {
  if (!c || side < 0 || side > 1 || !host || ld < c->dim)
    return fail(c, FRECSYS_ERR_INVALID, "get_gramian: bad arguments");
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, hipMemcpy2DAsync(host, sizeof(float) * ld, c->gram[side], sizeof(float) * c->Dp,
                              sizeof(float) * c->dim, c->dim, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return FRECSYS_OK;
}

int frecsys_gram_groups(const frecsys_ctx* c, int32_t side, int32_t* n_groups, int32_t* own_lo,
                        int32_t* own_hi, int64_t* floats_per_group) {
  if (!c || side < 0 || side > 1) return FRECSYS_ERR_INVALID;
  const GramPlan pl = gram_plan(c->Dp, c->n[side]);
  int lo, hi;
  gram_owned_groups(pl, c->world, c->rank, &lo, &hi);
  if (n_groups) *n_groups = pl.ngroup;
  if (own_lo) *own_lo = lo;
  if (own_hi) *own_hi = hi;
  if (floats_per_group) *floats_per_group = (int64_t)pl.slab_floats;
  return FRECSYS_OK;
}

int frecsys_get_gram_groups(frecsys_ctx* c, int32_t side, float* host) {
  if (!c || side < 0 || side > 1 || !host)
    return fail(c, FRECSYS_ERR_INVALID, "get_gram_groups: bad arguments");
  const GramPlan& pl = c->gplan[side];
  if (!c->d_gslabs[side] || pl.n != c->n[side])
    return fail(c, FRECSYS_ERR_INVALID, "get_gram_groups: no Gramian formed for side");
  HIP_TRY(c, hipSetDevice(c->device));
  if (pl.ngroup)
    HIP_TRY(c, hipMemcpyAsync(host, c->d_gslabs[side], sizeof(float) * pl.ngroup * pl.slab_floats,
                              hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return FRECSYS_OK;
}

int frecsys_set_gram_groups(frecsys_ctx* c, int32_t side, const float* host) {
  if (!c || side < 0 || side > 1 || !host)
    return fail(c, FRECSYS_ERR_INVALID, "set_gram_groups: bad arguments");
  HIP_TRY(c, hipSetDevice(c->device));
  int rc = join_eager(c, 1 << side, c->stream);
  if (rc) return rc;
  const GramPlan pl = gram_plan(c->Dp, c->n[side]);
  rc = ensure(c, &c->d_gslabs[side], &c->cap_gslabs[side],
              std::max<size_t>((size_t)pl.ngroup * pl.slab_floats, 1));
  if (rc) return rc;
  if (pl.ngroup)
    HIP_TRY(c, hipMemcpyAsync(c->d_gslabs[side], host, sizeof(float) * pl.ngroup * pl.slab_floats,
                              hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, launch_gram_final(c->Dp, pl, c->d_gslabs[side], c->gram[side], c->stream));
  c->gplan[side] = pl;
  c->gram_ver[side] = ++c->ver_counter;
  c->gram_src[side] = 0;
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return FRECSYS_OK;
}

int frecsys_comm_world(const frecsys_ctx* c, int32_t* world, int32_t* rank, int32_t* comm_ranks) {
  if (!c) return FRECSYS_ERR_INVALID;
  if (world) *world = c->world;
  if (rank) *rank = c->rank;
  if (comm_ranks) {
    int n = 0;
    if (c->comm && ncclCommCount(c->comm, &n) != ncclSuccess) return FRECSYS_ERR_RCCL;
    *comm_ranks = n;  // 0: no communicator
  }
  return FRECSYS_OK;
}

int frecsys_set_gramian(frecsys_ctx* c, int32_t side, const float* host, int64_t ld) {
  if (!c || side < 0 || side > 1 || !host || ld < c->dim)
    return fail(c, FRECSYS_ERR_INVALID, "set_gramian: bad arguments");
  HIP_TRY(c, hipSetDevice(c->device));
  int rc = join_eager(c, 1 << side, c->stream);
  if (rc) return rc;
  c->gram_ver[side] = ++c->ver_counter;
  c->gram_src[side] = 0;
  HIP_TRY(c, hipMemsetAsync(c->gram[side], 0, sizeof(float) * c->Dp * c->Dp, c->stream));
  HIP_TRY(c, hipMemcpy2DAsync(c->gram[side], sizeof(float) * c->Dp, host, sizeof(float) * ld,
                              sizeof(float) * c->dim, c->dim, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return FRECSYS_OK;
}

}  // extern "C"

namespace {
// The d-space solve of the queue prefix ap.order[0..ap.n_rows): the tiled
// one-workgroup-per-entity kernels (long histories split) up to Dp = 256,
// the HBM-workspace batches of wide.hip at Dp = 512 / 1024.
// aux (Dp <= 256, optional): an idle stream for the long histories' slabs
// and then their entities' solves, so the slabs run beside the other
// entities' solve instead of before it (s waits for aux at the end).
int launch_dspace(frecsys_ctx* c, SolveArgs ap, const std::vector<int32_t>& hs,
                  const std::function<int64_t(int64_t)>& heff, hipStream_t s,
                  const std::string& pre, bool can_split, int side, bool vq,
                  hipStream_t aux = nullptr) {
  if (wide_dim(c->Dp)) {
    const size_t slot = wide_slot_floats(c->Dp);
    const int64_t budget =
        (int64_t)(ws_budget(c, c->cap_wide_ws * sizeof(float)) / (slot * sizeof(float)));
    int64_t batch = std::max<int64_t>(1, std::min<int64_t>(ap.n_rows, budget));
    int rc = ensure_batch(c, &c->wide_ws, &c->cap_wide_ws, slot, &batch);
    if (rc) return rc;
    if (can_split) {  // long histories of the first batch cut into slabs (a budget of their own)
      const size_t sf = wide_slab_floats(c->Dp);
      rc = plan_split(c, hs, batch, heff, &ap, wide_slab_rows(), sf,
                      (int64_t)(ws_budget(c, c->cap_slabs * sizeof(float)) / (sf * sizeof(float))),
                      s, true);
      if (rc) return rc;
    }
    static const bool wprof = getenv("FRECSYS_DUAL_PROF") != nullptr;
    static unsigned long long* w_prof = nullptr;
    if (wprof && !w_prof) {
      HIP_TRY(c, hipMalloc((void**)&w_prof, sizeof(unsigned long long) * 16));
      HIP_TRY(c, hipMemset(w_prof, 0, sizeof(unsigned long long) * 16));
    }
    ap.prof = wprof ? w_prof : nullptr;
    char* xs = nullptr;
    if (c->wide_presplit && ap.n_rows > 0) {
      // no room for the table: the register-staged SYRK (bit-identical)
      bool oom = false;
      rc = try_ensure(c, &c->wide_xs, &c->cap_wide_xs, wide_xsplit_bytes(c->Dp, ap.n_other), &oom);
      if (rc) return rc;
      if (oom) ++c->ws_shrinks;
      xs = c->wide_xs;
    }
    const size_t k = ktimer_begin(c, pre + ".dspace", s);
    HIP_TRY(c, launch_wide_solve(c->Dp, ap, c->wide_ws, batch, s, xs));
    ktimer_end(c, k, s);
    if (wprof) {  // diagnostics (ablation builds): wide SYRK cycles per chunk and phase
      unsigned long long hp[16];
      HIP_TRY(c, hipStreamSynchronize(s));
      HIP_TRY(c, hipMemcpy(hp, w_prof, sizeof(hp), hipMemcpyDeviceToHost));
      HIP_TRY(c, hipMemset(w_prof, 0, sizeof(hp)));
      for (int pt = 0; pt < 2; ++pt)
        for (int wv = 0; wv < 2; ++wv) {
          const unsigned long long* q = hp + 8 * pt + 4 * wv;
          const double n = (double)std::max<unsigned long long>(q[3], 1);
          fprintf(stderr, "[wide-prof] %s %s wave %d chunks %llu cycles/chunk: mfma+stage %.0f "
                  "ring+loads %.0f barrier %.0f\n", pre.c_str(), pt ? "diag" : "offdiag",
                  wv ? 7 : 0, q[3], q[0] / n, q[1] / n, q[2] / n);
        }
    }
    // SURVEY 8(d) per entity: dspace_syrk_flops + dspace_solve_flops, gather_bytes
    // (empty histories untouched); both linear in h, so from the prefix sums
    const double d = c->dim;
    const HeffSums hsum = heff_sums(c, side, vq, 0, ap.n_rows);
    add_work(c, pre + ".dspace", d * (d + 1.0) * hsum.h1 + hsum.nz * dspace_solve_flops(d),
             (d * 4.0 + 4.0) * hsum.h1 + hsum.nz * (8.0 + d * 4.0), hsum.nz);  // one timed call
    return FRECSYS_OK;
  }
  if (can_split) {
    int rc = plan_split(c, hs, ap.n_rows, heff, &ap, c->split_rows, split_slab_floats(c->Dp),
                        INT64_MAX, s);
    if (rc) return rc;
  }
  const bool side_split = ap.n_work > 0 && aux != nullptr;
  if (side_split) {
    // slabs, then the split entities' solves (they start from the slabs) on
    // aux; the other entities on s meanwhile
    HIP_TRY(c, hipEventRecord(c->ev_fork, s));
    HIP_TRY(c, hipStreamWaitEvent(aux, c->ev_fork, 0));
    const size_t k = ktimer_begin(c, pre + ".split", aux);
    HIP_TRY(c, launch_split_syrk(c->Dp, ap, aux));
    ktimer_end(c, k, aux);
  } else if (ap.n_work > 0) {
    const size_t k = ktimer_begin(c, pre + ".split", s);
    HIP_TRY(c, launch_split_syrk(c->Dp, ap, s));
    ktimer_end(c, k, s);
  }
  static const bool dprof = getenv("FRECSYS_DUAL_PROF") != nullptr;
  static unsigned long long* d_prof = nullptr;
  if (dprof && !d_prof) {
    HIP_TRY(c, hipMalloc((void**)&d_prof, sizeof(unsigned long long) * 16));
    HIP_TRY(c, hipMemset(d_prof, 0, sizeof(unsigned long long) * 16));
  }
  ap.prof = dprof ? d_prof : nullptr;
  const size_t k = ktimer_begin(c, pre + ".dspace", s);
  if (side_split) {
    SolveArgs af = ap;  // queue positions [0, n_split): the split entities
    af.n_rows = ap.n_split;
    HIP_TRY(c, launch_solve(c->Dp, af, aux));
    HIP_TRY(c, hipEventRecord(c->ev_join, aux));
    SolveArgs ar = ap;  // positions [n_split, n_rows)
    ar.order = ap.order + ap.n_split;
    ar.n_rows = ap.n_rows - ap.n_split;
    ar.split = nullptr;
    ar.n_split = 0;
    ar.work = nullptr;
    ar.n_work = 0;
    HIP_TRY(c, launch_solve(c->Dp, ar, s));
    HIP_TRY(c, hipStreamWaitEvent(s, c->ev_join, 0));
  } else {
    HIP_TRY(c, launch_solve(c->Dp, ap, s));
  }
  ktimer_end(c, k, s);
  {  // the split entities' SYRK is the split kernel's work, their solve this one's
    const double d = c->dim;
    const HeffSums sp = heff_sums(c, side, vq, 0, ap.n_split);
    const HeffSums rest = heff_sums(c, side, vq, ap.n_split, ap.n_rows);
    const int64_t ne = sp.nz + rest.nz;
    add_work(c, pre + ".dspace",
             d * (d + 1.0) * rest.h1 + (double)ne * dspace_solve_flops(d),
             (d * 4.0 + 4.0) * rest.h1 + (double)ne * (8.0 + d * 4.0), ne);
    if (ap.n_work > 0)
      add_work(c, pre + ".split", d * (d + 1.0) * sp.h1, (d * 4.0 + 4.0) * sp.h1, sp.nz);
  }
  if (dprof) {  // diagnostics: mean cycles per entity and phase
    unsigned long long hp[16];
    HIP_TRY(c, hipStreamSynchronize(s));
    HIP_TRY(c, hipMemcpy(hp, d_prof, sizeof(hp), hipMemcpyDeviceToHost));
    HIP_TRY(c, hipMemset(d_prof, 0, sizeof(hp)));
    const double n = (double)std::max<unsigned long long>(hp[4], 1);
    fprintf(stderr, "[dspace-prof] %s n %llu mean h %.0f cycles/entity: setup %.0f syrk %.0f "
            "epilogue %.0f (rhs %.0f tiles %.0f) chol %.0f | chain %.0f workers %.0f factored %.0f\n",
            pre.c_str(), hp[4], hp[8] / n, hp[0] / n, hp[1] / n, (hp[2] + hp[9] + hp[10]) / n,
            hp[9] / n, hp[10] / n, hp[3] / n, hp[5] / n, hp[6] / n, hp[7] / n);
    fprintf(stderr, "[dspace-prof] %s chain: waits %.0f trsm %.0f update %.0f factor %.0f | "
            "worker waits %.0f\n",
            pre.c_str(), hp[11] / n, hp[12] / n, hp[13] / n, hp[14] / n, hp[15] / n);
  }
  return FRECSYS_OK;
}

int solve_side_impl(frecsys_ctx* c, int32_t side, const frecsys_solve_params* p,
                    bool force_dspace) {
  if (!c || !valid_side(side) || !p) return fail(c, FRECSYS_ERR_INVALID, "solve: bad arguments");
  if (!c->rp[side]) return fail(c, FRECSYS_ERR_INVALID, "solve: no CSR loaded for side");
  const int kind = p->kind;
  if (kind < FRECSYS_KIND_IALS || kind > FRECSYS_KIND_CVAR_GRAD_V)
    return fail(c, FRECSYS_ERR_INVALID, "solve: bad kind");
  const bool vkind = kind == FRECSYS_KIND_WEIGHTED_V || kind == FRECSYS_KIND_CVAR_GRAD_V;
  const bool ukind = kind == FRECSYS_KIND_WEIGHTED_U || kind == FRECSYS_KIND_CVAR_GRAD_U;
  const bool grad = kind == FRECSYS_KIND_CVAR_GRAD_U || kind == FRECSYS_KIND_CVAR_GRAD_V;
  if (vkind && (!p->entity_reg || !p->other_weight))
    return fail(c, FRECSYS_ERR_INVALID, "solve: V kinds need entity_reg and other_weight");
  if (grad && side == 2) return fail(c, FRECSYS_ERR_INVALID, "solve: CVaR step on EVAL side");
  const int other = side == 1 ? 0 : 1;
  if (p->from_snapshot && !c->snap[other])
    return fail(c, FRECSYS_ERR_INVALID, "solve: from_snapshot without a snapshot");
  HIP_TRY(c, hipSetDevice(c->device));
  int rc = join_eager(c, side < 2 ? 1 << side : 0, c->stream);  // a build still reading emb[side]
  if (rc) return rc;
  if (ukind && p->entity_weight) {
    rc = upload(c, &c->d_entity_weight, &c->cap_entity_weight, p->entity_weight,
                (size_t)c->n[side]);
    if (rc) return rc;
  }
  if (vkind) {
    rc = upload(c, &c->d_entity_reg, &c->cap_entity_reg, p->entity_reg, (size_t)c->n[side]);
    if (rc) return rc;
    rc = upload(c, &c->d_other_weight, &c->cap_other_weight, p->other_weight,
                (size_t)c->n[other]);
    if (rc) return rc;
  }
  int64_t lo, hi;
  shard(c, side, &lo, &hi);
  rc = build_order(c, side);
  if (rc) return rc;
  SolveArgs a{};
  a.kind = kind;
  a.order = c->d_order[side];
  a.counter = c->d_counter;
  a.quirk = c->quirks;
  a.row_ptr = c->rp[side];
  a.col = c->col[side];
  a.row_lo = lo;
  a.n_rows = hi - lo;
  a.X = p->from_snapshot ? c->snap[other] : c->emb[other];
  a.n_other = c->n[other];
  a.G = c->gram[other];
  a.E = c->emb[side];
  a.out = c->emb[side];
  a.reg = p->reg;
  a.reg_exp = p->reg_exp;
  a.w = p->unobserved_weight;
  a.alpha = p->alpha;
  a.eta = p->stepsize;
  a.lambda_is_reg = p->lambda_is_reg;
  a.entity_weight = (ukind && p->entity_weight) ? c->d_entity_weight : nullptr;
  a.entity_reg = vkind ? c->d_entity_reg : nullptr;
  a.other_weight = vkind ? c->d_other_weight : nullptr;
  a.fail = c->d_fail;
  a.split = nullptr;
  a.n_split = 0;
  a.slabs = nullptr;
  a.work = nullptr;
  a.n_work = 0;
  a.debug_skip = c->debug_skip;
  const unsigned long long none = ~0ull;
  // ~0ull by a device-side fill: an H2D copy from host memory at this point
  // was observed starting only after the early basis build queued on another
  // stream had finished, holding back the fork of the d-space solve
  HIP_TRY(c, hipMemsetAsync(c->d_fail, 0xFF, sizeof(none), c->stream));
  // Queue split: the queue is sorted by decreasing history, and h_eff (the
  // rows the assembly reads, tail-quirk rows included) is monotone in h, so
  // the d-space entities are a prefix, then the history-space buckets
  // (32*(t-1) < h_eff <= 32*t, t = 8..1), then the empty histories.
  const std::vector<int32_t>& hs = c->order_h[side];
  auto heff = [&](int64_t h) -> int64_t {
    return (vkind && c->quirks && h > 128 && (h % 128) != 0) ? h + 128 - (h % 128) : h;
  };
  auto first_le = [&](int64_t lim) {  // first queue index with h_eff <= lim
    return (int64_t)(std::partition_point(hs.begin(), hs.end(),
                                          [&](int32_t h) { return heff(h) > lim; }) -
                     hs.begin());
  };
  // The history-space form needs M = mu*G + lam*I SPD for every entity:
  // lam > 0 and mu >= 0 (G is PSD).  Otherwise (and when it reports a
  // non-positive pivot) the call runs the d-space solve for everyone.
  bool m_spd = p->reg > 0.0f && p->unobserved_weight >= 0.0f;
  if (m_spd && ukind && p->entity_weight)
    for (int64_t i = 0; i < c->n[side] && m_spd; ++i) m_spd = p->entity_weight[i] >= 0.0f;
  if (m_spd && vkind && !p->lambda_is_reg) {
    const float base = p->alpha * p->unobserved_weight * (float)c->n[other];
    for (int64_t i = 0; i < c->n[side] && m_spd; ++i) m_spd = p->entity_reg[i] + base > 0.0f;
  }
  const bool dual = c->dual_on && !force_dspace && m_spd && !grad && c->Dp >= 64 &&
                    c->dual_max_h_side[side] > 0 && (int64_t)hs.size() == c->order_n[side];
  const int64_t n_dspace = dual ? first_le(c->dual_max_h_side[side]) : a.n_rows;
  c->dual_used[side] = dual;
  if (side < 2) emb_written(c, side);
  const int64_t n_nonempty = dual ? first_le(0) : a.n_rows;
  {
    static const char* names[3] = {"solve_user", "solve_item", "solve_eval"};
    const std::string pre = names[side];
    ScopedTimer t(c, names[side]);
    if (!dual || n_dspace >= n_nonempty) {
      // stream2 (the mixed path's d-space stream) is idle here: the slabs of
      // the long histories run on it beside the other entities' solve
      rc = launch_dspace(c, a, hs, heff, c->stream, pre,
                         c->Dp >= 32 && (int64_t)hs.size() == c->order_n[side], side, vkind,
                         c->dual_serial ? nullptr : c->stream2);
      if (rc) return rc;
    } else {
      // d-space solve of the long histories on stream2, concurrently with
      // the basis change + history-space solve of the rest on stream
      // the basis (one-workgroup tridiagonalisation first) is queued before
      // the d-space kernels so its workgroup is not left waiting for a CU
      // behind them; stream2 waits only for what preceded the fork
      hipStream_t s2 = c->dual_serial ? c->stream : c->stream2;
      if (n_dspace > 0) HIP_TRY(c, hipEventRecord(c->ev_fork, c->stream));
      // one M = mu*G + lam*I for every entity (iALS with l2_reg_exp = 0, or
      // lambda = reg: ials.h:310-315): the Cholesky basis, no tridiagonal
      // reduction, no per-entity LDL -- at every Dp the history space runs
      // at (64..256, 512, 1024: chol_basis_kernel<T>, launch_chol_basis)
      int bmode = 0;
      float bmu = 0.f, blam = 0.f;
      if (c->chol_basis_on && kind == FRECSYS_KIND_IALS &&
          (p->lambda_is_reg || p->reg_exp == 0.0f)) {
        bmode = 1;
        bmu = p->unobserved_weight;
        blam = p->reg;
      }
      c->want_mode[other] = bmode;
      c->want_mu[other] = bmu;
      c->want_lam[other] = blam;
      const QueueRec* hrows = nullptr;
      int64_t nhrows = 0;
      uint64_t hsub = 0;
      rc = hspace_rows(c, side, other, n_dspace, n_nonempty, &hrows, &nhrows, &hsub);
      if (rc) return rc;
      size_t k = ktimer_begin(c, pre + ".basis", c->stream);
      rc = prepare_basis(c, other, a.X, c->stream, bmode, bmu, blam, hrows, nhrows, hsub);
      if (rc) return rc;
      ktimer_end(c, k, c->stream);
      if (n_dspace > 0) {
        HIP_TRY(c, hipStreamWaitEvent(s2, c->ev_fork, 0));
        SolveArgs ap = a;
        ap.n_rows = n_dspace;
        rc = launch_dspace(c, ap, hs, heff, s2, pre, true, side, vkind);
        if (rc) return rc;
        HIP_TRY(c, hipEventRecord(c->ev_join, s2));
      }
      DualArgs d{};
      d.kind = kind;
      d.quirk = c->quirks;
      d.Dp = c->Dp;
      d.col = a.col;
      d.Xrot = c->xrot[other];
      d.tdiag = c->tri[other];
      d.toff = c->tri[other] + c->Dp;
      d.unit_m = bmode;
      d.basis_status = c->tri[other];
      d.n_other = a.n_other;
      d.reg = a.reg;
      d.reg_exp = a.reg_exp;
      d.w = a.w;
      d.alpha = a.alpha;
      d.lambda_is_reg = a.lambda_is_reg;
      d.entity_weight = a.entity_weight;
      d.entity_reg = a.entity_reg;
      d.other_weight = a.other_weight;
      d.fail = a.fail;
      d.debug_skip = a.debug_skip;
      static const bool dprof = getenv("FRECSYS_DUAL_PROF") != nullptr;
      unsigned long long*& d_prof = g_dual_prof;
      if (dprof && !d_prof) {
        HIP_TRY(c, hipMalloc((void**)&d_prof, sizeof(unsigned long long) * 16 * 9));
        HIP_TRY(c, hipMemset(d_prof, 0, sizeof(unsigned long long) * 16 * 9));
      }
      const int64_t n_hs = n_nonempty - n_dspace;
      const size_t n_blk = (size_t)((n_hs + 63) / 64) * 64;  // position-blocked buffers
      rc = ensure(c, &c->dual_table, &c->cap_dual_table, n_blk * 3 * c->Dp);
      if (rc) return rc;
      rc = ensure(c, &c->out_rot[side], &c->cap_out_rot[side], n_blk * c->Dp);
      if (rc) return rc;
      d.out_rot = c->out_rot[side];
      k = ktimer_begin(c, pre + ".hspace", c->stream);
      d.order = a.order + n_dspace;
      d.n_rows = n_hs;
      d.table = c->dual_table;
      d.pos0 = 0;
      HIP_TRY(c, launch_dual_ldl(d, c->stream));
      // buckets in two lanes (the long ones on stream, the short ones on
      // stream3) so one bucket's tail and resource shape overlap another's
      const bool two_lanes = !c->dual_serial;
      if (two_lanes) {
        HIP_TRY(c, hipEventRecord(c->ev_fork3, c->stream));
        HIP_TRY(c, hipStreamWaitEvent(c->stream3, c->ev_fork3, 0));
      }
      int64_t lo = n_dspace;
      if (c->dual_max_h_side[side] > 32 * kDualMaxTiles && lo < n_nonempty) {
        // the wide bucket, 256 < h_eff <= 512, in batches of its workspace
        const int64_t hi = std::min(n_nonempty, first_le(32 * kDualMaxTiles));
        const size_t per = dual_wide_zs_bytes(c->Dp) + sizeof(float) * (dual_wide_slot_floats() + 512);
        const size_t held = c->cap_dw_zs + sizeof(float) * (c->cap_dw_slots + c->cap_dw_z);
        int64_t nbat = std::max<int64_t>(
            1, std::min<int64_t>(hi - lo, (int64_t)(ws_budget(c, held) / per)));
        if (hi > lo) {
          rc = ensure_batch(c, &c->dw_zs, &c->cap_dw_zs, dual_wide_zs_bytes(c->Dp), &nbat);
          if (rc) return rc;
          rc = ensure_batch(c, &c->dw_slots, &c->cap_dw_slots, dual_wide_slot_floats(), &nbat);
          if (rc) return rc;
          rc = ensure_batch(c, &c->dw_z, &c->cap_dw_z, (size_t)512, &nbat);
          if (rc) return rc;
        }
        for (int64_t b0 = lo; b0 < hi; b0 += nbat) {
          d.order = a.order + b0;
          d.n_rows = std::min(nbat, hi - b0);
          d.pos0 = b0 - n_dspace;
          d.prof = nullptr;
          HIP_TRY(c, launch_dual_wide(d, c->dw_zs, c->dw_slots, c->dw_z, a.fail, c->stream));
        }
        lo = std::max(lo, hi);
      }
      for (int tiles = kDualMaxTiles; tiles >= 1 && lo < n_nonempty; --tiles) {
        const int64_t hi = std::min(n_nonempty, first_le(32 * (tiles - 1)));
        if (hi > lo) {
          d.order = a.order + lo;
          d.n_rows = hi - lo;
          d.pos0 = lo - n_dspace;
          d.prof = dprof ? d_prof + 16 * tiles : nullptr;
          hipStream_t ls = (two_lanes && tiles <= 4) ? c->stream3 : c->stream;
          HIP_TRY(c, launch_dual(tiles, d, ls));
        }
        lo = std::max(lo, hi);
      }
      if (two_lanes) {
        HIP_TRY(c, hipEventRecord(c->ev_join3, c->stream3));
        HIP_TRY(c, hipStreamWaitEvent(c->stream, c->ev_join3, 0));
      }
      d.order = a.order + n_dspace;
      d.n_rows = n_hs;
      d.pos0 = 0;
      if (!bmode) HIP_TRY(c, launch_dual_sweep(d, c->stream));  // unit table: identity
      ktimer_end(c, k, c->stream);
      {  // h x h system per entity: S = I + Z D^-1 Z^T (h^2 d), its LLT (h^3 / 3),
         // the recurrence and Y^T z (4 h d); rows read twice, the LDL row
        const double dd = c->dim;
        const HeffSums hsum = heff_sums(c, side, vkind, n_dspace, n_nonempty);
        const double ne = (double)(n_nonempty - n_dspace);
        add_work(c, pre + ".hspace", hsum.h2 * dd + hsum.h3 / 3.0 + 4.0 * hsum.h1 * dd,
                 (2.0 * dd * 4.0 + 4.0) * hsum.h1 + ne * (8.0 + 3.0 * dd * 4.0 + dd * 4.0),
                 n_nonempty - n_dspace);
      }
      k = ktimer_begin(c, pre + ".rotate", c->stream);
      HIP_TRY(c, launch_rotate(c->out_rot[side], a.order + n_dspace, 0, n_nonempty - n_dspace,
                               c->qsplit[other][1], a.out, c->Dp, c->stream, 1));
      ktimer_end(c, k, c->stream);
      if (n_dspace > 0) HIP_TRY(c, hipStreamWaitEvent(c->stream, c->ev_join, 0));
    }
    t.stop();
  }
  const bool collective = side < 2 && c->comm;
  if (collective) {
    // every rank takes the same retry / NOT_SPD decision below (the
    // smallest failing entity over all ranks), so the collectives of a
    // rerun stay matched
    NCCL_TRY(c, ncclAllReduce(c->d_fail, c->d_fail, 1, ncclUint64, ncclMin, c->comm, c->stream));
  }
  unsigned long long f = none;
  HIP_TRY(c, hipMemcpyAsync(&f, c->d_fail, sizeof(f), hipMemcpyDeviceToHost, c->stream));
  if (side < 2 && (c->world > 1 || c->comm)) {
    ScopedTimer t(c, "allgather");
    rc = allgather_rows(c, c->emb[side], side, c->Dp);
    if (rc) return rc;
    t.stop();
  }
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  flush_ktimers(c);
  if (getenv("FRECSYS_DUAL_PROF") && dual && g_dual_prof) {
    // diagnostics: mean cycles per entity and phase of the workgroup kernel
    unsigned long long hp[16 * 9];
    HIP_TRY(c, hipMemcpy(hp, g_dual_prof, sizeof(hp), hipMemcpyDeviceToHost));
    HIP_TRY(c, hipMemset(g_dual_prof, 0, sizeof(hp)));
    for (int t = 1; t <= 8; ++t) {
      const unsigned long long n = hp[16 * t + 4];
      if (!n) continue;
      fprintf(stderr, "[dual-prof] side %d tiles %d n %llu cycles/entity: setup %.0f slabs %.0f chol %.0f "
              "yz %.0f | chain %.0f workers %.0f factored %.0f\n", side, t, n,
              (double)hp[16 * t] / n, (double)hp[16 * t + 1] / n, (double)hp[16 * t + 2] / n,
              (double)hp[16 * t + 3] / n, (double)hp[16 * t + 5] / n, (double)hp[16 * t + 6] / n,
              (double)hp[16 * t + 7] / n);
    }
  }
  if (f != none && c->debug_skip) {
    // ablation builds only (FRECSYS_DEBUG_SKIP): the skipped phases leave
    // garbage matrices by design, so a failed pivot is expected and ignored
    // -- a timing run must reach the end of the epoch, not abort on NOT_SPD
    return FRECSYS_OK;
  }
  if (f != none && dual && (collective || n_dspace < n_nonempty)) {
    // a history-space pivot failed (or a poisoned basis after a tagged-poll
    // timeout): the verdict is the d-space solve's.  Counted (frecsys_counter
    // "hspace_reruns"): the whole side pays a d-space solve
    ++c->hspace_reruns;
    return solve_side_impl(c, side, p, true);
  }
  if (f != none) {
    c->err_entity = (int64_t)f - 1;
    return fail(c, FRECSYS_ERR_NOT_SPD,
                "LLT failed (matrix not SPD) for entity " + std::to_string(c->err_entity));
  }
  return FRECSYS_OK;
}

}  // namespace

extern "C" {

int frecsys_solve_side(frecsys_ctx* c, int32_t side, const frecsys_solve_params* p) {
  return solve_side_impl(c, side, p, false);
}

int frecsys_user_loss(frecsys_ctx* c, int32_t side, float beta, int32_t half, float* host_out) {
  if (!c || (side != 0 && side != 2)) return fail(c, FRECSYS_ERR_INVALID, "loss: bad side");
  if (!c->rp[side]) return fail(c, FRECSYS_ERR_INVALID, "loss: no CSR loaded");
  HIP_TRY(c, hipSetDevice(c->device));
  const size_t rows = (size_t)c->n[side];
  const bool fresh = c->cap_loss < rows || !c->d_loss;
  int rc = ensure(c, &c->d_loss, &c->cap_loss, rows);
  if (rc) return rc;
  if (fresh || side == 2)
    HIP_TRY(c, hipMemsetAsync(c->d_loss, 0, sizeof(float) * std::max<size_t>(rows, 1), c->stream));
  int64_t lo, hi;
  shard(c, side, &lo, &hi);
  // Dp = 64..256: u^T G u by the rotation kernel (column-block partials; it
  // measured faster than quad_kernel's f32 MFMA, which keeps the other widths)
  const bool qr = !wide_dim(c->Dp) && c->Dp >= 64 && c->Dp % 32 == 0;
  rc = ensure(c, &c->d_quad, &c->cap_quad,
              std::max<size_t>(wide_dim(c->Dp) ? wide_quad_floats(c->Dp, hi - lo)
                               : qr ? (size_t)rotate_quad_parts(c->Dp) * (size_t)(hi - lo)
                                    : rows,
                               1));
  if (rc) return rc;
  LossArgs a{};
  a.quad = c->d_quad;
  a.quad_parts = qr ? rotate_quad_parts(c->Dp) : 0;
  if (wide_dim(c->Dp) || qr) {
    if (!c->gsplit) HIP_TRY(c, hipMalloc(&c->gsplit, basis_split_bytes(c->Dp)));
    a.gsplit = c->gsplit;
  }
  a.row_ptr = c->rp[side];
  a.col = c->col[side];
  a.row_lo = lo;
  a.n_rows = hi - lo;
  a.U = c->emb[side];
  a.V = c->emb[1];
  a.G = c->gram[1];
  a.beta = beta;
  a.half = half;
  a.out = c->d_loss;
  {
    // user_loss: both kernels; user_loss.gather: the gather kernel alone (its
    // own rate for the loss_gather roofline)
    frecsys_ctx::Pending g{"user_loss.gather", pool_event(c), pool_event(c)};
    a.ev_gather = c->Dp > 16 ? g.a : nullptr;
    ScopedTimer t(c, "user_loss");
    HIP_TRY(c, launch_user_loss(c->Dp, a, c->stream));
    if (a.ev_gather) {
      (void)hipEventRecord(g.b, c->stream);
      c->pending.push_back(g);
    } else {
      c->event_pool.push_back(g.a);
      c->event_pool.push_back(g.b);
    }
    t.stop();
    flush_ktimers(c);
  }
  if (side == 0) {  // gather of the item rows + u^T G u: SURVEY 8(d) bytes with a 1-float output
    const std::vector<int64_t>& rp = c->host_rp[0];
    const double nnz = rp.empty() ? 0.0 : (double)(rp[hi] - rp[lo]), n = (double)(hi - lo);
    const double dd = c->dim;
    add_work(c, "user_loss", 2.0 * nnz * dd + 2.0 * n * dd * dd,
             nnz * dd * 4.0 + nnz * 4.0 + (n + 1.0) * 8.0 + n * 4.0, hi - lo);
  }
  if (host_out) {
    if (side == 0 && (c->world > 1 || c->comm)) {
      rc = allgather_rows(c, c->d_loss, 0, 1);
      if (rc) return rc;
    }
    if (rows)
      HIP_TRY(c, hipMemcpyAsync(host_out, c->d_loss, sizeof(float) * rows, hipMemcpyDeviceToHost,
                                c->stream));
  }
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return FRECSYS_OK;
}

int frecsys_eval_topk(frecsys_ctx* c, int32_t k, int32_t* topk) {
  if (!c || !topk) return fail(c, FRECSYS_ERR_INVALID, "eval_topk: bad arguments");
  if (!c->rp[2] || !c->emb[2]) return fail(c, FRECSYS_ERR_INVALID, "eval_topk: no EVAL side loaded");
  const int64_t n = c->n[2], m = c->n[1];
  if (k < 1 || k > 1024 || k > m)
    return fail(c, FRECSYS_ERR_INVALID, "eval_topk: k must be in [1, min(1024, items)]");
  if (n == 0) return FRECSYS_OK;
  HIP_TRY(c, hipSetDevice(c->device));
  // scores in batches of rows bounded to 1 GiB of workspace
  const int64_t nb = std::max<int64_t>(1, std::min<int64_t>(n, ((int64_t)1 << 28) / m));
  int rc = ensure(c, &c->d_scores, &c->cap_scores, (size_t)nb * m);
  if (rc) return rc;
  rc = ensure(c, &c->d_topk, &c->cap_topk, (size_t)n * k);
  if (rc) return rc;
  {
    ScopedTimer t(c, "eval_topk");
    for (int64_t r0 = 0; r0 < n; r0 += nb) {
      const int64_t cnt = std::min(nb, n - r0);
      HIP_TRY(c, launch_eval_topk(c->emb[2], r0, cnt, c->emb[1], m, c->Dp, c->rp[2], c->col[2], k,
                                  c->d_scores, c->d_topk + r0 * k, c->stream));
    }
    t.stop();
  }
  HIP_TRY(c, hipMemcpyAsync(topk, c->d_topk, sizeof(int32_t) * n * k, hipMemcpyDeviceToHost,
                            c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return FRECSYS_OK;
}

int frecsys_pp_set_rating_index(frecsys_ctx* c, int32_t side, const int32_t* rix) {
  if (!c || (side != 0 && side != 1) || !rix)
    return fail(c, FRECSYS_ERR_INVALID, "pp_set_rating_index: bad arguments");
  if (!c->rp[side]) return fail(c, FRECSYS_ERR_INVALID, "pp_set_rating_index: no CSR");
  HIP_TRY(c, hipSetDevice(c->device));
  const int64_t nnz = c->nnz[side];
  for (int64_t k = 0; k < nnz; ++k)
    if (rix[k] < 0 || rix[k] >= nnz)
      return fail(c, FRECSYS_ERR_INVALID, "pp_set_rating_index: index out of range");
  if (c->d_rix[side]) HIP_TRY(c, hipFree(c->d_rix[side]));
  c->d_rix[side] = nullptr;
  HIP_TRY(c, hipMalloc((void**)&c->d_rix[side], sizeof(int32_t) * std::max<int64_t>(nnz, 1)));
  if (nnz)
    HIP_TRY(c, hipMemcpy(c->d_rix[side], rix, sizeof(int32_t) * nnz, hipMemcpyHostToDevice));
  return ensure(c, &c->d_pred[0], &c->cap_pred[0], (size_t)std::max<int64_t>(nnz, 1));
}

namespace {
PPArgs pp_args(frecsys_ctx* c, int side) {
  const int other = side == 1 ? 0 : 1;
  PPArgs a{};
  a.col = c->col[side];
  a.rix = side == 2 ? nullptr : c->d_rix[side];
  a.pred = c->d_pred[side == 2 ? 1 : 0];
  a.X = c->emb[other];
  a.G = c->gram[other];
  a.E = c->emb[side];
  a.Dp = c->Dp;
  a.n_other = c->n[other];
  a.fail = c->d_fail;
  return a;
}
}  // namespace

int frecsys_pp_predict(frecsys_ctx* c, int32_t side) {
  if (!c || (side != 0 && side != 2)) return fail(c, FRECSYS_ERR_INVALID, "pp_predict: bad side");
  if (!c->rp[side]) return fail(c, FRECSYS_ERR_INVALID, "pp_predict: no CSR");
  if (side == 0 && !c->d_rix[0])
    return fail(c, FRECSYS_ERR_INVALID, "pp_predict: no rating index (pp_set_rating_index)");
  if (c->pp_old_side != -1)  // the other ranks' updates of the last block are not in yet
    return fail(c, FRECSYS_ERR_INVALID, "pp_predict: pp_sync pending for the last sharded block step");
  HIP_TRY(c, hipSetDevice(c->device));
  if (side == 2) {
    int rc = ensure(c, &c->d_pred[1], &c->cap_pred[1], (size_t)std::max<int64_t>(c->nnz[2], 1));
    if (rc) return rc;
  }
  PPArgs a = pp_args(c, side);
  HIP_TRY(c, launch_pp_predict(a, c->rp[side], c->n[side], c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return FRECSYS_OK;
}

int frecsys_pp_step(frecsys_ctx* c, int32_t side, int32_t start, int32_t end,
                    const frecsys_solve_params* p, double* residual) {
  if (!c || !valid_side(side) || !p) return fail(c, FRECSYS_ERR_INVALID, "pp_step: bad arguments");
  if (start < 0 || end > c->dim || end - start < 1 || end - start > 128)
    return fail(c, FRECSYS_ERR_INVALID, "pp_step: block must satisfy 0 <= start < end <= dim, "
                                        "end - start <= 128");
  if (!c->rp[side]) return fail(c, FRECSYS_ERR_INVALID, "pp_step: no CSR");
  if (side != 2 && !c->d_rix[side])
    return fail(c, FRECSYS_ERR_INVALID, "pp_step: no rating index (pp_set_rating_index)");
  if (!c->d_pred[side == 2 ? 1 : 0])
    return fail(c, FRECSYS_ERR_INVALID, "pp_step: no prediction vector (pp_predict)");
  const int kind = p->kind;
  if (kind != FRECSYS_KIND_IALS && kind != FRECSYS_KIND_WEIGHTED_U &&
      kind != FRECSYS_KIND_WEIGHTED_V)
    return fail(c, FRECSYS_ERR_INVALID, "pp_step: kind must be IALS, WEIGHTED_U or WEIGHTED_V");
  if (kind == FRECSYS_KIND_WEIGHTED_V && (!p->entity_reg || !p->other_weight))
    return fail(c, FRECSYS_ERR_INVALID, "pp_step: WEIGHTED_V needs entity_reg and other_weight");
  // external-exchange mode: a second step before frecsys_pp_sync would
  // overwrite the snapshot the other ranks' prediction updates are replayed
  // from, and this rank's predictions would drift from theirs
  if (c->pp_old_side != -1)
    return fail(c, FRECSYS_ERR_INVALID, "pp_step: pp_sync pending for the last sharded block step");
  HIP_TRY(c, hipSetDevice(c->device));
  const int other = side == 1 ? 0 : 1;
  {
    int rc = join_eager(c, 3, c->stream);
    if (rc) return rc;
  }
  if (side < 2) emb_written(c, side);
  if (kind == FRECSYS_KIND_WEIGHTED_U && p->entity_weight) {
    int rc = upload(c, &c->d_entity_weight, &c->cap_entity_weight, p->entity_weight,
                    (size_t)c->n[side]);
    if (rc) return rc;
  }
  if (kind == FRECSYS_KIND_WEIGHTED_V) {
    int rc = upload(c, &c->d_entity_reg, &c->cap_entity_reg, p->entity_reg, (size_t)c->n[side]);
    if (rc) return rc;
    rc = upload(c, &c->d_other_weight, &c->cap_other_weight, p->other_weight,
                (size_t)c->n[other]);
    if (rc) return rc;
  }
  // world > 1 (USER / ITEM): this rank's shard of the rows -- the per-row
  // block steps are independent given the predictions, which every rank then
  // brings up to date for the other ranks' rows (pp_refresh_kernel, bitwise
  // the owner's update); EVAL rows are not sharded
  const bool sharded = side < 2 && c->world > 1;
  const bool xchg = sharded && in_call_exchange(c);  // RCCL or the caller's transport
  int64_t lo = 0, hi = c->n[side];
  if (sharded) shard(c, side, &lo, &hi);
  const int bw = end - start;
  if (sharded) {  // the block columns before the step: the refresh replays Delta from them
    int rc = ensure(c, &c->d_pp_old, &c->cap_pp_old,
                    (size_t)std::max<int64_t>(c->n[side], 1) * bw);
    if (rc) return rc;
    if (c->n[side])
      HIP_TRY(c, hipMemcpy2DAsync(c->d_pp_old, sizeof(float) * bw, c->emb[side] + start,
                                  sizeof(float) * c->Dp, sizeof(float) * bw, c->n[side],
                                  hipMemcpyDeviceToDevice, c->stream));
  }
  std::vector<QueueRec> recs((size_t)(hi - lo));
  const std::vector<int64_t>& rp = side == 2 ? c->host_rp_eval : c->host_rp[side];
  for (int64_t i = lo; i < hi; ++i) recs[i - lo] = QueueRec{(int32_t)i, (int32_t)(rp[i + 1] - rp[i]), rp[i]};
  std::stable_sort(recs.begin(), recs.end(),
                   [](const QueueRec& x, const QueueRec& y) { return x.h > y.h; });
  QueueRec* d_q = nullptr;
  HIP_TRY(c, hipMalloc((void**)&d_q, sizeof(QueueRec) * std::max<size_t>(recs.size(), 1)));
  HIP_TRY(c, hipMemcpyAsync(d_q, recs.data(), sizeof(QueueRec) * recs.size(), hipMemcpyHostToDevice,
                            c->stream));
  int rc = ensure(c, &c->d_resid, &c->cap_resid, std::max<size_t>(recs.size(), 1));
  if (rc) return rc;
  PPArgs a = pp_args(c, side);
  a.order = d_q;
  a.n_rows = (int64_t)recs.size();
  a.start = start;
  a.bw = end - start;
  a.kind = kind;
  a.reg = p->reg;
  a.reg_exp = p->reg_exp;
  a.w = p->unobserved_weight;
  a.alpha = p->alpha;
  a.entity_weight =
      (kind == FRECSYS_KIND_WEIGHTED_U && p->entity_weight) ? c->d_entity_weight : nullptr;
  a.entity_reg = kind == FRECSYS_KIND_WEIGHTED_V ? c->d_entity_reg : nullptr;
  a.other_weight = kind == FRECSYS_KIND_WEIGHTED_V ? c->d_other_weight : nullptr;
  a.resid = c->d_resid;
  const unsigned long long none = ~0ull;
  // ~0ull by a device-side fill: an H2D copy from host memory at this point
  // was observed starting only after the early basis build queued on another
  // stream had finished, holding back the fork of the d-space solve
  HIP_TRY(c, hipMemsetAsync(c->d_fail, 0xFF, sizeof(none), c->stream));
  {
    ScopedTimer t(c, "pp_step");
    HIP_TRY(c, launch_pp_step(a, c->stream));
    if (sharded && !xchg) {  // the caller exchanges the rows, then frecsys_pp_sync
      c->pp_old_side = side;
      c->pp_old_start = start;
      c->pp_old_bw = bw;
    }
    if (xchg) {
      // the rows of every rank, then the other ranks' prediction updates
      rc = xchg_rows(c, c->emb[side], side, c->Dp);
      if (rc) return rc;
      HIP_TRY(c, launch_pp_refresh(a, c->rp[side], c->d_pp_old, c->n[side], lo, hi, c->stream));
    }
    t.stop();
  }
  if (xchg) {  // every rank takes the same NOT_SPD verdict
    rc = xchg_min_u64(c, c->d_fail);
    if (rc) return rc;
  }
  std::vector<float> res(recs.size());
  unsigned long long f = none;
  HIP_TRY(c, hipMemcpyAsync(&f, c->d_fail, sizeof(f), hipMemcpyDeviceToHost, c->stream));
  if ((residual || xchg) && !recs.empty())
    HIP_TRY(c, hipMemcpyAsync(res.data(), c->d_resid, sizeof(float) * recs.size(),
                              hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  HIP_TRY(c, hipFree(d_q));
  if (f != none) {
    c->err_entity = (int64_t)(f - 1);
    return fail(c, FRECSYS_ERR_NOT_SPD, "pp_step: block matrix not SPD");
  }
  double s = 0.0;
  if (xchg) {
    // every rank's per-row residuals (all-gathered as a one-column table,
    // whether or not this rank asked for the sum: the ranks' exchanges stay
    // in step), summed in the single-rank queue order -- every row of the
    // side by decreasing h: the world-1 sum bit for bit
    const int64_t n = c->n[side];
    std::vector<int32_t>& all = c->pp_order_all[side];
    if ((int64_t)all.size() != n) {
      all.resize((size_t)n);
      for (int64_t i = 0; i < n; ++i) all[i] = (int32_t)i;
      std::stable_sort(all.begin(), all.end(), [&](int32_t x, int32_t y) {
        return rp[x + 1] - rp[x] > rp[y + 1] - rp[y];
      });
    }
    std::vector<float> ent((size_t)std::max<int64_t>(n, 1), 0.0f);
    for (size_t i = 0; i < recs.size(); ++i) ent[recs[i].entity] = res[i];
    rc = ensure(c, &c->d_resid_e, &c->cap_resid_e, (size_t)std::max<int64_t>(n, 1));
    if (rc) return rc;
    if (n) HIP_TRY(c, hipMemcpyAsync(c->d_resid_e, ent.data(), sizeof(float) * n,
                                     hipMemcpyHostToDevice, c->stream));
    rc = xchg_rows(c, c->d_resid_e, side, 1);
    if (rc) return rc;
    if (n) HIP_TRY(c, hipMemcpyAsync(ent.data(), c->d_resid_e, sizeof(float) * n,
                                     hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    for (int32_t e : all) s += (double)ent[e];
  } else {
    for (float v : res) s += (double)v;  // zero rows (empty histories) stay 0
  }
  if (residual) *residual = s;
  return FRECSYS_OK;
}

int frecsys_pp_get_predictions(frecsys_ctx* c, int32_t side, float* host) {
  if (!c || (side != 0 && side != 2) || !host)
    return fail(c, FRECSYS_ERR_INVALID, "pp_get_predictions: bad arguments");
  const float* p = c->d_pred[side == 2 ? 1 : 0];
  if (!p) return fail(c, FRECSYS_ERR_INVALID, "pp_get_predictions: no prediction vector");
  HIP_TRY(c, hipSetDevice(c->device));
  const int64_t nnz = c->nnz[side];
  if (nnz)
    HIP_TRY(c, hipMemcpyAsync(host, p, sizeof(float) * nnz, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return FRECSYS_OK;
}

int frecsys_set_transport(frecsys_ctx* c, const frecsys_transport* t) {
  if (!c) return FRECSYS_ERR_INVALID;
  if (t && (!t->allgather_rows || !t->allreduce_min_u64))
    return fail(c, FRECSYS_ERR_INVALID, "set_transport: every callback is required");
  if (c->pp_old_side != -1)
    return fail(c, FRECSYS_ERR_INVALID, "set_transport: pp_sync pending");
  c->has_transport = t != nullptr;
  c->transport = t ? *t : frecsys_transport{};
  return FRECSYS_OK;
}

int frecsys_pp_sync(frecsys_ctx* c, int32_t side) {
  if (!c || (side != 0 && side != 1)) return fail(c, FRECSYS_ERR_INVALID, "pp_sync: bad side");
  if (c->pp_old_side != side)
    return fail(c, FRECSYS_ERR_INVALID, "pp_sync: no sharded block step of this side pending");
  HIP_TRY(c, hipSetDevice(c->device));
  int64_t lo, hi;
  shard(c, side, &lo, &hi);
  PPArgs a = pp_args(c, side);
  a.start = c->pp_old_start;
  a.bw = c->pp_old_bw;
  HIP_TRY(c, launch_pp_refresh(a, c->rp[side], c->d_pp_old, c->n[side], lo, hi, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  c->pp_old_side = -1;
  return FRECSYS_OK;
}

int frecsys_train_stats(frecsys_ctx* c, double* observed, double* unobserved,
                        float* user_norm2, float* item_norm2) {
  if (!c) return fail(c, FRECSYS_ERR_INVALID, "train_stats: null ctx");
  if (observed && !c->rp[0]) return fail(c, FRECSYS_ERR_INVALID, "train_stats: no USER CSR");
  HIP_TRY(c, hipSetDevice(c->device));
  const int64_t nu = c->n[0], ni = c->n[1];
  const int Dp = c->Dp;
  int rc = ensure(c, &c->d_rows, &c->cap_rows, (size_t)std::max<int64_t>(std::max(nu, ni), 1));
  if (rc) return rc;
  ScopedTimer t(c, "train_stats");
  if (observed) {
    LossArgs a{};
    a.row_ptr = c->rp[0];
    a.col = c->col[0];
    a.row_lo = 0;
    a.n_rows = nu;
    a.U = c->emb[0];
    a.V = c->emb[1];
    a.G = c->gram[1];
    a.out = c->d_rows;
    a.raw = 1;
    HIP_TRY(c, hipMemsetAsync(c->d_rows, 0, sizeof(float) * std::max<int64_t>(nu, 1), c->stream));
    HIP_TRY(c, launch_user_loss(Dp, a, c->stream));
    std::vector<float> h((size_t)nu);
    if (nu)
      HIP_TRY(c, hipMemcpyAsync(h.data(), c->d_rows, sizeof(float) * nu, hipMemcpyDeviceToHost,
                                c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    double s = 0.0;
    for (float v : h) s += (double)v;
    *observed = s;
  }
  if (unobserved) {
    rc = ensure(c, &c->d_gstat, &c->cap_gstat, (size_t)2 * Dp * Dp);
    if (rc) return rc;
    rc = ensure(c, &c->d_dot, &c->cap_dot, 1);
    if (rc) return rc;
    for (int s = 0; s < 2; ++s) {
      rc = form_gramian(c, 2, c->emb[s], c->n[s], nullptr, c->d_gstat + (size_t)s * Dp * Dp, true);
      if (rc) return rc;
    }
    HIP_TRY(c, launch_gram_dot(c->d_gstat, c->d_gstat + (size_t)Dp * Dp, Dp, c->d_dot, c->stream));
    HIP_TRY(c, hipMemcpyAsync(unobserved, c->d_dot, sizeof(double), hipMemcpyDeviceToHost,
                              c->stream));
  }
  for (int s = 0; s < 2; ++s) {
    float* host = s == 0 ? user_norm2 : item_norm2;
    if (!host || c->n[s] == 0) continue;
    HIP_TRY(c, launch_row_norm2(c->emb[s], c->n[s], Dp, c->d_rows, c->stream));
    HIP_TRY(c, hipMemcpyAsync(host, c->d_rows, sizeof(float) * c->n[s], hipMemcpyDeviceToHost,
                              c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
  }
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  t.stop();
  return FRECSYS_OK;
}

int frecsys_synchronize(frecsys_ctx* c) {
  if (!c) return FRECSYS_ERR_INVALID;
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, hipStreamSynchronize(c->stream5));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return FRECSYS_OK;
}

int frecsys_release_workspaces(frecsys_ctx* c) {
  if (!c) return FRECSYS_ERR_INVALID;
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, hipStreamSynchronize(c->stream5));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  auto rel = [&](auto** p, size_t* cap) -> int {
    if (*p) HIP_TRY(c, hipFree(*p));
    *p = nullptr;
    *cap = 0;
    return FRECSYS_OK;
  };
  int rc = rel(&c->wide_ws, &c->cap_wide_ws);
  if (!rc) rc = rel(&c->wide_xs, &c->cap_wide_xs);
  if (!rc) rc = rel(&c->d_slabs, &c->cap_slabs);
  if (!rc) rc = rel(&c->dw_zs, &c->cap_dw_zs);
  if (!rc) rc = rel(&c->dw_slots, &c->cap_dw_slots);
  if (!rc) rc = rel(&c->dw_z, &c->cap_dw_z);
  return rc;
}

int frecsys_timing(const frecsys_ctx* c, const char* what, double* total_ms, int64_t* launches) {
  if (!c || !what) return FRECSYS_ERR_INVALID;
  auto it = c->timers.find(what);
  if (total_ms) *total_ms = it == c->timers.end() ? 0.0 : it->second.total_ms;
  if (launches) *launches = it == c->timers.end() ? 0 : it->second.launches;
  return FRECSYS_OK;
}

int frecsys_work(const frecsys_ctx* c, const char* what, double* flops, double* bytes,
                 int64_t* entities, int64_t* launches) {
  if (!c || !what) return FRECSYS_ERR_INVALID;
  auto it = c->work.find(what);
  const Work w = it == c->work.end() ? Work{} : it->second;
  if (flops) *flops = w.flops;
  if (bytes) *bytes = w.bytes;
  if (entities) *entities = w.entities;
  if (launches) *launches = w.launches;
  return FRECSYS_OK;
}

int frecsys_debug_diag_factor(frecsys_ctx* c, int32_t blocked, int32_t n_tiles, const float* a,
                              float* linv, int32_t* ok) {
  if (!c || n_tiles < 0 || (n_tiles && (!a || !linv || !ok)))
    return fail(c, FRECSYS_ERR_INVALID, "debug_diag_factor: bad arguments");
  if (n_tiles == 0) return FRECSYS_OK;
  HIP_TRY(c, hipSetDevice(c->device));
  float *dA = nullptr, *dL = nullptr;
  int* dok = nullptr;
  const size_t bytes = sizeof(float) * 1024 * (size_t)n_tiles;
  HIP_TRY(c, hipMalloc((void**)&dA, bytes));
  HIP_TRY(c, hipMalloc((void**)&dL, bytes));
  HIP_TRY(c, hipMalloc((void**)&dok, sizeof(int) * (size_t)n_tiles));
  HIP_TRY(c, hipMemcpyAsync(dA, a, bytes, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, launch_debug_diag(dA, dL, dok, n_tiles, blocked ? 1 : 0, c->stream));
  HIP_TRY(c, hipMemcpyAsync(linv, dL, bytes, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipMemcpyAsync(ok, dok, sizeof(int) * (size_t)n_tiles, hipMemcpyDeviceToHost,
                            c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  HIP_TRY(c, hipFree(dA));
  HIP_TRY(c, hipFree(dL));
  HIP_TRY(c, hipFree(dok));
  return FRECSYS_OK;
}

int frecsys_debug_basis(frecsys_ctx* c, int32_t side, float* q, float* diag, float* sub) {
  if (!c || side < 0 || side > 1 || !q || !diag || !sub)
    return fail(c, FRECSYS_ERR_INVALID, "debug_basis: bad arguments");
  if (c->Dp < 64) return fail(c, FRECSYS_ERR_UNSUPPORTED, "debug_basis: Dp < 64");
  HIP_TRY(c, hipSetDevice(c->device));
  int rc = prepare_basis(c, side, c->emb[side], c->stream);
  if (rc) return rc;
  const size_t Dp = (size_t)c->Dp;
  HIP_TRY(c, hipMemcpyAsync(q, c->q[side], sizeof(float) * Dp * Dp, hipMemcpyDeviceToHost,
                            c->stream));
  HIP_TRY(c, hipMemcpyAsync(diag, c->tri[side], sizeof(float) * Dp, hipMemcpyDeviceToHost,
                            c->stream));
  HIP_TRY(c, hipMemcpyAsync(sub, c->tri[side] + Dp, sizeof(float) * Dp, hipMemcpyDeviceToHost,
                            c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return FRECSYS_OK;
}

int32_t frecsys_history_space_max_h(const frecsys_ctx* c) {
  return c && c->dual_on && c->Dp >= 64 ? c->dual_max_h : 0;
}

int32_t frecsys_history_space_max_h_side(const frecsys_ctx* c, int32_t side) {
  if (!c || !c->dual_on || c->Dp < 64 || (side != FRECSYS_SIDE_USER && side != FRECSYS_SIDE_ITEM))
    return 0;
  return c->dual_max_h_side[side];
}

int frecsys_counter(frecsys_ctx* c, const char* what, int64_t* value) {
  if (!c || !what || !value) return fail(c, FRECSYS_ERR_INVALID, "counter: bad arguments");
  if (!strcmp(what, "hspace_reruns")) {
    *value = c->hspace_reruns;
    return FRECSYS_OK;
  }
  if (!strcmp(what, "ws_shrinks")) {
    *value = c->ws_shrinks;
    return FRECSYS_OK;
  }
  if (!strcmp(what, "tagged_timeouts")) {
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipStreamSynchronize(c->stream5));
    unsigned ev[4] = {0, 0, 0, 0};
    HIP_TRY(c, hipMemcpyAsync(ev, c->d_events, sizeof(ev), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    *value = (int64_t)ev[0];
    return FRECSYS_OK;
  }
  return fail(c, FRECSYS_ERR_INVALID, std::string("counter: unknown counter ") + what);
}

int frecsys_snapshot_residual(frecsys_ctx* c, int32_t side, double* sq) {
  if (!c || side < 0 || side > 1 || !sq) return fail(c, FRECSYS_ERR_INVALID, "snapshot_residual: bad arguments");
  if (!c->snap[side]) return fail(c, FRECSYS_ERR_INVALID, "snapshot_residual: no snapshot taken");
  HIP_TRY(c, hipSetDevice(c->device));
  const int64_t n = c->n[side];
  int rc = ensure(c, &c->d_rows, &c->cap_rows, (size_t)std::max<int64_t>(n, 1));
  if (rc) return rc;
  *sq = 0.0;
  if (n == 0) return FRECSYS_OK;
  HIP_TRY(c, launch_row_diff2(c->emb[side], c->snap[side], n, c->Dp, c->d_rows, c->stream));
  std::vector<float> h((size_t)n);
  HIP_TRY(c, hipMemcpyAsync(h.data(), c->d_rows, sizeof(float) * n, hipMemcpyDeviceToHost,
                            c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  double s = 0.0;
  for (float v : h) s += (double)v;
  *sq = s;
  return FRECSYS_OK;
}

int frecsys_timing_reset(frecsys_ctx* c) {
  if (!c) return FRECSYS_ERR_INVALID;
  c->timers.clear();
  c->work.clear();
  return FRECSYS_OK;
}

}  // extern "C"
