// kernels.h -- launch interface between the C-ABI host code (capi.hip) and
// the gfx950 kernels (solve.hip, gramian.hip, loss.hip).  Internal header.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace frecsys_hip {

// One entry of the solve queue: entity row, its history length and the
// offset of its history in the CSR column array (16 B, one load).
struct QueueRec {
  int32_t entity;
  int32_t h;
  int64_t p0;
};

// One partial SYRK of a long history: queue position, virtual history
// positions [k0, k1), output slab.
struct SplitWork {
  int32_t pos;
  int32_t k0;
  int32_t k1;
  int32_t slab;
};

// Everything one launch of the per-entity solve needs (device pointers).
struct SolveArgs {
  int kind;                 // FRECSYS_KIND_*
  int quirk;                // reproduce the ProjectV tail double-count
  const int64_t* row_ptr;   // CSR of the solved side
  const int32_t* col;
  int64_t row_lo;           // first entity of this launch (small kernel)
  int64_t n_rows;           // entities in this launch
  const QueueRec* order;    // [n_rows] longest history first (tiled kernel)
  unsigned int* counter;    // work-queue head, zeroed by the launcher
  const float* X;           // other side's embeddings, ld = Dp
  int64_t n_other;          // rows of the other side (for lambda)
  const float* G;           // Dp x Dp Gramian of the other side
  const float* E;           // current embeddings of the solved side (CVaR)
  float* out;               // solved side's embeddings, ld = Dp
  float reg, reg_exp, w, alpha, eta;
  int lambda_is_reg;           // lambda = reg for every entity
  const float* entity_weight;  // [rows of side] omega, or nullptr (-> 1)
  const float* entity_reg;     // [rows of side] item_reg_
  const float* other_weight;   // [rows of other side] nu
  unsigned long long* fail;    // atomicMin(entity + 1) on a non-SPD pivot
  int debug_skip;              // diagnostic ablation mask (0 in production)
  unsigned long long* prof;    // diagnostics: per-phase cycle sums [16] (nullptr = off)
  // long-history split (tiled and wide kernels; nullptr / 0 = none)
  const int2* split;           // [n_split] per queue position: first slab, slab count
  int64_t n_split;
  float* slabs;                // [slabs][split_slab_floats(Dp)]
  const SplitWork* work;       // [n_work] partial SYRK items
  int64_t n_work;
  // wide dims: the pre-split copy of X (wide.h wide_xsplit_*), or nullptr
  const char* xsplit;
};

// Partition-independent Gramian.  The rows of a side are cut
// into fixed leaves (rows per leaf from the side's row count alone) and the
// leaves into ngroup = min(kGramGroups, leaves) runs of consecutive leaves.
// A leaf's partial is one workgroup's fixed-order accumulation, a group's
// slab the sum of its leaves in leaf order, and G the sum of the group slabs
// in group order: the same additions whichever rank computes which group, so
// G is bitwise the same at every world size (ranks own whole groups and
// exchange group slabs, never partially reduced sums).
constexpr int kGramGroups = 16;
struct GramPlan {
  int64_t n = 0;        // rows of the side
  int64_t rpl = 0;      // rows per leaf
  int64_t nleaf = 0;
  int ngroup = 0;
  size_t slab_floats = 0;  // floats of one leaf / group slab (lower tiles, or Dp^2 at Dp <= 16)
};
GramPlan gram_plan(int Dp, int64_t n);
inline int64_t gram_group_leaf(const GramPlan& p, int g) {
  return p.ngroup ? (int64_t)g * p.nleaf / p.ngroup : 0;
}
// Groups [lo, hi) of rank `rank` of `world` (contiguous, balanced by count).
inline void gram_owned_groups(const GramPlan& p, int world, int rank, int* lo, int* hi) {
  *lo = (int)((int64_t)p.ngroup * rank / world);
  *hi = (int)((int64_t)p.ngroup * (rank + 1) / world);
}
// Leaf-workspace floats for computing groups [g_lo, g_hi).
size_t gram_leaf_floats(const GramPlan& p, int g_lo, int g_hi);

struct GramArgs {
  const float* X;        // ld = Dp
  const float* w;        // per-row weight (absolute row index) or nullptr
  float* partials;       // leaf workspace (gram_leaf_floats)
  float* gslabs;         // [plan.ngroup][plan.slab_floats] group slabs
  GramPlan plan;
  int g_lo, g_hi;        // groups this launch computes
  // set by the launcher: rows [row0, row0 + n) = the leaves of the groups
  int64_t row0;
  int64_t n;
};

struct LossArgs {
  const int64_t* row_ptr;
  const int32_t* col;
  int64_t row_lo, n_rows;
  const float* U;        // ld = Dp (rows of the side)
  const float* V;        // items, ld = Dp
  const float* G;        // Dp x Dp
  float beta;
  int half;
  float* out;            // [rows of side]
  float* quad;           // [rows of side] scratch: u^T G u (Dp >= 32); with quad_parts > 0
                         // [quad_parts][n_rows] partial sums by launch row (rotate_quad)
  int quad_parts;
  void* gsplit;          // Dp = 512 / 1024: scratch for G's split image (basis_split_bytes)
  int raw;               // 1: out[e] = sum_j (x_j . u - 1)^2 only (train stats)
  hipEvent_t ev_gather;  // recorded right before the gather kernel (timing), or nullptr
};


// History-space ("dual") solve of the short-history entities (dual.hip).
// With G = Q T Q^T (Q orthogonal, T tridiagonal) and M = mu*G + lam*I,
// A = M + Xt^T Xt, b = Xt^T s  (Xt = the history rows scaled by sqrt of
// their A-weight, s = the matching rhs coefficients) is solved as
//   x = Q (mu*T + lam*I)^-1 Y^T z,  z = (I + Y (mu*T + lam*I)^-1 Y^T)^-1 s,
// Y = Xt Q (push-through identity): an h x h SPD system instead of d x d.
struct DualArgs {
  int kind;                 // FRECSYS_KIND_IALS / WEIGHTED_U / WEIGHTED_V
  int quirk;
  int Dp;
  const QueueRec* order;    // [n_rows] this launch's entities
  int64_t n_rows;
  const int32_t* col;       // CSR columns of the solved side
  const float* Xrot;        // other side rotated into the T basis: X Q, ld Dp
  const float* tdiag;       // [Dp] diagonal of T
  const float* toff;        // [Dp] T(k+1, k)
  // Cholesky basis (launch_chol_basis: one M for every entity, Xrot = X L^-T):
  // the LDL table is the unit one and *basis_status = 0 fails the launch
  int unit_m;
  const float* basis_status;
  int64_t n_other;
  // position-blocked buffers (64 positions per block, k-major inside a
  // block: every access by consecutive positions is coalesced), position =
  // pos0 + index in this launch's order slice:
  //   out_rot[blk][k][64]     Y^T (c.*z), then x'
  //   table[blk][3][Dp][64]   l_k, D^-1/2, D^-1 of mu*T + lam*I
  float* out_rot;
  float* table;
  int64_t pos0;
  float reg, reg_exp, w, alpha;
  int lambda_is_reg;
  const float* entity_weight;
  const float* entity_reg;
  const float* other_weight;
  unsigned long long* fail;
  int debug_skip;  // ablation only: 1 SYRK, 2/4/8/16 Cholesky parts, 64 Y^T z, 128 recurrence
  unsigned long long* prof;  // diagnostics: per-phase cycle sums [16] (nullptr = off)
};

// Largest history-space tile count built (h_eff <= 32 * kDualMaxTiles).
constexpr int kDualMaxTiles = 8;

hipError_t launch_solve(int Dp, const SolveArgs& a, hipStream_t s);
// Diagnostics: n 32x32 tiles (row-major) -> L^-1 of each (blk: the
// MFMA-blocked diagonal factor, else the lane recurrence), ok[n].
hipError_t launch_debug_diag(const float* A, float* Linv, int* ok, int n, int blk, hipStream_t s);
// Partial SYRKs of the split entities (a.work[0..n_work)) into a.slabs.
hipError_t launch_split_syrk(int Dp, const SolveArgs& a, hipStream_t s);
size_t split_slab_floats(int Dp);
// LDL^T of every entity's tridiagonal mu*T + lam*I (one thread per entity,
// a.order[0..n_rows)) into a.table.
hipError_t launch_dual_ldl(const DualArgs& a, hipStream_t s);
// out_rot rows of a.order[0..n_rows): v -> L^-T D^-1 L^-1 v (one thread per
// entity, table rows as written by launch_dual_ldl).
hipError_t launch_dual_sweep(const DualArgs& a, hipStream_t s);
// One launch per history bucket: every entity of a.order has
// 32*(tiles-1) < h_eff <= 32*tiles.
hipError_t launch_dual(int tiles, const DualArgs& a, hipStream_t s);
// The wide bucket (dual.hip): 256 < h_eff <= 512 at Dp = 512 / 1024, the
// entities a.order[0..n_rows) (positions a.pos0..) through HBM workspaces:
// zs (dual_wide_zs_bytes per entity), slots (dual_wide_slot_floats per
// entity), zbuf (512 floats per entity); Cholesky failures into fail.
constexpr int kDualWideMaxH = 512;
size_t dual_wide_zs_bytes(int Dp);
size_t dual_wide_slot_floats();
hipError_t launch_dual_wide(const DualArgs& a, void* zs, float* slots, float* zbuf,
                            unsigned long long* fail, hipStream_t s);
// wide_chol_kernel<16> over n Cholesky slots (row-major 32 x 32 tiles of a
// 512 x 512 SPD matrix + its rhs): solution of slot i into out[512 i ..),
// a failure reported as order[i].entity; only the tiles holding the
// h_eff = order[i].h (+ the tail quirk's rows when quirk_v) rows are factored.
hipError_t launch_wide_chol_slots(const QueueRec* order, int64_t n, float* slots, float* out,
                                  unsigned long long* fail, int quirk_v, hipStream_t s);
// Householder tridiagonalisation G = Q T Q^T of a Dp x Dp symmetric matrix
// (one workgroup): T's diagonal / subdiagonal, the reflectors (row k of Vh,
// entries k+1..Dp-1) and their tau.  With Q (only when tridiag_forms_q(Dp)):
// Q itself too, row-major, formed by workgroups of the same launch as the
// reflectors are published (work: tridiag_work_floats(Dp)), and with
// img_q / img_qt the split images of Q and Q^T (launch_split_basis's layout).
hipError_t launch_tridiag(const float* G, int Dp, float* tdiag, float* toff, float* Vh,
                          float* tau, hipStream_t s, float* work = nullptr, float* Q = nullptr,
                          void* img_q = nullptr, void* img_qt = nullptr,
                          unsigned* tcount = nullptr);
bool tridiag_forms_q(int Dp);
size_t tridiag_work_floats(int Dp);
// Q = H_0 H_1 ... H_{Dp-3} from the reflectors, row-major Dp x Dp; with
// img_q / img_qt also the split images of Q and Q^T (launch_split_basis's
// layout, basis_split_bytes each; Dp a multiple of 32).
hipError_t launch_form_q(const float* Vh, const float* tau, int Dp, float* Q, hipStream_t s,
                         void* img_q = nullptr, void* img_qt = nullptr);
// The split image of B = (trans ? Q^T : Q) for launch_rotate: Dp * Dp * 3
// bf16 (16-B granules in MFMA fragment order).
size_t basis_split_bytes(int Dp);
hipError_t launch_split_basis(const float* Q, int Dp, int trans, void* out, hipStream_t s);
// Cholesky basis of M = mu*G + lam*I (one workgroup): XT = L^-T (Dp x Dp,
// row-major, upper triangular) with M = L L^T; status[0] = 1, or 0 on a
// non-positive pivot.  work: chol_basis_work_floats(Dp).  Dp = 64..256, 512,
// 1024 (T = 32: 7 staging tiles beside the 31-tile panel in the 160 KB of
// LDS, spectral.hip chol_basis_stage_tiles).
size_t chol_basis_work_floats(int Dp);
hipError_t launch_chol_basis(const float* G, int Dp, float mu, float lam, float* work, float* XT,
                             float* status, hipStream_t s);
// Y[row] = X[row] * B with B given by its split image (launch_split_basis),
// fp32-accurate products on the bf16 matrix cores,
// for rows r0..r0+n-1, or for the entities rows[0..n) when rows != nullptr
// (Y: ld Dp; X: ld Dp, or with x_blocked the position-blocked layout of
// DualArgs::out_rot, X row r = position r).  Dp = 64 .. 256, 512, 1024.
// Rows of the other side that a side's history-space entities read (the
// forward rotation's subset): mark[col[p]] = 1 over their histories.
hipError_t launch_mark_rows(const QueueRec* order, int64_t n, const int32_t* col, uint8_t* mark,
                            hipStream_t s);
hipError_t launch_rotate(const float* X, const QueueRec* rows, int64_t r0, int64_t n,
                         const void* bsplit, float* Y, int Dp, hipStream_t s, int x_blocked = 0);
// Dp = 512 / 1024: qpart[b * n + r] = sum over the columns of 128-block b of
// (X B)[r] .* X[r] for rows r0 .. r0+n-1 (u^T G u partials, B = G).
hipError_t launch_rotate_quad(const float* X, int64_t r0, int64_t n, const void* bsplit,
                              float* qpart, int Dp, hipStream_t s);
// Column blocks (partial sums per row) launch_rotate_quad writes at Dp.
int rotate_quad_parts(int Dp);

__host__ __device__ inline int64_t blk_v(int64_t p, int k, int Dp) {
  return ((p >> 6) * Dp + k) * 64 + (p & 63);
}
__host__ __device__ inline int64_t blk_t(int64_t p, int j, int k, int Dp) {
  return ((p >> 6) * 3 * Dp + j * Dp + k) * 64 + (p & 63);
}
// The leaves of groups [a.g_lo, a.g_hi) into a.partials, each group summed
// into its slab a.gslabs[g].
hipError_t launch_gramian(int Dp, const GramArgs& a, hipStream_t s);
// G = sum of the plan's group slabs in group order, mirrored (Dp x Dp).
hipError_t launch_gram_final(int Dp, const GramPlan& p, const float* gslabs, float* G,
                             hipStream_t s);

// iALS++ block step (pp.hip; ialspp.h:85-145, 351-424).
struct PPArgs {
  const QueueRec* order;    // entities of the launch (LPT order)
  int64_t n_rows;
  const int32_t* col;       // CSR columns of the solved side
  const int32_t* rix;       // rating index per CSR entry (nullptr: the CSR position)
  float* pred;              // prediction vector, by rating index
  const float* X;           // other side, ld Dp
  const float* G;           // Gramian of the other side, Dp x Dp
  float* E;                 // solved side, ld Dp (block updated in place)
  int Dp, start, bw;        // block columns [start, start + bw), bw <= 128
  int kind;                 // KIND_IALS (iALS++), KIND_WEIGHTED_U / _V (SAFER2++)
  float reg, reg_exp, w, alpha;
  const float* entity_weight;  // U: omega (nullptr -> 1)
  const float* entity_reg;     // V: item_reg_
  const float* other_weight;   // V: nu_u = omega_u / |H_u|
  int64_t n_other;
  float* resid;             // [n_rows] squared delta norms, or nullptr
  unsigned long long* fail;
};
// Sharded block step: the prediction updates of rows [0, n) outside [lo, hi)
// replayed from old ([n][bw], the block before the step) and a.E (after).
hipError_t launch_pp_refresh(const PPArgs& a, const int64_t* row_ptr, const float* old,
                             int64_t n, int64_t lo, int64_t hi, hipStream_t s);
hipError_t launch_pp_step(const PPArgs& a, hipStream_t s);
// PredictDataset over the CSR rows 0..n_rows-1 (E = the rows' embeddings).
hipError_t launch_pp_predict(const PPArgs& a, const int64_t* row_ptr, int64_t n_rows,
                             hipStream_t s);

// Fold-in scoring + top-k (topk.hip): rows r0..r0+n-1 of X against the m
// rows of Y; S: [n][m] workspace; out: [n][k].
hipError_t launch_eval_topk(const float* X, int64_t r0, int64_t n, const float* Y, int64_t m,
                            int Dp, const int64_t* row_ptr, const int32_t* col, int k, float* S,
                            int32_t* out, hipStream_t s);

// Wide dims, Dp = 512 / 1024 (wide.hip).  d-space solve with A in an HBM
// workspace ([batch][wide_slot_floats(Dp)]), entities a.order[0..n_rows)
// in batches; Gramian by 128x128 block pairs; per-step tridiagonalisation
// (work: wide_tridiag_work_floats); rotations; user loss (a.quad holds
// wide_quad_floats partials).
bool wide_dim(int Dp);
size_t wide_slot_floats(int Dp);
// Long-history split of the wide d-space SYRK: entities of the first batch
// with more than 2 * wide_slab_rows() assembly rows have their SYRK cut into
// slabs of wide_slab_rows() (the two-level accumulation block, so the slab
// sums fold into exactly the unsplit result) in a.work / a.split / a.slabs
// ([slabs][wide_slab_floats(Dp)]), computed by their own workgroups first.
int64_t wide_slab_rows();
size_t wide_slab_floats(int Dp);
int64_t wide_rows_per_leaf(int64_t n);
// Leaves of g (rows [g.row0, g.row0 + g.n), leaf size g.plan.rpl) into g.partials.
hipError_t launch_wide_gram_leaves(int Dp, const GramArgs& g, hipStream_t s);
hipError_t launch_wide_gram_final(int Dp, const float* gslabs, int64_t ngroup, float* G,
                                  hipStream_t s);
// xsplit: a buffer of wide_xsplit_bytes(Dp, a.n_other) (wide.h) for the SYRK
// from the pre-split table, or nullptr for the register-staged SYRK
hipError_t launch_wide_solve(int Dp, const SolveArgs& a, float* ws, int64_t batch,
                             hipStream_t s, char* xsplit = nullptr);
size_t wide_tridiag_work_floats(int Dp);
bool wide_tridiag_tagged();
hipError_t launch_wide_tridiag(const float* G, int Dp, float* tdiag, float* toff, float* Vh,
                               float* tau, float* work, hipStream_t s, float* Q = nullptr,
                               void* img_q = nullptr, void* img_qt = nullptr,
                               unsigned* tcount = nullptr);
size_t wide_quad_floats(int Dp, int64_t rows);
hipError_t launch_wide_user_loss(int Dp, const LossArgs& a, hipStream_t s);
hipError_t launch_user_loss(int Dp, const LossArgs& a, hipStream_t s);
hipError_t launch_zero_gram(int Dp, float* G, hipStream_t s);
// Train-loss diagnostics: out[r] = ||X[r]||^2 for n rows; dot = sum_ij A_ij B_ij
// (double, Dp x Dp).
hipError_t launch_row_norm2(const float* X, int64_t n, int Dp, float* out, hipStream_t s);
// ||X[r] - Y[r]||^2 per row (the print_residual_stats norms)
hipError_t launch_row_diff2(const float* X, const float* Y, int64_t n, int Dp, float* out,
                            hipStream_t s);
hipError_t launch_gram_dot(const float* A, const float* B, int Dp, double* dot, hipStream_t s);

// Padded leading dimension for a logical dimension (8, 16, multiples of 32
// up to 256, then 512 and 1024).  Returns 0 when unsupported.
int padded_dim(int dim);
// true (default): the SYRK kernels run fp32-accurate split-bf16 MFMA
// (common.h mfma_x6); FRECSYS_SYRK_F32=1 selects v_mfma_f32_32x32x2_f32.
bool syrk_split_bf16();
// true when a gather over `rows` rows of ld Dp needs 64-bit element offsets
// (rows * Dp >= 2^32), or FRECSYS_GATHER64=1 forces them (tests: the two
// widths are bit-identical).
bool gather_off64(int64_t rows, int Dp);

}  // namespace frecsys_hip
