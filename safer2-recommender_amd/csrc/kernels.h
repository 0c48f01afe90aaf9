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
};

struct GramArgs {
  const float* X;        // ld = Dp
  int64_t row0;          // first row
  int64_t n;             // rows
  const float* w;        // per-row weight (absolute row index) or nullptr
  float* partials;       // workspace
  float* G;              // Dp x Dp output (full, symmetric)
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
};

// Number of workgroups / partial slabs the Gramian of n rows uses.
int64_t gram_num_blocks(int Dp, int64_t n);
// Partial workspace floats needed for n rows at padded dim Dp.
size_t gram_workspace_floats(int Dp, int64_t n);

hipError_t launch_solve(int Dp, const SolveArgs& a, hipStream_t s);
hipError_t launch_gramian(int Dp, const GramArgs& a, hipStream_t s);
hipError_t launch_user_loss(int Dp, const LossArgs& a, hipStream_t s);
hipError_t launch_zero_gram(int Dp, float* G, hipStream_t s);

// Padded leading dimension for a logical dimension (8, 16, then multiples
// of 32 up to 256).  Returns 0 when unsupported.
int padded_dim(int dim);

}  // namespace frecsys_hip
