// wide.h -- helpers shared by the wide-dimension kernels (Dp = 512 / 1024):
// wide.hip (Gramian, Cholesky, tridiagonalisation, the register-staged SYRK)
// and wide_syrk.hip (the SYRK from the pre-split table).  Internal header.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.h"

namespace frecsys_hip {

// History position of virtual assembly row k: rows past h are the ProjectV
// tail quirk's re-read of the last h % 128 rows (safer2.h:181-199).
__device__ __forceinline__ int64_t wide_virt_pos(int64_t k, int64_t h) {
  return k < h ? k : (h - 128 + (k - h));
}

// XCD-aware grid: workgroup b runs on XCD b % 8 (round-robin dispatch), so
// the P workgroups of one unit (entity / slab / row block) are given
// consecutive slots of ONE XCD's sequence -- they run together and the unit's
// rows are fetched from HBM once into that XCD's L2 instead of once per
// workgroup.  Placement is a speed matter only: nothing depends on it.
__device__ __forceinline__ bool xcd_unit(int P, int64_t n_units, int64_t& unit, int& pidx) {
  const int64_t bid = blockIdx.x;
  const int64_t s = bid >> 3;
  pidx = (int)(s % P);
  unit = (s / P) * 8 + (bid & 7);
  return unit < n_units;
}
inline unsigned xcd_grid(int64_t n_units, int P) {
  return (unsigned)(((n_units + 7) / 8) * 8 * P);
}

// rows of one two-level accumulation block of the wide SYRKs: 128 chunks of
// 16 rows summed from zero, then added into the unit's output tiles (the
// long-history slab size, wide_slab_rows())
constexpr int kWideChunk = 16;
constexpr int kWideFlush = 128;

// ---- the pre-split copy of the other side (wide_syrk.hip) ----
// Row r: the three bf16 pieces (hi, mid, lo; common.h split3) of
// x~ = sa_r * X[r] (sa_r = sqrt(nu_r) for the V kinds, else 1), each Dp
// values, then a 128-B tail whose first float is the rhs weight nu_r / sa_r
// (V kinds).  Row n_other is all zero: the rows past a unit's end read it.
__host__ __device__ inline int64_t wide_xsplit_row_bytes(int Dp) { return 6 * (int64_t)Dp + 128; }
inline size_t wide_xsplit_bytes(int Dp, int64_t n_other) {
  return (size_t)(n_other + 1) * (size_t)wide_xsplit_row_bytes(Dp);
}
// The pre-split table of a.X (with a.other_weight for the V kinds) into xs.
hipError_t launch_wide_presplit(int Dp, const SolveArgs& a, char* xs, hipStream_t s);
// MODE 2: the long-history slabs a.work[0..n_work); MODE 1: entities
// a.order[pos0 .. pos0 + n) into the workspace ws (a.xsplit set).
hipError_t launch_wide_syrk3(int Dp, const SolveArgs& a, int mode, int64_t pos0, int64_t n,
                             float* ws, hipStream_t s);

}  // namespace frecsys_hip
