// gramian.hip -- G = X^T diag(w) X on gfx950.
//
// Replaces Eigen's dense GEMM `X.transpose() * X` (ials.h:321, ials.h:371,
// safer2.h:55, safer2.h:294-295) and the weighted `U^T (U .* omega)`
// (safer2.h:504-509).  Dense and regular, so it is the one MFMA-shaped op of
// the loop: split-K over row blocks, each workgroup accumulating the lower
// 32x32 tiles of its block with v_mfma_f32_32x32x2_f32 (rows staged through
// LDS by coalesced float4 loads), one partial slab per leaf of rows; the
// leaves of a group are summed in leaf order into the group's slab, and the
// group slabs in group order into G, mirrored (kernels.h GramPlan: the leaf
// and group cuts depend only on the row count, so the sum is the same at
// every world size).  Deterministic, no atomics.  Dp = 8, 16 use a VALU path.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "common.h"
#include "kernels.h"

namespace frecsys_hip {

namespace {

template <int T>
struct GramCfg {
  static constexpr int Dp = 32 * T;
  static constexpr int NT = T * (T + 1) / 2;
  static constexpr int NW = (T <= 2) ? 4 : 8;
  static constexpr int NTHR = NW * 64;
  static constexpr int MT = (NT + NW - 1) / NW;
  static constexpr int R = 32;
  static constexpr int NSLOT = R * Dp / 4;
  static constexpr int NQ = (NSLOT + NTHR - 1) / NTHR;
};

constexpr int kMaxBlocks = 512;

int64_t rows_per_block(int64_t n) {
  int64_t rpb = (n + kMaxBlocks - 1) / kMaxBlocks;
  if (rpb < 64) rpb = 64;
  return (rpb + 31) / 32 * 32;
}

template <int T>
__global__ void __launch_bounds__(GramCfg<T>::NTHR)
    gram_tiled_kernel(GramArgs a, int64_t rpb) {
  using C = GramCfg<T>;
  constexpr int Dp = C::Dp, NT = C::NT, NW = C::NW, NTHR = C::NTHR, MT = C::MT;
  constexpr int R = C::R, NQ = C::NQ, NSLOT = C::NSLOT;
  __shared__ __attribute__((aligned(16))) float stage[2][R * Dp];
  __shared__ float wsc[2][R];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lo = lane & 31, hi = lane >> 5;
  const int64_t r0 = a.row0 + (int64_t)blockIdx.x * rpb;
  int64_t r1 = r0 + rpb;
  if (r1 > a.row0 + a.n) r1 = a.row0 + a.n;
  const int nchunks = (int)((r1 - r0 + R - 1) / R);

  float4 regs[NQ];
  float wreg = 0.0f;
  auto load = [&](int c) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int sidx = tid + q * NTHR;
      regs[q] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (NSLOT % NTHR == 0 || sidx < NSLOT) {
        const int64_t row = r0 + (int64_t)c * R + sidx / (Dp / 4);
        if (row < r1)
          regs[q] = *reinterpret_cast<const float4*>(a.X + row * Dp + 4 * (sidx % (Dp / 4)));
      }
    }
    if (tid < R) {
      const int64_t row = r0 + (int64_t)c * R + tid;
      wreg = (row < r1) ? (a.w ? a.w[row] : 1.0f) : 0.0f;
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int sidx = tid + q * NTHR;
      if (NSLOT % NTHR == 0 || sidx < NSLOT)
        *reinterpret_cast<float4*>(&stage[buf][4 * sidx]) = regs[q];
    }
    if (tid < R) wsc[buf][tid] = wreg;
  };

  f32x16 acc[MT];
  int aoff[MT], boff[MT];
  bool valid[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    acc[m] = f32x16{0.f};
    const int t = wave + m * NW;
    valid[m] = t < NT;
    int I = 0;
    while ((I + 1) * (I + 2) / 2 <= t) ++I;
    const int J = t - I * (I + 1) / 2;
    aoff[m] = 32 * I + lo;
    boff[m] = 32 * J + lo;
  }
  if (nchunks > 0) {
    load(0);
    store(0);
  }
  __syncthreads();
  for (int c = 0; c < nchunks; ++c) {
    const int buf = c & 1;
    const bool more = c + 1 < nchunks;
    if (more) load(c + 1);
#pragma unroll 4
    for (int s = 0; s < R / 2; ++s) {
      const float* rowp = &stage[buf][(2 * s + hi) * Dp];
      const float wr = wsc[buf][2 * s + hi];
#pragma unroll
      for (int m = 0; m < MT; ++m)
        if (valid[m]) acc[m] = mfma32(rowp[aoff[m]], rowp[boff[m]] * wr, acc[m]);
    }
    if (more) store(buf ^ 1);
    __syncthreads();
  }
  float* P = a.partials + (int64_t)blockIdx.x * NT * 1024;
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    if (valid[m]) {
      const int I = (aoff[m] - lo) >> 5, J = (boff[m] - lo) >> 5;
      float* tile = P + tidx(I, J) * 1024;
#pragma unroll
      for (int q = 0; q < 16; ++q) tile[acc_row(q, hi) * 32 + lo] = acc[m][q];
    }
  }
}

// Sum of the nblk partial slabs, four consecutive elements (one float4) of
// the lower tiles per output.  The blocks are cut into kRedChains contiguous
// ranges summed as independent chains -- one thread per (chain, float4), so
// 8 x NT workgroups share the read (bandwidth-, not latency-bound: 36 one-
// chain-set workgroups left 220 CUs idle, 102 us) -- then combined in chain
// order through LDS: a fixed order, so the result is deterministic.  Then
// mirrored into G.
constexpr int kRedChains = 8;
template <int T>
__global__ void __launch_bounds__(256)
    gram_reduce_kernel(const float* __restrict__ P, int64_t nblk, float* __restrict__ G) {
  constexpr int Dp = 32 * T, NT = T * (T + 1) / 2, QW = 256 / kRedChains;
  __shared__ float4 part[kRedChains][QW];
  const int c = threadIdx.x / QW, qq = threadIdx.x % QW;
  const int q = blockIdx.x * QW + qq;  // float4 index within a slab (NT * 256 is a multiple of QW)
  const int64_t stride = (int64_t)NT * 1024;
  const int64_t per = (nblk + kRedChains - 1) / kRedChains;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int64_t i = 0; i < per; ++i) {
    const int64_t b = c * per + i;
    if (b < nblk) {
      const float4 v = reinterpret_cast<const float4*>(P + b * stride)[q];
      acc.x += v.x;
      acc.y += v.y;
      acc.z += v.z;
      acc.w += v.w;
    }
  }
  part[c][qq] = acc;
  __syncthreads();
  if (c != 0) return;
  float4 s = part[0][qq];
#pragma unroll
  for (int k = 1; k < kRedChains; ++k) {
    const float4 v = part[k][qq];
    s.x += v.x;
    s.y += v.y;
    s.z += v.z;
    s.w += v.w;
  }
  const int t = q >> 8, e0 = (q & 255) * 4;  // tile, first element (row-major 32 x 32)
  int I = 0;
  while ((I + 1) * (I + 2) / 2 <= t) ++I;
  const int J = t - I * (I + 1) / 2;
  const float sv[4] = {s.x, s.y, s.z, s.w};
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int gi = 32 * I + ((e0 + u) >> 5), gj = 32 * J + ((e0 + u) & 31);
    if (gi < gj) continue;  // diagonal tiles: the lower half only
    G[gi * Dp + gj] = sv[u];
    G[gj * Dp + gi] = sv[u];
  }
}

// Dp = 8, 16: thread (i, j) of one Dp x Dp partial per workgroup.
template <int Dp>
__global__ void __launch_bounds__(256) gram_small_kernel(GramArgs a, int64_t rpb) {
  const int el = threadIdx.x;
  const int64_t r0 = a.row0 + (int64_t)blockIdx.x * rpb;
  int64_t r1 = r0 + rpb;
  if (r1 > a.row0 + a.n) r1 = a.row0 + a.n;
  if (el >= Dp * Dp) return;
  const int i = el / Dp, j = el % Dp;
  float s = 0.0f;
  for (int64_t r = r0; r < r1; ++r) {
    const float* x = a.X + r * Dp;
    const float wr = a.w ? a.w[r] : 1.0f;
    s += x[i] * (x[j] * wr);
  }
  a.partials[(int64_t)blockIdx.x * Dp * Dp + el] = s;
}

template <int Dp>
__global__ void __launch_bounds__(256)
    gram_small_reduce_kernel(const float* __restrict__ P, int64_t nblk, float* __restrict__ G) {
  const int el = threadIdx.x;
  if (el >= Dp * Dp) return;
  const int i = el / Dp, j = el % Dp;
  if (i < j) return;
  float s = 0.0f;
  for (int64_t b = 0; b < nblk; ++b) s += P[b * Dp * Dp + el];
  G[i * Dp + j] = s;
  G[j * Dp + i] = s;
}

// Sum of a group's leaf partials in leaf order, one thread per float4 of
// the slab (blockIdx.y = group - g_lo; leaves indexed from the first leaf of
// group g_lo, as the leaf kernels wrote them).
__global__ void __launch_bounds__(256)
    gram_group_kernel(const float4* __restrict__ P, int64_t slab4, int64_t nleaf, int ngroup,
                      int g_lo, float4* __restrict__ out) {
  const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (q >= slab4) return;
  const int g = g_lo + (int)blockIdx.y;
  const int64_t base = (int64_t)g_lo * nleaf / ngroup;
  const int64_t l0 = (int64_t)g * nleaf / ngroup - base, l1 = (int64_t)(g + 1) * nleaf / ngroup - base;
  float4 acc = P[l0 * slab4 + q];
  for (int64_t l = l0 + 1; l < l1; ++l) {
    const float4 v = P[l * slab4 + q];
    acc.x += v.x;
    acc.y += v.y;
    acc.z += v.z;
    acc.w += v.w;
  }
  out[(int64_t)g * slab4 + q] = acc;
}

template <int T>
void launch_tiled_leaves(const GramArgs& a, hipStream_t s, int64_t nblk) {
  hipLaunchKernelGGL(gram_tiled_kernel<T>, dim3((unsigned)nblk), dim3(GramCfg<T>::NTHR), 0, s, a,
                     a.plan.rpl);
}

template <int T>
void launch_tiled_final(const float* gslabs, int64_t ngroup, float* G, hipStream_t s) {
  constexpr int NT = T * (T + 1) / 2;
  hipLaunchKernelGGL(gram_reduce_kernel<T>, dim3(NT * 256 / (256 / kRedChains)), dim3(256), 0, s,
                     gslabs, ngroup, G);
}

}  // namespace

GramPlan gram_plan(int Dp, int64_t n) {
  GramPlan p;
  p.n = n;
  p.rpl = wide_dim(Dp) ? wide_rows_per_leaf(n) : rows_per_block(n);
  p.nleaf = n > 0 ? (n + p.rpl - 1) / p.rpl : 0;
  p.ngroup = (int)std::min<int64_t>(kGramGroups, p.nleaf);
  const int T = Dp / 32;
  p.slab_floats = Dp <= 16 ? (size_t)Dp * Dp : (size_t)(T * (T + 1) / 2) * 1024;
  return p;
}

size_t gram_leaf_floats(const GramPlan& p, int g_lo, int g_hi) {
  const int64_t nl = g_hi > g_lo ? gram_group_leaf(p, g_hi) - gram_group_leaf(p, g_lo) : 0;
  return (size_t)std::max<int64_t>(nl, 1) * p.slab_floats;
}

hipError_t launch_gramian(int Dp, const GramArgs& in, hipStream_t s) {
  if (in.g_hi <= in.g_lo) return hipSuccess;
  GramArgs a = in;
  const int64_t l0 = gram_group_leaf(a.plan, a.g_lo), l1 = gram_group_leaf(a.plan, a.g_hi);
  a.row0 = l0 * a.plan.rpl;
  a.n = std::min(a.plan.n, l1 * a.plan.rpl) - a.row0;
  const int64_t nblk = l1 - l0;
  if (wide_dim(Dp)) {
    hipError_t e = launch_wide_gram_leaves(Dp, a, s);
    if (e != hipSuccess) return e;
  } else {
    switch (Dp) {
      case 8: hipLaunchKernelGGL(gram_small_kernel<8>, dim3((unsigned)nblk), dim3(256), 0, s, a,
                                 a.plan.rpl); break;
      case 16: hipLaunchKernelGGL(gram_small_kernel<16>, dim3((unsigned)nblk), dim3(256), 0, s, a,
                                  a.plan.rpl); break;
      case 32: launch_tiled_leaves<1>(a, s, nblk); break;
      case 64: launch_tiled_leaves<2>(a, s, nblk); break;
      case 96: launch_tiled_leaves<3>(a, s, nblk); break;
      case 128: launch_tiled_leaves<4>(a, s, nblk); break;
      case 160: launch_tiled_leaves<5>(a, s, nblk); break;
      case 192: launch_tiled_leaves<6>(a, s, nblk); break;
      case 224: launch_tiled_leaves<7>(a, s, nblk); break;
      case 256: launch_tiled_leaves<8>(a, s, nblk); break;
      default: return hipErrorInvalidValue;
    }
  }
  const int64_t slab4 = (int64_t)(a.plan.slab_floats / 4);
  hipLaunchKernelGGL(gram_group_kernel, dim3((unsigned)((slab4 + 255) / 256), (unsigned)(a.g_hi - a.g_lo)),
                     dim3(256), 0, s, reinterpret_cast<const float4*>(a.partials), slab4,
                     a.plan.nleaf, a.plan.ngroup, a.g_lo, reinterpret_cast<float4*>(a.gslabs));
  return hipGetLastError();
}

hipError_t launch_gram_final(int Dp, const GramPlan& p, const float* gslabs, float* G,
                             hipStream_t s) {
  if (p.ngroup == 0) return hipMemsetAsync(G, 0, sizeof(float) * Dp * Dp, s);
  if (wide_dim(Dp)) return launch_wide_gram_final(Dp, gslabs, p.ngroup, G, s);
  switch (Dp) {
    case 8: hipLaunchKernelGGL(gram_small_reduce_kernel<8>, dim3(1), dim3(256), 0, s, gslabs,
                               (int64_t)p.ngroup, G); break;
    case 16: hipLaunchKernelGGL(gram_small_reduce_kernel<16>, dim3(1), dim3(256), 0, s, gslabs,
                                (int64_t)p.ngroup, G); break;
    case 32: launch_tiled_final<1>(gslabs, p.ngroup, G, s); break;
    case 64: launch_tiled_final<2>(gslabs, p.ngroup, G, s); break;
    case 96: launch_tiled_final<3>(gslabs, p.ngroup, G, s); break;
    case 128: launch_tiled_final<4>(gslabs, p.ngroup, G, s); break;
    case 160: launch_tiled_final<5>(gslabs, p.ngroup, G, s); break;
    case 192: launch_tiled_final<6>(gslabs, p.ngroup, G, s); break;
    case 224: launch_tiled_final<7>(gslabs, p.ngroup, G, s); break;
    case 256: launch_tiled_final<8>(gslabs, p.ngroup, G, s); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_zero_gram(int Dp, float* G, hipStream_t s) {
  return hipMemsetAsync(G, 0, sizeof(float) * Dp * Dp, s);
}

}  // namespace frecsys_hip
