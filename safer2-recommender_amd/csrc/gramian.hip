// gramian.hip -- G = X^T diag(w) X on gfx950.
//
// Replaces Eigen's dense GEMM `X.transpose() * X` (ials.h:321, ials.h:371,
// safer2.h:55, safer2.h:294-295) and the weighted `U^T (U .* omega)`
// (safer2.h:504-509).  Dense and regular, so it is the one MFMA-shaped op of
// the loop: split-K over row blocks, each workgroup accumulating the lower
// 32x32 tiles of its block with v_mfma_f32_32x32x2_f32 (rows staged through
// LDS by coalesced float4 loads), partial slabs written in block order, then
// a reduce kernel that sums the slabs in that fixed order (deterministic,
// no atomics) and mirrors the lower triangle.  Dp = 8, 16 use a VALU path.
#include <hip/hip_runtime.h>

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

template <int T>
hipError_t launch_tiled(const GramArgs& a, hipStream_t s) {
  const int64_t rpb = rows_per_block(a.n);
  const int64_t nblk = (a.n + rpb - 1) / rpb;
  constexpr int Dp = 32 * T;
  if (nblk > 0)
    hipLaunchKernelGGL(gram_tiled_kernel<T>, dim3((unsigned)nblk), dim3(GramCfg<T>::NTHR), 0, s,
                       a, rpb);
  else
    return hipMemsetAsync(a.G, 0, sizeof(float) * Dp * Dp, s);
  constexpr int NT = T * (T + 1) / 2;
  hipLaunchKernelGGL(gram_reduce_kernel<T>, dim3(NT * 256 / (256 / kRedChains)), dim3(256), 0, s,
                     a.partials, nblk, a.G);
  return hipGetLastError();
}

template <int Dp>
hipError_t launch_small(const GramArgs& a, hipStream_t s) {
  const int64_t rpb = rows_per_block(a.n);
  const int64_t nblk = (a.n + rpb - 1) / rpb;
  if (nblk == 0) return hipMemsetAsync(a.G, 0, sizeof(float) * Dp * Dp, s);
  hipLaunchKernelGGL(gram_small_kernel<Dp>, dim3((unsigned)nblk), dim3(256), 0, s, a, rpb);
  hipLaunchKernelGGL(gram_small_reduce_kernel<Dp>, dim3(1), dim3(256), 0, s, a.partials, nblk,
                     a.G);
  return hipGetLastError();
}

}  // namespace

int64_t gram_num_blocks(int Dp, int64_t n) {
  (void)Dp;
  const int64_t rpb = rows_per_block(n);
  return (n + rpb - 1) / rpb;
}

size_t gram_workspace_floats(int Dp, int64_t n) {
  const int64_t nblk = wide_dim(Dp) ? wide_gram_num_blocks(n) : gram_num_blocks(Dp, n);
  if (Dp <= 16) return (size_t)(nblk > 0 ? nblk : 1) * Dp * Dp;
  const int T = Dp / 32;
  return (size_t)(nblk > 0 ? nblk : 1) * (T * (T + 1) / 2) * 1024;
}

hipError_t launch_gramian(int Dp, const GramArgs& a, hipStream_t s) {
  if (wide_dim(Dp)) return launch_wide_gramian(Dp, a, s);
  switch (Dp) {
    case 8: return launch_small<8>(a, s);
    case 16: return launch_small<16>(a, s);
    case 32: return launch_tiled<1>(a, s);
    case 64: return launch_tiled<2>(a, s);
    case 96: return launch_tiled<3>(a, s);
    case 128: return launch_tiled<4>(a, s);
    case 160: return launch_tiled<5>(a, s);
    case 192: return launch_tiled<6>(a, s);
    case 224: return launch_tiled<7>(a, s);
    case 256: return launch_tiled<8>(a, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_zero_gram(int Dp, float* G, hipStream_t s) {
  return hipMemsetAsync(G, 0, sizeof(float) * Dp * Dp, s);
}

}  // namespace frecsys_hip
