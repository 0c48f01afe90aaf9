// Microbenchmark of the 32x32 diagonal-block factor + inverse variants of
// chol.h on gfx950: cycles per call (one wave, 20 calls) and the max
// deviation of L^-1 from the plain recurrence (diagnostics only).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 diag_bench2.hip -o diag_bench2
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>

#include "../../safer2-recommender_amd/csrc/chol.h"
using namespace frecsys_hip;


// Variant: row k of L broadcast through LDS (all lanes read one address)
// instead of k v_readlanes; only the newest element by v_readlane.
__device__ __noinline__ bool diag_factor_inv_rb(lds_float* tile, int lane) {
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) f32x4 lds_f4;
  const int r = lane & 31;
  const bool fl = lane < 32;
  float a[32];
  load_factor_rows<8>(tile, r, fl, a);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  lds_float* R = tile;  // [32][32] rows of L (row-major), lanes < 32 write
  bool ok = true;
  auto column = [&](int k, int m0) __attribute__((always_inline)) {
    float l[32];
    // row k, m in [m0, k-1): written by earlier columns
#pragma unroll
    for (int m = m0 & ~3; m + 4 <= k - 1 + 3 && m < k - 1; m += 4) {
      const f32x4 v = *(const lds_f4*)(R + k * 32 + m);
      l[m] = v[0]; l[m + 1] = v[1]; l[m + 2] = v[2]; l[m + 3] = v[3];
    }
    float p0 = 0.f, p1 = 0.f;
#pragma unroll
    for (int m = m0; m < k - 1; m += 2) {
      p0 += a[m] * l[m];
      if (m + 1 < k - 1) p1 += a[m + 1] * l[m + 1];
    }
    float t = a[k] - (p0 + p1);
    if (k - 1 >= m0) t -= a[k - 1] * rdlane(a[k - 1], k);
    const float piv = rdlane(t, k);
    ok = ok && (piv > 0.0f);
    a[k] = t * __builtin_amdgcn_rsqf(piv);
    if (fl) R[r * 32 + k] = a[k];
  };
#pragma unroll
  for (int k = 0; k < 16; ++k) column(k, 0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  lds_float* U = tile;
#pragma unroll
  for (int m = 0; m < 16; m += 4)
    *reinterpret_cast<__attribute__((address_space(3))) f32x4*>(U + lane * 16 + m) =
        f32x4{a[m], a[m + 1], a[m + 2], a[m + 3]};
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  const int li = lane & 15, lk = lane >> 4;
  f32x4 w[4] = {f32x4{0.f}, f32x4{0.f}, f32x4{0.f}, f32x4{0.f}};
#pragma unroll
  for (int k0 = 0; k0 < 4; ++k0) {
    const float av = U[(16 + li) * 16 + 4 * k0 + lk];
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
      const float bv = U[(16 * nb + li) * 16 + 4 * k0 + lk];
      w[nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, w[nb], 0, 0, 0);
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int nb = 0; nb < 4; ++nb)
    *reinterpret_cast<__attribute__((address_space(3))) f32x4*>(U + (16 * nb + li) * 16 + 4 * lk) =
        w[nb];
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int c = 0; c < 16; c += 4) {
    const f32x4 x = *reinterpret_cast<const __attribute__((address_space(3))) f32x4*>(
        U + lane * 16 + c);
    a[16 + c] -= x[0];
    a[17 + c] -= x[1];
    a[18 + c] -= x[2];
    a[19 + c] -= x[3];
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int k = 16; k < 32; ++k) column(k, 16);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  const int j = r;
#pragma unroll
  for (int k = 0; k < 32; ++k)
    if (!fl) tile[sw(k, j)] = (k >= j) ? a[k] : 0.0f;
  return ok;
}


// Variant rb2: row k+1 of L prefetched from LDS (broadcast b128 reads)
// while column k runs; the newest element by v_readlane.  Rows stored as
// (r, m) at r*32 + (m ^ 4*((r >> 1) & 7)): groups of 4 stay aligned, the
// 32 lanes' column writes hit 16 bank pairs.
__device__ __forceinline__ int rbx(int r, int m) { return r * 32 + (m ^ (((r >> 1) & 7) << 2)); }
__device__ __noinline__ bool diag_factor_inv_rb2(lds_float* tile, int lane) {
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) f32x4 lds_f4;
  const int r = lane & 31;
  const bool fl = lane < 32;
  float a[32];
  load_factor_rows<8>(tile, r, fl, a);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  lds_float* R = tile;
  bool ok = true;
  auto half = [&](int m0) __attribute__((always_inline)) {
    float pre[32], nxt[32];
#pragma unroll
    for (int k = m0; k < m0 + 16; ++k) {
      // prefetch row k+1, entries [m0, k) (entry k-1 was written by column k-1)
      if (k + 1 < m0 + 16) {
#pragma unroll
        for (int m = m0; m < k; m += 4) {
          const f32x4 v = *(const lds_f4*)(R + rbx(k + 1, m));
          nxt[m] = v[0]; nxt[m + 1] = v[1]; nxt[m + 2] = v[2]; nxt[m + 3] = v[3];
        }
      }
      float p0 = 0.f, p1 = 0.f;
#pragma unroll
      for (int m = m0; m < k - 1; m += 2) {
        p0 += a[m] * pre[m];
        if (m + 1 < k - 1) p1 += a[m + 1] * pre[m + 1];
      }
      float t = a[k] - (p0 + p1);
      if (k - 1 >= m0) t -= a[k - 1] * rdlane(a[k - 1], k);
      const float piv = rdlane(t, k);
      ok = ok && (piv > 0.0f);
      a[k] = t * __builtin_amdgcn_rsqf(piv);
      if (fl) R[rbx(r, k)] = a[k];
#pragma unroll
      for (int m = m0; m < 32; ++m) pre[m] = nxt[m];
    }
  };
  half(0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  lds_float* U = tile;
#pragma unroll
  for (int m = 0; m < 16; m += 4)
    *reinterpret_cast<__attribute__((address_space(3))) f32x4*>(U + lane * 16 + m) =
        f32x4{a[m], a[m + 1], a[m + 2], a[m + 3]};
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  const int li = lane & 15, lk = lane >> 4;
  f32x4 w[4] = {f32x4{0.f}, f32x4{0.f}, f32x4{0.f}, f32x4{0.f}};
#pragma unroll
  for (int k0 = 0; k0 < 4; ++k0) {
    const float av = U[(16 + li) * 16 + 4 * k0 + lk];
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
      const float bv = U[(16 * nb + li) * 16 + 4 * k0 + lk];
      w[nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, w[nb], 0, 0, 0);
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int nb = 0; nb < 4; ++nb)
    *reinterpret_cast<__attribute__((address_space(3))) f32x4*>(U + (16 * nb + li) * 16 + 4 * lk) =
        w[nb];
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int c = 0; c < 16; c += 4) {
    const f32x4 x = *reinterpret_cast<const __attribute__((address_space(3))) f32x4*>(
        U + lane * 16 + c);
    a[16 + c] -= x[0];
    a[17 + c] -= x[1];
    a[18 + c] -= x[2];
    a[19 + c] -= x[3];
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  half(16);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  const int j = r;
#pragma unroll
  for (int k = 0; k < 32; ++k)
    if (!fl) tile[sw(k, j)] = (k >= j) ? a[k] : 0.0f;
  return ok;
}

__device__ __noinline__ bool diag_factor_inv_b2(lds_float* tile, int lane) {
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  const int r = lane & 31;
  const bool fl = lane < 32;
  float a[32];
  load_factor_rows<8>(tile, r, fl, a);
  // pivots checked on the scalar unit: piv > 0 and not NaN <=> its bits as
  // an int lie in (0, 0x7f800000]
  int pmin = 0x7fffffff, pmax = 0;
  auto column = [&](int k, int m0) {  // column k from the terms m in [m0, k)
    float p0 = 0.f, p1 = 0.f;
#pragma unroll
    for (int m = m0; m < k; m += 2) {
      const float b0 = rdlane(a[m], k);
      const float b1 = m + 1 < k ? rdlane(a[m + 1], k) : 0.0f;
      p0 += a[m] * b0;
      if (m + 1 < k) p1 += a[m + 1] * b1;
    }
    const float t = a[k] - (p0 + p1);
    const float piv = rdlane(t, k);
    const int pi = __builtin_amdgcn_readfirstlane(__float_as_int(piv));
    pmin = min(pmin, pi);
    pmax = max(pmax, pi);
    a[k] = t * __builtin_amdgcn_rsqf(piv);  // lane k: t = piv -> sqrt(piv)
  };
#pragma unroll
  for (int k = 0; k < 16; ++k) column(k, 0);
  // ---- cross terms on the matrix cores ----
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  lds_float* U = tile;  // [64][16]: lane l's a[0..15]; rows 16..31 = L21
#pragma unroll
  for (int m = 0; m < 16; m += 4)
    *reinterpret_cast<__attribute__((address_space(3))) f32x4*>(U + lane * 16 + m) =
        f32x4{a[m], a[m + 1], a[m + 2], a[m + 3]};
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  const int li = lane & 15, lk = lane >> 4;
  f32x4 w[4] = {f32x4{0.f}, f32x4{0.f}, f32x4{0.f}, f32x4{0.f}};
#pragma unroll
  for (int k0 = 0; k0 < 4; ++k0) {
    // A[i][k] = L21[i][4k0+k], B[k][n] = U[16nb+n][4k0+k]; D[c'][n] -> W[16nb+n][c']
    const float av = U[(16 + li) * 16 + 4 * k0 + lk];
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
      const float bv = U[(16 * nb + li) * 16 + 4 * k0 + lk];
      w[nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, w[nb], 0, 0, 0);
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // U's reads done before W overwrites it
#pragma unroll
  for (int nb = 0; nb < 4; ++nb)
    *reinterpret_cast<__attribute__((address_space(3))) f32x4*>(U + (16 * nb + li) * 16 + 4 * lk) =
        w[nb];
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int c = 0; c < 16; c += 4) {
    const f32x4 x = *reinterpret_cast<const __attribute__((address_space(3))) f32x4*>(
        U + lane * 16 + c);
    a[16 + c] -= x[0];
    a[17 + c] -= x[1];
    a[18 + c] -= x[2];
    a[19 + c] -= x[3];
  }
#pragma unroll
  for (int k = 16; k < 32; ++k) column(k, 16);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  const int j = r;
#pragma unroll
  for (int k = 0; k < 32; ++k)
    if (!fl) tile[sw(k, j)] = (k >= j) ? a[k] : 0.0f;
  return pmin > 0 && pmax <= 0x7f800000;
}


template <int V, bool CONT>
__global__ void __launch_bounds__(320) bench(const float* A, unsigned long long* cyc, float* Linv) {
  __shared__ __attribute__((aligned(16))) float tile[1024], src[1024];
  __shared__ int done;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (threadIdx.x == 0) done = 0;
  __syncthreads();
  if (wave == 4) {  // a worker wave on wave 0's SIMD: MFMA products until wave 0 is done
    f32x16 acc = f32x16{0.f};
    float x = (float)lane;
    int it = 0;
    while (*(volatile int*)&done == 0 && it < 100000) {
#pragma unroll
      for (int i = 0; i < 8; ++i) acc = mfma32(x, x + 1.0f, acc);
      ++it;
    }
    if (acc[0] == 12345.f) Linv[0] = acc[1];
    return;
  }
  if (wave != 0) return;
  for (int i = lane; i < 1024; i += 64) src[sw(i >> 5, i & 31)] = A[i];
  unsigned long long t0 = 0, t1 = 0;
  bool ok = true;
  if (CONT) __builtin_amdgcn_s_setprio(2);
  for (int it = 0; it < 21; ++it) {
    for (int i = lane; i < 1024; i += 64) tile[i] = src[i];
    wave_lds_sync();
    if (it == 1) t0 = clock64();
    if constexpr (V == 0) ok = diag_factor_inv_lds((lds_float*)tile, lane);
    else if constexpr (V == 1) ok = diag_factor_inv_blk((lds_float*)tile, lane);
    else if constexpr (V == 2) ok = diag_factor_inv_rb((lds_float*)tile, lane);
    else if constexpr (V == 3) ok = diag_factor_inv_rb2((lds_float*)tile, lane);
    else ok = diag_factor_inv_b2((lds_float*)tile, lane);
    wave_lds_sync();
  }
  t1 = clock64();
  if (lane == 0) done = 1;
  if (lane == 0) cyc[0] = (t1 - t0) / 20;
  for (int i = lane; i < 1024; i += 64) Linv[i] = tile[sw(i >> 5, i & 31)];
  if (lane == 0 && !ok) cyc[1] = 1;
}

int main() {
  float hA[1024];
  // SPD test matrix with a realistic spread: B B^T / 32 + 1e-3 I
  unsigned s = 12345;
  float B[32][32];
  for (int i = 0; i < 32; ++i)
    for (int j = 0; j < 32; ++j) {
      s = s * 1664525u + 1013904223u;
      B[i][j] = (float)((s >> 8) & 0xFFFF) / 65536.0f - 0.5f;
    }
  for (int i = 0; i < 32; ++i)
    for (int j = 0; j < 32; ++j) {
      double t = 0;
      for (int k = 0; k < 32; ++k) t += (double)B[i][k] * B[j][k];
      hA[i * 32 + j] = (float)(t / 32.0 + (i == j ? 1e-2 : 0.0));
    }
  float *dA, *dL;
  unsigned long long* dc;
  hipMalloc(&dA, 4096);
  hipMalloc(&dL, 6 * 4096);
  hipMalloc(&dc, 6 * 16);
  hipMemset(dc, 0, 96);
  hipMemcpy(dA, hA, 4096, hipMemcpyHostToDevice);
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL((bench<0, false>), dim3(1), dim3(64), 0, 0, dA, dc, dL);
    hipLaunchKernelGGL((bench<1, false>), dim3(1), dim3(64), 0, 0, dA, dc + 2, dL + 1024);
    hipLaunchKernelGGL((bench<2, false>), dim3(1), dim3(64), 0, 0, dA, dc + 4, dL + 2048);
    hipLaunchKernelGGL((bench<3, false>), dim3(1), dim3(64), 0, 0, dA, dc + 6, dL + 3072);
    hipLaunchKernelGGL((bench<1, true>), dim3(1), dim3(320), 0, 0, dA, dc + 8, dL + 4096);
    hipLaunchKernelGGL((bench<4, false>), dim3(1), dim3(64), 0, 0, dA, dc + 10, dL + 5120);
  }
  unsigned long long hc[12];
  float hL[6 * 1024];
  hipMemcpy(hc, dc, 96, hipMemcpyDeviceToHost);
  hipMemcpy(hL, dL, 6 * 4096, hipMemcpyDeviceToHost);
  const char* names[6] = {"lds (plain)", "blk (16+16)", "rb (LDS rows)", "rb2 (prefetch)", "blk+worker", "b2 (salu ok, 2 chains)"};
  for (int v = 0; v < 6; ++v) {
    double md = 0, mx = 0;
    for (int i = 0; i < 1024; ++i) {
      md = fmax(md, fabs((double)hL[v * 1024 + i] - hL[i]));
      mx = fmax(mx, fabs((double)hL[i]));
    }
    // residual of L^-1 A L^-T - I
    double res = 0;
    const float* Li = hL + v * 1024;
    for (int i = 0; i < 32; ++i)
      for (int j = 0; j < 32; ++j) {
        double t = 0;
        for (int k = 0; k < 32; ++k)
          for (int l = 0; l < 32; ++l) t += (double)Li[i * 32 + k] * hA[k * 32 + l] * Li[j * 32 + l];
        res = fmax(res, fabs(t - (i == j ? 1.0 : 0.0)));
      }
    printf("%-12s %6llu cycles  fail=%llu  max|dLinv| %.3g (max|Linv| %.3g)  max|Linv A Linv^T - I| %.3g\n",
           names[v], hc[2 * v], hc[2 * v + 1], md, mx, res);
  }
  return 0;
}
