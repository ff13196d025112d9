// Batched candidate-block inversion for the pivot search (gfx950).
//
// Reference: inverse_block (main.cpp:746-820, scalar Gauss-Jordan with partial pivoting, "first
// max wins", singular when |a_kk| < EPS*norm) + block_norm (main.cpp:669-683), called for every
// candidate block of the current block column at main.cpp:1039-1066.
//
// One workgroup per candidate block.  The m x m block (padded to MP = 32/64/128/256) lives in
// REGISTERS (16 elements per thread for MP = 64/128, measured 4x faster per step than 64 elements
// per thread at one wave per SIMD): thread (tr, tc) owns rows i = tc + 32*qi and columns
// j = tr + TR*cj, so the global load
// from the K-major multiplier panel is coalesced along i.  Each of the m elimination steps needs two
// workgroup barriers: column k is published to LDS, every wave redundantly computes the pivot argmax
// (no third barrier), the pivot-row owners publish the scaled pivot row, then every thread applies
// its rank-1 update.  The elimination is the in-place "sweep" form without row swaps (pivot rows are
// recorded in prow/kinv and the inverse is written permuted), which needs no augmented identity.
// Outputs: the inverse (transposed, ready to be the K-major GEMM operand H^T), ||inv||_inf, validity.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "kernels.hpp"

namespace gj {
namespace kern {

// ---- wave-wide max of a double without LDS round trips: DPP quad/row permutes for the first
// 16 lanes, v_permlane16_swap / v_permlane32_swap (gfx950) for the rest.
template <int CTRL>
__device__ __forceinline__ double dpp64(double x) {
  const uint64_t b = __builtin_bit_cast(uint64_t, x);
  const int lo = __builtin_amdgcn_mov_dpp((int)(uint32_t)b, CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(uint32_t)(b >> 32), CTRL, 0xF, 0xF, false);
  return __builtin_bit_cast(double, ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
__device__ __forceinline__ double join64(unsigned lo, unsigned hi) {
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ double wave_max_f64(double v) {
  v = fmax(v, dpp64<0xB1>(v));   // quad_perm [1,0,3,2]
  v = fmax(v, dpp64<0x4E>(v));   // quad_perm [2,3,0,1]
  v = fmax(v, dpp64<0x141>(v));  // row_half_mirror (8)
  v = fmax(v, dpp64<0x140>(v));  // row_mirror (16)
  {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const auto l = __builtin_amdgcn_permlane16_swap((unsigned)b, (unsigned)b, false, false);
    const auto h = __builtin_amdgcn_permlane16_swap((unsigned)(b >> 32), (unsigned)(b >> 32), false, false);
    v = fmax(join64(l[0], h[0]), join64(l[1], h[1]));
  }
  {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const auto l = __builtin_amdgcn_permlane32_swap((unsigned)b, (unsigned)b, false, false);
    const auto h = __builtin_amdgcn_permlane32_swap((unsigned)(b >> 32), (unsigned)(b >> 32), false, false);
    v = fmax(join64(l[0], h[0]), join64(l[1], h[1]));
  }
  return v;
}
// Pivot key: |a| with its lowest 8 mantissa bits replaced by (255 - row), so one wave-wide double
// max yields the largest magnitude and, among (near-)equal magnitudes, the lowest row.
__device__ __forceinline__ double pivot_key(double a, int row) {
  if (!(a == a)) a = 0.0;
  const uint64_t b = (__builtin_bit_cast(uint64_t, a) & ~uint64_t(0xFF)) | (uint64_t)(255 - row);
  return __builtin_bit_cast(double, b);
}
__device__ __forceinline__ int pivot_key_row(double key) {
  return 255 - (int)(__builtin_bit_cast(uint64_t, key) & 0xFF);
}

template <typename T, int MP, int NTH>
__global__ __launch_bounds__(NTH) void block_inverse_kernel(const T* __restrict__ Lt, int64_t ldl,
                                                            T* __restrict__ inv_t,
                                                            double* __restrict__ scores,
                                                            int32_t* __restrict__ valid,
                                                            const int32_t* __restrict__ used,
                                                            int m, int64_t p, int64_t k,
                                                            double thresh) {
  constexpr int TR = NTH / 32;   // thread rows (column groups)
  constexpr int RI = MP / 32;    // rows per thread
  constexpr int CJ = MP / TR;    // columns per thread
  constexpr int SCAN = (MP + 63) / 64;
  static_assert(RI >= 1 && CJ >= 1, "bad geometry");

  const int b = blockIdx.x;
  const int64_t g = (int64_t)b * p + k;
  if (used[g]) {
    if (threadIdx.x == 0) {
      valid[b] = 0;
      scores[b] = 0.0;
    }
    return;
  }
  const int tid = threadIdx.x, lane = tid & 63, tc = tid & 31, tr = tid >> 5;

  __shared__ T colv[2][MP];
  __shared__ T rowv[2][MP];
  __shared__ int prow[MP];
  __shared__ int kinv[MP];
  __shared__ double red[MP];
  __shared__ double wmax[NTH / 64];

  T w[RI][CJ];
#pragma unroll
  for (int qi = 0; qi < RI; ++qi) {
    const int i = tc + 32 * qi;
#pragma unroll
    for (int cj = 0; cj < CJ; ++cj) {
      const int j = tr + TR * cj;
      w[qi][cj] = (i < m && j < m) ? -Lt[(int64_t)j * ldl + (int64_t)b * m + i]
                                   : (i == j ? T(1) : T(0));
    }
  }
  for (int i = tid; i < MP; i += NTH) red[i] = 0.0;

  bool lused[SCAN];
#pragma unroll
  for (int s = 0; s < SCAN; ++s) lused[s] = false;

  bool singular = false;
  for (int kk = 0; kk < m; ++kk) {
    const int par = kk & 1;
    const int kcj = kk / TR;
    const bool col_owner = (tr == kk % TR);
    // (1) publish column kk (one half-wave owns it)
    if (col_owner) {
#pragma unroll
      for (int qi = 0; qi < RI; ++qi) {
        T v = T(0);
#pragma unroll
        for (int cj = 0; cj < CJ; ++cj)
          if (cj == kcj) v = w[qi][cj];
        colv[par][tc + 32 * qi] = v;
      }
    }
    __syncthreads();
    // (2) argmax |colv| over unused real rows, lowest row on ties (every wave, redundantly, with
    // register-only cross-lane moves); r is wave-uniform -> scalar branches below
    double key = -1.0;
#pragma unroll
    for (int s = 0; s < SCAN; ++s) {
      const int i = lane + 64 * s;
      const double kv = (i < m && !lused[s]) ? pivot_key(fabs((double)colv[par][i]), i) : -1.0;
      key = fmax(key, kv);
    }
    key = wave_max_f64(key);
    const int r = __builtin_amdgcn_readfirstlane(pivot_key_row(key));
    const T pivv = colv[par][r];
    if (!(fabs((double)pivv) >= thresh)) {  // uniform across the workgroup
      singular = true;
      break;
    }
#pragma unroll
    for (int s = 0; s < SCAN; ++s)
      if (lane + 64 * s == r) lused[s] = true;
    if (tid == 0) {
      prow[kk] = r;
      kinv[r] = kk;
    }
    const T inv = T(1) / pivv;
    const int rq = r >> 5;
    const bool row_owner = (tc == (r & 31));
    // (3) publish the scaled pivot row (rowv[kk] = inv)
    if (row_owner) {
#pragma unroll
      for (int qi = 0; qi < RI; ++qi)
        if (qi == rq) {
#pragma unroll
          for (int cj = 0; cj < CJ; ++cj) {
            const int j = tr + TR * cj;
            rowv[par][j] = (j == kk) ? inv : w[qi][cj] * inv;
          }
        }
    }
    __syncthreads();
    // (4) rank-1 update: column kk enters as 0 (-> -f*inv), pivot row fixed up afterwards
    if (col_owner) {
#pragma unroll
      for (int qi = 0; qi < RI; ++qi)
#pragma unroll
        for (int cj = 0; cj < CJ; ++cj)
          if (cj == kcj) w[qi][cj] = T(0);
    }
    T rv[CJ];
#pragma unroll
    for (int cj = 0; cj < CJ; ++cj) rv[cj] = rowv[par][tr + TR * cj];
#pragma unroll
    for (int qi = 0; qi < RI; ++qi) {
      const T nf = -colv[par][tc + 32 * qi];
#pragma unroll
      for (int cj = 0; cj < CJ; ++cj) w[qi][cj] = __builtin_fma(nf, rv[cj], w[qi][cj]);
    }
    if (row_owner) {
#pragma unroll
      for (int qi = 0; qi < RI; ++qi)
        if (qi == rq) {
#pragma unroll
          for (int cj = 0; cj < CJ; ++cj) w[qi][cj] = rv[cj];
        }
    }
  }

  if (singular) {
    if (tid == 0) {
      valid[b] = 0;
      scores[b] = 0.0;
    }
    return;
  }

  // ||inv||_inf = max row abs-sum of the swept block (row/column permutations do not change it)
#pragma unroll
  for (int qi = 0; qi < RI; ++qi) {
    const int i = tc + 32 * qi;
    double s = 0.0;
#pragma unroll
    for (int cj = 0; cj < CJ; ++cj) {
      const int j = tr + TR * cj;
      if (j < m) s += fabs((double)w[qi][cj]);
    }
    if (i < m) atomicAdd(&red[i], s);
  }
  __syncthreads();
  double mx = 0.0;
  for (int i = tid; i < m; i += NTH) mx = fmax(mx, red[i]);
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) mx = fmax(mx, __shfl_xor(mx, off, 64));
  if (lane == 0) wmax[tid >> 6] = mx;

  // inverse, transposed: inv(W)[kinv[i]][prow[u]] = W_swept[i][u]  ->  inv_t[prow[u]*m + kinv[i]]
  T* out = inv_t + (int64_t)b * m * m;
#pragma unroll
  for (int qi = 0; qi < RI; ++qi) {
    const int i = tc + 32 * qi;
    if (i >= m) continue;
    const int ki = kinv[i];
#pragma unroll
    for (int cj = 0; cj < CJ; ++cj) {
      const int u = tr + TR * cj;
      if (u < m) out[(int64_t)prow[u] * m + ki] = w[qi][cj];
    }
  }
  __syncthreads();
  if (tid == 0) {
    double sc = 0.0;
    for (int q = 0; q < NTH / 64; ++q) sc = fmax(sc, wmax[q]);
    scores[b] = sc;
    valid[b] = isfinite(sc) ? 1 : 0;
  }
}

// Generic path for m > 256: the working block lives in a global scratch area (one m*m slab per
// workgroup), 256 threads.  Correct for any m; only used when the block exceeds the register path.
template <typename T>
__global__ __launch_bounds__(256) void block_inverse_generic(const T* __restrict__ Lt, int64_t ldl,
                                                             T* __restrict__ inv_t,
                                                             double* __restrict__ scores,
                                                             int32_t* __restrict__ valid,
                                                             const int32_t* __restrict__ used,
                                                             int m, int64_t p, int64_t k,
                                                             double thresh, T* scratch,
                                                             int* iscratch) {
  const int b = blockIdx.x;
  const int64_t g = (int64_t)b * p + k;
  const int tid = threadIdx.x;
  if (used[g]) {
    if (tid == 0) {
      valid[b] = 0;
      scores[b] = 0.0;
    }
    return;
  }
  T* W = scratch + (int64_t)b * m * m;
  int* prow = iscratch + (int64_t)b * 3 * m;
  int* kinv = prow + m;
  int* usedr = kinv + m;
  __shared__ double sv[256];
  __shared__ int si[256];
  __shared__ T s_inv;
  __shared__ int s_r;
  __shared__ int s_sing;
  for (int64_t e = tid; e < (int64_t)m * m; e += 256) {
    const int i = (int)(e / m), j = (int)(e % m);
    W[e] = -Lt[(int64_t)j * ldl + (int64_t)b * m + i];
  }
  for (int i = tid; i < m; i += 256) usedr[i] = 0;
  __threadfence_block();
  __syncthreads();
  for (int kk = 0; kk < m; ++kk) {
    double best = -1.0;
    int bi = m;
    for (int i = tid; i < m; i += 256)
      if (!usedr[i]) {
        const double v = fabs((double)W[(int64_t)i * m + kk]);
        if (v > best) {
          best = v;
          bi = i;
        }
      }
    sv[tid] = best;
    si[tid] = bi;
    __syncthreads();
    if (tid == 0) {
      double bb = -1.0;
      int ib = m;
      for (int q = 0; q < 256; ++q)
        if (sv[q] > bb || (sv[q] == bb && si[q] < ib)) {
          bb = sv[q];
          ib = si[q];
        }
      s_sing = !(bb >= thresh);
      s_r = ib;
      if (!s_sing) {
        usedr[ib] = 1;
        prow[kk] = ib;
        kinv[ib] = kk;
        s_inv = T(1) / W[(int64_t)ib * m + kk];
      }
    }
    __threadfence_block();
    __syncthreads();
    if (s_sing) break;
    const int r = s_r;
    const T inv = s_inv;
    for (int j = tid; j < m; j += 256) W[(int64_t)r * m + j] = (j == kk) ? inv : W[(int64_t)r * m + j] * inv;
    __threadfence_block();
    __syncthreads();
    for (int64_t e = tid; e < (int64_t)m * m; e += 256) {
      const int i = (int)(e / m), j = (int)(e % m);
      if (i == r) continue;
      const T f = W[(int64_t)i * m + kk];
      if (j == kk) continue;
      W[e] -= f * W[(int64_t)r * m + j];
    }
    __threadfence_block();
    __syncthreads();
    for (int i = tid; i < m; i += 256)
      if (i != r) W[(int64_t)i * m + kk] = -W[(int64_t)i * m + kk] * inv;
    __threadfence_block();
    __syncthreads();
  }
  if (s_sing) {
    if (tid == 0) {
      valid[b] = 0;
      scores[b] = 0.0;
    }
    return;
  }
  double mx = 0.0;
  for (int i = tid; i < m; i += 256) {
    double s = 0.0;
    for (int j = 0; j < m; ++j) s += fabs((double)W[(int64_t)i * m + j]);
    mx = fmax(mx, s);
  }
  sv[tid] = mx;
  T* out = inv_t + (int64_t)b * m * m;
  for (int64_t e = tid; e < (int64_t)m * m; e += 256) {
    const int i = (int)(e / m), u = (int)(e % m);
    out[(int64_t)prow[u] * m + kinv[i]] = W[e];
  }
  __syncthreads();
  if (tid == 0) {
    double sc = 0.0;
    for (int q = 0; q < 256; ++q) sc = fmax(sc, sv[q]);
    scores[b] = sc;
    valid[b] = isfinite(sc) ? 1 : 0;
  }
}

template <typename T>
static void launch_bi(const void* Lt, int64_t ldl, void* inv_t, double* scores, int32_t* valid,
                      const int32_t* used, const Layout& L, double thresh, hipStream_t s,
                      void* scratch, int* iscratch) {
  const int m = (int)L.m;
  const unsigned grid = (unsigned)L.nblk;
  const T* lt = static_cast<const T*>(Lt);
  T* it = static_cast<T*>(inv_t);
  if (m <= 32)
    hipLaunchKernelGGL((block_inverse_kernel<T, 32, 256>), dim3(grid), dim3(256), 0, s, lt, ldl, it,
                       scores, valid, used, m, L.p, L.k, thresh);
  else if (m <= 64)
    hipLaunchKernelGGL((block_inverse_kernel<T, 64, 256>), dim3(grid), dim3(256), 0, s, lt, ldl, it,
                       scores, valid, used, m, L.p, L.k, thresh);
  else if (m <= 128)  // 16 elements per thread, 4 waves per SIMD to hide the per-step latency chain
    hipLaunchKernelGGL((block_inverse_kernel<T, 128, 1024>), dim3(grid), dim3(1024), 0, s, lt, ldl,
                       it, scores, valid, used, m, L.p, L.k, thresh);
  else if (m <= 256 && sizeof(T) == 4)  // 256x256 fp32 = 64 VGPRs/lane at 1024 threads
    hipLaunchKernelGGL((block_inverse_kernel<T, 256, 1024>), dim3(grid), dim3(1024), 0, s, lt, ldl,
                       it, scores, valid, used, m, L.p, L.k, thresh);
  else
    hipLaunchKernelGGL((block_inverse_generic<T>), dim3(grid), dim3(256), 0, s, lt, ldl, it, scores,
                       valid, used, m, L.p, L.k, thresh, static_cast<T*>(scratch), iscratch);
}

static bool generic_path(DType dt, int64_t m) { return dt == DType::F64 ? m > 128 : m > 256; }

size_t block_inverse_scratch_bytes(DType dt, const Layout& L) {
  if (!generic_path(dt, L.m)) return 0;
  return (size_t)L.nblk * L.m * L.m * dtype_size(dt);
}
size_t block_inverse_iscratch_bytes(const Layout& L) {
  return (size_t)L.nblk * 3 * L.m * sizeof(int);
}

void block_inverse(DType dt, const void* Lt, int64_t ldl, void* inv_t, double* scores,
                   int32_t* valid, const int32_t* used, const Layout& L, double thresh,
                   hipStream_t s, void* scratch, int* iscratch) {
  if (L.nblk <= 0) return;
  if (dt == DType::F64)
    launch_bi<double>(Lt, ldl, inv_t, scores, valid, used, L, thresh, s, scratch, iscratch);
  else
    launch_bi<float>(Lt, ldl, inv_t, scores, valid, used, L, thresh, s, scratch, iscratch);
}

}  // namespace kern
}  // namespace gj
