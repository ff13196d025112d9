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

#include <stdexcept>

#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <string>

#include "kernels.hpp"
#include "wave_ops.hpp"

namespace gj {
namespace kern {

// Same for non-negative keys compared as integers (no NaN canonicalisation on the chain).
__device__ __forceinline__ uint64_t umax64(uint64_t a, uint64_t b) { return a > b ? a : b; }
template <int CTRL>
__device__ __forceinline__ uint64_t dppu64(uint64_t b) {
  const int lo = __builtin_amdgcn_mov_dpp((int)(uint32_t)b, CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(uint32_t)(b >> 32), CTRL, 0xF, 0xF, false);
  return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
  v = umax64(v, dppu64<0xB1>(v));
  v = umax64(v, dppu64<0x4E>(v));
  v = umax64(v, dppu64<0x141>(v));
  v = umax64(v, dppu64<0x140>(v));
  {
    const auto l = __builtin_amdgcn_permlane16_swap((unsigned)v, (unsigned)v, false, false);
    const auto h = __builtin_amdgcn_permlane16_swap((unsigned)(v >> 32), (unsigned)(v >> 32), false, false);
    v = umax64(((uint64_t)h[0] << 32) | l[0], ((uint64_t)h[1] << 32) | l[1]);
  }
  {
    const auto l = __builtin_amdgcn_permlane32_swap((unsigned)v, (unsigned)v, false, false);
    const auto h = __builtin_amdgcn_permlane32_swap((unsigned)(v >> 32), (unsigned)(v >> 32), false, false);
    v = umax64(((uint64_t)h[0] << 32) | l[0], ((uint64_t)h[1] << 32) | l[1]);
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
                                                            double thresh, int32_t* __restrict__ piv_out,
                                                            int live_nblk) {
  constexpr int TR = NTH / 32;   // thread rows (column groups)
  constexpr int RI = MP / 32;    // rows per thread
  constexpr int CJ = MP / TR;    // columns per thread
  constexpr int SCAN = (MP + 63) / 64;
  static_assert(RI >= 1 && CJ >= 1, "bad geometry");

  const int b = live_nblk ? live_block(used, live_nblk, p, k) : (int)blockIdx.x;  // see live_block
  const int64_t g = (int64_t)b * p + k;
  if (b < 0 || used[g]) {
    if (threadIdx.x == 0 && b >= 0) {
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
  __shared__ int pos[MP];     // current position of every row under the reference's swaps
  __shared__ int posrow[MP];  // row at every position
  __shared__ double red[NTH / 64][MP];  // per-wave partial row abs-sums (fixed-order reduction)
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
  for (int i = tid; i < MP; i += NTH) {
    pos[i] = i;
    posrow[i] = i;
  }

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
    // (2) argmax |colv| over unused real rows — the reference's scan exactly (main.cpp:756-763):
    // the largest magnitude (64-bit keys), on equal magnitudes the lowest CURRENT position under
    // its row swaps (pos); every wave redundantly, register-only butterfly; r is wave-uniform
    uint64_t bk = 0;
    int bp = 0x7fffffff, br = -1;
#pragma unroll
    for (int s = 0; s < SCAN; ++s) {
      const int i = lane + 64 * s;
      if (i < m && !lused[s]) {
        const uint64_t key = __builtin_bit_cast(uint64_t, fabs((double)colv[par][i])) & 0x7FFFFFFFFFFFFFFFull;
        const int ps = pos[i];
        if (br < 0 || key > bk || (key == bk && ps < bp)) {
          bk = key;
          bp = ps;
          br = i;
        }
      }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      const uint64_t ok = __shfl_xor(bk, o, 64);
      const int op = __shfl_xor(bp, o, 64), orr = __shfl_xor(br, o, 64);
      if (orr >= 0 && (br < 0 || ok > bk || (ok == bk && op < bp))) {
        bk = ok;
        bp = op;
        br = orr;
      }
    }
    const int r = __builtin_amdgcn_readfirstlane(br < 0 ? kk : br);
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
    if (tid == 0) {  // the reference's swap of step kk (every wave has finished this step's scan)
      const int r2 = posrow[kk], pr = pos[r];
      pos[r2] = pr;
      posrow[pr] = r2;
      pos[r] = kk;
      posrow[kk] = r;
    }
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

  if (piv_out)  // test probe: the pivot row of every column
    for (int c = tid; c < m; c += NTH) piv_out[(int64_t)b * m + c] = prow[c];
  // ||inv||_inf = max row abs-sum of the swept block (row/column permutations do not change it).
  // Summed in a fixed order (the reference's block_norm is a sequential sum, main.cpp:669-683), so
  // the score -- and with it the pivot sequence -- is the same bits on every run: the two half-waves
  // of a wave (thread rows tr = 2w, 2w + 1) meet by one commutative exchange, then every row adds
  // its per-wave partials in wave order.
  const int wv = tid >> 6;
#pragma unroll
  for (int qi = 0; qi < RI; ++qi) {
    const int i = tc + 32 * qi;
    double s = 0.0;
#pragma unroll
    for (int cj = 0; cj < CJ; ++cj) {
      const int j = tr + TR * cj;
      if (j < m) s += fabs((double)w[qi][cj]);
    }
    s += __shfl_xor(s, 32, 64);
    if (i < m && lane < 32) red[wv][i] = s;
  }
  __syncthreads();
  double mx = 0.0;
  for (int i = tid; i < m; i += NTH) {
    double rs = 0.0;
#pragma unroll
    for (int q = 0; q < NTH / 64; ++q) rs += red[q][i];
    mx = fmax(mx, rs);
  }
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
                                                             int* iscratch, int live_nblk) {
  const int b = live_nblk ? live_block(used, live_nblk, p, k) : (int)blockIdx.x;  // see live_block
  const int64_t g = (int64_t)b * p + k;
  const int tid = threadIdx.x;
  if (b < 0 || used[g]) {
    if (tid == 0 && b >= 0) {
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

// Panel-blocked sweep for the large blocks (256 < m <= 4096, fp64 and fp32): reference
// inverse_block (main.cpp:746-820) + block_norm (main.cpp:669-683), same pivot rule as the
// matrix-core kernels (largest magnitude, ties to the lowest current position under the
// reference's row swaps).  256 threads; thread tid owns block rows tid + 256 s (s < RPT).
//  * The working block lives column-major in a global (L2-resident) scratch slab, so every pass
//    over it is coalesced (threads = consecutive rows).
//  * A panel of PB columns is factored in REGISTERS (each thread its rows x PB): per step a
//    block-wide exact argmax (wave butterfly on (magnitude bits, position), 4 partials in LDS), the
//    pivot row broadcast through LDS, and the rank-1 update of the thread's own panel rows — two
//    barriers per step, no global traffic.
//  * The rest of the block then takes the panel as ONE rank-PB update, X += U R (U = the panel's
//    multipliers, still in the owners' registers; R = the PB pivot rows before the panel, staged in
//    LDS as [column][PB] so every thread reads the same column: broadcast), i.e. one read-modify-
//    write pass over the block per PB steps instead of per step, and the panel's own columns
//    become U + E (same panel algebra as blockinv_mfma.hip).
// Replaces the per-step global sweep (block_inverse_generic, kept for m > 4096 and as the reference
// timing of GJ_BI_VARIANT 6).  m > 1024 takes 6 or 8 rows per thread and 4-column panels, m > 2048
// 12 or 16 rows and 2-column panels (the [m][PB] R image + 4 m ints of book-keeping: <= 128 KiB of
// the 160 KiB LDS at m = 4096, one workgroup per CU).
// Branch-free buffer access for the blocked kernel: a masked lane passes an out-of-range offset
// (load returns 0, store is dropped) — a per-lane branch around a load makes the compiler drain
// vmcnt at the merge, which serialises the batched loads below.
constexpr int kBbRecords = 0x7ffffff0, kBbOOB = 0x7ffffff8;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t bb_rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, kBbRecords, 0x00020000);
}
template <typename T>
__device__ __forceinline__ T bb_load(__amdgpu_buffer_rsrc_t r, int off) {
  if constexpr (sizeof(T) == 8) {
    typedef unsigned int u2 __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(T, (u2)__builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
  } else {
    return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
  }
}
template <typename T>
__device__ __forceinline__ void bb_store(T v, __amdgpu_buffer_rsrc_t r, int off) {
  if constexpr (sizeof(T) == 8) {
    typedef unsigned int u2 __attribute__((ext_vector_type(2)));
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, v), r, off, 0, 0);
  } else {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned int, v), r, off, 0, 0);
  }
}

template <typename T, int RPT, int PB>
__global__ __launch_bounds__(256) void block_inverse_blocked(const T* __restrict__ Lt, int64_t ldl,
                                                             T* __restrict__ inv_t, double* __restrict__ scores,
                                                             int32_t* __restrict__ valid,
                                                             const int32_t* __restrict__ used, int m, int64_t p,
                                                             int64_t k, double thresh, T* __restrict__ scratch,
                                                             int32_t* __restrict__ piv_out, int live_nblk) {
  extern __shared__ __attribute__((aligned(16))) unsigned char bb_smem[];
  const int b = live_nblk ? live_block(used, live_nblk, p, k) : (int)blockIdx.x;  // see live_block
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (b < 0 || used[(int64_t)b * p + k]) {
    if (tid == 0 && b >= 0) {
      valid[b] = 0;
      scores[b] = 0.0;
    }
    return;
  }
  T* R = reinterpret_cast<T*>(bb_smem);                 // [m][PB]: pivot rows before the panel
  int* pos = reinterpret_cast<int*>(R + (size_t)m * PB);  // current position of every row
  int* posrow = pos + m;                                  // row at every position
  int* prow = posrow + m;                                 // prow[c] = pivot row of column c
  int* kinv = prow + m;                                   // kinv[r] = column pivoted on row r
  __shared__ T rowb[PB];
  __shared__ int rsel[PB];
  __shared__ unsigned long long redk[4];
  __shared__ int redp[4], redr[4];
  __shared__ double redn[4];

  T* Wc = scratch + (int64_t)b * m * m;  // column-major: Wc[j * m + i] = W[i][j]
  constexpr int ES = (int)sizeof(T);
  const __amdgpu_buffer_rsrc_t rw = bb_rsrc(Wc), rl = bb_rsrc(Lt + (int64_t)b * m);
  auto woff = [&](int j, int i, bool ok) { return ok ? (j * m + i) * ES : kBbOOB; };
  // every loop over the block below keeps JB independent loads in flight per thread (one wave per
  // SIMD: a load-use chain per element would leave the loop latency-bound); JB x RPT loads in
  // registers, so fewer columns per batch when every thread holds more rows
  constexpr int JB = RPT > 8 ? 2 : RPT > 4 ? 4 : 8;
  for (int j0 = 0; j0 < m; j0 += JB) {
    T x[JB][RPT];
#pragma unroll
    for (int jb = 0; jb < JB; ++jb)
#pragma unroll
      for (int s = 0; s < RPT; ++s) {
        const int i = tid + 256 * s, j = j0 + jb;
        x[jb][s] = bb_load<T>(rl, (i < m && j < m) ? (int)(((int64_t)j * ldl + i) * ES) : kBbOOB);
      }
#pragma unroll
    for (int jb = 0; jb < JB; ++jb)
#pragma unroll
      for (int s = 0; s < RPT; ++s) {
        const int i = tid + 256 * s, j = j0 + jb;
        bb_store<T>(-x[jb][s], rw, woff(j, i, i < m && j < m));
      }
  }
  for (int i = tid; i < m; i += 256) {
    pos[i] = i;
    posrow[i] = i;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");

  bool mine_used[RPT];
#pragma unroll
  for (int s = 0; s < RPT; ++s) mine_used[s] = (tid + 256 * s >= m);
  bool sing = false;
  for (int c0 = 0; c0 < m && !sing; c0 += PB) {
    const int pb = min(PB, m - c0);
    T P[RPT][PB];
#pragma unroll
    for (int s = 0; s < RPT; ++s) {
      const int i = tid + 256 * s;
#pragma unroll
      for (int kk = 0; kk < PB; ++kk) P[s][kk] = bb_load<T>(rw, woff(c0 + kk, i, i < m && kk < pb));
    }
#pragma unroll
    for (int jj = 0; jj < PB; ++jj) {
      if (jj >= pb || sing) break;
      // block-wide argmax of |column jj| over the unused rows: larger magnitude, then lower position
      unsigned long long bk = 0;
      int bp = 0x7fffffff, br = -1;
#pragma unroll
      for (int s = 0; s < RPT; ++s) {
        const int i = tid + 256 * s;
        if (mine_used[s]) continue;
        const unsigned long long key =
            __builtin_bit_cast(unsigned long long, (double)P[s][jj]) & 0x7FFFFFFFFFFFFFFFull;
        const int ps = pos[i];
        if (br < 0 || key > bk || (key == bk && ps < bp)) {
          bk = key;
          bp = ps;
          br = i;
        }
      }
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) {
        const unsigned long long ok = __shfl_xor(bk, o, 64);
        const int op = __shfl_xor(bp, o, 64), orr = __shfl_xor(br, o, 64);
        if (orr >= 0 && (br < 0 || ok > bk || (ok == bk && op < bp))) {
          bk = ok;
          bp = op;
          br = orr;
        }
      }
      if (lane == 0) {
        redk[wave] = bk;
        redp[wave] = bp;
        redr[wave] = br;
      }
      __syncthreads();  // B1: partials published (and every read of pos / rowb of the last step done)
      int r = -1;
      {
        unsigned long long fk = 0;
        int fp = 0x7fffffff;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          const int wr = redr[w];
          if (wr >= 0 && (r < 0 || redk[w] > fk || (redk[w] == fk && redp[w] < fp))) {
            fk = redk[w];
            fp = redp[w];
            r = wr;
          }
        }
      }
      if (r < 0) r = c0 + jj;  // no free row (cannot happen for jj < m): any row, singular below
      if (tid == (r & 255)) {
#pragma unroll
        for (int s = 0; s < RPT; ++s)
          if ((r >> 8) == s) {
#pragma unroll
            for (int kk = 0; kk < PB; ++kk) rowb[kk] = P[s][kk];
          }
      }
      if (tid == 0) {  // the reference's swap of step c0 + jj: pivot row <-> row at that position
        const int kp = c0 + jj, r2 = posrow[kp], pr = pos[r];
        pos[r2] = pr;
        posrow[pr] = r2;
        pos[r] = kp;
        posrow[kp] = r;
        prow[kp] = r;
        kinv[r] = kp;
        rsel[jj] = r;
      }
      __syncthreads();  // B2: pivot row and book-keeping published
      T rv[PB];
#pragma unroll
      for (int kk = 0; kk < PB; ++kk) rv[kk] = rowb[kk];
      const T piv = rv[jj];
      if (!(fabs((double)piv) >= thresh)) {
        sing = true;  // every thread read the same pivot: a uniform exit
        break;
      }
      const T inv = fast_recip(piv);
#pragma unroll
      for (int s = 0; s < RPT; ++s) {
        const int i = tid + 256 * s;
        const T u = (i == r) ? inv - T(1) : -P[s][jj] * inv;
#pragma unroll
        for (int kk = 0; kk < PB; ++kk)
          if (kk != jj) P[s][kk] = __builtin_fma(u, rv[kk], P[s][kk]);
        P[s][jj] = u;
        if (i == r) mine_used[s] = true;
      }
    }
    if (sing) break;
    // R = the panel's pivot rows over every column, before the panel (Wc is still untouched)
    for (int j = tid; j < m; j += 256)
#pragma unroll
      for (int kk = 0; kk < PB; ++kk) R[j * PB + kk] = bb_load<T>(rw, woff(j, rsel[kk < pb ? kk : 0], kk < pb));
    __syncthreads();  // B3: R staged; every thread is done reading Wc for this panel
    // X += U R outside the panel (own rows, every column); the panel's columns := U + E
    for (int j0 = 0; j0 < m; j0 += JB) {
      T x[JB][RPT];
#pragma unroll
      for (int jb = 0; jb < JB; ++jb)
#pragma unroll
        for (int s = 0; s < RPT; ++s) {
          const int i = tid + 256 * s, j = j0 + jb;
          x[jb][s] = bb_load<T>(rw, woff(j, i, i < m && j < m));
        }
#pragma unroll
      for (int jb = 0; jb < JB; ++jb) {
        const int j = j0 + jb;
        if (j >= m || (j >= c0 && j < c0 + pb)) continue;  // uniform
        T rj[PB];
#pragma unroll
        for (int kk = 0; kk < PB; ++kk) rj[kk] = R[j * PB + kk];
#pragma unroll
        for (int s = 0; s < RPT; ++s) {
          const int i = tid + 256 * s;
          T v = x[jb][s];
#pragma unroll
          for (int kk = 0; kk < PB; ++kk) v = __builtin_fma(P[s][kk], rj[kk], v);
          bb_store<T>(v, rw, woff(j, i, i < m));
        }
      }
    }
#pragma unroll
    for (int s = 0; s < RPT; ++s) {
      const int i = tid + 256 * s;
#pragma unroll
      for (int kk = 0; kk < PB; ++kk)
        bb_store<T>(P[s][kk] + (i == rsel[kk < pb ? kk : 0] ? T(1) : T(0)), rw, woff(c0 + kk, i, i < m && kk < pb));
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();  // B4: the block is consistent again (the next R reads other threads' rows)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  }
  if (sing) {
    if (tid == 0) {
      valid[b] = 0;
      scores[b] = 0.0;
    }
    return;
  }
  if (piv_out)  // test probe: the pivot row of every column
    for (int c = tid; c < m; c += 256) piv_out[(int64_t)b * m + c] = prow[c];
  // inverse, transposed: inv(W)[kinv[i]][prow[u]] = W_swept[i][u] -> inv_t[prow[u]][kinv[i]]; the
  // row abs-sums of W_swept are those of the inverse (block_norm)
  const __amdgpu_buffer_rsrc_t ro = bb_rsrc(inv_t + (int64_t)b * m * m);
  double rs[RPT];
#pragma unroll
  for (int s = 0; s < RPT; ++s) rs[s] = 0.0;
  int ki[RPT];
#pragma unroll
  for (int s = 0; s < RPT; ++s) ki[s] = (tid + 256 * s < m) ? kinv[tid + 256 * s] : 0;
  for (int u0 = 0; u0 < m; u0 += JB) {
    T x[JB][RPT];
#pragma unroll
    for (int ub = 0; ub < JB; ++ub)
#pragma unroll
      for (int s = 0; s < RPT; ++s) {
        const int i = tid + 256 * s, u = u0 + ub;
        x[ub][s] = bb_load<T>(rw, woff(u, i, i < m && u < m));
      }
#pragma unroll
    for (int ub = 0; ub < JB; ++ub) {
      const int u = u0 + ub;
      if (u >= m) continue;
      const int o = prow[u] * m;
#pragma unroll
      for (int s = 0; s < RPT; ++s) {
        const bool ok = tid + 256 * s < m;
        bb_store<T>(x[ub][s], ro, ok ? (o + ki[s]) * ES : kBbOOB);
        rs[s] += fabs((double)x[ub][s]);  // masked lanes hold 0
      }
    }
  }
  double mx = 0.0;
#pragma unroll
  for (int s = 0; s < RPT; ++s) mx = fmax(mx, rs[s]);
  mx = wave_max_f64(mx);
  if (lane == 0) redn[wave] = mx;
  __syncthreads();
  if (tid == 0) {
    const double sc = fmax(fmax(redn[0], redn[1]), fmax(redn[2], redn[3]));
    scores[b] = sc;
    valid[b] = isfinite(sc) ? 1 : 0;
  }
}

template <typename T>
static bool launch_blocked(const void* Lt, int64_t ldl, void* inv_t, double* scores, int32_t* valid,
                           const int32_t* used, const Layout& L, double thresh, int64_t nlive, hipStream_t s, void* scratch) {
  const int m = (int)L.m;
  if (m <= 256 || m > 4096) return false;
  const unsigned grid = (unsigned)(nlive >= 0 ? std::max<int64_t>(nlive, 1) : L.nblk);
  const int live_nblk = nlive >= 0 ? (int)L.nblk : 0;
  const int RPT = m <= 1024 ? (m + 255) / 256 : m <= 1536 ? 6 : m <= 2048 ? 8 : m <= 3072 ? 12 : 16;
  const int PBv = RPT <= 2 ? 16 : RPT <= 4 ? 8 : RPT <= 8 ? 4 : 2;
  const size_t lds = (size_t)m * PBv * sizeof(T) + 4 * (size_t)m * sizeof(int);
  const T* lt = static_cast<const T*>(Lt);
  T* it = static_cast<T*>(inv_t);
  T* sc = static_cast<T*>(scratch);
  int32_t* probe = block_inverse_probe();
#define GJ_BB(RP, PBB)                                                                               \
  do {                                                                                                \
    static bool attr = false;                                                                         \
    if (!attr) {                                                                                      \
      if (hipFuncSetAttribute(reinterpret_cast<const void*>(&block_inverse_blocked<T, RP, PBB>),      \
                              hipFuncAttributeMaxDynamicSharedMemorySize,                             \
                              256 * (RP) * ((PBB) * (int)sizeof(T) + 16)) != hipSuccess) {             \
        (void)hipGetLastError();                                                                      \
        throw Error(Status::BadArgs, "block inverse: dynamic LDS attribute refused");                 \
      }                                                                                               \
      attr = true;                                                                                    \
    }                                                                                                 \
    hipLaunchKernelGGL((block_inverse_blocked<T, RP, PBB>), dim3(grid), dim3(256), lds, s, lt, ldl,   \
                       it, scores, valid, used, m, L.p, L.k, thresh, sc, probe, live_nblk);           \
  } while (0)
  if (RPT == 2) GJ_BB(2, 16);
  else if (RPT == 3) GJ_BB(3, 8);
  else if (RPT == 4) GJ_BB(4, 8);
  else if (RPT == 6) GJ_BB(6, 4);
  else if (RPT == 8) GJ_BB(8, 4);
  else if (RPT == 12) GJ_BB(12, 2);
  else GJ_BB(16, 2);
#undef GJ_BB
  return true;
}

// 0 = matrix-core panels (default: blockinv_mfma.hip for 16 < m <= 128, blockinv_big.hip for fp64
// 128 < m <= 256, the panel-blocked kernel up to 4096, the GPU-wide panel / GEMM form above),
// 1 = the per-step register sweep, 5 = the co-resident L2-image kernel (fp64 32 < m <= 128;
// GJ_BI_VARIANT=co), 6 = the per-step global sweep for m > 256 (reference timing), 7 = the GPU-wide
// form for every m > 256 (GJ_BI_VARIANT=huge; tests), 8 = the panel-blocked kernel for every
// 256 < m <= 4096 whatever the live count (GJ_BI_VARIANT=blocked; tests)
static int g_bi_variant = -1;
int block_inverse_variant_id(const char* name) {
  const std::string v(name);
  if (v == "panel") return 0;
  if (v == "sweep") return 1;
  if (v == "co") return 5;
  if (v == "generic") return 6;
  if (v == "huge") return 7;
  if (v == "blocked") return 8;
  throw std::invalid_argument("unknown block-inverse variant '" + v + "' (panel | sweep | co | generic | huge | blocked)");
}
static int bi_variant() {
  if (g_bi_variant < 0) {
    const char* e = getenv("GJ_BI_VARIANT");
    g_bi_variant = (e && *e) ? block_inverse_variant_id(e) : 0;  // a typo throws
  }
  return g_bi_variant;
}
void set_block_inverse_variant(int v) { g_bi_variant = v; }
int block_inverse_variant() { return bi_variant(); }

// The GPU-wide form (one candidate at a time, every CU) against the panel-blocked kernel (every
// candidate at once, one workgroup each), by the live candidate count: per batch, measured
// (scripts/runs/r6_bi_large.sh, fp64, ms) panel 6.7 / 43 / 578 / 8160 at m = 512 / 1024 / 2048 /
// 4096 whatever the count, GPU-wide 4.7 / 12.5 / 41 / 150 per candidate.
static bool huge_preferred(int64_t m, int64_t nlive) {
  if (m > 4096) return true;
  if (m > 2048) return nlive <= 48;
  if (m > 1536) return nlive <= 12;
  if (m >= 1024) return nlive <= 3;
  return false;
}

template <typename T>
static void launch_bi(const void* Lt, int64_t ldl, void* inv_t, double* scores, int32_t* valid,
                      const int32_t* used, const Layout& L, double thresh, int64_t nlive, hipStream_t s,
                      void* scratch, int* iscratch, int variant) {
  const int m = (int)L.m;
  const unsigned grid = (unsigned)(nlive >= 0 ? std::max<int64_t>(nlive, 1) : L.nblk);
  const int live_nblk = nlive >= 0 ? (int)L.nblk : 0;
  const T* lt = static_cast<const T*>(Lt);
  T* it = static_cast<T*>(inv_t);
  const int g_bi_variant = variant >= 0 ? variant : bi_variant();
  if (g_bi_variant == 5 && block_inverse_co(sizeof(T) == 8 ? DType::F64 : DType::F32, Lt, ldl, inv_t, scores,
                                            valid, used, L, thresh, nlive, s, scratch))
    return;
  if (g_bi_variant == 0 &&
      block_inverse_mfma(sizeof(T) == 8 ? DType::F64 : DType::F32, Lt, ldl, inv_t, scores, valid, used,
                         L, thresh, nlive, s))
    return;
  if (g_bi_variant != 1 && block_inverse_big(sizeof(T) == 8 ? DType::F64 : DType::F32, Lt, ldl, inv_t, scores,
                                              valid, used, L, thresh, nlive, s, scratch))
    return;
  if (m <= 32)
    hipLaunchKernelGGL((block_inverse_kernel<T, 32, 256>), dim3(grid), dim3(256), 0, s, lt, ldl, it,
                       scores, valid, used, m, L.p, L.k, thresh, block_inverse_probe(), live_nblk);
  else if (m <= 64)
    hipLaunchKernelGGL((block_inverse_kernel<T, 64, 256>), dim3(grid), dim3(256), 0, s, lt, ldl, it,
                       scores, valid, used, m, L.p, L.k, thresh, block_inverse_probe(), live_nblk);
  else if (m <= 128)  // 16 elements per thread, 4 waves per SIMD to hide the per-step latency chain
    hipLaunchKernelGGL((block_inverse_kernel<T, 128, 1024>), dim3(grid), dim3(1024), 0, s, lt, ldl,
                       it, scores, valid, used, m, L.p, L.k, thresh, block_inverse_probe(), live_nblk);
  else if (m <= 256 && sizeof(T) == 4)  // 256x256 fp32 = 64 VGPRs/lane at 1024 threads
    hipLaunchKernelGGL((block_inverse_kernel<T, 256, 1024>), dim3(grid), dim3(1024), 0, s, lt, ldl,
                       it, scores, valid, used, m, L.p, L.k, thresh, block_inverse_probe(), live_nblk);
  else if ((m > 4096 && g_bi_variant != 6) || (g_bi_variant == 0 && huge_preferred(m, nlive >= 0 ? nlive : L.nblk)) ||
           (g_bi_variant == 7 && m > 256)) {
    // large m, few live candidates: the GPU-wide panel / GEMM form, one candidate at a time
    // (blockinv_huge.hip)
    block_inverse_huge(sizeof(T) == 8 ? DType::F64 : DType::F32, Lt, ldl, inv_t, scores, valid, used, L, thresh,
                       nlive, s, scratch);
    return;
  } else if (g_bi_variant != 6 && launch_blocked<T>(Lt, ldl, inv_t, scores, valid, used, L, thresh, nlive, s, scratch))
    return;
  else
    hipLaunchKernelGGL((block_inverse_generic<T>), dim3(grid), dim3(256), 0, s, lt, ldl, it, scores,
                       valid, used, m, L.p, L.k, thresh, static_cast<T*>(scratch), iscratch, live_nblk);
}

// The kernel launch_bi picks (same decision tree), for the engine's policy report.
const char* block_inverse_kernel_name(DType dt, int64_t m, int variant) {
  const int v = variant >= 0 ? variant : bi_variant();
  const bool f64 = dt == DType::F64;
  if (v == 5 && f64 && m > 32 && m <= 128) return "l2_coresident";
  if (v == 0 && m > 16 && m <= 128) return "mfma_register";
  if (v != 1 && f64 && m > 128 && m <= 256) return "l2_image";
  if (m <= 128 || (m <= 256 && !f64)) return "register_sweep";
  if ((m > 4096 && v != 6) || v == 7) return "gpu_panel_gemm";
  if (v == 0 && m >= 1024) return "panel_blocked|gpu_panel_gemm (by live candidates)";
  if (v != 6 && m <= 4096) return "panel_blocked";
  return "generic";
}

static bool generic_path(DType dt, int64_t m) { return dt == DType::F64 ? m > 128 : m > 256; }

size_t block_inverse_scratch_bytes(DType dt, const Layout& L, int variant) {
  const int v = variant >= 0 ? variant : bi_variant();
  if (v == 5 && dt == DType::F64 && L.m > 32 && L.m <= 128) return block_inverse_big_scratch_bytes(dt, L);
  if (!generic_path(dt, L.m)) return 0;
  if (const size_t big = block_inverse_big_scratch_bytes(dt, L)) return big;
  return (size_t)L.nblk * L.m * L.m * dtype_size(dt);
}
size_t block_inverse_iscratch_bytes(const Layout& L) {
  return (size_t)L.nblk * 3 * L.m * sizeof(int);
}

bool block_inverse_select(DType dt, const void* Lt, int64_t ldl, void* inv_t, double* scores,
                          int32_t* valid, const int32_t* used, const Layout& L, double thresh, int64_t nlive,
                          hipStream_t s, const PivotSelectArgs& sel, int variant, void* scratch) {
  const int v = variant >= 0 ? variant : bi_variant();
  if (L.nblk <= 0) return false;
  PivotSelectArgs sa = sel;
  sa.sysfence = host_fence();
  if (v == 5)
    return scratch && block_inverse_co(dt, Lt, ldl, inv_t, scores, valid, used, L, thresh, nlive, s, scratch, &sa);
  if (v != 0) return false;
  return block_inverse_mfma(dt, Lt, ldl, inv_t, scores, valid, used, L, thresh, nlive, s, &sa);
}

void block_inverse(DType dt, const void* Lt, int64_t ldl, void* inv_t, double* scores,
                   int32_t* valid, const int32_t* used, const Layout& L, double thresh, int64_t nlive,
                   hipStream_t s, void* scratch, int* iscratch, int variant) {
  if (L.nblk <= 0) return;
  if (dt == DType::F64)
    launch_bi<double>(Lt, ldl, inv_t, scores, valid, used, L, thresh, nlive, s, scratch, iscratch, variant);
  else
    launch_bi<float>(Lt, ldl, inv_t, scores, valid, used, L, thresh, nlive, s, scratch, iscratch, variant);
}

}  // namespace kern
}  // namespace gj
