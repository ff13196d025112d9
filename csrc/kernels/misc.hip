// Memory-bound helper kernels of the engine (gfx950).
//
//   generate        <- init_matrix / f / f_i            (main.cpp:47-64, :128-149)
//   extract_neg_t   <- get(a, E, i, t) of the hot loop  (main.cpp:690-708, :1172) — here one tiled
//                      transpose of block column t into the K-major multiplier panel
//   pivot_local     <- local candidate scan             (main.cpp:1039-1066)
//   pivot_global    <- pivot_op over all ranks          (main.cpp:729-744, :1074)
//   permute_blocks  <- the row swaps (main.cpp:1100-1131) done once at the end
//   row_abs_max     <- norm()                           (main.cpp:643-667)
//   residual_reduce <- norm() of the residual strip     (main.cpp:494-507)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

#include "gj/gen.hpp"
#include "kernels.hpp"
#include "pivot_select.hpp"
#include "wave_ops.hpp"

namespace gj {
namespace kern {

namespace {
inline unsigned grid_for(int64_t work, int per_block, int64_t cap = 1 << 20) {
  int64_t g = (work + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

// atomic max for non-negative doubles: their IEEE bit patterns order like the values
__device__ inline void atomic_max_nonneg(double* addr, double v) {
  if (!(v >= 0.0)) v = __longlong_as_double(0x7ff8000000000000ll);  // NaN propagates as max
  atomicMax(reinterpret_cast<unsigned long long*>(addr), (unsigned long long)__double_as_longlong(v));
}
}  // namespace

// ---------------------------------------------------------------- generate
template <typename T>
__global__ void generate_kernel(T* X, int64_t rows, int64_t npad, int64_t n, int64_t m, int64_t p,
                                int64_t k, int kind, uint64_t seed) {
  const int64_t total = rows * npad;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / npad, j = e - r * npad;
    const int64_t gr = ((r / m) * p + k) * m + r % m;
    X[e] = (T)gen_value(kind, seed, n, gr, j);
  }
}

// One workgroup per local row: the row's values are generated column by column (no 64-bit index
// division per element, as in the flat kernel above) and their magnitudes summed in the order of
// row_abs_kernel below (thread t: columns t, t + 256, ...; then the same wave / workgroup
// reduction), so the norm is bit-identical to generate() followed by row_abs_max().
template <typename T>
__global__ __launch_bounds__(256) void generate_norm_kernel(T* X, int64_t npad, int64_t n, int64_t m, int64_t p,
                                                            int64_t k, int kind, uint64_t seed, double* out) {
  const int64_t r = blockIdx.x;
  const int64_t gr = ((r / m) * p + k) * m + r % m;
  T* row = X + r * npad;
  double s = 0.0;
  for (int64_t j = threadIdx.x; j < npad; j += 256) {
    const T v = (T)gen_value(kind, seed, n, gr, j);
    row[j] = v;
    if (j < n) s += fabs((double)v);
  }
  if (gr >= n) return;  // padding row: generated, not part of the norm (row_abs_kernel)
  __shared__ double sh[4];
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off, 64);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) atomic_max_nonneg(out, sh[0] + sh[1] + sh[2] + sh[3]);
}

void generate_norm(DType dt, void* X, const Layout& L, int kind, uint64_t seed, double* out, hipStream_t s) {
  (void)hipMemsetAsync(out, 0, sizeof(double), s);
  if (L.rows <= 0) return;
  if (dt == DType::F64)
    hipLaunchKernelGGL(generate_norm_kernel<double>, dim3((unsigned)L.rows), dim3(256), 0, s,
                       static_cast<double*>(X), L.npad, L.n, L.m, L.p, L.k, kind, seed, out);
  else
    hipLaunchKernelGGL(generate_norm_kernel<float>, dim3((unsigned)L.rows), dim3(256), 0, s,
                       static_cast<float*>(X), L.npad, L.n, L.m, L.p, L.k, kind, seed, out);
}

void generate(DType dt, void* X, const Layout& L, int kind, uint64_t seed, hipStream_t s) {
  const int64_t total = L.rows * L.npad;
  if (total <= 0) return;
  const unsigned grid = grid_for(total, 256 * 4);
  if (dt == DType::F64)
    hipLaunchKernelGGL(generate_kernel<double>, dim3(grid), dim3(256), 0, s, static_cast<double*>(X),
                       L.rows, L.npad, L.n, L.m, L.p, L.k, kind, seed);
  else
    hipLaunchKernelGGL(generate_kernel<float>, dim3(grid), dim3(256), 0, s, static_cast<float*>(X),
                       L.rows, L.npad, L.n, L.m, L.p, L.k, kind, seed);
}

// ---------------------------------------------------------------- upload_convert
template <typename T>
__global__ void upload_kernel(T* X, int64_t ldx, const double* src, int64_t ld, int64_t rows,
                              int64_t cols) {
  const int64_t total = rows * cols;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / cols, j = e - r * cols;
    X[r * ldx + j] = (T)src[r * ld + j];
  }
}

void upload_convert(DType dt, void* X, int64_t ldx, const double* src, int64_t src_ld, int64_t rows,
                    int64_t cols, hipStream_t s) {
  if (rows <= 0 || cols <= 0) return;
  const unsigned grid = grid_for(rows * cols, 256 * 4);
  if (dt == DType::F64)
    hipLaunchKernelGGL(upload_kernel<double>, dim3(grid), dim3(256), 0, s, static_cast<double*>(X),
                       ldx, src, src_ld, rows, cols);
  else
    hipLaunchKernelGGL(upload_kernel<float>, dim3(grid), dim3(256), 0, s, static_cast<float*>(X), ldx,
                       src, src_ld, rows, cols);
}

// dst[r*ldd + j] = (double)X[r*ldx + j]  (fp64 residual / refinement of an fp32 solve)
template <typename T>
__global__ void widen_kernel(double* dst, int64_t ldd, const T* X, int64_t ldx, int64_t rows, int64_t cols) {
  const int64_t total = rows * cols;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / cols, j = e - r * cols;
    dst[r * ldd + j] = (double)X[r * ldx + j];
  }
}

void widen(DType dt, double* dst, int64_t ldd, const void* X, int64_t ldx, int64_t rows, int64_t cols,
           hipStream_t s) {
  if (rows <= 0 || cols <= 0) return;
  const unsigned grid = grid_for(rows * cols, 256 * 4);
  if (dt == DType::F64)
    hipLaunchKernelGGL(widen_kernel<double>, dim3(grid), dim3(256), 0, s, dst, ldd,
                       static_cast<const double*>(X), ldx, rows, cols);
  else
    hipLaunchKernelGGL(widen_kernel<float>, dim3(grid), dim3(256), 0, s, dst, ldd,
                       static_cast<const float*>(X), ldx, rows, cols);
}

// ---------------------------------------------------------------- extract_neg_t (tiled transpose)
template <typename T>
__global__ __launch_bounds__(256) void extract_kernel(T* __restrict__ Lt, int64_t ldl,
                                                      const T* __restrict__ X, int64_t ldx,
                                                      int64_t rows, int64_t col0, int64_t m) {
  __shared__ T tile[64][65];
  const int64_t r0 = (int64_t)blockIdx.x * 64, c0 = (int64_t)blockIdx.y * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;  // 64 x 4
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int i = ty + 4 * q;
    const int64_t r = r0 + i, c = c0 + tx;
    tile[i][tx] = (r < rows && c < m) ? X[r * ldx + col0 + c] : T(0);
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int j = ty + 4 * q;
    const int64_t c = c0 + j, r = r0 + tx;
    if (r < rows && c < m) Lt[c * ldl + r] = -tile[tx][j];
  }
}

void extract_neg_t(DType dt, void* Lt, int64_t ldl, const void* X, int64_t ldx, int64_t rows,
                   int64_t col0, int64_t m, hipStream_t s) {
  if (rows <= 0 || m <= 0) return;
  dim3 grid((unsigned)((rows + 63) / 64), (unsigned)((m + 63) / 64));
  if (dt == DType::F64)
    hipLaunchKernelGGL(extract_kernel<double>, grid, dim3(256), 0, s, static_cast<double*>(Lt), ldl,
                       static_cast<const double*>(X), ldx, rows, col0, m);
  else
    hipLaunchKernelGGL(extract_kernel<float>, grid, dim3(256), 0, s, static_cast<float*>(Lt), ldl,
                       static_cast<const float*>(X), ldx, rows, col0, m);
}

// ---------------------------------------------------------------- add_diag / h_block
// Keep a stream busy for `ticks` of the 100 MHz wall clock on every launched workgroup (per-rank
// start jitter of the asynchronous virtual ranks; the CU footprint of a transfer in ShadowComm's
// communication-cost model).  Every wave leaves when the time is up.
// lds_bytes > 0: 256-thread workgroups holding that much LDS (the footprint of an RCCL channel).
__global__ __launch_bounds__(256) void spin_kernel(uint64_t ticks) {
  const uint64_t t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(4);
}

// An RCCL channel workgroup's footprint for the communication-cost model (ShadowComm): 256 threads,
// 140 VGPRs per wave (the v139 clobber makes the allocation), the LDS passed at launch -- measured on
// rcclGenericKernel<2, false> of a p = 2 solve (profiles/rccl_footprint_r5.md).
__global__ __launch_bounds__(256) void spin_channel_kernel(uint64_t ticks) {
  asm volatile("v_mov_b32 v139, 0" ::: "v139");
  const uint64_t t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(4);
}

void spin(int nwg, double us, hipStream_t s, int lds_bytes) {
  if (nwg <= 0 || !(us > 0)) return;
  const uint64_t ticks = (uint64_t)(us * 100.0);  // wall_clock64: 100 MHz
  if (lds_bytes > 0)
    hipLaunchKernelGGL(spin_channel_kernel, dim3((unsigned)nwg), dim3(256), (size_t)lds_bytes, s, ticks);
  else
    hipLaunchKernelGGL(spin_kernel, dim3((unsigned)nwg), dim3(64), 0, s, ticks);
}

// The receiving channels of a modelled transfer write its bytes (ShadowComm): zeros, 16-byte vector
// stores spread over the launched workgroups, the same 140-VGPR / LDS footprint as spin_channel_kernel.
__global__ __launch_bounds__(256) void zero_channel_kernel(uint4* p, size_t n16, unsigned char* tail, int ntail) {
  asm volatile("v_mov_b32 v139, 0" ::: "v139");
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  const uint4 z = make_uint4(0u, 0u, 0u, 0u);
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) p[i] = z;
  if (blockIdx.x == 0 && (int)threadIdx.x < ntail) tail[threadIdx.x] = 0;
}

void zero_channels(void* p, size_t bytes, int nwg, int lds_bytes, hipStream_t s) {
  if (!bytes || nwg <= 0) return;
  // the engine's buffers are 16-byte aligned; a misaligned head goes to hipMemsetAsync
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  if (a & 15) {
    (void)hipMemsetAsync(p, 0, bytes, s);
    return;
  }
  const size_t n16 = bytes / 16;
  const int ntail = (int)(bytes % 16);
  hipLaunchKernelGGL(zero_channel_kernel, dim3((unsigned)nwg), dim3(256), (size_t)lds_bytes, s,
                     static_cast<uint4*>(p), n16, static_cast<unsigned char*>(p) + n16 * 16, ntail);
}

template <typename T>
__global__ void add_diag_kernel(T* A, int64_t ld, int64_t nd, double alpha) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nd) A[i * ld + i] += (T)alpha;
}

void add_diag(DType dt, void* A, int64_t ld, int64_t nd, double alpha, hipStream_t s) {
  if (nd <= 0) return;
  const unsigned grid = grid_for(nd, 256);
  if (dt == DType::F64)
    hipLaunchKernelGGL(add_diag_kernel<double>, dim3(grid), dim3(256), 0, s, static_cast<double*>(A),
                       ld, nd, alpha);
  else
    hipLaunchKernelGGL(add_diag_kernel<float>, dim3(grid), dim3(256), 0, s, static_cast<float*>(A), ld,
                       nd, alpha);
}

template <typename T>
__global__ void h_block_kernel(T* R, int64_t ldr, const T* Ht, int64_t m) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= m * m) return;
  const int64_t i = e / m, j = e - i * m;
  R[i * ldr + j] = Ht[j * m + i];
}

void h_block(DType dt, void* R, int64_t ldr, const void* Ht, int64_t m, hipStream_t s) {
  const unsigned grid = grid_for(m * m, 256);
  if (dt == DType::F64)
    hipLaunchKernelGGL(h_block_kernel<double>, dim3(grid), dim3(256), 0, s, static_cast<double*>(R), ldr,
                       static_cast<const double*>(Ht), m);
  else
    hipLaunchKernelGGL(h_block_kernel<float>, dim3(grid), dim3(256), 0, s, static_cast<float*>(R), ldr,
                       static_cast<const float*>(Ht), m);
}

// ---------------------------------------------------------------- pivot selection
// GJ_HOST_FENCE=1: publish the host's pivot mirror behind system-scope fences (the round-4 form)
// instead of system-scope relaxed stores (pivot_select.hpp pivot_finish).
int host_fence() {
  static const int v = [] {
    const char* e = std::getenv("GJ_HOST_FENCE");
    return (e && *e) ? (std::atoi(e) != 0) : 0;
  }();
  return v;
}

__global__ __launch_bounds__(64) void pivot_local_kernel(const double* scores, const int32_t* valid,
                                                         const int32_t* used, const int32_t* pos,
                                                         int64_t nblk, int64_t p, int64_t k,
                                                         PivotRec* out) {
  const PivotRec best = pivot_local_wave(scores, valid, used, pos, nblk, p, k);
  if (threadIdx.x == 0) *out = best;
}

void pivot_local(const double* scores, const int32_t* valid, const int32_t* used, const int32_t* pos,
                 const Layout& L, PivotRec* out, hipStream_t s) {
  hipLaunchKernelGGL(pivot_local_kernel, dim3(1), dim3(64), 0, s, scores, valid, used, pos, L.nblk,
                     L.p, L.k, out);
}

__global__ __launch_bounds__(64) void pivot_global_kernel(const PivotRec* recs, int32_t p, int32_t t,
                                                          int32_t* pos, int32_t* phys_at, int32_t* used,
                                                          int32_t* seq, PivotResult* out,
                                                          PivotResult* host_out, int sysfence) {
  const PivotRec best = pivot_gathered_wave(recs, p);
  if (threadIdx.x != 0) return;
  pivot_finish(best, p, t, pos, phys_at, used, seq, out, host_out, sysfence);
}

// p == 1: local argmin and global book-keeping in one launch (the rank's record is the gathered set).
__global__ __launch_bounds__(64) void pivot_select_single_kernel(
    const double* scores, const int32_t* valid, int64_t nblk, int32_t t, int32_t* pos,
    int32_t* phys_at, int32_t* used, int32_t* seq, PivotRec* rec, PivotResult* out,
    PivotResult* host_out, int sysfence) {
  const PivotRec best = pivot_local_wave(scores, valid, used, pos, nblk, 1, 0);
  if (threadIdx.x != 0) return;
  *rec = best;
  pivot_finish(best, 1, t, pos, phys_at, used, seq, out, host_out, sysfence);
}

void pivot_select_single(const double* scores, const int32_t* valid, const Layout& L, int32_t t,
                         int32_t* pos, int32_t* phys_at, int32_t* used, int32_t* seq, PivotRec* rec,
                         PivotResult* out, PivotResult* host_out, hipStream_t s) {
  hipLaunchKernelGGL(pivot_select_single_kernel, dim3(1), dim3(64), 0, s, scores, valid, L.nblk, t, pos,
                     phys_at, used, seq, rec, out, host_out, host_fence());
}

void pivot_global(const PivotRec* recs, int32_t p, int32_t t, int32_t* pos, int32_t* phys_at,
                  int32_t* used, int32_t* seq, PivotResult* out, PivotResult* host_out, hipStream_t s) {
  hipLaunchKernelGGL(pivot_global_kernel, dim3(1), dim3(64), 0, s, recs, p, t, pos, phys_at, used, seq,
                     out, host_out, host_fence());
}

// ---------------------------------------------------------------- partial pivoting (--pivot partial)
// Score of every local candidate block W_b = -(Lt block b)^T: its largest magnitude (scores[b] =
// -max|W_b|, so the common argmin picks the largest), valid when that is >= thresh.  One
// workgroup per block: each thread scans a strided part of the m x m block (K-major: column c of
// W_b is the contiguous run Lt[c*ldl + b*m .. + m)).
template <typename T>
__global__ __launch_bounds__(256) void candidate_maxabs_kernel(const T* __restrict__ Lt, int64_t ldl, int m,
                                                               int64_t p, int64_t k, double thresh,
                                                               const int32_t* __restrict__ used,
                                                               double* __restrict__ scores,
                                                               int32_t* __restrict__ valid) {
  const int b = blockIdx.x;
  if (used[(int64_t)b * p + k]) {
    if (threadIdx.x == 0) {
      valid[b] = 0;
      scores[b] = 0.0;
    }
    return;
  }
  double mx = 0.0;
  const int64_t total = (int64_t)m * m;
  for (int64_t e = threadIdx.x; e < total; e += blockDim.x) {
    const int64_t c = e / m, i = e - c * m;
    mx = fmax(mx, fabs((double)Lt[c * ldl + (int64_t)b * m + i]));
  }
  __shared__ double red[4];
  mx = wave_max_f64(mx);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) mx = fmax(mx, red[w]);
    mx = fmax(mx, red[0]);
    scores[b] = -mx;
    valid[b] = (mx >= thresh && isfinite(mx)) ? 1 : 0;
  }
}

void candidate_maxabs(DType dt, const void* Lt, int64_t ldl, double* scores, int32_t* valid,
                      const int32_t* used, const Layout& L, double thresh, hipStream_t s) {
  if (L.nblk <= 0) return;
  if (dt == DType::F64)
    hipLaunchKernelGGL(candidate_maxabs_kernel<double>, dim3((unsigned)L.nblk), dim3(256), 0, s,
                       static_cast<const double*>(Lt), ldl, (int)L.m, L.p, L.k, thresh, used, scores, valid);
  else
    hipLaunchKernelGGL(candidate_maxabs_kernel<float>, dim3((unsigned)L.nblk), dim3(256), 0, s,
                       static_cast<const float*>(Lt), ldl, (int)L.m, L.p, L.k, thresh, used, scores, valid);
}

// The chosen local candidate (rec, from pivot_local) copied out of Lt into sel (K-major m x m,
// ld m: the single-block operand of block_inverse); an invalid record gives -I (W = I).
template <typename T>
__global__ __launch_bounds__(256) void gather_candidate_kernel(T* __restrict__ sel, const T* __restrict__ Lt,
                                                               int64_t ldl, int m, int64_t p,
                                                               const PivotRec* __restrict__ rec) {
  const bool ok = rec->valid != 0;
  const int64_t b = ok ? (int64_t)rec->phys / p : 0;
  const int64_t total = (int64_t)m * m;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = e / m, i = e - c * m;
    sel[e] = ok ? Lt[c * ldl + b * m + i] : (c == i ? T(-1) : T(0));
  }
}

void gather_candidate(DType dt, void* sel, const void* Lt, int64_t ldl, const PivotRec* rec, const Layout& L,
                      hipStream_t s) {
  const unsigned grid = grid_for(L.m * L.m, 256, 64);
  if (dt == DType::F64)
    hipLaunchKernelGGL(gather_candidate_kernel<double>, dim3(grid), dim3(256), 0, s, static_cast<double*>(sel),
                       static_cast<const double*>(Lt), ldl, (int)L.m, L.p, rec);
  else
    hipLaunchKernelGGL(gather_candidate_kernel<float>, dim3(grid), dim3(256), 0, s, static_cast<float*>(sel),
                       static_cast<const float*>(Lt), ldl, (int)L.m, L.p, rec);
}

// After block_inverse on sel: the chosen candidate's slot of inv_t := inv1, and the record stays
// valid only if that inverse exists (rec->valid &= valid1[0]).
template <typename T>
__global__ __launch_bounds__(256) void commit_candidate_kernel(T* __restrict__ inv_t, const T* __restrict__ inv1,
                                                               const int32_t* __restrict__ valid1,
                                                               const double* __restrict__ score1, double growth,
                                                               int m, int64_t p, PivotRec* __restrict__ rec) {
  // growth guard (SolveOptions::pivot_growth): ||inv(W)||_inf * max|W| above the bound = singular
  const bool ok = rec->valid != 0 && valid1[0] != 0 && (growth <= 0.0 || score1[0] * -rec->score <= growth);
  const int64_t b = (int64_t)rec->phys / p;
  const int64_t total = (int64_t)m * m;
  if (ok)
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * blockDim.x)
      inv_t[b * total + e] = inv1[e];
  __syncthreads();  // every thread has read rec before thread 0 of block 0 rewrites it
  if (blockIdx.x == 0 && threadIdx.x == 0 && !ok) rec->valid = 0;
}

void commit_candidate(DType dt, void* inv_t, const void* inv1, const int32_t* valid1, const double* score1, double growth, PivotRec* rec,
                      const Layout& L, hipStream_t s) {
  // one workgroup: rec is read by every thread before thread 0 may clear it
  if (dt == DType::F64)
    hipLaunchKernelGGL(commit_candidate_kernel<double>, dim3(1), dim3(256), 0, s, static_cast<double*>(inv_t),
                       static_cast<const double*>(inv1), valid1, score1, growth, (int)L.m, L.p, rec);
  else
    hipLaunchKernelGGL(commit_candidate_kernel<float>, dim3(1), dim3(256), 0, s, static_cast<float*>(inv_t),
                       static_cast<const float*>(inv1), valid1, score1, growth, (int)L.m, L.p, rec);
}

// ---------------------------------------------------------------- owner edits (one launch)
// The pivot comes from device memory (the step's pivot-sequence entry): the launch can be enqueued
// before the host has seen the pivot, and is a no-op on ranks that do not own it.
// Work items in one flat range: the At row edits, the H copy, then (PieceMove) the pivot row's
// piece moved out of X and the identity block.
template <typename T>
__global__ __launch_bounds__(256) void owner_edits_kernel(T* At, int64_t ldl, const int32_t* __restrict__ phys,
                                                          int64_t p, int64_t k, int64_t j, int64_t m, T* lrow, T* ht,
                                                          const T* inv, PieceMove mv) {
  const int64_t g = *phys;
  if (g < 0 || g % p != k) return;
  const int64_t b = g / p, row0 = b * m;
  const T* inv_blk = inv + b * m * m;
  // the flat index space in 32 bits (every section is far below 2^31 elements): a 32-bit division
  // per element instead of the 64-bit division routine (the pivot chain waits for this launch)
  const uint32_t mu = (uint32_t)m, wu = (uint32_t)(mv.w > 0 ? mv.w : 1), jm = (uint32_t)(j * m);
  const uint32_t total = (uint32_t)((j + 1) * m * m), e1 = total + mu * mu, e2 = e1 + mu * (uint32_t)mv.w,
                 e3 = e2 + (mv.eye ? mu * mu : 0u);
  for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < e3; e += gridDim.x * blockDim.x) {
    if (e < total) {
      const uint32_t kk = e / mu, c = e - kk * mu;
      T* x = At + (int64_t)kk * ldl + row0 + c;
      if (kk < jm) lrow[e] = *x;  // lrow[kk * m + c]
      *x = (kk - jm == c) ? T(1) : T(0);
    } else if (e < e1) {
      ht[e - total] = inv_blk[e - total];
    } else if (e < e2) {
      const uint32_t r = (e - e1) / wu, c = (e - e1) - r * wu;
      T* x = static_cast<T*>(mv.X) + (row0 + r) * mv.ldx + mv.col0 + c;
      static_cast<T*>(mv.dst)[(int64_t)r * mv.ldd + c] = *x;
      *x = T(0);
    } else {
      const uint32_t r = (e - e2) / mu, c = (e - e2) - r * mu;
      static_cast<T*>(mv.eye)[(int64_t)r * mv.ld_eye + c] = (r == c) ? T(1) : T(0);
    }
  }
}

void owner_edits(DType dt, void* At, int64_t ldl, const int32_t* phys, int64_t p, int64_t k, int64_t j,
                 int64_t m, void* lrow, void* ht, const void* inv, const PieceMove& mv, hipStream_t s) {
  const int64_t work = (j + 2) * m * m + m * mv.w + (mv.eye ? m * m : 0);
  const unsigned grid = grid_for(work, 256, 256);
  if (dt == DType::F64)
    hipLaunchKernelGGL(owner_edits_kernel<double>, dim3(grid), dim3(256), 0, s, static_cast<double*>(At), ldl, phys,
                       p, k, j, m, static_cast<double*>(lrow), static_cast<double*>(ht),
                       static_cast<const double*>(inv), mv);
  else
    hipLaunchKernelGGL(owner_edits_kernel<float>, dim3(grid), dim3(256), 0, s, static_cast<float*>(At), ldl, phys, p,
                       k, j, m, static_cast<float*>(lrow), static_cast<float*>(ht), static_cast<const float*>(inv),
                       mv);
}

// The pivot row's piece of the panel's later columns, moved out (copied, then zeroed in X).
template <typename T>
__global__ __launch_bounds__(256) void take_rows_kernel(T* dst, int64_t ldd, T* X, int64_t ldx,
                                                        const int32_t* __restrict__ phys, int64_t p, int64_t k,
                                                        int64_t col0, int64_t w, int64_t m) {
  const int64_t g = *phys;
  if (g < 0 || g % p != k) return;
  const int64_t row0 = (g / p) * m, total = m * w;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / w, c = e - r * w;
    T* x = X + (row0 + r) * ldx + col0 + c;
    dst[r * ldd + c] = *x;
    *x = T(0);
  }
}

void take_rows(DType dt, void* dst, int64_t ldd, void* X, int64_t ldx, const int32_t* phys, int64_t p, int64_t k,
               int64_t col0, int64_t w, int64_t m, hipStream_t s) {
  if (w <= 0 || m <= 0) return;
  const unsigned grid = grid_for(m * w, 256, 256);
  if (dt == DType::F64)
    hipLaunchKernelGGL(take_rows_kernel<double>, dim3(grid), dim3(256), 0, s, static_cast<double*>(dst), ldd,
                       static_cast<double*>(X), ldx, phys, p, k, col0, w, m);
  else
    hipLaunchKernelGGL(take_rows_kernel<float>, dim3(grid), dim3(256), 0, s, static_cast<float*>(dst), ldd,
                       static_cast<float*>(X), ldx, phys, p, k, col0, w, m);
}

// ---------------------------------------------------------------- root-agnostic exchange helpers
template <typename T>
__global__ __launch_bounds__(256) void sum_slices_kernel(T* __restrict__ dst, const T* __restrict__ src, int64_t count,
                                                         int64_t nslices) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (int64_t)gridDim.x * blockDim.x) {
    T acc = src[i];
    for (int64_t q = 1; q < nslices; ++q) acc += src[q * count + i];
    dst[i] = acc;
  }
}

void sum_slices(DType dt, void* dst, const void* src, int64_t count, int64_t nslices, hipStream_t s) {
  if (count <= 0) return;
  const unsigned grid = grid_for(count, 256, 1024);
  if (dt == DType::F64)
    hipLaunchKernelGGL(sum_slices_kernel<double>, dim3(grid), dim3(256), 0, s, static_cast<double*>(dst),
                       static_cast<const double*>(src), count, nslices);
  else
    hipLaunchKernelGGL(sum_slices_kernel<float>, dim3(grid), dim3(256), 0, s, static_cast<float*>(dst),
                       static_cast<const float*>(src), count, nslices);
}

template <typename T>
__global__ __launch_bounds__(256) void zero_unless_owner_kernel(T* buf, int64_t count, const int32_t* __restrict__ phys,
                                                                int64_t p, int64_t k) {
  const int64_t g = *phys;
  if (g >= 0 && g % p == k) return;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (int64_t)gridDim.x * blockDim.x)
    buf[i] = T(0);
}

void zero_unless_owner(DType dt, void* buf, int64_t count, const int32_t* phys, int64_t p, int64_t k, hipStream_t s) {
  if (count <= 0) return;
  const unsigned grid = grid_for(count, 256, 1024);
  if (dt == DType::F64)
    hipLaunchKernelGGL(zero_unless_owner_kernel<double>, dim3(grid), dim3(256), 0, s, static_cast<double*>(buf), count,
                       phys, p, k);
  else
    hipLaunchKernelGGL(zero_unless_owner_kernel<float>, dim3(grid), dim3(256), 0, s, static_cast<float*>(buf), count,
                       phys, p, k);
}

// ---------------------------------------------------------------- permute_blocks
template <typename T>
__global__ __launch_bounds__(256) void permute_kernel(T* __restrict__ dst, int64_t ldd,
                                                      const T* __restrict__ X, int64_t ldx, int m,
                                                      int64_t ncols, const int32_t* dst_blk,
                                                      const int32_t* colsrc) {
  const int64_t row = blockIdx.x;  // local row of X
  const int64_t b = row / m, r = row - b * m;
  T* d = dst + ((int64_t)dst_blk[b] * m + r) * ldd;
  const T* s = X + row * ldx;
  // whole column blocks per iteration (no per-element index division): block c of the output row is
  // block colsrc[c] of the input row, m contiguous elements each
  const int64_t nb = ncols / m;
  const int per = 256 / m > 0 ? 256 / m : 1;  // column blocks handled together by the 256 threads
  const int lb = (int)threadIdx.x / m, jj = (int)threadIdx.x - lb * m;
  if (m <= 256) {
    for (int64_t c = (int64_t)blockIdx.y * per + lb; c < nb; c += (int64_t)gridDim.y * per)
      if (lb < per) d[c * m + jj] = s[(int64_t)colsrc[c] * m + jj];
  } else {
    for (int64_t c = blockIdx.y; c < nb; c += gridDim.y)
      for (int j = threadIdx.x; j < m; j += 256) d[c * m + j] = s[(int64_t)colsrc[c] * m + j];
  }
}

// 16-byte form: each thread moves UNR vectors per trip, all loads issued before the stores (the
// scalar form above held one 8-byte load in flight per thread: N = 32768 fp64 3.9 ms = 4.4 TB/s,
// N = 8192 308 us).  vpb = 16-byte vectors per column block.
template <int UNR>
__global__ __launch_bounds__(256) void permute_vec_kernel(uint4* __restrict__ dst, int64_t ldd4,
                                                          const uint4* __restrict__ X, int64_t ldx4,
                                                          int m, unsigned vpb, unsigned nvec,
                                                          const int32_t* dst_blk, const int32_t* colsrc) {
  const int64_t row = blockIdx.x;
  const int64_t b = row / m, r = row - b * m;
  uint4* d = dst + ((int64_t)dst_blk[b] * m + r) * ldd4;
  const uint4* s = X + row * ldx4;
  const unsigned stride = gridDim.y * 256u;
  for (unsigned i0 = blockIdx.y * 256u + threadIdx.x; i0 < nvec; i0 += stride * UNR) {
    uint4 v[UNR];
    unsigned at[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const unsigned i = i0 + (unsigned)u * stride;
      at[u] = i;
      if (i < nvec) {
        const unsigned c = i / vpb, j = i - c * vpb;
        v[u] = s[(int64_t)colsrc[c] * vpb + j];
      }
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u)
      if (at[u] < nvec) d[at[u]] = v[u];
  }
}

void permute_blocks(DType dt, void* dst, int64_t ldd, const void* X, int64_t ldx, int64_t nblk,
                    int64_t m, int64_t Nr, const int32_t* dst_blk, const int32_t* colsrc,
                    hipStream_t s) {
  if (nblk <= 0) return;
  const int64_t ncols = Nr * m;
  const int64_t es = dt == DType::F64 ? 8 : 4;
  const bool aligned = (m * es) % 16 == 0 && (ldd * es) % 16 == 0 && (ldx * es) % 16 == 0 &&
                       (reinterpret_cast<uintptr_t>(dst) % 16) == 0 && (reinterpret_cast<uintptr_t>(X) % 16) == 0 &&
                       ncols * es / 16 < (int64_t(1) << 31);
  if (aligned) {
    constexpr int kUnr = 4;
    const unsigned vpb = (unsigned)(m * es / 16), nvec = (unsigned)(ncols * es / 16);
    const unsigned gy = (unsigned)std::max<int64_t>(1, std::min<int64_t>((nvec + 256 * kUnr - 1) / (256 * kUnr), 64));
    hipLaunchKernelGGL(permute_vec_kernel<kUnr>, dim3((unsigned)(nblk * m), gy), dim3(256), 0, s,
                       static_cast<uint4*>(dst), ldd * es / 16, static_cast<const uint4*>(X), ldx * es / 16, (int)m,
                       vpb, nvec, dst_blk, colsrc);
    return;
  }
  const int64_t per = std::max<int64_t>(1, 256 / m);
  const unsigned gy = (unsigned)std::min<int64_t>((Nr + per * 4 - 1) / (per * 4), 64);
  dim3 grid((unsigned)(nblk * m), gy);
  if (dt == DType::F64)
    hipLaunchKernelGGL(permute_kernel<double>, grid, dim3(256), 0, s, static_cast<double*>(dst), ldd,
                       static_cast<const double*>(X), ldx, (int)m, ncols, dst_blk, colsrc);
  else
    hipLaunchKernelGGL(permute_kernel<float>, grid, dim3(256), 0, s, static_cast<float*>(dst), ldd,
                       static_cast<const float*>(X), ldx, (int)m, ncols, dst_blk, colsrc);
}

// ---------------------------------------------------------------- verification hash
// parts[g] = sum (mod 2^64) of hash_term over the words workgroup g visits (grid-stride); every
// workgroup writes its own part with one vector store (no atomics), the host adds the parts.
__global__ __launch_bounds__(256) void hash_rows_kernel(const uint8_t* base, int64_t ld_bytes, int64_t wwords,
                                                        int64_t rows, uint64_t* parts) {
  const int64_t total = wwords * rows;
  uint64_t h = 0;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int64_t r = e / wwords, w = e - r * wwords;
    const uint32_t v = *reinterpret_cast<const uint32_t*>(base + r * ld_bytes + 4 * w);
    h += hash_term(v, (uint64_t)e);
  }
  __shared__ uint64_t sh[256];
  sh[threadIdx.x] = h;
  __syncthreads();
  for (int o = 128; o >= 1; o >>= 1) {
    if ((int)threadIdx.x < o) sh[threadIdx.x] += sh[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) parts[blockIdx.x] = sh[0];
}

void hash_rows(const void* base, int64_t ld_bytes, int64_t width_bytes, int64_t rows, uint64_t* parts,
               int nparts, hipStream_t s) {
  hipLaunchKernelGGL(hash_rows_kernel, dim3((unsigned)nparts), dim3(256), 0, s, static_cast<const uint8_t*>(base),
                     ld_bytes, width_bytes / 4, rows, parts);
}

// ---------------------------------------------------------------- norms
template <typename T>
__global__ __launch_bounds__(256) void row_abs_kernel(const T* X, int64_t ldx, int64_t n, int64_t m,
                                                      int64_t p, int64_t k, double* out, int minus_i) {
  const int64_t r = blockIdx.x;
  const int64_t gr = ((r / m) * p + k) * m + r % m;
  if (gr >= n) return;
  double s = 0.0;
  for (int64_t j = threadIdx.x; j < n; j += 256)
    s += fabs((double)X[r * ldx + j] - ((minus_i && j == gr) ? 1.0 : 0.0));
  __shared__ double sh[4];
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off, 64);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) atomic_max_nonneg(out, sh[0] + sh[1] + sh[2] + sh[3]);
}

void row_abs_max(DType dt, const void* X, int64_t ldx, const Layout& L, double* out, hipStream_t s,
                 bool minus_identity) {
  (void)hipMemsetAsync(out, 0, sizeof(double), s);
  if (L.rows <= 0) return;
  const int mi = minus_identity ? 1 : 0;
  if (dt == DType::F64)
    hipLaunchKernelGGL(row_abs_kernel<double>, dim3((unsigned)L.rows), dim3(256), 0, s,
                       static_cast<const double*>(X), ldx, L.n, L.m, L.p, L.k, out, mi);
  else
    hipLaunchKernelGGL(row_abs_kernel<float>, dim3((unsigned)L.rows), dim3(256), 0, s,
                       static_cast<const float*>(X), ldx, L.n, L.m, L.p, L.k, out, mi);
}

__global__ __launch_bounds__(256) void residual_reduce_kernel(const double* partial, int nparts,
                                                              int64_t rows, int64_t n, int64_t m,
                                                              int64_t p, int64_t k, double* out) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  double s = 0.0;
  bool real = false;
  if (r < rows) {
    const int64_t gr = ((r / m) * p + k) * m + r % m;
    real = gr < n;
    if (real)
      for (int q = 0; q < nparts; ++q) s += partial[r * nparts + q];
  }
  double v = real ? s : 0.0;
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = fmax(v, __shfl_xor(v, off, 64));
  if ((threadIdx.x & 63) == 0) atomic_max_nonneg(out, v);
}

void residual_reduce(const double* partial, int nparts, const Layout& L, double* out, hipStream_t s) {
  (void)hipMemsetAsync(out, 0, sizeof(double), s);
  if (L.rows <= 0) return;
  hipLaunchKernelGGL(residual_reduce_kernel, dim3((unsigned)((L.rows + 255) / 256)), dim3(256), 0, s,
                     partial, nparts, L.rows, L.n, L.m, L.p, L.k, out);
}

}  // namespace kern
}  // namespace gj
