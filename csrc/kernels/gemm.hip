// gfx950 MFMA GEMM for the Gauss-Jordan engine.
//
//   MODE_ACC   : C[M x N] += A * B       (the elimination update, reference mult_substr_block
//                                          main.cpp:151-206 called from the hot loop :1165-1194)
//   MODE_STORE : C[M x N]  = A * B       (pivot-row normalisation, reference mult_block
//                                          main.cpp:888-950 called at :1136-1159)
//   MODE_RESID : per-row partial sums of |A*B - I| (residual, reference matrix_mult_matrix +
//                                          minus_i + norm, main.cpp:534-667, fused: no D matrix)
//
// Tiling (CDNA4, wave64): 128 x 128 output tile per 256-thread workgroup, 4 waves in a 2 x 2 grid,
// each wave owns 64 x 64 = 4 x 4 MFMA tiles of 16 x 16.  fp64 uses v_mfma_f64_16x16x4_f64 (C/D map
// col = lane&15, row = (lane>>4) + 4*reg), fp32 uses v_mfma_f32_16x16x4_f32 (row = 4*(lane>>4) + reg).
// The accumulator is initialised straight from C in the MFMA C/D layout (MODE_ACC), so the
// read-modify-write needs no separate epilogue pass.  K is staged through LDS in BK = 16 slices,
// double-buffered (one barrier per slice); both operands are stored K-major in LDS with a 16-element
// pad so the fragment reads (lanes 0-15 / 16-31 on consecutive k rows) are bank-conflict free.
// Launch bounds allow 2 workgroups per CU (73.7 KiB LDS each) so one workgroup's C load/store
// overlaps the other's MFMA stream.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.hpp"

namespace gj {
namespace kern {

constexpr int BM = 128, BN = 128, BK = 16, NT = 256, PADL = 16;
constexpr int LDSR = BM + PADL;  // LDS row length (elements) of a K-major slice

template <typename T>
struct Mfma;

template <>
struct Mfma<double> {
  typedef double acc_t __attribute__((ext_vector_type(4)));
  static __device__ __forceinline__ acc_t op(double a, double b, acc_t c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ int row_of(int lane, int q) { return (lane >> 4) + 4 * q; }
};

template <>
struct Mfma<float> {
  typedef float acc_t __attribute__((ext_vector_type(4)));
  static __device__ __forceinline__ acc_t op(float a, float b, acc_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ int row_of(int lane, int q) { return 4 * (lane >> 4) + q; }
};

enum { MODE_ACC = 0, MODE_STORE = 1, MODE_RESID = 2 };

struct GemmArgs {
  int64_t M, N, K;
  const void* A;
  int64_t lda;
  const void* B;
  int64_t ldb;
  void* C;
  int64_t ldc;
  int tiles_m, tiles_n;
  // MODE_ACC extras: C columns [zc0, zc1) enter as 0 (the pivot block column: X[i,t] := -L_i H),
  // rows [pr0, pr0 + K) are the pivot block row: they are written with B (= R) instead of C + A*B.
  int64_t zc0, zc1, pr0;
  // residual
  int64_t n_real, blk_m, p, k;
  double* partial;  // [M][nparts]
  int nparts;
};

// XCD-aware bijective remap: blocks b and b+8 share an XCD (MI355X_MICROARCH.md §Workgroup
// dispatch); give every XCD a contiguous range of tiles so neighbouring tiles share L2 lines.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8, x = bid % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
}

template <typename T, int AL, int MODE>
__global__ __launch_bounds__(NT, 2) void gemm_kernel(GemmArgs g) {
  using MF = Mfma<T>;
  using acc_t = typename MF::acc_t;
  __shared__ T lds[2][2][BK][LDSR];  // [buf][A/B][k][row or col]

  const int nwg = g.tiles_m * g.tiles_n;
  const int tile = xcd_remap((int)blockIdx.x, nwg);
  // within an XCD's contiguous range, walk the N tiles fastest (they share the A slab)
  const int tm = tile / g.tiles_n, tn = tile % g.tiles_n;
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const T* __restrict__ A = static_cast<const T*>(g.A);
  const T* __restrict__ B = static_cast<const T*>(g.B);
  T* __restrict__ C = static_cast<T*>(g.C);

  acc_t acc[4][4];
  if (MODE == MODE_ACC) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t col = n0 + wn * 64 + j * 16 + (lane & 15);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int64_t row = m0 + wm * 64 + i * 16 + MF::row_of(lane, q);
          const bool zero = (col >= g.zc0 && col < g.zc1);
          acc[i][j][q] = (row < g.M && col < g.N && !zero) ? C[row * g.ldc + col] : T(0);
        }
      }
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = acc_t{0, 0, 0, 0};
  }

  // ---- global -> register staging of one K slice (8 A + 8 B elements per thread)
  T ra[8], rb[8];
  auto load_slice = [&](int64_t k0) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int idx = e * NT + tid;
      // B: [BK][BN], coalesced along n
      {
        const int kk = idx / BN, nn = idx % BN;
        const int64_t gk = k0 + kk, gn = n0 + nn;
        rb[e] = (gk < g.K && gn < g.N) ? B[gk * g.ldb + gn] : T(0);
      }
      if (AL == 1) {  // K-major A: At[k][i], coalesced along i
        const int kk = idx / BM, ii = idx % BM;
        const int64_t gk = k0 + kk, gi = m0 + ii;
        ra[e] = (gk < g.K && gi < g.M) ? A[gk * g.lda + gi] : T(0);
      } else {  // row-major A: A[i][k], 16 consecutive k per row
        const int ii = idx / BK, kk = idx % BK;
        const int64_t gk = k0 + kk, gi = m0 + ii;
        ra[e] = (gk < g.K && gi < g.M) ? A[gi * g.lda + gk] : T(0);
      }
    }
  };
  auto store_slice = [&](int buf) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int idx = e * NT + tid;
      lds[buf][1][idx / BN][idx % BN] = rb[e];
      if (AL == 1)
        lds[buf][0][idx / BM][idx % BM] = ra[e];
      else
        lds[buf][0][idx % BK][idx / BK] = ra[e];
    }
  };

  const int nk = (int)((g.K + BK - 1) / BK);
  load_slice(0);
  store_slice(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load_slice((int64_t)(kt + 1) * BK);
#pragma unroll
    for (int kk = 0; kk < BK; kk += 4) {
      T a[4], b[4];
      const int kr = kk + (lane >> 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = lds[cur][0][kr][wm * 64 + i * 16 + (lane & 15)];
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = lds[cur][1][kr][wn * 64 + j * 16 + (lane & 15)];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = MF::op(a[i], b[j], acc[i][j]);
    }
    if (kt + 1 < nk) store_slice(cur ^ 1);
    __syncthreads();
  }

  if (MODE == MODE_ACC || MODE == MODE_STORE) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t col = n0 + wn * 64 + j * 16 + (lane & 15);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int64_t row = m0 + wm * 64 + i * 16 + MF::row_of(lane, q);
          if (row < g.M && col < g.N) {
            T v = acc[i][j][q];
            if (MODE == MODE_ACC && row >= g.pr0 && row < g.pr0 + g.K) v = B[(row - g.pr0) * g.ldb + col];
            C[row * g.ldc + col] = v;
          }
        }
      }
  } else {  // MODE_RESID: per-row partial sum of |acc - I| over this wave's 64 real columns
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int64_t row = m0 + wm * 64 + i * 16 + MF::row_of(lane, q);
        const int64_t gr = ((row / g.blk_m) * g.p + g.k) * g.blk_m + row % g.blk_m;
        double s = 0.0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int64_t col = n0 + wn * 64 + j * 16 + (lane & 15);
          if (col < g.n_real) {
            const double v = (double)acc[i][j][q] - (col == gr ? 1.0 : 0.0);
            s += fabs(v);
          }
        }
        // sum across the 16 lanes that share this row (lane & 15)
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) s += __shfl_xor(s, off, 64);
        if ((lane & 15) == 0 && row < g.M)
          g.partial[row * g.nparts + (int64_t)tn * 2 + wn] = s;
      }
  }
}

template <typename T, int AL, int MODE>
static void launch(const GemmArgs& a0, hipStream_t s) {
  GemmArgs a = a0;
  a.tiles_m = (int)((a.M + BM - 1) / BM);
  a.tiles_n = (int)((a.N + BN - 1) / BN);
  const int64_t nwg = (int64_t)a.tiles_m * a.tiles_n;
  if (nwg <= 0) return;
  hipLaunchKernelGGL((gemm_kernel<T, AL, MODE>), dim3((unsigned)nwg), dim3(NT), 0, s, a);
}

void gemm(DType dt, int op, int a_kmajor, int64_t M, int64_t N, int64_t K, const void* A,
          int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, hipStream_t s,
          int64_t zc0, int64_t zc1, int64_t pr0) {
  if (M <= 0 || N <= 0) return;
  GemmArgs a{};
  a.M = M; a.N = N; a.K = K; a.A = A; a.lda = lda; a.B = B; a.ldb = ldb; a.C = C; a.ldc = ldc;
  a.zc0 = zc0; a.zc1 = zc1; a.pr0 = pr0 < 0 ? -(int64_t(1) << 62) : pr0;
  const int mode = op == 0 ? MODE_ACC : MODE_STORE;
#define GJ_DISPATCH(T)                                                        \
  if (a_kmajor) {                                                             \
    if (mode == MODE_ACC) launch<T, 1, MODE_ACC>(a, s);                       \
    else launch<T, 1, MODE_STORE>(a, s);                                      \
  } else {                                                                    \
    if (mode == MODE_ACC) launch<T, 0, MODE_ACC>(a, s);                       \
    else launch<T, 0, MODE_STORE>(a, s);                                      \
  }
  if (dt == DType::F64) {
    GJ_DISPATCH(double)
  } else {
    GJ_DISPATCH(float)
  }
#undef GJ_DISPATCH
}

int residual_nparts(int64_t N) { return (int)(((N + BN - 1) / BN) * 2); }

void residual_partial(DType dt, int64_t M, int64_t N, int64_t K, const void* A, int64_t lda,
                      const void* B, int64_t ldb, int64_t n_real, int64_t blk_m, int64_t p,
                      int64_t k, double* partial, hipStream_t s) {
  if (M <= 0 || N <= 0) return;
  GemmArgs a{};
  a.M = M; a.N = N; a.K = K; a.A = A; a.lda = lda; a.B = B; a.ldb = ldb; a.C = nullptr; a.ldc = 0;
  a.zc0 = a.zc1 = 0; a.pr0 = -(int64_t(1) << 62);
  a.n_real = n_real; a.blk_m = blk_m; a.p = p; a.k = k; a.partial = partial;
  a.nparts = residual_nparts(N);
  if (dt == DType::F64)
    launch<double, 0, MODE_RESID>(a, s);
  else
    launch<float, 0, MODE_RESID>(a, s);
}

}  // namespace kern
}  // namespace gj
