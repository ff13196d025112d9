// gfx950 fp64 elimination GEMM on the VALU (v_fma_f64), an alternative to the MFMA kernel in
// gemm.hip with identical semantics (MODE_ACC with zero columns / pivot rows, MODE_STORE).
//
// Why: measured on MI355X (bench/mfma_peak.hip, profiles/mfma_peak.md) the fp64 VALU sustains
// ~66 TF/s while v_mfma_f64_16x16x4_f64 sustains ~49-52 TF/s — unlike bf16/fp32, fp64 matrix-core
// issue is slower than the fp64 vector pipe on CDNA4.  This kernel register-blocks 8 x 8 outputs per
// thread (64 independent FMA chains), streams A^T / B K-slices through LDS with conflict-free reads
// (A: 4 x ds_read_b128 per k, 4 distinct addresses per wave; B: 8 x ds_read_b64 per k, 128 B
// contiguous per 16 lanes) and keeps the same tile-relative buffer addressing as the MFMA kernel.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.hpp"

namespace gj {
namespace kern {

namespace {
constexpr int VBM = 128, VBN = 128, VBK = 16, VNT = 256, VPAD = 8;
constexpr int VLA = VBM + VPAD, VLB = VBN + VPAD;
constexpr int kRec = 0x7ffffff0;
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef double d2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t vrsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, kRec, 0x00020000);
}
__device__ __forceinline__ double vload(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0));
}
__device__ __forceinline__ void vstore(double v, __amdgpu_buffer_rsrc_t r, int voff, int soff) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, voff, soff, 0);
}
__device__ __forceinline__ int vremap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8, x = bid % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
}
}  // namespace

struct VArgs {
  int64_t M, N, K;
  const double* At;  // K-major A: At[k*lda + i]
  int64_t lda;
  const double* B;
  int64_t ldb;
  double* C;
  int64_t ldc;
  int tiles_m, tiles_n;
  int64_t zc0, zc1;
  int64_t zr[GemmExtra::kMaxZeroRows];
  int64_t zh;
  int store;  // 1: C = A*B, 0: C += A*B
};

__global__ __launch_bounds__(VNT, 2) void gemm_valu_f64(VArgs g) {
  __shared__ double lA[2][VBK][VLA];
  __shared__ double lB[2][VBK][VLB];
  const int nwg = g.tiles_m * g.tiles_n;
  const int tile = vremap((int)blockIdx.x, nwg);
  const int tm = tile / g.tiles_n, tn = tile % g.tiles_n;
  const int64_t m0 = (int64_t)tm * VBM, n0 = (int64_t)tn * VBN;
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;  // rows ty*8 + r, cols tx + 16*c
  const int ldc = (int)g.ldc, ldb = (int)g.ldb, lda = (int)g.lda;

  const int Mt = (int)((g.M - m0) < VBM ? (g.M - m0) : VBM);
  const int Nt = (int)((g.N - n0) < VBN ? (g.N - n0) : VBN);
  const int64_t zlo = g.zc0 - n0, zhi = g.zc1 - n0;
  const int z0 = (int)(zlo < 0 ? 0 : (zlo > VBN ? VBN : zlo)), z1 = (int)(zhi < 0 ? 0 : (zhi > VBN ? VBN : zhi));
  int zr0[GemmExtra::kMaxZeroRows], zr1[GemmExtra::kMaxZeroRows];
#pragma unroll
  for (int z = 0; z < GemmExtra::kMaxZeroRows; ++z) {
    const int64_t lo = g.zr[z] - m0, hi = g.zr[z] + g.zh - m0;
    zr0[z] = (int)(lo < 0 ? 0 : (lo > VBM ? VBM : lo));
    zr1[z] = (int)(hi < 0 ? 0 : (hi > VBM ? VBM : hi));
  }

  __amdgpu_buffer_rsrc_t rc = vrsrc(g.C + m0 * g.ldc + n0);
  const int cvoff = ((ty * 8) * ldc + tx) * 8;

  double acc[8][8];
  if (!g.store) {
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int rr = ty * 8 + r;
      bool zrow = false;
#pragma unroll
      for (int z = 0; z < GemmExtra::kMaxZeroRows; ++z) zrow |= (rr >= zr0[z] && rr < zr1[z]);
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const int cc = tx + 16 * c;
        const bool ok = rr < Mt && cc < Nt && !zrow && !(cc >= z0 && cc < z1);
        acc[r][c] = ok ? vload(rc, cvoff + c * 16 * 8, r * ldc * 8) : 0.0;
      }
    }
  } else {
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
      for (int c = 0; c < 8; ++c) acc[r][c] = 0.0;
  }

  // staging: 8 A + 8 B elements per thread per 16-deep slice; (k = e*2 + tid/128, i = tid%128)
  const int sk = tid >> 7, si = tid & 127;
  const bool a_ok = (m0 + si) < g.M, b_ok = (n0 + si) < g.N;
  const int a_voff = (sk * lda + si) * 8, b_voff = (sk * ldb + si) * 8;
  double ra[8], rb[8];
  auto load_slice = [&](int64_t k0) {
    __amdgpu_buffer_rsrc_t rar = vrsrc(g.At + k0 * g.lda + m0);
    __amdgpu_buffer_rsrc_t rbr = vrsrc(g.B + k0 * g.ldb + n0);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const bool kok = (k0 + e * 2 + sk) < g.K;
      ra[e] = (kok && a_ok) ? vload(rar, a_voff, e * 2 * lda * 8) : 0.0;
      rb[e] = (kok && b_ok) ? vload(rbr, b_voff, e * 2 * ldb * 8) : 0.0;
    }
  };
  auto store_slice = [&](int buf) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      lA[buf][e * 2 + sk][si] = ra[e];
      lB[buf][e * 2 + sk][si] = rb[e];
    }
  };

  const int nk = (int)((g.K + VBK - 1) / VBK);
  load_slice(0);
  store_slice(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load_slice((int64_t)(kt + 1) * VBK);
#pragma unroll 4
    for (int k = 0; k < VBK; ++k) {
      double a[8], b[8];
      const d2* ap = reinterpret_cast<const d2*>(&lA[cur][k][ty * 8]);
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        const d2 v = ap[h];
        a[2 * h] = v.x;
        a[2 * h + 1] = v.y;
      }
#pragma unroll
      for (int c = 0; c < 8; ++c) b[c] = lB[cur][k][tx + 16 * c];
#pragma unroll
      for (int r = 0; r < 8; ++r)
#pragma unroll
        for (int c = 0; c < 8; ++c) acc[r][c] = __builtin_fma(a[r], b[c], acc[r][c]);
    }
    if (kt + 1 < nk) store_slice(cur ^ 1);
    __syncthreads();
  }

#pragma unroll
  for (int r = 0; r < 8; ++r)
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int rr = ty * 8 + r, cc = tx + 16 * c;
      if (rr < Mt && cc < Nt) vstore(acc[r][c], rc, cvoff + c * 16 * 8, r * ldc * 8);
    }
}

void gemm_valu(int op, int64_t M, int64_t N, int64_t K, const void* At, int64_t lda, const void* B,
               int64_t ldb, void* C, int64_t ldc, hipStream_t s, const GemmExtra* ex) {
  if (M <= 0 || N <= 0) return;
  VArgs a{};
  a.M = M; a.N = N; a.K = K;
  a.At = static_cast<const double*>(At); a.lda = lda;
  a.B = static_cast<const double*>(B); a.ldb = ldb;
  a.C = static_cast<double*>(C); a.ldc = ldc;
  a.tiles_m = (int)((M + VBM - 1) / VBM);
  a.tiles_n = (int)((N + VBN - 1) / VBN);
  constexpr int64_t kNone = -(int64_t(1) << 62);
  a.zc0 = ex ? ex->zc0 : 0;
  a.zc1 = ex ? ex->zc1 : 0;
  a.zh = ex ? ex->zh : 0;
  for (int z = 0; z < GemmExtra::kMaxZeroRows; ++z) a.zr[z] = (ex && z < ex->nzr) ? ex->zr[z] : kNone;
  a.store = op == 1;
  hipLaunchKernelGGL(gemm_valu_f64, dim3((unsigned)(a.tiles_m * a.tiles_n)), dim3(VNT), 0, s, a);
}

}  // namespace kern
}  // namespace gj
