// Candidate-block inversion for 128 < m <= 256 in fp64 (gfx950) — the blocks that no longer fit a
// workgroup's registers (a 256 x 256 fp64 block is 512 KiB: the whole VGPR file of a CU).
//
// Reference: inverse_block (main.cpp:746-820: scalar Gauss-Jordan, partial pivoting with the first
// maximum winning, singular when |a_kk| < EPS*norm) + block_norm (main.cpp:669-683), run for every
// candidate block of the pivot search (main.cpp:1039-1066).  Output contract as blockinv.hip: the
// inverse transposed (the K-major GEMM operand H^T), ||inv||_inf, validity.
//
// One workgroup per candidate block: 8 BLOCK waves + 1 PIVOT wave.  The block lives in an
// L2-resident scratch image in MFMA fragment order (tile (rt, ct) = 64 lanes x 4 consecutive
// values, so every tile load / store is one fully coalesced 2 KiB access).  Block wave w owns the
// column tiles w and w + 8 for the whole kernel, so the only cross-wave traffic is LDS:
//  * the pivot wave factors a 256 x 16 panel in registers (4 rows per lane; the software-pipelined
//    PivotPanel of blockinv_mfma.hip: exact wave argmax, v_rcp + Newton, updates in the gaps) and
//    publishes the multipliers U (LDS) and the 16 pivot rows;
//  * every block wave reads the panel's pivot rows over ITS columns from its own tiles (R), then
//    applies X += U R tile by tile with v_mfma_f64_16x16x4f64 (4 per tile), and the panel's own
//    column tile becomes U + E;
//  * look-ahead: the owner of the next panel's column tile updates that tile FIRST and hands it to
//    the pivot wave through LDS (barrier B0), so the next panel's factorisation runs while the
//    block waves update the rest (barrier B1 when it is done): two barriers per panel.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstdint>

#include "kernels.hpp"
#include "pivot_panel.hpp"
#include "pivot_select.hpp"
#include "wave_ops.hpp"

namespace gj {
namespace kern {

namespace {

constexpr int kBigLDU = 17;   // padded row of the U / panel images

// v_mfma_f64_16x16x4f64: A lane l = A[l & 15][l >> 4], B lane l = B[l >> 4][l & 15],
// C/D lane l register r = D[(l >> 4) + 4 r][l & 15].
typedef double acc4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int frow(int lane, int r) { return (lane >> 4) + 4 * r; }

// element (row, col) of the fragment image (tile-major; 16 x 16 tiles of 64 lanes x 4 values)
template <int NT>
__device__ __forceinline__ int64_t fidx(int row, int col) {
  const int rt = row >> 4, ct = col >> 4, ri = row & 15, ci = col & 15;
  const int lane = 16 * (ri & 3) + ci, r = ri >> 2;
  return ((int64_t)(rt * NT + ct) * 64 + lane) * 4 + r;
}

__device__ __forceinline__ double sum16(double v) {  // sum over the 16 lanes of a row group
  v += __shfl_xor(v, 1, 16);
  v += __shfl_xor(v, 2, 16);
  v += __shfl_xor(v, 4, 16);
  v += __shfl_xor(v, 8, 16);
  return v;
}

}  // namespace

// MP = padded block order, NB = block waves (+ 1 pivot wave).  <256, 8>: the m <= 256 kernel;
// <128, 3> / <64, 3>: the CO-RESIDENT form for m <= 128 — 4 waves (one per SIMD), <= 176 VGPRs and
// ~72 KiB of LDS, i.e. the footprint ONE retiring trailing-update workgroup frees on a CU (4 x 112
// VGPRs per SIMD of GEMM + 64 spare; 4 x 26 KiB LDS + 56 spare), so a batch of candidate
// inverses starts inside a running trailing update instead of waiting for whole CUs.
// LAY = 1 (NB = 8): 11 hardware waves with 4 and 8 idle, so the pivot wave (hardware wave 0) has
// SIMD 0 to itself (waves are placed on SIMDs round-robin), as in blockinv_mfma.hip.
template <int MP, int NB, int LAY = 0>
__global__ __launch_bounds__(64 * (NB + 1 + (LAY ? (NB - 1) / 3 : 0))) void block_inverse_l2_kernel(
    const double* __restrict__ Lt, int64_t ldl, double* __restrict__ inv_t, double* __restrict__ scores,
    int32_t* __restrict__ valid, const int32_t* __restrict__ used, int m, int64_t p, int64_t k,
    double thresh, double* __restrict__ scratch, int32_t* __restrict__ piv_out, PivotSelectArgs sel,
    int live_nblk) {
  constexpr int NT = MP / 16;               // tiles per dimension = panels
  constexpr int CPW = (NT + NB - 1) / NB;    // column tiles per block wave (ct = wave + NB j < NT)
  constexpr int RPL = MP / 64;               // pivot-wave rows per lane
  constexpr int LDU = kBigLDU;
  constexpr int RWC = 16 * CPW + 1;
  static_assert(MP % 64 == 0 && NB <= NT && 2 * LDU >= NB, "geometry");

  // the fused selection (select_tail, one whole wave per workgroup) as in blockinv_mfma.hip
  const int nblk = live_nblk ? live_nblk : (int)gridDim.x;
  const int b = live_nblk ? live_block(used, live_nblk, p, k) : (int)blockIdx.x;  // see live_block
  if (b < 0 || used[(int64_t)b * p + k]) {
    if (threadIdx.x < 64) {
      if (threadIdx.x == 0 && b >= 0) {
        valid[b] = 0;
        scores[b] = 0.0;
      }
      select_tail(sel, scores, valid, used, nblk, p, k);
    }
    return;
  }
  double* S = scratch + (int64_t)b * MP * MP;

  __shared__ double Ub[2][MP][LDU];   // U of the last two panels (after the last: row abs-sums)
  __shared__ double Pb[MP][LDU];      // the next panel's columns, for the pivot wave
  __shared__ double Rw[NB][16][RWC];  // per block wave: the panel's pivot rows over its columns
  __shared__ int rsel[2][16];
  __shared__ int prow[MP];            // prow[c] = pivot row of column c
  __shared__ int kinv[MP];            // kinv[r] = column pivoted on row r
  __shared__ int s_sing;

  const int hw = (int)(threadIdx.x >> 6), lane = (int)(threadIdx.x & 63);
  int wave = hw;
  if constexpr (LAY == 1) {
    if (hw > 0 && (hw & 3) == 0) {
      // idle wave: the pivot wave's barrier sequence, no work
      __syncthreads();  // B0(0)
      for (int q = 0; q < NT; ++q) {
        __syncthreads();  // B1(q)
        if (s_sing) break;
        if (q + 1 < NT) __syncthreads();  // B0(q+1)
      }
      if (!s_sing) {
        __syncthreads();  // E0
        __syncthreads();  // E1
      }
      return;
    }
    wave = hw == 0 ? NB : hw - 1 - (hw >> 2);
  }
  const int tid = wave * 64 + lane;
  for (int i = tid; i < MP; i += 64 * (NB + 1)) kinv[i] = -1;
  if (tid == 0) s_sing = 0;

  if (wave == NB) {
    // ================= pivot wave
    __builtin_amdgcn_s_setprio(3);
    uint64_t keymask[RPL];
#pragma unroll
    for (int s = 0; s < RPL; ++s) keymask[s] = 0x7FFFFFFFFFFFFFFFull;
    int pos[RPL];  // current position of each row under the reference's row swaps (PivotPanel)
#pragma unroll
    for (int s = 0; s < RPL; ++s) pos[s] = lane + 64 * s;
    __syncthreads();  // B0(0)
    for (int q = 0; q < NT; ++q) {
      const int c0 = 16 * q, ub = q & 1;
      double W[RPL][16];
#pragma unroll
      for (int s = 0; s < RPL; ++s)
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) W[s][jj] = Pb[lane + 64 * s][jj];
      int rr[16];
      bool sing = false;
      pivot_panel_il<double, RPL>(W, keymask, pos, lane, c0, m, thresh, rr, sing);
#pragma unroll
      for (int s = 0; s < RPL; ++s)
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) Ub[ub][lane + 64 * s][jj] = W[s][jj];
      int myr = 0;
#pragma unroll
      for (int jj = 0; jj < 16; ++jj) myr = (lane == jj) ? rr[jj] : myr;
      if (lane < 16) {
        rsel[ub][lane] = myr;
        prow[c0 + lane] = myr;
        kinv[myr] = c0 + lane;
      }
      if (sing && lane == 0) s_sing = 1;
      __syncthreads();  // B1(q)
      if (s_sing) break;
      if (q + 1 < NT) __syncthreads();  // B0(q+1)
    }
    if (piv_out && !s_sing)  // test probe: the pivot row of every column
      for (int c = lane; c < m; c += 64) piv_out[(int64_t)b * m + c] = prow[c];
    if (!s_sing) {
      __syncthreads();  // E0: every panel applied
      __syncthreads();  // E1: row abs-sums published
      double mx = 0.0;
      double(*red)[MP] = reinterpret_cast<double(*)[MP]>(&Ub[0][0][0]);
      for (int i = lane; i < m; i += 64) {
        double sm = 0.0;
#pragma unroll
        for (int w = 0; w < NB; ++w) sm += red[w][i];
        mx = fmax(mx, sm);
      }
      mx = wave_max_f64(mx);
      if (lane == 0) {
        scores[b] = mx;
        valid[b] = isfinite(mx) ? 1 : 0;
      }
    } else if (lane == 0) {
      valid[b] = 0;
      scores[b] = 0.0;
    }
    select_tail(sel, scores, valid, used, nblk, p, k);
    return;
  }

  // ================= block waves: column tiles ct = wave + NB j
  const int cl = lane & 15, g = lane >> 4;
  // initial image: W = -(Lt block b)^T, identity in the padding
  for (int j = 0; j < CPW; ++j) {
    const int ct = wave + NB * j;
    if (ct >= NT) break;
    const int jc = 16 * ct + cl;
    const double* src = Lt + (int64_t)jc * ldl + (int64_t)b * m;
    for (int rt = 0; rt < NT; ++rt) {
      acc4 x;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = 16 * rt + frow(lane, r);
        x[r] = (i < m && jc < m) ? -src[i] : (i == jc ? 1.0 : 0.0);
        if (ct == 0) Pb[i][cl] = x[r];
      }
      *reinterpret_cast<acc4*>(S + ((int64_t)(rt * NT + ct) * 64 + lane) * 4) = x;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __syncthreads();  // B0(0)
  __syncthreads();  // B1(0)
  bool sing_exit = (s_sing != 0);
  for (int q = 0; q < NT && !sing_exit; ++q) {
    const int ub = q & 1;
    const bool look = (q + 1 < NT);
    // (1) the panel's pivot rows over my columns, before this panel touches them
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    for (int e = lane; e < 16 * 16 * CPW; e += 64) {
      const int kk = e / (16 * CPW), cc = e % (16 * CPW);
      const int ctc = wave + NB * (cc >> 4);
      if (ctc < NT) Rw[wave][kk][cc] = S[fidx<NT>(rsel[ub][kk], 16 * ctc + (cc & 15))];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // (2) my column tiles, the next panel's first (if it is mine)
    int first = 0;
    for (int j = 0; j < CPW; ++j)
      if (wave + NB * j == q + 1) first = j;
    for (int jj = 0; jj < CPW; ++jj) {
      const int j = jj == 0 ? first : (jj == first ? 0 : jj);
      const int ct = wave + NB * j;
      if (ct >= NT) continue;
      double* tile0 = S + ((int64_t)ct * 64 + lane) * 4;
      if (ct == q) {  // the panel's own columns: U + E
        const int rs = rsel[ub][cl];
        for (int rt = 0; rt < NT; ++rt) {
          acc4 x;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int i = 16 * rt + frow(lane, r);
            x[r] = Ub[ub][i][cl] + (i == rs ? 1.0 : 0.0);
          }
          *reinterpret_cast<acc4*>(tile0 + (int64_t)rt * NT * 256) = x;
        }
      } else {
        double bop[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) bop[s] = Rw[wave][4 * s + g][16 * j + cl];
        const bool to_pb = look && ct == q + 1;
        acc4 xn = *reinterpret_cast<const acc4*>(tile0);
        for (int rt = 0; rt < NT; ++rt) {
          acc4 x = xn;
          if (rt + 1 < NT) xn = *reinterpret_cast<const acc4*>(tile0 + (int64_t)(rt + 1) * NT * 256);
          double a[4];
#pragma unroll
          for (int s = 0; s < 4; ++s) a[s] = Ub[ub][16 * rt + cl][4 * s + g];
#pragma unroll
          for (int s = 0; s < 4; ++s) x = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s], bop[s], x, 0, 0, 0);
          *reinterpret_cast<acc4*>(tile0 + (int64_t)rt * NT * 256) = x;
          if (to_pb) {
#pragma unroll
            for (int r = 0; r < 4; ++r) Pb[16 * rt + frow(lane, r)][cl] = x[r];
          }
        }
      }
      if (jj == 0 && look) __syncthreads();  // B0(q+1): the next panel's columns are in Pb
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (look) {
      __syncthreads();  // B1(q+1)
      sing_exit = (s_sing != 0);
    }
  }
  if (sing_exit) return;
  __syncthreads();  // E0: every panel applied, Ub free
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  // inverse, transposed: inv(W)[kinv[i]][prow[u]] = W_swept[i][u] -> inv_t[prow[u]][kinv[i]];
  // row abs-sums of W_swept = row abs-sums of the inverse (block_norm)
  double(*red)[MP] = reinterpret_cast<double(*)[MP]>(&Ub[0][0][0]);
  double* out = inv_t + (int64_t)b * m * m;
  for (int rt = 0; rt < NT; ++rt) {
    double rs[4] = {0.0, 0.0, 0.0, 0.0};
    for (int j = 0; j < CPW; ++j) {
      const int ct = wave + NB * j;
      if (ct >= NT) break;
      const int u = 16 * ct + cl;
      const acc4 x = *reinterpret_cast<const acc4*>(S + ((int64_t)(rt * NT + ct) * 64 + lane) * 4);
      const int o = u < m ? prow[u] : -1;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = 16 * rt + frow(lane, r);
        if (o >= 0 && i < m) {
          out[(int64_t)o * m + kinv[i]] = x[r];
          rs[r] += fabs(x[r]);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const double sm = sum16(rs[r]);
      if (cl == 0) red[wave][16 * rt + frow(lane, r)] = sm;
    }
  }
  __syncthreads();  // E1
}

bool block_inverse_big(DType dt, const void* Lt, int64_t ldl, void* inv_t, double* scores, int32_t* valid,
                       const int32_t* used, const Layout& L, double thresh, int64_t nlive, hipStream_t s, void* scratch) {
  const int m = (int)L.m;
  if (dt != DType::F64 || m <= 128 || m > 256) return false;
  if (L.nblk == 0) return true;
  const unsigned grid = (unsigned)(nlive >= 0 ? std::max<int64_t>(nlive, 1) : L.nblk);
  const int live_nblk = nlive >= 0 ? (int)L.nblk : 0;
  // the pivot wave alone on its SIMD (11-wave layout): -6 to -7 % per batch against the 9-wave one
  hipLaunchKernelGGL((block_inverse_l2_kernel<256, 8, 1>), dim3(grid), dim3(64 * 11), 0, s,
                     static_cast<const double*>(Lt), ldl, static_cast<double*>(inv_t), scores, valid, used, m,
                     L.p, L.k, thresh, static_cast<double*>(scratch), block_inverse_probe(), PivotSelectArgs{},
                     live_nblk);
  return true;
}

bool block_inverse_co(DType dt, const void* Lt, int64_t ldl, void* inv_t, double* scores, int32_t* valid,
                      const int32_t* used, const Layout& L, double thresh, int64_t nlive, hipStream_t s, void* scratch,
                      const PivotSelectArgs* sel) {
  const int m = (int)L.m;
  if (dt != DType::F64 || m <= 32 || m > 128) return false;
  if (L.nblk == 0) return true;
  const unsigned grid = (unsigned)(nlive >= 0 ? std::max<int64_t>(nlive, 1) : L.nblk);
  const int live_nblk = nlive >= 0 ? (int)L.nblk : 0;
  const PivotSelectArgs tail = sel ? *sel : PivotSelectArgs{};
  if (m <= 64)
    hipLaunchKernelGGL((block_inverse_l2_kernel<64, 3>), dim3(grid), dim3(64 * 4), 0, s,
                       static_cast<const double*>(Lt), ldl, static_cast<double*>(inv_t), scores, valid, used, m,
                       L.p, L.k, thresh, static_cast<double*>(scratch), block_inverse_probe(), tail, live_nblk);
  else
    hipLaunchKernelGGL((block_inverse_l2_kernel<128, 3>), dim3(grid), dim3(64 * 4), 0, s,
                       static_cast<const double*>(Lt), ldl, static_cast<double*>(inv_t), scores, valid, used, m,
                       L.p, L.k, thresh, static_cast<double*>(scratch), block_inverse_probe(), tail, live_nblk);
  return true;
}

size_t block_inverse_big_scratch_bytes(DType dt, const Layout& L) {
  if (dt != DType::F64 || L.m <= 32 || L.m > 256) return 0;
  const int64_t MP = L.m <= 64 ? 64 : L.m <= 128 ? 128 : 256;
  return (size_t)std::max<int64_t>(L.nblk, 1) * MP * MP * sizeof(double);
}

}  // namespace kern
}  // namespace gj
