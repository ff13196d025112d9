// Candidate-block inversion with the bulk of the work on the matrix cores (gfx950).
//
// Reference: inverse_block (main.cpp:746-820: scalar Gauss-Jordan, partial pivoting with the
// first maximum winning, singular when |a_kk| < EPS*norm) + block_norm (main.cpp:669-683), run for
// every candidate block of the pivot search (main.cpp:1039-1066).  Output contract as
// blockinv.hip: the inverse transposed (the K-major GEMM operand H^T), ||inv||_inf, validity.
//
// One workgroup per candidate block, NW + 1 waves (MP = 16 NW, MP = 32 / 64 / 128):
//  * NW BLOCK waves hold the MP x MP block as MFMA accumulator tiles.  Block wave w keeps every
//    row of 16 columns, PER = 16 / NW of each 16-column panel, so every panel is spread over all
//    block waves.  Per panel they apply the panel's 16 sweep steps as ONE rank-16 update
//    X += U R (U: the panel's MP x 16 multipliers, R: its 16 pivot rows before the panel) with
//    v_mfma_f64_16x16x4 / v_mfma_f32_16x16x4 (MP/16 x 4 instructions per wave), and the panel's
//    own columns become U + E.
//  * The PIVOT wave (the last one, s_setprio 3) factors a panel in registers: rows lane and
//    lane + 64, 16 columns, the multipliers overwriting the consumed columns in place.  A step's
//    pivot is found by an exact wave max + ballot (largest magnitude, lowest row on ties, like the
//    reference's strict '>' scan); the pivot value and the next column's entry come by v_readlane
//    (the chain of the next step needs only those), the rest of the pivot row through LDS.
// Panels overlap: while the pivot wave factors panel k+1, the block waves apply panel k.  The
// only other work on the chain per panel is one 16 x 16 MFMA tile per block wave that brings
// panel k+1's columns up to date (4 instructions) — two workgroup barriers per panel.
//
// Panel algebra (the in-place sweep, no row swaps): a step with pivot (r, c) acts on every other
// column x as x <- x + u x[r] with u_i = -a_ic / a_rc (i != r), u_r = 1/a_rc - 1, and column c
// becomes u + e_r.  16 steps compose to X <- X + U (E^T X) on the other columns, U + E on the
// panel's own; pivot rows are recorded (prow / kinv) and the inverse is written permuted.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstdint>
#include <type_traits>
#include <utility>

#include "kernels.hpp"
#include "pivot_panel.hpp"
#include "pivot_select.hpp"
#include "wave_ops.hpp"

namespace gj {
namespace kern {

#ifdef GJ_BI_PROBE  // shader-clock stamps of workgroup 0 (bench/blockinv_mfma_probe.hip)
__device__ unsigned long long g_bim_probe[1024];
#define BIM_PROBE(slot)                                                                       \
  do {                                                                                        \
    if (blockIdx.x == 0 && lane == 0) g_bim_probe[(slot)] = __builtin_amdgcn_s_memtime();     \
  } while (0)
#else
#define BIM_PROBE(slot) \
  do {                  \
  } while (0)
#endif

namespace {

template <typename T>
struct BiTile;

// v_mfma_f64_16x16x4_f64: C/D lane l, register r -> row (l>>4) + 4r, column l&15
template <>
struct BiTile<double> {
  typedef double acc_t __attribute__((ext_vector_type(4)));
  static __device__ __forceinline__ acc_t mfma(double a, double b, acc_t c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ int row(int lane, int r) { return (lane >> 4) + 4 * r; }
};

// v_mfma_f32_16x16x4_f32: C/D lane l, register r -> row 4(l>>4) + r, column l&15
template <>
struct BiTile<float> {
  typedef float acc_t __attribute__((ext_vector_type(4)));
  static __device__ __forceinline__ acc_t mfma(float a, float b, acc_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ int row(int lane, int r) { return 4 * (lane >> 4) + r; }
};

}  // namespace


// LAY = 1: the pivot wave gets a SIMD of its own.  The waves of a workgroup are placed on the four
// SIMDs round-robin (hardware wave w -> SIMD w % 4), so hardware waves 4, 8, ... are left idle (they
// only take part in the barriers): the pivot wave (hardware wave 0) then never shares its SIMD's
// fp64 datapath with block-wave MFMAs.
template <int MP, int LAY>
constexpr int bim_hw_waves() { return MP / 16 + 1 + (LAY ? (MP / 16 - 1) / 3 : 0); }

template <typename T, int MP, int LAY = 0>
__global__ __launch_bounds__(64 * (MP / 16 + 1 + (LAY ? (MP / 16 - 1) / 3 : 0))) void block_inverse_mfma_kernel(
    const T* __restrict__ Lt, int64_t ldl, T* __restrict__ inv_t, double* __restrict__ scores,
    int32_t* __restrict__ valid, const int32_t* __restrict__ used, int m, int64_t p, int64_t k,
    double thresh, int32_t* __restrict__ piv_out, PivotSelectArgs sel, int live_nblk) {
  using TL = BiTile<T>;
  using acc_t = typename TL::acc_t;
  constexpr int NW = MP / 16;     // block waves = row tiles = panels
  constexpr int NP = MP / 16;
  constexpr int PER = 16 / NW;    // columns of each panel per block wave
  constexpr int NTH = 64 * (NW + 1);
  constexpr int LDR = sizeof(T) == 8 ? 18 : 20;  // [row][panel column] images: 16-B aligned rows
  constexpr int RPL = MP > 64 ? 2 : 1;           // pivot wave: rows lane (+ 64)
  constexpr int SR = MP / 2;                     // output rows staged per pass
  constexpr int LDS_S = MP + 2;                  // staging row (bank spread across output rows)
  static_assert(NW * 16 == MP && PER * NW == 16, "MP must be 32, 64 or 128");
  static_assert(SR * LDS_S <= 4 * MP * LDR, "staging does not fit");

  // live_nblk > 0: the grid covers only the live candidates (live_block); 0: one per local block
  const int nblk = live_nblk ? live_nblk : (int)gridDim.x;
  const int b = live_nblk ? live_block(used, live_nblk, p, k) : (int)blockIdx.x;
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

  // Ub[2][MP][LDR]: U of the last two panels | Pb[MP][LDR]: the panel the pivot wave factors next
  // | Xn[MP][LDR]: the next panel's columns before the current panel.  After the last panel the
  // same bytes stage the permuted output (S[SR][MP]).
  __shared__ __attribute__((aligned(16))) T big[4 * MP * LDR];
  T(*Ub)[MP][LDR] = reinterpret_cast<T(*)[MP][LDR]>(big);
  T(*Pb)[LDR] = reinterpret_cast<T(*)[LDR]>(big + 2 * MP * LDR);
  T(*Xn)[LDR] = reinterpret_cast<T(*)[LDR]>(big + 3 * MP * LDR);
  T* S = big;
  __shared__ T Rw[NW][16][16];   // per block wave: the current panel's pivot rows over its columns
  __shared__ int rsel[2][16];    // pivot rows of the last two panels
  __shared__ int prow[MP];       // prow[c] = pivot row of column c
  __shared__ int kinv[MP];       // kinv[r] = column pivoted on row r (-1 = not yet)
  __shared__ double redg[64 * NW / MP][MP];  // partial row abs-sums of the inverse
  __shared__ int s_sing;

  const int hw = (int)(threadIdx.x >> 6), lane = (int)(threadIdx.x & 63);
  int wave = hw;
  if constexpr (LAY == 1) {
    if (hw > 0 && (hw & 3) == 0) {
      // idle wave: the pivot wave's barrier sequence, no work
      __syncthreads();  // B0(0)
      for (int q = 0; q < NP; ++q) {
        __syncthreads();  // B1(q)
        if (s_sing) break;
        if (q + 1 < NP) __syncthreads();  // B0(q+1)
      }
      __syncthreads();  // E0
      if (!s_sing)
        for (int h = 0; h < 2; ++h) {
          __syncthreads();  // E1(h)
          __syncthreads();  // E2(h)
        }
      return;
    }
    wave = hw == 0 ? NW : hw - 1 - (hw >> 2);
  }
  const int tid = wave * 64 + lane;
  if (wave == 0) BIM_PROBE(1002);
  for (int i = tid; i < MP; i += NTH) kinv[i] = -1;
  if (tid == 0) s_sing = 0;

  // Block-wave register tiles: lane l, register r of tile t holds row 16t + 4(l>>4) + r (four
  // consecutive rows per lane; for f64 this permutes the instruction's row order (l>>4) + 4r, so
  // the A operand's row m is row arow(m) of the tile) and column jcol(l & 15).
  auto arow = [](int mrow) { return sizeof(T) == 8 ? 4 * (mrow & 3) + (mrow >> 2) : mrow; };

  // The two roles run separate loops with the same barrier sequence (B0 before a panel's
  // factorisation, B1 after it), so their register sets do not overlap.
  bool sing_exit = false;
  if (wave == NW) {
    // ================= pivot wave: panel rows lane + 64 s, multipliers overwrite consumed columns
    __builtin_amdgcn_s_setprio(3);
    uint64_t keymask[RPL];  // 0x7FFF.. for rows still free, 0 for pivot rows and padding
#pragma unroll
    for (int s = 0; s < RPL; ++s) keymask[s] = (lane + 64 * s >= MP) ? 0ull : 0x7FFFFFFFFFFFFFFFull;
    int pos[RPL];  // current position of each row under the reference's row swaps (PivotPanel)
#pragma unroll
    for (int s = 0; s < RPL; ++s) pos[s] = lane + 64 * s;
    BIM_PROBE(0);
    __syncthreads();  // B0(0)
    for (int q = 0; q < NP; ++q) {
      const int c0 = 16 * q, ub = q & 1;
      BIM_PROBE(8 + 24 * q);
      T W[RPL][16];
#pragma unroll
      for (int s = 0; s < RPL; ++s)
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) W[s][jj] = (lane + 64 * s < MP) ? Pb[lane + 64 * s][jj] : T(0);
      int rr[16];
      bool sing = false;
      pivot_panel_il<T, RPL>(W, keymask, pos, lane, c0, m, thresh, rr, sing);
      // publish U and the panel's pivot rows
#pragma unroll
      for (int s = 0; s < RPL; ++s)
        if (lane + 64 * s < MP) {
#pragma unroll
          for (int jj = 0; jj < 16; ++jj) Ub[ub][lane + 64 * s][jj] = W[s][jj];
        }
      int myr = 0;
#pragma unroll
      for (int jj = 0; jj < 16; ++jj) myr = (lane == jj) ? rr[jj] : myr;
      if (lane < 16) {
        rsel[ub][lane] = myr;
        prow[c0 + lane] = myr;
        kinv[myr] = c0 + lane;
      }
      if (sing && lane == 0) s_sing = 1;
      BIM_PROBE(25 + 24 * q);
      __syncthreads();  // B1(q)
      BIM_PROBE(26 + 24 * q);
      if (s_sing) break;
      if (q + 1 < NP) __syncthreads();  // B0(q+1)
    }
    if (piv_out && !s_sing)  // test probe: the pivot row of every column
      for (int c = lane; c < m; c += 64) piv_out[(int64_t)b * m + c] = prow[c];
  } else {
    // ================= block waves: every row of 16 columns as MFMA accumulator tiles
    const int cl = lane & 15;
    const int g4 = 4 * (lane >> 4);
    const int jpan = cl / PER;                             // my column's panel
    const int jcol = 16 * jpan + PER * wave + (cl % PER);  // my column
    acc_t X[NW];
    {
      // four consecutive rows per lane and tile: one 16-byte (f32) or two 16-byte (f64) loads
      // when the panel is 16-byte aligned, else element loads
      const T* src = Lt + (int64_t)jcol * ldl + (int64_t)b * m;
      constexpr int VEC = 16 / sizeof(T);
      const bool vec = (jcol < m) && ((((uintptr_t)src) & 15) == 0) && (m % 4 == 0);
      if (vec) {
#pragma unroll
        for (int t = 0; t < NW; ++t) {
          const int i0 = 16 * t + g4;
          if (i0 < m) {
            typedef T vec_t __attribute__((ext_vector_type(VEC)));
#pragma unroll
            for (int h = 0; h < 4 / VEC; ++h) {
              const vec_t v = *reinterpret_cast<const vec_t*>(src + i0 + VEC * h);
#pragma unroll
              for (int e = 0; e < VEC; ++e) X[t][VEC * h + e] = -v[e];
            }
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) X[t][r] = (i0 + r == jcol) ? T(1) : T(0);
          }
        }
      } else {
#pragma unroll
        for (int t = 0; t < NW; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int i = 16 * t + g4 + r;
            X[t][r] = (i < m && jcol < m) ? -src[i] : (i == jcol ? T(1) : T(0));
          }
      }
    }
    if (jpan == 0) {
#pragma unroll
      for (int t = 0; t < NW; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) Pb[16 * t + g4 + r][jcol] = X[t][r];
    }
    if (NP > 1 && jpan == 1) {
#pragma unroll
      for (int t = 0; t < NW; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) Xn[16 * t + g4 + r][jcol - 16] = X[t][r];
    }

    // X += U_q R_q for panel q (R_q = its pivot rows before the panel, extracted from X first);
    // panel q's own columns := U_q + E.
    auto apply_panel = [&](int q) {
      const int ub = q & 1, c0 = 16 * q;
#pragma unroll
      for (int t = 0; t < NW; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int kc = kinv[16 * t + g4 + r] - c0;
          if (kc >= 0 && kc < 16) Rw[wave][kc][cl] = X[t][r];
        }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      T bop[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) bop[s] = Rw[wave][4 * s + (lane >> 4)][cl];
      const int ar = arow(lane & 15);
#pragma unroll
      for (int t = 0; t < NW; ++t) {
        // one tile's A fragments at a time (hoisting all of them costs 2 NW x 4 VGPRs)
        T a[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) a[s] = Ub[ub][16 * t + ar][4 * s + (lane >> 4)];
#pragma unroll
        for (int s = 0; s < 4; ++s) X[t] = TL::mfma(a[s], bop[s], X[t]);
        __builtin_amdgcn_sched_barrier(0);
      }
      if (jpan == q) {
        const int c = jcol - c0;
        const int rs = rsel[ub][c];
#pragma unroll
        for (int t = 0; t < NW; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int i = 16 * t + g4 + r;
            X[t][r] = Ub[ub][i][c] + (i == rs ? T(1) : T(0));
          }
      }
    };

    if (wave == 0) BIM_PROBE(512);
    __syncthreads();  // B0(0)
    for (int q = 0; q < NP; ++q) {
      const int c0 = 16 * q, ub = q & 1;
      if (wave == 0) BIM_PROBE(520 + 8 * q);
      if (q > 0) apply_panel(q - 1);
      if (wave == 0) BIM_PROBE(521 + 8 * q);
      // the next panel's columns, as they are before panel q -> Xn
      if (q + 1 < NP && jpan == q + 1) {
#pragma unroll
        for (int t = 0; t < NW; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) Xn[16 * t + g4 + r][jcol - c0 - 16] = X[t][r];
      }
      if (wave == 0) BIM_PROBE(522 + 8 * q);
      __syncthreads();  // B1(q): panel q factored, Xn complete
      if (wave == 0) BIM_PROBE(523 + 8 * q);
      if (s_sing) {
        sing_exit = true;
        break;
      }
      if (q + 1 < NP) {
        // rows 16 wave .. +15 of panel q+1 brought up to date: Xn + U_q Xn[pivot rows of q]
        acc_t c;
#pragma unroll
        for (int r = 0; r < 4; ++r) c[r] = Xn[16 * wave + g4 + r][cl];
        const int ar = 16 * wave + arow(cl);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const T a = Ub[ub][ar][4 * s + (lane >> 4)];
          const T bb = Xn[rsel[ub][4 * s + (lane >> 4)]][cl];
          c = TL::mfma(a, bb, c);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) Pb[16 * wave + g4 + r][cl] = c[r];
        if (wave == 0) BIM_PROBE(524 + 8 * q);
        __syncthreads();  // B0(q+1)
      }
    }
    if (!sing_exit) apply_panel(NP - 1);
    if (wave == 0) BIM_PROBE(1000);
    __syncthreads();  // E0: every panel applied; the LDS images are free
    if (!s_sing) {
      // inverse, transposed: inv(W)[kinv[i]][prow[u]] = W_swept[i][u]  ->  inv_t[prow[u]][kinv[i]],
      // staged in LDS by output row (two passes of SR rows) so that the global stores coalesce;
      // the column abs-sums of inv_t are the row abs-sums of the inverse (block_norm)
      const int orow = jcol < m ? prow[jcol] : -1;
      T* out = inv_t + (int64_t)b * m * m;
      constexpr int NG = 64 * NW / MP;  // copy-out thread groups (one column each)
      const int cc = tid % MP, grp = tid / MP;
      double csum = 0.0;
      for (int h = 0; h < 2; ++h) {
        const int r0 = h * SR, nrow = max(0, min(SR, m - r0));
        if (orow >= r0 && orow < r0 + SR) {
#pragma unroll
          for (int t = 0; t < NW; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int i = 16 * t + g4 + r;
              if (i < m) S[(orow - r0) * LDS_S + kinv[i]] = X[t][r];
            }
        }
        __syncthreads();  // E1(h)
        if (cc < m) {
          for (int ro = grp; ro < nrow; ro += NG) {
            const T v = S[ro * LDS_S + cc];
            out[(int64_t)(r0 + ro) * m + cc] = v;
            csum += fabs((double)v);
          }
        }
        __syncthreads();  // E2(h)
      }
      if (cc < m) redg[grp][cc] = csum;
      if (wave == 0) BIM_PROBE(1001);
      __syncthreads();  // E3: the row sums are in LDS before the pivot wave reads them
    }
  }
  if (wave == NW) {
    __syncthreads();  // E0
    if (!s_sing) {
      for (int h = 0; h < 2; ++h) {
        __syncthreads();  // E1(h)
        __syncthreads();  // E2(h)
      }
      __syncthreads();  // E3
    }
  }
  (void)sing_exit;
  if (s_sing) {
    if (wave == 0) {
      if (lane == 0) {
        valid[b] = 0;
        scores[b] = 0.0;
      }
      select_tail(sel, scores, valid, used, nblk, p, k);
    }
    return;
  }
  if (wave == NW) {
    double mx = 0.0;
    for (int i = lane; i < m; i += 64) {
      double sm = 0.0;
#pragma unroll
      for (int gq = 0; gq < 64 * NW / MP; ++gq) sm += redg[gq][i];
      mx = fmax(mx, sm);
    }
    mx = wave_max_f64(mx);
    if (lane == 0) {
      scores[b] = mx;
      valid[b] = isfinite(mx) ? 1 : 0;
    }
    select_tail(sel, scores, valid, used, nblk, p, k);
  }
}

static int32_t* g_piv_probe = nullptr;
void set_block_inverse_probe(int32_t* piv_out) { g_piv_probe = piv_out; }
int32_t* block_inverse_probe() { return g_piv_probe; }

bool block_inverse_mfma(DType dt, const void* Lt, int64_t ldl, void* inv_t, double* scores,
                        int32_t* valid, const int32_t* used, const Layout& L, double thresh, int64_t nlive,
                        hipStream_t s, const PivotSelectArgs* sel) {
  const int m = (int)L.m;
  if (m <= 16 || m > 128) return false;
  if (L.nblk == 0) return true;
  // one workgroup per live candidate (at least one: the fused selection tail must run)
  const unsigned grid = (unsigned)(nlive >= 0 ? std::max<int64_t>(nlive, 1) : L.nblk);
  const int live_nblk = nlive >= 0 ? (int)L.nblk : 0;
  const int MP = m <= 32 ? 32 : m <= 64 ? 64 : 128;
  const PivotSelectArgs tail = sel ? *sel : PivotSelectArgs{};
  // MP = 128: the pivot wave alone on its SIMD (LAY 1), where 8 block waves' MFMAs would share it:
  // 96.0 -> 86.4 us per batch of 64 fp64 128 x 128 candidates (MP = 64: no change, 9-wave layout)
#define GJ_BI_LAUNCH(T, MPV, LAYV)                                                                       \
  hipLaunchKernelGGL((block_inverse_mfma_kernel<T, MPV, LAYV>), dim3(grid), dim3(64 * bim_hw_waves<MPV, LAYV>()), \
                     0, s, static_cast<const T*>(Lt), ldl, static_cast<T*>(inv_t), scores, valid, used, m, L.p,   \
                     L.k, thresh, g_piv_probe, tail, live_nblk)
  if (dt == DType::F64) {
    if (MP == 32) GJ_BI_LAUNCH(double, 32, 0);
    else if (MP == 64) GJ_BI_LAUNCH(double, 64, 0);
    else GJ_BI_LAUNCH(double, 128, 1);
  } else {
    if (MP == 32) GJ_BI_LAUNCH(float, 32, 0);
    else if (MP == 64) GJ_BI_LAUNCH(float, 64, 0);
    else GJ_BI_LAUNCH(float, 128, 1);
  }
#undef GJ_BI_LAUNCH
  return true;
}

}  // namespace kern
}  // namespace gj
