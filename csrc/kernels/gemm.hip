// gfx950 MFMA GEMM for the Gauss-Jordan engine.
//
//   MODE_ACC   : C[M x N] += A * B       (the elimination update, reference mult_substr_block
//                                          main.cpp:151-206 called from the hot loop :1165-1194)
//                with fused extras: C enters as 0 in columns [zc0, zc1) (the panel's pivot block
//                columns, X[i,t] := sum -L_i H) and in up to 8 row blocks (the panel's pivot rows,
//                whose multiplier rows the engine turned into [0 .. I .. L] coefficients)
//   MODE_STORE : C[M x N]  = A * B       (pivot-row normalisation, reference mult_block
//                                          main.cpp:888-950 called at :1136-1159)
//   MODE_RESID : per-row partial sums of |A*B - I| (residual, reference matrix_mult_matrix +
//                                          minus_i + norm, main.cpp:534-667, fused: no D matrix)
//
// Kernels (all wave64, v_mfma_f64_16x16x4_f64 with C/D map col = lane&15, row = (lane>>4) + 4*reg
// for fp64; v_mfma_f32_16x16x4_f32, row = 4*(lane>>4) + reg, or v_mfma_f32_32x32x2_f32 for fp32;
// the accumulator is loaded straight from C in the C/D layout, so the read-modify-write needs no
// separate epilogue pass):
//   * gemm_glds_f64 — the fp64 trailing update (K = depth*m >= 256, enough tiles to fill the chip):
//     128 x 64 tile per 256-thread workgroup, 2 x 2 waves of 64 x 32, operands staged global -> LDS
//     by LDS-DMA (buffer_load_dwordx4 ... lds) into a 2-stage ring, counted vmcnt + raw s_barrier,
//     4 workgroups per CU (82 % MFMA busy at 2.3 GHz: profiles/gemm_variants_k512.md).
//   * gemm_glds_f32 — the fp32 trailing update: the same LDS-DMA ring, 128 x 128 tile of 2 x 2
//     waves of 64 x 64, v_mfma_f32_32x32x2_f32, 126-132 TF/s (squarepf register staging 118-122).
//   * gemm_kernel<T, A-layout, MODE, Cfg> — register-staged tiles for everything else
//     (latency-bound panel GEMMs the small 64 x 32 tile; the residual the 128 x 128 tile; fp32
//     deep updates the glds32 kernel cannot take the 128 x 128 "squarepf" tile).  K is staged
//     through LDS in BK-deep slices, double-buffered, with a 16-element row pad so the fragment
//     reads (lanes 0-15 / 16-31 on consecutive k rows) are bank-conflict free; Cfg::PF = 2 keeps
//     two slices in registers.
// All global traffic uses buffer instructions on a per-tile (or per-slice) resource with one 32-bit
// per-lane offset plus SGPR offsets (no 64-bit address registers, no spills), and masking is done
// with out-of-range offsets instead of branches (see kOOB).  Tiles are mapped XCD-aware (xcd_remap).
#include <hip/hip_runtime.h>

#include <stdexcept>

#include <cstdint>
#include <cstdlib>
#include <string>
#include <type_traits>
#include <utility>

#include "kernels.hpp"

namespace gj {
namespace kern {

constexpr int PADL = 16;                          // LDS row pad (elements): conflict-free frag reads
constexpr int kRecords = 0x7ffffff0;              // buffer extent of every resource
// Masked-off lanes use this per-lane offset (>= kRecords): the buffer unit returns 0 for such a load
// and drops such a store, so no access needs a branch.  Branch-free loads matter: a load behind a
// per-lane condition makes hipcc wait vmcnt(0) at the next use of ANY load result, which drains the
// K-slice prefetch every iteration.
constexpr int kOOB = 0x7ffffff8;

// Tile configurations.  WM x WN waves, each owning a (BM/WM) x (BN/WN) block of 16x16 MFMA tiles.
// OCC = workgroups per CU the launch bounds are written for.
template <int BM_, int BN_, int BK_, int WM_, int WN_, int OCC_, int PF_ = 1>
struct Cfg {
  static constexpr int BM = BM_, BN = BN_, BK = BK_, WM = WM_, WN = WN_, OCC = OCC_;
  static constexpr int PF = PF_;  // K slices in flight in registers (1 or 2) ahead of the LDS slice
  static constexpr int NT = 64 * WM * WN;
  static constexpr int TM = BM / WM, TN = BN / WN;
  static constexpr int MI = TM / 16, NJ = TN / 16;
  static constexpr int SPA = BK * BM / NT, SPB = BK * BN / NT;  // staged elements per thread
  static constexpr int LDA = BM + PADL, LDB = BN + PADL;         // LDS row lengths
  static constexpr int WAVES_PER_SIMD = OCC * WM * WN / 4;
  static_assert(NT % BM == 0 && NT % BN == 0, "thread count must tile the slice rows");
  static_assert(SPA >= 1 && SPB >= 1 && MI >= 1 && NJ >= 1, "bad tile config");
};
// The tiles the solver selects (profiles/gemm_variants_k512.md; the round-1 tuning candidates
// tall / narrowpf / square / wide / big8 / valu were measured slower everywhere and removed):
using CfgBig = Cfg<128, 128, 16, 2, 4, 2>;   // 512 threads, 2 WG/CU: the residual GEMM
using CfgNarrow = Cfg<128, 64, 8, 2, 2, 4>;  // 256 threads, 4 WG/CU: shallow / narrow updates
using CfgSmall = Cfg<64, 32, 16, 2, 1, 8>;   // 128 threads: latency-bound panel GEMMs (few tiles)
using CfgSquarePf = Cfg<128, 128, 8, 2, 2, 2, 2>;  // fp32 deep trailing updates (110.5 TF/s)
using CfgBigPf = Cfg<128, 128, 16, 2, 4, 2, 2>;    // fp64 deep updates the LDS-DMA kernel cannot take

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

template <typename T>
struct Mfma;

template <>
struct Mfma<double> {
  typedef double acc_t __attribute__((ext_vector_type(4)));
  static __device__ __forceinline__ acc_t op(double a, double b, acc_t c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  }
  // row_of(lane, q) = rl(lane) + rq(q)
  static __device__ __forceinline__ int rl(int lane) { return lane >> 4; }
  static constexpr int rq(int q) { return 4 * q; }
};

template <>
struct Mfma<float> {
  typedef float acc_t __attribute__((ext_vector_type(4)));
  static __device__ __forceinline__ acc_t op(float a, float b, acc_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ int rl(int lane) { return 4 * (lane >> 4); }
  static constexpr int rq(int q) { return q; }
};

// ---- buffer load/store of one element (32-bit lane offset + SGPR offset, both in bytes)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, kRecords, 0x00020000);
}
template <typename T>
__device__ __forceinline__ T bload(__amdgpu_buffer_rsrc_t r, int voff, int soff);
template <>
__device__ __forceinline__ double bload<double>(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0);
  return __builtin_bit_cast(double, v);
}
template <>
__device__ __forceinline__ float bload<float>(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
}
__device__ __forceinline__ void bstore(double v, __amdgpu_buffer_rsrc_t r, int voff, int soff) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, voff, soff, 0);
}
__device__ __forceinline__ void bstore(float v, __amdgpu_buffer_rsrc_t r, int voff, int soff) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned int, v), r, voff, soff, 0);
}
// the same with the non-temporal cache policy when nt (GemmArgs::c_nt; a uniform branch)
__device__ __forceinline__ float bload_c32(__amdgpu_buffer_rsrc_t r, int voff, int soff, bool nt) {
  return __builtin_bit_cast(float, nt ? __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 2)
                                      : __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
}
__device__ __forceinline__ void bstore_c(float v, __amdgpu_buffer_rsrc_t r, int voff, int soff, bool nt) {
  if (nt)
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned int, v), r, voff, soff, 2);
  else
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned int, v), r, voff, soff, 0);
}
__device__ __forceinline__ double bload_c(__amdgpu_buffer_rsrc_t r, int voff, int soff, bool nt) {
  const u32x2 v = nt ? __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 2)
                     : __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0);
  return __builtin_bit_cast(double, v);
}
__device__ __forceinline__ void bstore_c(double v, __amdgpu_buffer_rsrc_t r, int voff, int soff, bool nt) {
  if (nt)
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, voff, soff, 2);
  else
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, voff, soff, 0);
}

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
  // MODE_ACC extras (see GemmExtra): zero-input columns [zc0, zc1) and row blocks [zr, zr + zh)
  int64_t zc0, zc1;
  int64_t zr[GemmExtra::kMaxZeroRows];
  int64_t zh;
  // residual
  int64_t n_real, blk_m, p, k;
  double* partial;  // [M][nparts]
  int nparts;
  bool latency;     // GemmExtra::latency -> CfgSmall for few-tile launches
  bool lat_wide;    // GemmExtra::lat_wide
  bool lat_reg;     // GemmExtra::lat_reg
  bool c_overlap;   // LDS-DMA fp64 kernel: C loads overlapped with the first slices (GJ_GLDS_COVL)
  int group;        // LDS-DMA kernel: tile rows per column-walk group (1 = row-major tile order)
  void* tneg;       // GemmExtra::tneg: -C^T of the columns < tncols also written here
  int64_t ldt, tncols;
  const int32_t* pred;  // GemmExtra::owner_phys: skip unless *pred % pred_p == pred_k
  int64_t pred_p, pred_k;
  bool dense;           // GemmExtra::dense: the 5-workgroups-per-CU LDS-DMA build
  int build;            // GemmExtra::glds_build: this launch's LDS-DMA build (0 = auto)
  int tile;             // GemmExtra::glds_tile: this launch's LDS-DMA tile width (0 = auto)
  uint64_t rsel[GemmExtra::kRselWords];  // GemmExtra::rsel / rsel_m: row-block selection
  int64_t rsel_m;
  int64_t skc0, skc1;   // GemmExtra::skip_c0 / skip_c1 (whole tiles)
  const void* cin;      // GemmExtra::c_in (MODE_ACC input array, ld ldcin; null: C itself)
  int64_t ldcin;
  int c_nt;             // LDS-DMA fp64 kernel: C loads (bit 0) / stores (bit 1) non-temporal (GJ_GLDS_CNT)
};

// GemmExtra::rsel: physical first row of the tile whose logical first row is r (the block height
// rsel_m is a multiple of the tile height, so a tile never straddles two selected blocks)
__device__ __forceinline__ int64_t rsel_map(const GemmArgs& g, int64_t r) {
  int64_t bl = r / g.rsel_m;
  const int64_t off = r - bl * g.rsel_m;
#pragma unroll
  for (int w = 0; w < GemmExtra::kRselWords; ++w) {
    uint64_t x = g.rsel[w];
    const int c = __popcll(x);
    if (bl < c) {
      for (; bl > 0; --bl) x &= x - 1;
      return (64 * w + __ffsll((unsigned long long)x) - 1) * g.rsel_m + off;
    }
    bl -= c;
  }
  return 0;
}

// GemmExtra::owner_phys: the whole launch is a no-op on ranks that do not own the pivot
__device__ __forceinline__ bool gemm_skipped(const GemmArgs& g) {
  if (g.pred == nullptr) return false;
  const int64_t gg = *g.pred;
  return gg < 0 || gg % g.pred_p != g.pred_k;
}

// XCD-aware bijective remap: blocks b and b+8 share an XCD (MI355X_MICROARCH.md §Workgroup
// dispatch); give every XCD a contiguous range of tiles so neighbouring tiles share L2 lines.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8, x = bid % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
}

// One output tile of C (+)= A B (register-staged K slices, double-buffered LDS).  `tile` indexes the
// tiles_m x tiles_n grid with the N tiles fastest (they share the A slab).
template <typename T, int AL, int MODE, typename CF>
__device__ __forceinline__ void gemm_tile(const GemmArgs& g, const int tile) {
  using MF = Mfma<T>;
  using acc_t = typename MF::acc_t;
  constexpr int ES = sizeof(T);
  constexpr int BM = CF::BM, BN = CF::BN, BK = CF::BK, WN = CF::WN, NT = CF::NT;
  constexpr int TM = CF::TM, TN = CF::TN, MI = CF::MI, NJ = CF::NJ;
  __shared__ T ldsA[2][BK][CF::LDA];  // K-major A slices (double-buffered)
  __shared__ T ldsB[2][BK][CF::LDB];  // B slices

  const int tm = tile / g.tiles_n, tn = tile % g.tiles_n;
  if ((int64_t)tn * BN >= g.skc0 && (int64_t)(tn + 1) * BN <= g.skc1) return;  // GemmExtra::skip_c0/c1
  // m0L: the tile's first row among the M rows of the product; m0: its physical row (they differ
  // only under a row-block selection, GemmExtra::rsel)
  const int64_t m0L = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const int64_t m0 = g.rsel_m > 0 ? rsel_map(g, m0L) : m0L;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const T* A = static_cast<const T*>(g.A);
  const T* B = static_cast<const T*>(g.B);
  T* C = static_cast<T*>(g.C);
  const int ldc = (int)g.ldc, ldb = (int)g.ldb, lda = (int)g.lda;

  // C addressing: tile resource, one per-lane offset, (i, q) row offsets in SGPRs, j as immediate
  const int rlane = wm * TM + MF::rl(lane);  // row within the tile (minus i*16 + rq)
  const int clane = wn * TN + (lane & 15);   // col within the tile (minus j*16)
  // all masks in 32-bit tile-relative form (row/col bounds and the pivot rows/zero columns)
  const int Mt = (int)((g.M - m0L) < BM ? (g.M - m0L) : BM);
  const int Nt = (int)((g.N - n0) < BN ? (g.N - n0) : BN);
  const int64_t zlo = g.zc0 - n0, zhi = g.zc1 - n0;
  const int z0 = (int)(zlo < 0 ? 0 : (zlo > BN ? BN : zlo)), z1 = (int)(zhi < 0 ? 0 : (zhi > BN ? BN : zhi));
  int zr0[GemmExtra::kMaxZeroRows], zr1[GemmExtra::kMaxZeroRows];
#pragma unroll
  for (int z = 0; z < GemmExtra::kMaxZeroRows; ++z) {
    const int64_t lo = g.zr[z] - m0, hi = g.zr[z] + g.zh - m0;
    zr0[z] = (int)(lo < 0 ? 0 : (lo > BM ? BM : lo));
    zr1[z] = (int)(hi < 0 ? 0 : (hi > BM ? BM : hi));
  }
  __amdgpu_buffer_rsrc_t rc = rsrc(MODE == MODE_RESID ? (const void*)A : (const void*)(C + m0 * g.ldc + n0));
  const int cvoff = (rlane * ldc + clane) * ES;

  acc_t acc[MI][NJ];
  if (MODE == MODE_ACC) {
    // the accumulator's input: C itself, or GemmExtra::c_in
    const int ldi = g.cin ? (int)g.ldcin : ldc;
    const __amdgpu_buffer_rsrc_t rci =
        g.cin ? rsrc(static_cast<const T*>(g.cin) + m0 * g.ldcin + n0) : rc;
    const int civoff = (rlane * ldi + clane) * ES;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = rlane + i * 16 + MF::rq(q);
        const int soff = (i * 16 + MF::rq(q)) * ldi * ES;
        bool zrow = false;
#pragma unroll
        for (int z = 0; z < GemmExtra::kMaxZeroRows; ++z) zrow |= (r >= zr0[z] && r < zr1[z]);
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int c = clane + j * 16;
          const bool ok = r < Mt && c < Nt && !zrow && !(c >= z0 && c < z1);
          acc[i][j][q] = bload<T>(rci, ok ? civoff + j * 16 * ES : kOOB, soff);
        }
      }
  } else {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = acc_t{0, 0, 0, 0};
  }

  // ---- global -> register staging of one K slice (SPA A + SPB B elements per thread)
  // B slice [BK][BN]: element idx = e*NT + tid -> (k = e*(NT/BN) + tid/BN, n = tid%BN)
  // A slice K-major [BK][BM]: (k = e*(NT/BM) + tid/BM, i = tid%BM); row-major A: (i = idx/BK, k = idx%BK)
  constexpr int KPB = NT / BN, KPA = NT / BM;  // k rows covered per staging step
  const int bk_l = tid / BN, bn_l = tid % BN;
  const int ak_l = tid / BM, am_l = tid % BM;
  const bool b_col_ok = (n0 + bn_l) < g.N;
  const bool a_col_ok = (m0L + am_l) < g.M;
  const int b_voff = (bk_l * ldb + bn_l) * ES;
  const int a_voff = (AL == 1) ? (ak_l * lda + am_l) * ES : 0;
  T ra[CF::PF][CF::SPA], rb[CF::PF][CF::SPB];
  // column masks folded into the per-lane offsets once; the K bound is a 32-bit compare against
  // the (scalar) rows left in the slice, so the staging needs no 64-bit temporaries
  const int b_vo = b_col_ok ? b_voff : kOOB;
  const int a_vo = a_col_ok ? a_voff : kOOB;
  auto load_slice = [&](int64_t k0, auto slot) {
    constexpr int S = decltype(slot)::value;
    const int krem = (int)((g.K - k0) < BK ? (g.K - k0) : BK);
    __amdgpu_buffer_rsrc_t rbr = rsrc(B + k0 * g.ldb + n0);
#pragma unroll
    for (int e = 0; e < CF::SPB; ++e)
      rb[S][e] = bload<T>(rbr, (e * KPB + bk_l < krem) ? b_vo : kOOB, e * KPB * ldb * ES);
    if (AL == 1) {
      __amdgpu_buffer_rsrc_t rar = rsrc(A + k0 * g.lda + m0);
#pragma unroll
      for (int e = 0; e < CF::SPA; ++e)
        ra[S][e] = bload<T>(rar, (e * KPA + ak_l < krem) ? a_vo : kOOB, e * KPA * lda * ES);
    } else {
      __amdgpu_buffer_rsrc_t rar = rsrc(A + m0 * g.lda + k0);
#pragma unroll
      for (int e = 0; e < CF::SPA; ++e) {
        const int idx = e * NT + tid;
        const int ii = idx / BK, kk = idx % BK;
        const bool ok = (k0 + kk) < g.K && (m0L + ii) < g.M;
        ra[S][e] = bload<T>(rar, ok ? (ii * lda + kk) * ES : kOOB, 0);
      }
    }
  };
  auto store_slice = [&](int buf, auto slot) {
    constexpr int S = decltype(slot)::value;
#pragma unroll
    for (int e = 0; e < CF::SPB; ++e) ldsB[buf][e * KPB + bk_l][bn_l] = rb[S][e];
#pragma unroll
    for (int e = 0; e < CF::SPA; ++e) {
      if (AL == 1) {
        ldsA[buf][e * KPA + ak_l][am_l] = ra[S][e];
      } else {
        const int idx = e * NT + tid;
        ldsA[buf][idx % BK][idx / BK] = ra[S][e];
      }
    }
  };
  auto compute = [&](int cur) {
#pragma unroll
    for (int kk = 0; kk < BK; kk += 4) {
      T a[MI], b[NJ];
      const int kr = kk + (lane >> 4);
#pragma unroll
      for (int i = 0; i < MI; ++i) a[i] = ldsA[cur][kr][wm * TM + i * 16 + (lane & 15)];
#pragma unroll
      for (int j = 0; j < NJ; ++j) b[j] = ldsB[cur][kr][wn * TN + j * 16 + (lane & 15)];
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = MF::op(a[i], b[j], acc[i][j]);
    }
  };
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, (CF::PF > 1 ? 1 : 0)>;

  const int nk = (int)((g.K + BK - 1) / BK);
  load_slice(0, S0{});
  store_slice(0, S0{});
  // The C loads were issued before slice 0, so they are complete here; say so to the compiler:
  // otherwise the accumulators' pending loads merge into the loop header and hipcc waits vmcnt(0)
  // inside every iteration, draining the prefetch of the next K slice.
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) asm volatile("" ::"v"(acc[i][j][q]));
  if (CF::PF > 1 && nk > 1) load_slice((int64_t)BK, S1{});
  __syncthreads();
  if (CF::PF == 1) {
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < nk ) load_slice((int64_t)(kt + 1) * BK, S0{});
      compute(cur);
      if (kt + 1 < nk ) store_slice(cur ^ 1, S0{});
      __syncthreads();
    }
  } else {
    // slice s lives in register slot s & 1: slice kt+2 is fetched while slice kt is multiplied
    // and slice kt+1 (fetched one iteration earlier) is written to the other LDS buffer.
    auto body = [&](int kt, auto ld_slot, auto st_slot) {
      if (kt + 2 < nk ) load_slice((int64_t)(kt + 2) * BK, ld_slot);
      compute(kt & 1);
      if (kt + 1 < nk ) store_slice((kt & 1) ^ 1, st_slot);
      __syncthreads();
    };
    for (int kt = 0; kt < nk; kt += 2) {
      body(kt, S0{}, S1{});
      if (kt + 1 < nk) body(kt + 1, S1{}, S0{});
    }
  }

  if (MODE == MODE_ACC || MODE == MODE_STORE) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = rlane + i * 16 + MF::rq(q);
        const int soff = (i * 16 + MF::rq(q)) * ldc * ES;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int c = clane + j * 16;
          bstore(acc[i][j][q], rc, (r < Mt && c < Nt) ? cvoff + j * 16 * ES : kOOB, soff);
        }
      }
    if (g.tneg && n0 < g.tncols) {  // -C^T: lanes 0-15 of a row group write 16 rows of the transpose
      __amdgpu_buffer_rsrc_t rt = rsrc(static_cast<T*>(g.tneg) + n0 * g.ldt + m0);
      const int ldt = (int)g.ldt;
      const int Ntn = (int)((g.tncols - n0) < Nt ? (g.tncols - n0) : Nt);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int r = rlane + i * 16 + MF::rq(q);
#pragma unroll
          for (int j = 0; j < NJ; ++j) {
            const int c = clane + j * 16;
            bstore(-acc[i][j][q], rt, (r < Mt && c < Ntn) ? (c * ldt + r) * ES : kOOB, 0);
          }
        }
    }
  } else {  // MODE_RESID: per-row partial sum of |acc - I| over this wave's TN real columns
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int64_t row = m0 + rlane + i * 16 + MF::rq(q);
        const int64_t gr = ((row / g.blk_m) * g.p + g.k) * g.blk_m + row % g.blk_m;
        double s = 0.0;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int64_t col = n0 + clane + j * 16;
          if (col < g.n_real) s += fabs((double)acc[i][j][q] - (col == gr ? 1.0 : 0.0));
        }
        // sum across the 16 lanes that share this row (lane & 15)
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) s += __shfl_xor(s, off, 64);
        if ((lane & 15) == 0 && row < g.M) g.partial[row * g.nparts + (int64_t)tn * WN + wn] = s;
      }
  }
}

template <typename T, int AL, int MODE, typename CF>
__global__ __launch_bounds__(CF::NT, CF::WAVES_PER_SIMD) void gemm_kernel(GemmArgs g) {
  if (gemm_skipped(g)) return;
  gemm_tile<T, AL, MODE, CF>(g, xcd_remap((int)blockIdx.x, g.tiles_m * g.tiles_n));
}

// Several independent small GEMMs in one launch (the panel-piece products of one pivot step): the
// launch latency and the wait for a free CU slot are paid once instead of per product.  Workgroup
// b works on tile b - start[i] of product i (start[] = prefix sums of the tile counts).  Every
// product is C += A B with K-major A; C = A B is the same with all columns masked on input.
constexpr int kMaxBatch = 4;
struct GemmBatch {
  GemmArgs a[kMaxBatch];
  int start[kMaxBatch];
  int n;
};

template <typename T, typename CF>
__global__ __launch_bounds__(CF::NT, CF::WAVES_PER_SIMD) void gemm_batch_kernel(GemmBatch b) {
  if (gemm_skipped(b.a[0])) return;  // one predicate per batch (fill: every product's, identical)
  const int bid = (int)blockIdx.x;
  int i = 0;
#pragma unroll
  for (int k = 1; k < kMaxBatch; ++k) i += (k < b.n && bid >= b.start[k]) ? 1 : 0;
  // constant-index copies (a dynamically indexed kernel-argument array would go through scratch)
  switch (i) {
    case 0: gemm_tile<T, 1, MODE_ACC, CF>(b.a[0], bid - b.start[0]); break;
    case 1: gemm_tile<T, 1, MODE_ACC, CF>(b.a[1], bid - b.start[1]); break;
    case 2: gemm_tile<T, 1, MODE_ACC, CF>(b.a[2], bid - b.start[2]); break;
    default: gemm_tile<T, 1, MODE_ACC, CF>(b.a[3], bid - b.start[3]); break;
  }
}

// ---- fp64 trailing-update GEMM with LDS-DMA staging (buffer_load_dwordx4 ... lds).
//
// Same tile as CfgNarrow (128 x 64 per 256-thread workgroup, 2 x 2 waves of 64 x 32) but the K
// slices go global -> LDS without registers: each wave issues three 1-KiB LDS-DMA pieces per
// 8-deep slice (two A rows, then two B rows) into an NS-stage LDS ring, and the only waits in the
// loop are a counted vmcnt and a raw s_barrier.  Freeing the staging registers lets five
// workgroups share a CU.  Measured at 32768 x 4096 x 512: 62.6 TF/s (register staging 57.6; the
// same tile with no staging at all, a round-2 timing probe, 66.8).  Masked elements come back as zeros
// from out-of-range buffer offsets.
// LDS images: A [k][128 + 16 pad] (one DMA piece = one k row); B [k][64] with the two 128-B halves
// of every odd row swapped (element n of row k at n ^ 16(k&1)), so the four k rows read by one
// ds_read_b64 land on distinct bank halves; the swizzle is applied to the global source address.
// Requirements (checked by the dispatcher): K-major A, M, N, lda, ldb even, A/B 16-byte aligned.
// Round 6: BN = 128 (2 x 2 waves of 64 x 64, 16 accumulator tiles per wave) as a template
// option -- half the LDS fragment reads per MFMA (8 per 16 MFMAs instead of 6 per 8) and half the
// A-slab traffic per flop; B rows are then 1 KiB, one DMA piece each, like A's
// (profiles/gemm_tile128_r6.md).
namespace glds {
constexpr int BM = 128, BN = 64, NT = 256;
constexpr int LDA = BM + 16;  // A row stride (doubles)
template <int BK, int BN_ = BN>
struct Geo {
  static constexpr int SA = BK * LDA, SB = BK * BN_;  // stage sizes (doubles)
  static constexpr int STAGE = SA + SB;
  static constexpr int PIECES = BK / 4 + (BN_ == 128 ? BK / 4 : BK / 8);  // LDS-DMA instructions per wave per slice
};
}  // namespace glds

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, double* lds_wave_base, int voff, int soff = 0) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds_wave_base, 16,
                                           voff, soff, 0, 0);
}

// s_waitcnt vmcnt(P * n) for a runtime n <= 3: the pieces of the n most recent slices may stay in
// flight (P pieces per slice)
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// f(std::integral_constant<int, I>) for I = B .. E-1, unrolled at compile time
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

template <int P>
__device__ __forceinline__ void wait_pieces(int n) {
  static_assert(P >= 1 && 3 * P < 64, "pieces per slice");
  if (n <= 0) wait_vm<0>();
  else if (n == 1) wait_vm<P>();
  else if (n == 2) wait_vm<2 * P>();
  else wait_vm<3 * P>();
}

// PEEL = 1: the steady-state loop is unrolled over the NS stages (every LDS stage base, fragment
// offset and DMA destination a compile-time constant), its slices carry no K mask (the partial last
// slice, if any, takes the masked issue), and each DMA piece is one per-lane offset fixed for the
// whole launch plus the slice's byte offset in an SGPR (soffset): no per-slice VALU address or mask
// arithmetic, and a constant vmcnt per slice.
template <int MODE, int NS, int OCC, int BK, int PEEL = 0, int BNT = glds::BN>
__global__ __launch_bounds__(glds::NT, OCC) void gemm_glds_f64(GemmArgs g) {
  using namespace glds;
  if (gemm_skipped(g)) return;
  static_assert(NS >= 2 && NS <= 5, "stages");
  static_assert(BK == 8 || BK == 16, "slice depth");
  static_assert(BNT == 64 || BNT == 128, "tile width");
  constexpr int BN = BNT;  // (shadows glds::BN)
  constexpr int SA = Geo<BK, BN>::SA, STAGE = Geo<BK, BN>::STAGE, PIECES = Geo<BK, BN>::PIECES;
  using MF = Mfma<double>;
  using acc_t = MF::acc_t;
  constexpr int ES = 8, TM = 64, TN = BN / 2, MI = 4, NJ = TN / 16, WN = 2;
  // B DMA pieces per wave per slice: BN = 64 two k rows per piece (lane >> 5 picks the row), BN = 128
  // one k row per piece (like A)
  constexpr int BPW = BN == 128 ? BK / 4 : BK / 8;
  __shared__ double lds[NS * STAGE];

  const int nwg = g.tiles_m * g.tiles_n;
  const int tile = xcd_remap((int)blockIdx.x, nwg);
  // groups of G tile rows walked column by column: the tiles in flight on one XCD then share
  // G A-slabs and a narrow band of B instead of all of B
  const int G = g.group > 0 ? g.group : 1;
  const int grp = tile / (G * g.tiles_n), gr0 = grp * G;
  const int gsz = (g.tiles_m - gr0) < G ? (g.tiles_m - gr0) : G;
  const int rem = tile - grp * G * g.tiles_n;
  const int tm = gr0 + rem % gsz, tn = rem / gsz;
  if ((int64_t)tn * BN >= g.skc0 && (int64_t)(tn + 1) * BN <= g.skc1) return;  // GemmExtra::skip_c0/c1
  // m0L logical / m0 physical first row (GemmExtra::rsel, as in gemm_tile)
  const int64_t m0L = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const int64_t m0 = g.rsel_m > 0 ? rsel_map(g, m0L) : m0L;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const double* A = static_cast<const double*>(g.A);
  const double* B = static_cast<const double*>(g.B);
  double* C = static_cast<double*>(g.C);
  const int ldc = (int)g.ldc, ldb = (int)g.ldb, lda = (int)g.lda;

  const int rlane = wm * TM + MF::rl(lane);
  const int clane = wn * TN + (lane & 15);
  const int Mt = (int)((g.M - m0L) < BM ? (g.M - m0L) : BM);
  const int Nt = (int)((g.N - n0) < BN ? (g.N - n0) : BN);
  const int64_t zlo = g.zc0 - n0, zhi = g.zc1 - n0;
  const int z0 = (int)(zlo < 0 ? 0 : (zlo > BN ? BN : zlo)), z1 = (int)(zhi < 0 ? 0 : (zhi > BN ? BN : zhi));
  int zr0[GemmExtra::kMaxZeroRows], zr1[GemmExtra::kMaxZeroRows];
#pragma unroll
  for (int z = 0; z < GemmExtra::kMaxZeroRows; ++z) {
    const int64_t lo = g.zr[z] - m0, hi = g.zr[z] + g.zh - m0;
    zr0[z] = (int)(lo < 0 ? 0 : (lo > BM ? BM : lo));
    zr1[z] = (int)(hi < 0 ? 0 : (hi > BM ? BM : hi));
  }
  __amdgpu_buffer_rsrc_t rc = rsrc(C + m0 * g.ldc + n0);
  const int cvoff = (rlane * ldc + clane) * ES;

  acc_t acc[MI][NJ];
  const int ldi = g.cin ? (int)g.ldcin : ldc;
  const __amdgpu_buffer_rsrc_t rci = g.cin ? rsrc(static_cast<const double*>(g.cin) + m0 * g.ldcin + n0) : rc;
  const int civoff = (rlane * ldi + clane) * ES;
  // the accumulator input: C itself, or GemmExtra::c_in (ld ldcin); masked elements as 0
  auto load_c = [&]() {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = rlane + i * 16 + MF::rq(q);
        const int soff = (i * 16 + MF::rq(q)) * ldi * ES;
        bool zrow = false;
#pragma unroll
        for (int z = 0; z < GemmExtra::kMaxZeroRows; ++z) zrow |= (r >= zr0[z] && r < zr1[z]);
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int c = clane + j * 16;
          if (MODE == MODE_ACC) {
            const bool ok = r < Mt && c < Nt && !zrow && !(c >= z0 && c < z1);
            acc[i][j][q] = bload_c(rci, ok ? civoff + j * 16 * ES : kOOB, soff, g.c_nt & 1);
          } else {
            acc[i][j][q] = 0.0;
          }
        }
      }
  };
  // g.c_overlap: the C loads go out right behind the first slices' LDS-DMA pieces and the first
  // wait covers both (one memory latency at the tile's start instead of two); otherwise C lands
  // before the first piece is issued, as the hand-written waits count pieces only
  if (!(MODE == MODE_ACC && g.c_overlap)) {
    load_c();
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) asm volatile("" ::"v"(acc[i][j][q]));
  }

  // DMA piece geometry (per wave, per slice): A rows wid and wid + 4 (lane l -> columns 2l, 2l+1);
  // BN = 64: B rows 2 wid + (l >> 5), columns 2 (l & 31) of the swizzled image; BN = 128: B rows
  // wid + 4h, columns 2l of the swizzled image (row parity = wid's, as 4h is even).  h-th piece's
  // LDS row: bldsrow(h).
  const int acol = 2 * lane;
  const bool a_ok = (m0L + acol) < g.M;
  const int brow = BN == 128 ? wid : 2 * wid + (lane >> 5);
  const int bpos = BN == 128 ? 2 * lane : 2 * (lane & 31);
  const int bcol = bpos ^ ((brow & 1) * 16);
  const bool b_ok = (n0 + bcol) < g.N;
  auto brow_h = [&](int h) { return BN == 128 ? brow + 4 * h : brow + 8 * h; };       // global k row
  auto blds_h = [&](int h) { return BN == 128 ? (wid + 4 * h) * BN : 2 * (wid + 4 * h) * BN; };  // LDS offset
  __amdgpu_buffer_rsrc_t ra = rsrc(A + m0);
  __amdgpu_buffer_rsrc_t rb = rsrc(B + n0);
  const int Kd = (int)g.K;
  auto issue = [&](int kt) {
    double* st = lds + (kt % NS) * STAGE;
    const int k0 = kt * BK;
#pragma unroll
    for (int h = 0; h < BK / 4; ++h) {
      const int kr = wid + 4 * h;
      const bool ok = a_ok && (k0 + kr) < Kd;
      dma16(ra, st + kr * LDA, ok ? ((k0 + kr) * lda + acol) * ES : kOOB);
    }
#pragma unroll
    for (int h = 0; h < BPW; ++h) {
      const int br = brow_h(h);
      const bool okb = b_ok && (k0 + br) < Kd;
      dma16(rb, st + SA + blds_h(h), okb ? ((k0 + br) * ldb + bcol) * ES : kOOB);
    }
  };
  auto compute = [&](int kt) {
    const double* sa = lds + (kt % NS) * STAGE;
    const double* sb = sa + SA;
#pragma unroll
    for (int kk = 0; kk < BK; kk += 4) {
      double a[MI], b[NJ];
      const int kr = kk + (lane >> 4);
      const int sw = (kr & 1) * 16;
#pragma unroll
      for (int i = 0; i < MI; ++i) a[i] = sa[kr * LDA + wm * TM + i * 16 + (lane & 15)];
#pragma unroll
      for (int j = 0; j < NJ; ++j) b[j] = sb[kr * BN + ((wn * TN + j * 16 + (lane & 15)) ^ sw)];
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = MF::op(a[i], b[j], acc[i][j]);
    }
  };

  const int nk = (int)((g.K + BK - 1) / BK);
  const int pro = nk < NS - 1 ? nk : NS - 1;  // slices issued ahead
  if constexpr (PEEL == 0) {
    for (int kt = 0; kt < pro; ++kt) issue(kt);
    if (MODE == MODE_ACC && g.c_overlap) {
      load_c();
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the first slices and C landed
    } else {
      wait_pieces<PIECES>(pro - 1);  // slice 0 landed
    }
    __builtin_amdgcn_s_barrier();
    for (int kt = 0; kt < nk; ++kt) {
      if (kt + NS - 1 < nk) issue(kt + NS - 1);
      compute(kt);
      // slice kt+1 must have landed (this wave's pieces); the later issued ones may stay in flight
      const int last = (kt + NS - 1 < nk ? kt + NS - 1 : nk - 1);
      wait_pieces<PIECES>(last - (kt + 1) > 0 ? last - (kt + 1) : 0);
      // every wave's fragment reads of this stage complete before the barrier that lets a wave
      // refill it (hipcc sinks the last reads' wait below a raw s_barrier; measured free)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
  } else {
    const int nfull = Kd / BK;  // slices without a K mask
    int va[BK / 4], vb[BPW];
#pragma unroll
    for (int h = 0; h < BK / 4; ++h) va[h] = a_ok ? ((wid + 4 * h) * lda + acol) * ES : kOOB;
#pragma unroll
    for (int h = 0; h < BPW; ++h) vb[h] = b_ok ? (brow_h(h) * ldb + bcol) * ES : kOOB;
    const int sa_step = __builtin_amdgcn_readfirstlane(BK * lda * ES);
    const int sb_step = __builtin_amdgcn_readfirstlane(BK * ldb * ES);
    for (int kt = 0; kt < pro; ++kt) issue(kt);
    if (MODE == MODE_ACC && g.c_overlap) {
      load_c();
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the first slices and C landed
    } else {
      wait_pieces<PIECES>(pro - 1);  // slice 0 landed
    }
    __builtin_amdgcn_s_barrier();
    // steady state, NS slices per trip: every slice it issues (up to kt + 2 NS - 2) is full
    int kt = 0;
    for (; kt + 2 * NS - 2 < nfull; kt += NS) {
      static_for<0, NS>([&](auto s_c) {
        constexpr int S0 = decltype(s_c)::value, SI = (S0 + NS - 1) % NS;
        double* st = lds + SI * STAGE;
        const int kn = kt + S0 + NS - 1;
#pragma unroll
        for (int h = 0; h < BK / 4; ++h) dma16(ra, st + (wid + 4 * h) * LDA, va[h], kn * sa_step);
#pragma unroll
        for (int h = 0; h < BPW; ++h) dma16(rb, st + SA + blds_h(h), vb[h], kn * sb_step);
        const double* sa = lds + S0 * STAGE;
        const double* sb = sa + SA;
#pragma unroll
        for (int kk = 0; kk < BK; kk += 4) {
          double a[MI], b[NJ];
          const int kr = kk + (lane >> 4);
          const int sw = (kr & 1) * 16;
#pragma unroll
          for (int i = 0; i < MI; ++i) a[i] = sa[kr * LDA + wm * TM + i * 16 + (lane & 15)];
#pragma unroll
          for (int j = 0; j < NJ; ++j) b[j] = sb[kr * BN + ((wn * TN + j * 16 + (lane & 15)) ^ sw)];
#pragma unroll
          for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j) acc[i][j] = MF::op(a[i], b[j], acc[i][j]);
        }
        // slice kt + S0 + 1 landed; the NS - 2 newest may stay in flight
        wait_vm<PIECES * (NS - 2)>();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
      });
    }
    for (; kt < nk; ++kt) {  // the last slices: the general loop (runtime stage, masked issue)
      if (kt + NS - 1 < nk) issue(kt + NS - 1);
      compute(kt);
      const int last = (kt + NS - 1 < nk ? kt + NS - 1 : nk - 1);
      wait_pieces<PIECES>(last - (kt + 1) > 0 ? last - (kt + 1) : 0);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
  }

#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = rlane + i * 16 + MF::rq(q);
      const int soff = (i * 16 + MF::rq(q)) * ldc * ES;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int c = clane + j * 16;
        bstore_c(acc[i][j][q], rc, (r < Mt && c < Nt) ? cvoff + j * 16 * ES : kOOB, soff, g.c_nt & 2);
      }
    }
  if (g.tneg && n0 < g.tncols) {  // -C^T of the columns < tncols (GemmExtra::tneg)
    __amdgpu_buffer_rsrc_t rt = rsrc(static_cast<double*>(g.tneg) + n0 * g.ldt + m0);
    const int ldt = (int)g.ldt;
    const int Ntn = (int)((g.tncols - n0) < Nt ? (g.tncols - n0) : Nt);
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = rlane + i * 16 + MF::rq(q);
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int c = clane + j * 16;
          bstore(-acc[i][j][q], rt, (r < Mt && c < Ntn) ? (c * ldt + r) * ES : kOOB, 0);
        }
      }
  }
}

// ---- the pivot chain's small fp64 GEMMs (latency launches: panel pieces, look-ahead rows, column
// updates of a few row blocks).  The register-staged small tile walks K in 16-deep slices, each a
// global -> LDS -> MFMA round trip: 29 us for a 128 x 256 x 128 product on an idle GPU
// (bench/lat_gemm_probe.py).  Here every operand fragment goes straight from global memory into
// registers, a whole 32-deep K chunk per load burst and two chunks in flight (ping-pong register
// buffers): no LDS, no barrier, one memory latency per two chunks.  128 x 32 tile, 4 waves of
// 32 x 32 (v_mfma_f64_16x16x4, the same k order as every other kernel: bit-identical results).
template <int MODE>
__device__ __forceinline__ void lat_tile(const GemmArgs& g, int tile) {
  using MF = Mfma<double>;
  using acc_t = MF::acc_t;
  constexpr int BM = 128, BN = 32, KC = 32, NKK = KC / 4, ES = 8;
  const int tm = tile / g.tiles_n, tn = tile % g.tiles_n;
  if ((int64_t)tn * BN >= g.skc0 && (int64_t)(tn + 1) * BN <= g.skc1) return;  // GemmExtra::skip_c0/c1
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const int lane = (int)(threadIdx.x & 63);
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const double* A = static_cast<const double*>(g.A);
  const double* B = static_cast<const double*>(g.B);
  double* C = static_cast<double*>(g.C);
  const int lda = (int)g.lda, ldb = (int)g.ldb, ldc = (int)g.ldc, Kd = (int)g.K;
  const int Mt = (int)((g.M - m0) < BM ? (g.M - m0) : BM);
  const int Nt = (int)((g.N - n0) < BN ? (g.N - n0) : BN);
  const int64_t zlo = g.zc0 - n0, zhi = g.zc1 - n0;
  const int z0 = (int)(zlo < 0 ? 0 : (zlo > BN ? BN : zlo)), z1 = (int)(zhi < 0 ? 0 : (zhi > BN ? BN : zhi));
  int zr0[GemmExtra::kMaxZeroRows], zr1[GemmExtra::kMaxZeroRows];
#pragma unroll
  for (int z = 0; z < GemmExtra::kMaxZeroRows; ++z) {
    const int64_t lo = g.zr[z] - m0, hi = g.zr[z] + g.zh - m0;
    zr0[z] = (int)(lo < 0 ? 0 : (lo > BM ? BM : lo));
    zr1[z] = (int)(hi < 0 ? 0 : (hi > BM ? BM : hi));
  }
  // accumulator rows 32 w + 16 i + rl(lane) + rq(q), columns 16 j + (lane & 15)
  const int rbase = 32 * w + MF::rl(lane), cl = lane & 15;
  acc_t acc[2][2];
  {
    const __amdgpu_buffer_rsrc_t rci = rsrc(g.cin ? static_cast<const double*>(g.cin) + m0 * g.ldcin + n0
                                                  : static_cast<const double*>(C + m0 * g.ldc + n0));
    const int ldi = g.cin ? (int)g.ldcin : ldc;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = rbase + 16 * i + MF::rq(q);
        bool zrow = false;
#pragma unroll
        for (int z = 0; z < GemmExtra::kMaxZeroRows; ++z) zrow |= (r >= zr0[z] && r < zr1[z]);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int c = 16 * j + cl;
          if (MODE == MODE_ACC) {
            const bool ok = r < Mt && c < Nt && !zrow && !(c >= z0 && c < z1);
            acc[i][j][q] = bload<double>(rci, ok ? (r * ldi + c) * ES : kOOB, 0);
          } else {
            acc[i][j][q] = 0.0;
          }
        }
      }
  }
  // operand fragments: A row 32 w + 16 i + (lane & 15), B column 16 j + (lane & 15), k = 4 kk + (lane >> 4)
  const int ar = 32 * w + cl, kl = lane >> 4;
  const bool a_ok0 = ar < Mt, a_ok1 = ar + 16 < Mt, b_ok0 = cl < Nt, b_ok1 = cl + 16 < Nt;
  const __amdgpu_buffer_rsrc_t ra = rsrc(A + m0), rb = rsrc(B + n0);
  double fa0[NKK][2], fb0[NKK][2], fa1[NKK][2], fb1[NKK][2];
  auto load = [&](double (&fa)[NKK][2], double (&fb)[NKK][2], int k0) {
#pragma unroll
    for (int kk = 0; kk < NKK; ++kk) {
      const int k = k0 + 4 * kk + kl;
      const bool kok = k < Kd;
      fa[kk][0] = bload<double>(ra, (kok && a_ok0) ? (k * lda + ar) * ES : kOOB, 0);
      fa[kk][1] = bload<double>(ra, (kok && a_ok1) ? (k * lda + ar + 16) * ES : kOOB, 0);
      fb[kk][0] = bload<double>(rb, (kok && b_ok0) ? (k * ldb + cl) * ES : kOOB, 0);
      fb[kk][1] = bload<double>(rb, (kok && b_ok1) ? (k * ldb + cl + 16) * ES : kOOB, 0);
    }
  };
  auto compute = [&](const double (&fa)[NKK][2], const double (&fb)[NKK][2]) {
#pragma unroll
    for (int kk = 0; kk < NKK; ++kk)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = MF::op(fa[kk][i], fb[kk][j], acc[i][j]);
  };
  const int nch = (Kd + KC - 1) / KC;
  if (nch > 0) load(fa0, fb0, 0);
  if (nch > 1) load(fa1, fb1, KC);
  for (int c = 0; c < nch; c += 2) {
    compute(fa0, fb0);
    if (c + 2 < nch) load(fa0, fb0, (c + 2) * KC);
    if (c + 1 < nch) {
      compute(fa1, fb1);
      if (c + 3 < nch) load(fa1, fb1, (c + 3) * KC);
    }
  }
  const __amdgpu_buffer_rsrc_t rc = rsrc(C + m0 * g.ldc + n0);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = rbase + 16 * i + MF::rq(q);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int c = 16 * j + cl;
        bstore(acc[i][j][q], rc, (r < Mt && c < Nt) ? (r * ldc + c) * ES : kOOB, 0);
      }
    }
  if (g.tneg && n0 < g.tncols) {  // -C^T of the columns < tncols (GemmExtra::tneg)
    const __amdgpu_buffer_rsrc_t rt = rsrc(static_cast<double*>(g.tneg) + n0 * g.ldt + m0);
    const int ldt = (int)g.ldt;
    const int Ntn = (int)((g.tncols - n0) < Nt ? (g.tncols - n0) : Nt);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = rbase + 16 * i + MF::rq(q);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int c = 16 * j + cl;
          bstore(-acc[i][j][q], rt, (r < Mt && c < Ntn) ? (c * ldt + r) * ES : kOOB, 0);
        }
      }
  }
}

template <int MODE>
__global__ __launch_bounds__(256, 1) void gemm_lat_f64(GemmArgs g) {
  if (gemm_skipped(g)) return;
  lat_tile<MODE>(g, xcd_remap((int)blockIdx.x, g.tiles_m * g.tiles_n));
}

// gemm_batch_kernel with the register-fed tile (128 x 32 tiles: GemmArgs::tiles_* set for it)
__global__ __launch_bounds__(256, 1) void gemm_lat_batch_f64(GemmBatch b) {
  if (gemm_skipped(b.a[0])) return;
  const int bid = (int)blockIdx.x;
  int i = 0;
#pragma unroll
  for (int k = 1; k < kMaxBatch; ++k) i += (k < b.n && bid >= b.start[k]) ? 1 : 0;
  switch (i) {  // constant-index copies, as in gemm_batch_kernel
    case 0: lat_tile<MODE_ACC>(b.a[0], bid - b.start[0]); break;
    case 1: lat_tile<MODE_ACC>(b.a[1], bid - b.start[1]); break;
    case 2: lat_tile<MODE_ACC>(b.a[2], bid - b.start[2]); break;
    default: lat_tile<MODE_ACC>(b.a[3], bid - b.start[3]); break;
  }
}

// fp64 latency launches on gemm_lat_f64: per launch by GemmExtra::lat_reg (the engine sets it
// where CUs are reserved for the chain -- without a reservation its 208-register waves wait for
// room beside the trailing update: N = 32768 1069 -> 1096 ms), or forced for every launch by
// GJ_LAT_KERNEL=0/1 / set_lat_kernel(0 | 1); set_lat_kernel(-1) restores the per-launch choice
static int g_lat_kernel = -2;  // -2: not read yet, -1: per launch, 0 / 1: forced
static bool lat_kernel(const GemmArgs& a) {
  if (g_lat_kernel == -2) {
    const char* e = getenv("GJ_LAT_KERNEL");
    g_lat_kernel = e ? (std::atoi(e) != 0 ? 1 : 0) : -1;
  }
  return g_lat_kernel < 0 ? a.lat_reg : g_lat_kernel != 0;
}
void set_lat_kernel(int mode) { g_lat_kernel = mode < 0 ? -1 : (mode != 0 ? 1 : 0); }

template <int MODE>
static void launch_lat(const GemmArgs& a0, hipStream_t s) {
  GemmArgs a = a0;
  a.tiles_m = (int)((a.M + 127) / 128);
  a.tiles_n = (int)((a.N + 31) / 32);
  const int64_t nwg = (int64_t)a.tiles_m * a.tiles_n;
  if (nwg <= 0) return;
  hipLaunchKernelGGL((gemm_lat_f64<MODE>), dim3((unsigned)nwg), dim3(256), 0, s, a);
}

// GJ_GLDS_PEEL=0/1 or set_glds_peel(): the peeled, stage-unrolled main loop (PEEL template
// argument; default on since round 5).  32768 x 8192 x 512 alone, one box: 2 stages 63.65 -> 66.56
// TF/s, 3 stages 61.24 -> 67.57; the N = 32768 solve 1139 -> 1114 (2 stages) -> 1092-1093 ms
// (3 stages), two repetitions (scripts/runs/r5_ab.sh, profiles/gemm_peel_r5.md).
// GJ_GLDS_COVL=0/1 or set_glds_covl(): GemmArgs::c_overlap (default on; profiles/gemm_peel_r5.md)
static int g_glds_covl = -1;
static bool glds_covl() {
  if (g_glds_covl < 0) {
    const char* e = getenv("GJ_GLDS_COVL");
    g_glds_covl = e ? (std::atoi(e) != 0) : 1;
  }
  return g_glds_covl != 0;
}
void set_glds_covl(int on) { g_glds_covl = on ? 1 : 0; }
static int g_glds_peel = -1;
static int glds_peel() {
  if (g_glds_peel < 0) {
    const char* e = getenv("GJ_GLDS_PEEL");
    g_glds_peel = e ? (std::atoi(e) != 0) : 1;
  }
  return g_glds_peel;
}
void set_glds_peel(int on) { g_glds_peel = on ? 1 : 0; }
// GJ_GLDS_BUILD=<stages>.<waves-per-SIMD bound> (2.3 | 2.5 | 3.3) or set_glds_build(23 | 25 | 33):
// one build for every launch (A/B runs, tests); 0 = auto
static int g_glds_build = -1;
static int glds_build_forced() {
  if (g_glds_build < 0) {
    const char* e = getenv("GJ_GLDS_BUILD");
    const std::string v = e ? e : "";
    g_glds_build = v.empty() ? 0 : v == "2.5" ? 25 : v == "3.3" ? 33 : v == "2.3" ? 23 : v == "4.3" ? 43
                                                  : v == "16.2.3" ? 1623 : v == "3.2" ? 32 : -2;
    if (g_glds_build == -2) throw std::invalid_argument("GJ_GLDS_BUILD: 2.3 | 2.5 | 3.3 | 4.3 | 16.2.3 | 3.2");
  }
  return g_glds_build;
}
void set_glds_build(int b) {
  if (b != 0 && b != 23 && b != 25 && b != 33 && b != 43 && b != 1623 && b != 32)
    throw std::invalid_argument("glds build: 0 | 23 | 25 | 32 | 33 | 43 | 1623");
  g_glds_build = b;
}

// GJ_GLDS_TILE=64|128 or set_glds_tile(): the LDS-DMA kernel's tile width (BN) for the launches
// that take the 4-per-CU builds (the 5-per-CU dense build stays 128 x 64).  128 by default since
// round 6 (profiles/gemm_tile128_r6.md): 32768 x 8192 x 512 alone 64.4 -> 66.8-67.3 TF/s, the
// N = 32768 solve 1120.1 / 1119.9 -> 1083.7 / 1083.4 ms on one box (two repetitions, driver
// command), the shader clock at the same ~1370 W 2236 -> 2287 MHz: half the LDS fragment reads
// per MFMA and a third less operand traffic per flop buy clock under the power limit.
// Forced for every launch by GJ_GLDS_TILE / set_glds_tile(64 | 128); otherwise per launch
// (GemmArgs::tile from GemmExtra::glds_tile or the device hint), 128 when unnamed.  Under a CU
// reservation the engine names 64: N = 8192 22.68 / 22.69 ms (64) vs 23.52 / 23.53 (128), N = 16384
// even (scripts/runs/r6_small128.sh).
static int g_glds_tile = -1;  // -1 unread, 0 per launch, 64 / 128 forced
static int glds_tile(const GemmArgs& a) {
  if (g_glds_tile < 0) {
    const char* e = getenv("GJ_GLDS_TILE");
    const int v = e ? std::atoi(e) : 0;
    if (v != 0 && v != 64 && v != 128) throw std::invalid_argument("GJ_GLDS_TILE: 64 | 128");
    g_glds_tile = v;
  }
  return g_glds_tile ? g_glds_tile : a.tile == 64 ? 64 : 128;
}
void set_glds_tile(int bn) {
  if (bn != 0 && bn != 64 && bn != 128) throw std::invalid_argument("glds tile: 0 (per launch) | 64 | 128");
  g_glds_tile = bn;
}

// GemmArgs::c_nt: the fp64 LDS-DMA kernel's C loads (bit 0) / stores (bit 1) with the non-temporal
// cache policy, per launch from GemmExtra::c_nt (-1: unnamed, 0); GJ_GLDS_CNT=<bits> forces every
// launch (A/B runs).  N = 32768, every LDS-DMA launch, one box, two repetitions: 1129.9 / 1129.6 ms
// (0), 1123.5 / 1121.6 (loads), 1120.3 / 1117.4 (stores), 1111.7 / 1109.8 (both) -- the C tile is
// read and written once per panel, and streaming it leaves L2 to A and B (scripts/runs/r6_cnt.sh).
static int glds_cnt(int per_launch) {
  static const int forced = [] {
    const char* e = getenv("GJ_GLDS_CNT");
    return e ? (std::atoi(e) & 3) : -1;
  }();
  return forced >= 0 ? forced : per_launch > 0 ? (per_launch & 3) : 0;
}

// GJ_GLDS_GROUP=<G>: tile rows walked together per XCD (A/B runs; default 4)
static int glds_group() {
  static const int g = [] {
    const char* e = getenv("GJ_GLDS_GROUP");
    const int v = e ? std::atoi(e) : 4;
    return v > 0 ? v : 4;
  }();
  return g;
}

template <int MODE>
static void launch_glds(const GemmArgs& a0, hipStream_t s) {
  GemmArgs a = a0;
  const int forced0 = glds_build_forced();
  const int build0 = forced0 ? forced0 : a.build ? a.build : a.dense ? 25 : 23;
  if (glds_tile(a) == 128 && glds_peel() && build0 != 25) {
    // 128 x 128 tiles: 16 accumulator tiles per wave (128 VGPRs); <stages, W> 2.3 (auto) / 3.3 / 3.2.
    // Two stages by default: as fast alone as three (66.80 / 67.23 vs 66.83 / 67.25 TF/s), and 3 x
    // 34 KiB instead of 3 x 51 KiB per CU leaves 56 KiB of LDS free, so a co-resident candidate
    // inverse (72 KiB) starts when ONE trailing-update workgroup retires (profiles/gemm_tile128_r6.md)
    a.tiles_m = (int)((a.M + glds::BM - 1) / glds::BM);
    a.tiles_n = (int)((a.N + 127) / 128);
    const int64_t nwg = (int64_t)a.tiles_m * a.tiles_n;
    if (nwg <= 0) return;
    a.group = glds_group();
    a.c_nt = glds_cnt(a.c_nt);
    if (build0 == 33)
      hipLaunchKernelGGL((gemm_glds_f64<MODE, 3, 3, 8, 1, 128>), dim3((unsigned)nwg), dim3(glds::NT), 0, s, a);
    else if (build0 == 32)
      hipLaunchKernelGGL((gemm_glds_f64<MODE, 3, 2, 8, 1, 128>), dim3((unsigned)nwg), dim3(glds::NT), 0, s, a);
    else
      hipLaunchKernelGGL((gemm_glds_f64<MODE, 2, 3, 8, 1, 128>), dim3((unsigned)nwg), dim3(glds::NT), 0, s, a);
    return;
  }
  a.tiles_m = (int)((a.M + glds::BM - 1) / glds::BM);
  a.tiles_n = (int)((a.N + glds::BN - 1) / glds::BN);
  const int64_t nwg = (int64_t)a.tiles_m * a.tiles_n;
  if (nwg <= 0) return;
  // Template args <stages, W, slice>: W is __launch_bounds__' minimum waves per SIMD (a VGPR cap for
  // the compiler).  Residency = min(VGPR, LDS limits), from -Rpass-analysis=kernel-resource-usage:
  // <2,5,8> 96 VGPRs -> 5 workgroups/CU; <2,4,8> 111 and <2,3,8> 112 -> 4 (LDS would allow 6);
  // 3/4/5 stages -> 4/3/2.  Measured at 32768 x 4096 x 512 alone: <2,5,8> ("6") 62.6 TF/s, <2,4,8>
  // ("2") 61.2, <2,3,8> ("9") 60.5; 3/4/5 stages 59.4/59.1/53.7.  Inside the solver the order
  // flips: N=32768 <2,3,8> 1138 ms, <2,4,8> 1147, <2,5,8> 1205 (profiles/cu_reserve_sweep.md,
  // profiles/gemm_variants_k512.md): at 4 workgroups per CU the pivot-path kernels find room, and
  // the <2,3,8> schedule is the faster of the two 4-per-CU builds, so it is the only build.  Tile
  // rows are walked in groups of 4 (+0.5-1 %; groups 1-32 measured).
  a.group = 4;
  a.c_nt = glds_cnt(a.c_nt);
  // Round 5: with the peeled loop (constant vmcnt, no per-slice address / mask VALU) the third
  // stage pays -- it lets a slice's DMA stay in flight across a whole slice of MFMAs -- so 3.3 is
  // the default at 4 workgroups per CU; under a CU reservation the 5-per-CU build (2 stages: 5 x 3
  // stages would exceed the LDS) stays.  Without the peel, 2.3 (3.3 was slower, above).
  const int forced = glds_build_forced();
  const int build = forced ? forced : a.build ? a.build : a.dense ? 25 : glds_peel() ? 33 : 23;
  if (glds_peel()) {
    if (build == 25)
      hipLaunchKernelGGL((gemm_glds_f64<MODE, 2, 5, 8, 1>), dim3((unsigned)nwg), dim3(glds::NT), 0, s, a);
    else if (build == 33)
      hipLaunchKernelGGL((gemm_glds_f64<MODE, 3, 3, 8, 1>), dim3((unsigned)nwg), dim3(glds::NT), 0, s, a);
    else if (build == 43)  // 4 stages (53 KiB): 3 per CU
      hipLaunchKernelGGL((gemm_glds_f64<MODE, 4, 3, 8, 1>), dim3((unsigned)nwg), dim3(glds::NT), 0, s, a);
    else if (build == 1623)  // 16-deep slices, 2 stages (53 KiB): 3 per CU
      hipLaunchKernelGGL((gemm_glds_f64<MODE, 2, 3, 16, 1>), dim3((unsigned)nwg), dim3(glds::NT), 0, s, a);
    else
      hipLaunchKernelGGL((gemm_glds_f64<MODE, 2, 3, 8, 1>), dim3((unsigned)nwg), dim3(glds::NT), 0, s, a);
  } else if (build == 25)
    hipLaunchKernelGGL((gemm_glds_f64<MODE, 2, 5, 8>), dim3((unsigned)nwg), dim3(glds::NT), 0, s, a);
  else if (build == 33)
    hipLaunchKernelGGL((gemm_glds_f64<MODE, 3, 3, 8>), dim3((unsigned)nwg), dim3(glds::NT), 0, s, a);
  else
    hipLaunchKernelGGL((gemm_glds_f64<MODE, 2, 3, 8>), dim3((unsigned)nwg), dim3(glds::NT), 0, s, a);
}

static bool glds_ok(const GemmArgs& a) {
  const auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  return a.M % 2 == 0 && a.N % 2 == 0 && a.lda % 2 == 0 && a.ldb % 2 == 0 && al16(a.A) && al16(a.B) &&
         a.lda * a.K * 8 < kRecords && a.ldb * a.K * 8 < kRecords && a.ldc * 128 * 8 < kRecords;
}

// ---- fp32 trailing-update GEMM: the same LDS-DMA ring, built around v_mfma_f32_32x32x2_f32.
//
// The 32 x 32 x 2 instruction does the work of two 16 x 16 x 4 ones for the same two operand
// floats per lane, so a 64 x 64 wave tile (2 x 2 instructions) reads 4 LDS dwords per 256 MFMA
// cycles.  Its fragment reads are 32 consecutive floats of one k row per half-wave (the two lane
// groups of ds_read_b32), conflict-free without a pad or swizzle, so the LDS image of a slice is
// the plain [k][128] copy of A (K-major) and of B, and one 16-byte-per-lane DMA piece moves two
// whole k rows.  128 x 128 tile per 256-thread workgroup (2 x 2 waves).  Accumulator map of the
// 32 x 32 instruction: column lane & 31, register r -> row 8 (r >> 2) + 4 (lane >> 5) + (r & 3).
// Requirements (checked by glds32_ok): K-major A; M, N, lda, ldb multiples of 4; A/B 16-B aligned.
namespace glds32 {
constexpr int BM = 128, BN = 128, NT = 256;
}

__device__ __forceinline__ void dma16f(__amdgpu_buffer_rsrc_t r, float* lds_wave_base, int voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds_wave_base, 16, voff, soff,
                                           0, 0);
}
template <int P>
__device__ __forceinline__ void wait_slices(int n) {  // the pieces of the n newest slices may fly
  if (n <= 0) wait_vm<0>();
  else if (n == 1) wait_vm<P>();
  else if (n == 2) wait_vm<2 * P>();
  else wait_vm<3 * P>();
}

// PEEL = 1: the fp64 kernel's peeled, stage-unrolled steady state (gemm_glds_f64), for fp32.
// BNT = 256 (round 6, as the fp64 128 x 128 tile): 2 x 2 waves of 64 x 128, 128 accumulator VGPRs,
// a third fewer LDS fragment reads per MFMA and a quarter less staged operand traffic per flop; a B
// k row is then 1 KiB, one DMA piece (profiles/gemm_tile128_r6.md, fp32 section).
template <int MODE, int NS, int OCC, int BK, int PEEL = 0, int BNT = glds32::BN>
__global__ __launch_bounds__(glds32::NT, OCC) void gemm_glds_f32(GemmArgs g) {
  using namespace glds32;
  if (gemm_skipped(g)) return;
  static_assert(NS >= 2 && NS <= 4, "stages");
  static_assert(BK == 8 || BK == 16 || BK == 32, "slice depth");
  static_assert(BNT == 128 || BNT == 256, "tile width");
  constexpr int BN = BNT;  // (shadows glds32::BN)
  constexpr int SA = BK * BM, SB = BK * BN, STAGE = SA + SB;
  constexpr int BPW = BN == 256 ? BK / 4 : BK / 8;  // B pieces per wave per slice (1 / 2 k rows each)
  constexpr int PIECES = BK / 8 + BPW;  // per wave per slice: A rows (2 per piece), B rows
  typedef float acc_t __attribute__((ext_vector_type(16)));
  constexpr int ES = 4, TM = 64, TN = BN / 2, MI = 2, NJ = TN / 32, WN = 2;
  __shared__ float lds[NS * STAGE];

  const int nwg = g.tiles_m * g.tiles_n;
  const int tile = xcd_remap((int)blockIdx.x, nwg);
  const int G = g.group > 0 ? g.group : 1;
  const int grp = tile / (G * g.tiles_n), gr0 = grp * G;
  const int gsz = (g.tiles_m - gr0) < G ? (g.tiles_m - gr0) : G;
  const int rem = tile - grp * G * g.tiles_n;
  const int tm = gr0 + rem % gsz, tn = rem / gsz;
  if ((int64_t)tn * BN >= g.skc0 && (int64_t)(tn + 1) * BN <= g.skc1) return;  // GemmExtra::skip_c0/c1
  // m0L logical / m0 physical first row (GemmExtra::rsel, as in gemm_tile)
  const int64_t m0L = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const int64_t m0 = g.rsel_m > 0 ? rsel_map(g, m0L) : m0L;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const float* A = static_cast<const float*>(g.A);
  const float* B = static_cast<const float*>(g.B);
  float* C = static_cast<float*>(g.C);
  const int ldc = (int)g.ldc, ldb = (int)g.ldb, lda = (int)g.lda;

  const int rlane = wm * TM + 4 * (lane >> 5);
  const int clane = wn * TN + (lane & 31);
  const int Mt = (int)((g.M - m0L) < BM ? (g.M - m0L) : BM);
  const int Nt = (int)((g.N - n0) < BN ? (g.N - n0) : BN);
  const int64_t zlo = g.zc0 - n0, zhi = g.zc1 - n0;
  const int z0 = (int)(zlo < 0 ? 0 : (zlo > BN ? BN : zlo)), z1 = (int)(zhi < 0 ? 0 : (zhi > BN ? BN : zhi));
  int zr0[GemmExtra::kMaxZeroRows], zr1[GemmExtra::kMaxZeroRows];
#pragma unroll
  for (int z = 0; z < GemmExtra::kMaxZeroRows; ++z) {
    const int64_t lo = g.zr[z] - m0, hi = g.zr[z] + g.zh - m0;
    zr0[z] = (int)(lo < 0 ? 0 : (lo > BM ? BM : lo));
    zr1[z] = (int)(hi < 0 ? 0 : (hi > BM ? BM : hi));
  }
  __amdgpu_buffer_rsrc_t rc = rsrc(C + m0 * g.ldc + n0);
  const int cvoff = (rlane * ldc + clane) * ES;

  acc_t acc[MI][NJ];
  const int ldi = g.cin ? (int)g.ldcin : ldc;  // the accumulator's input: C or GemmExtra::c_in
  const __amdgpu_buffer_rsrc_t rci = g.cin ? rsrc(static_cast<const float*>(g.cin) + m0 * g.ldcin + n0) : rc;
  const int civoff = (rlane * ldi + clane) * ES;
  auto load_c = [&]() {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int dr = i * 32 + 8 * (q >> 2) + (q & 3);
        const int r = rlane + dr;
        bool zrow = false;
#pragma unroll
        for (int z = 0; z < GemmExtra::kMaxZeroRows; ++z) zrow |= (r >= zr0[z] && r < zr1[z]);
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int c = clane + j * 32;
          if (MODE == MODE_ACC) {
            const bool ok = r < Mt && c < Nt && !zrow && !(c >= z0 && c < z1);
            acc[i][j][q] = bload_c32(rci, ok ? civoff + j * 32 * ES : kOOB, dr * ldi * ES, g.c_nt & 1);
          } else {
            acc[i][j][q] = 0.0f;
          }
        }
      }
  };
  // g.c_overlap: C goes out right behind the first slices' DMA pieces (as in gemm_glds_f64)
  if (!(MODE == MODE_ACC && g.c_overlap)) {
    load_c();
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int q = 0; q < 16; ++q) asm volatile("" ::"v"(acc[i][j][q]));
  }

  // DMA piece (per wave): k rows 2 (wid + 4h) + (lane >> 5), floats 4 (lane & 31) .. + 3; B at
  // BN = 256: k rows wid + 4h, floats 4 lane .. + 3
  const int dcol = 4 * (lane & 31), drow = lane >> 5;
  const int bdcol = BN == 256 ? 4 * lane : dcol;
  const bool a_ok = (m0L + dcol) < g.M, b_ok = (n0 + bdcol) < g.N;
  auto bkp = [&](int h) { return BN == 256 ? wid + 4 * h : 2 * (wid + 4 * h); };   // LDS k row of piece h
  auto bkr = [&](int h) { return BN == 256 ? wid + 4 * h : 2 * (wid + 4 * h) + drow; };  // its global k row
  __amdgpu_buffer_rsrc_t ra = rsrc(A + m0);
  __amdgpu_buffer_rsrc_t rb = rsrc(B + n0);
  const int Kd = (int)g.K;
  auto issue = [&](int kt) {
    float* st = lds + (kt % NS) * STAGE;
    const int k0 = kt * BK;
#pragma unroll
    for (int h = 0; h < BK / 8; ++h) {
      const int kp = 2 * (wid + 4 * h), kr = kp + drow;
      const bool ok = a_ok && (k0 + kr) < Kd;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (__attribute__((address_space(3))) void*)(st + kp * BM), 16,
                                               ok ? ((k0 + kr) * lda + dcol) * ES : kOOB, 0, 0, 0);
    }
#pragma unroll
    for (int h = 0; h < BPW; ++h) {
      const int kp = bkp(h), kr = bkr(h);
      const bool ok = b_ok && (k0 + kr) < Kd;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (__attribute__((address_space(3))) void*)(st + SA + kp * BN),
                                               16, ok ? ((k0 + kr) * ldb + bdcol) * ES : kOOB, 0, 0, 0);
    }
  };
  // fragments of k step kk + 2 are read while the MFMAs of step kk run (two register sets)
  auto compute_st = [&](const int stage) {
    const float* sa = lds + stage * STAGE + wm * TM + (lane & 31) + (lane >> 5) * BM;
    const float* sb = lds + stage * STAGE + SA + wn * TN + (lane & 31) + (lane >> 5) * BN;
    float a[2][MI], b[2][NJ];
    auto frag = [&](int kk, int s) {
#pragma unroll
      for (int i = 0; i < MI; ++i) a[s][i] = sa[kk * BM + i * 32];
#pragma unroll
      for (int j = 0; j < NJ; ++j) b[s][j] = sb[kk * BN + j * 32];
    };
    frag(0, 0);
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
      const int s = (kk >> 1) & 1;
      if (kk + 2 < BK) frag(kk + 2, s ^ 1);
      __builtin_amdgcn_sched_barrier(0);  // keep the reads ahead of the MFMAs
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s][i], b[s][j], acc[i][j], 0, 0, 0);
    }
  };
  auto compute = [&](int kt) { compute_st(kt % NS); };

  const int nk = (int)((g.K + BK - 1) / BK);
  const int pro = nk < NS - 1 ? nk : NS - 1;
  for (int kt = 0; kt < pro; ++kt) issue(kt);
  if (MODE == MODE_ACC && g.c_overlap) {
    load_c();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the first slices and C landed
  } else {
    wait_slices<PIECES>(pro - 1);
  }
  __builtin_amdgcn_s_barrier();
  int kt = 0;
  if constexpr (PEEL == 1) {
    // steady state, NS slices per trip, every slice it issues (up to kt + 2 NS - 2) full: fixed
    // per-lane DMA offsets + the slice offset in an SGPR, compile-time stages, constant waits
    const int nfull = Kd / BK;
    int va[BK / 8], vb[BPW];
#pragma unroll
    for (int h = 0; h < BK / 8; ++h) {
      const int kr = 2 * (wid + 4 * h) + drow;
      va[h] = a_ok ? (kr * lda + dcol) * ES : kOOB;
    }
#pragma unroll
    for (int h = 0; h < BPW; ++h) vb[h] = b_ok ? (bkr(h) * ldb + bdcol) * ES : kOOB;
    const int sa_step = __builtin_amdgcn_readfirstlane(BK * lda * ES);
    const int sb_step = __builtin_amdgcn_readfirstlane(BK * ldb * ES);
    for (; kt + 2 * NS - 2 < nfull; kt += NS) {
      static_for<0, NS>([&](auto s_c) {
        constexpr int S0 = decltype(s_c)::value, SI = (S0 + NS - 1) % NS;
        float* st = lds + SI * STAGE;
        const int kn = kt + S0 + NS - 1;
#pragma unroll
        for (int h = 0; h < BK / 8; ++h) dma16f(ra, st + 2 * (wid + 4 * h) * BM, va[h], kn * sa_step);
#pragma unroll
        for (int h = 0; h < BPW; ++h) dma16f(rb, st + SA + bkp(h) * BN, vb[h], kn * sb_step);
        compute_st(S0);
        wait_vm<PIECES * (NS - 2)>();  // slice kt + S0 + 1 landed; the NS - 2 newest may fly
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
      });
    }
  }
  for (; kt < nk; ++kt) {
    if (kt + NS - 1 < nk) issue(kt + NS - 1);
    compute(kt);
    const int last = (kt + NS - 1 < nk ? kt + NS - 1 : nk - 1);
    wait_slices<PIECES>(last - (kt + 1) > 0 ? last - (kt + 1) : 0);
    // every wave's fragment reads of this stage are complete before anyone refills it
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }

#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int dr = i * 32 + 8 * (q >> 2) + (q & 3);
      const int r = rlane + dr;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int c = clane + j * 32;
        bstore_c(acc[i][j][q], rc, (r < Mt && c < Nt) ? cvoff + j * 32 * ES : kOOB, dr * ldc * ES, g.c_nt & 2);
      }
    }
}

template <int MODE>
static void launch_glds32(const GemmArgs& a0, hipStream_t s) {
  GemmArgs a = a0;
  // the wide tile where the engine (or GJ_GLDS_TILE=128) names the wide fp64 tile
  const bool skip_ok = !(a.skc1 > a.skc0) || (a.skc0 % 256 == 0 && a.skc1 % 256 == 0);  // whole tiles
  if (glds_tile(a) == 128 && glds_peel() && skip_ok) {
    a.tiles_m = (int)((a.M + glds32::BM - 1) / glds32::BM);
    a.tiles_n = (int)((a.N + 255) / 256);
    const int64_t nwg = (int64_t)a.tiles_m * a.tiles_n;
    if (nwg <= 0) return;
    a.group = 4;
    a.c_nt = glds_cnt(a.c_nt);
    hipLaunchKernelGGL((gemm_glds_f32<MODE, 2, 3, 16, 1, 256>), dim3((unsigned)nwg), dim3(glds32::NT), 0, s, a);
    return;
  }
  a.tiles_m = (int)((a.M + glds32::BM - 1) / glds32::BM);
  a.tiles_n = (int)((a.N + glds32::BN - 1) / glds32::BN);
  const int64_t nwg = (int64_t)a.tiles_m * a.tiles_n;
  if (nwg <= 0) return;
  a.group = 4;
  a.c_nt = glds_cnt(a.c_nt);
  // <stages, launch-bounds workgroups per CU, slice depth>; 8 KiB of LDS per 8 k rows.  Measured
  // (round 2, TF/s at 32768x16384x512 / 16384x65536x512 / 4096x65536x1024): <2,3,16>
  // 125.9 / 128.5 / 132.4 (4 WG/CU at 114 VGPRs), <2,2,16> 122.1 / 128.1 / 133.1, <3,2,16> 122.5 /
  // 125.0 / 129.1, <2,3,8> 125.3 / 127.7 / 131.4, <2,2,32> 116.2 / 118.4 / 124.1; squarepf 117.8 /
  // 119.8 / 122.3.
  // Round 5: the peeled steady state (set_glds_peel / GJ_GLDS_PEEL, shared with the fp64 kernel);
  // GJ_GLDS32_BUILD=2.3 / 2.4 / 3.3 (stages.launch-bound waves): A/B runs.  The peeled 2-stage loop
  // takes 152 VGPRs under a bound of 3 (3 per CU); 2.4 caps it at 128 for 4 per CU.
  static const int b32 = [] {
    const char* e = getenv("GJ_GLDS32_BUILD");
    const std::string v = e ? e : "";
    return v == "2.3" ? 23 : v == "3.3" ? 33 : 24;
  }();
  if (glds_peel()) {
    if (b32 == 33)
      hipLaunchKernelGGL((gemm_glds_f32<MODE, 3, 3, 16, 1>), dim3((unsigned)nwg), dim3(glds32::NT), 0, s, a);
    else if (b32 == 23)
      hipLaunchKernelGGL((gemm_glds_f32<MODE, 2, 3, 16, 1>), dim3((unsigned)nwg), dim3(glds32::NT), 0, s, a);
    else
      hipLaunchKernelGGL((gemm_glds_f32<MODE, 2, 4, 16, 1>), dim3((unsigned)nwg), dim3(glds32::NT), 0, s, a);
  } else {
    hipLaunchKernelGGL((gemm_glds_f32<MODE, 2, 3, 16>), dim3((unsigned)nwg), dim3(glds32::NT), 0, s, a);
  }
}

static bool glds32_ok(const GemmArgs& a) {
  const auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  return a.M % 4 == 0 && a.N % 4 == 0 && a.lda % 4 == 0 && a.ldb % 4 == 0 && al16(a.A) && al16(a.B) &&
         a.lda * a.K * 4 < kRecords && a.ldb * a.K * 4 < kRecords && a.ldc * 128 * 4 < kRecords;
}

template <typename T, int AL, int MODE, typename CF>
static void launch_cfg(const GemmArgs& a0, hipStream_t s) {
  GemmArgs a = a0;
  a.tiles_m = (int)((a.M + CF::BM - 1) / CF::BM);
  a.tiles_n = (int)((a.N + CF::BN - 1) / CF::BN);
  const int64_t nwg = (int64_t)a.tiles_m * a.tiles_n;
  if (nwg <= 0) return;
  hipLaunchKernelGGL((gemm_kernel<T, AL, MODE, CF>), dim3((unsigned)nwg), dim3(CF::NT), 0, s, a);
}

// Variant selection (GJ_GEMM_VARIANT=<name> or set_gemm_variant(); default "auto": per shape, by
// measurement — profiles/gemm_variants_k512.jsonl).
constexpr int kAutoVariant = 10;
static int g_variant = -1;
static int gemm_variant() {
  if (g_variant < 0) {
    const char* e = getenv("GJ_GEMM_VARIANT");
    g_variant = (e && *e) ? gemm_variant_id(e) : kAutoVariant;  // a typo throws: never a silent default
  }
  return g_variant;
}
int gemm_variant_id(const char* name) {
  const std::string s(name);
  static const char* names[] = {"big", "narrow", "", "", "", "", "squarepf", "", "", "bigpf", "auto", "glds"};
  for (int i = 0; i < (int)(sizeof(names) / sizeof(names[0])); ++i)
    if (*names[i] && s == names[i]) return i;
  throw std::invalid_argument("unknown GEMM variant '" + s + "' (big | narrow | squarepf | bigpf | glds | auto)");
}
void set_gemm_variant(int v) { g_variant = v; }

// Below this many narrow tiles the GEMM cannot fill the 256 CUs: use 8x smaller tiles instead
// (the panel-factorisation GEMMs: m x m .. m x d*m outputs, or rows x m column updates).
constexpr int64_t kSmallGridTiles = 512;

// GemmExtra::lat_wide (or set_lat_glds() for every launch, tests): latency launches of >=
// kLatGldsRows rows (the pivot chain's column updates: rows x m x j m) on the LDS-DMA kernel
// (128 x 64 tiles, 4 per CU) instead of the 64 x 32 register-staged latency tile
constexpr int64_t kLatGldsRows = 1024;
static int g_lat_glds = 0;
static bool lat_glds(const GemmArgs& a) { return a.lat_wide || g_lat_glds; }
void set_lat_glds(int on) { g_lat_glds = on ? 1 : 0; }

// the LDS-DMA kernel of T when it takes the shape (K-major A, no C_in; fp32: no -C^T epilogue)
template <typename T, int AL, int MODE>
static bool try_glds(const GemmArgs& a, hipStream_t s) {
  if constexpr (AL == 1 && MODE != MODE_RESID) {
    if (a.cin && a.ldcin * 128 * (int64_t)sizeof(T) >= kRecords) return false;
    if constexpr (sizeof(T) == 8) {
      if (glds_ok(a)) {
        launch_glds<MODE>(a, s);
        return true;
      }
    } else {
      if (!a.tneg && glds32_ok(a)) {
        launch_glds32<MODE>(a, s);
        return true;
      }
    }
  }
  return false;
}

template <typename T, int AL, int MODE>
static void launch(const GemmArgs& a, hipStream_t s) {
  if (MODE == MODE_RESID) return launch_cfg<T, AL, MODE, CfgBig>(a, s);
  if (a.rsel_m > 0) {  // row-block selection: LDS-DMA (128-row tiles) or register-staged tiles whose height divides the block
    const bool v_glds = gemm_variant() == kAutoVariant || gemm_variant() == 11;
    if (a.rsel_m % 128 == 0 && v_glds && (!a.latency || lat_glds(a)) && try_glds<T, AL, MODE>(a, s)) return;
    if (a.rsel_m % CfgNarrow::BM == 0 && !a.latency) return launch_cfg<T, AL, MODE, CfgNarrow>(a, s);
    if (a.rsel_m % CfgSmall::BM == 0) return launch_cfg<T, AL, MODE, CfgSmall>(a, s);
    throw Error(Status::BadArgs, "gemm: a row-block selection needs 64 | block height");
  }
  const int64_t narrow_tiles = ((a.M + CfgNarrow::BM - 1) / CfgNarrow::BM) * ((a.N + CfgNarrow::BN - 1) / CfgNarrow::BN);
  if (a.latency && narrow_tiles < kSmallGridTiles && gemm_variant() != 0) {
    if (lat_glds(a) && a.M >= kLatGldsRows && gemm_variant() == kAutoVariant && try_glds<T, AL, MODE>(a, s)) return;
    if constexpr (sizeof(T) == 8 && AL == 1 && MODE != MODE_RESID) {
      if (lat_kernel(a) && gemm_variant() == kAutoVariant && a.lda * a.K * 8 < kRecords && a.ldb * a.K * 8 < kRecords &&
          a.ldc * 128 * 8 < kRecords && (!a.cin || a.ldcin * 128 * 8 < kRecords))
        return launch_lat<MODE>(a, s);
    }
    return launch_cfg<T, AL, MODE, CfgSmall>(a, s);
  }
  // C_in (the chunk pass's normalisation input): the LDS-DMA kernels take it too since round 5 --
  // COMM's 128 x W x j m products ran 90-100 us on the register-staged tile at N = 8192
  static const bool cin_glds = !getenv("GJ_CIN_GLDS") || std::atoi(getenv("GJ_CIN_GLDS")) != 0;  // A/B knob
  if (a.cin && cin_glds && gemm_variant() == kAutoVariant && try_glds<T, AL, MODE>(a, s)) return;
  if (a.cin) return launch_cfg<T, AL, MODE, CfgNarrow>(a, s);
  int v = gemm_variant();
  int fallback = sizeof(T) == 8 ? 9 : 6;  // when the LDS-DMA kernel cannot take the shape
  if (v == kAutoVariant) {
    // Trailing updates (K >= 256) with enough 128x128 tiles to fill the chip: fp64 the LDS-DMA
    // kernel (61 TF/s vs 57.6 register-staged at 32768x4096x512; at the depth-2 K = 256 of
    // N = 8192 45.6 vs 43.1 TF/s at 8192x4096x256 and 26.9 vs 27.9 ms per inversion, round 3),
    // fp32 (K >= 384, as measured) the LDS-DMA 32x32x2 kernel.  Everything else keeps the
    // register-staged narrow tile.
    // Round 5, with the peeled LDS-DMA loop: every fp64 non-latency product takes it (the owners'
    // row normalisations of the chunk pass, the look-ahead update at N <= 16384 too): N = 8192
    // 25.54 / 24.95 -> 24.65 / 24.54 ms, N = 16384 153.4 / 152.7 -> 152.8 / 152.3, N = 32768 even
    // (scripts/runs/r5_fp32.sh, profiles/gemm_peel_r5.md).
    const int64_t big_tiles = ((a.M + 127) / 128) * ((a.N + 127) / 128);
    const bool deep = a.K >= (sizeof(T) == 8 ? 256 : 384) && big_tiles >= 512;
    v = (deep || sizeof(T) == 8) ? 11 : 1;
    if (!deep) fallback = 1;  // the round-4 rule's register-staged narrow tile
  }
  if (v == 11 && a.tneg && sizeof(T) == 4) v = 6;  // the fp32 LDS-DMA kernel has no -C^T epilogue
  if (v == 11) {  // LDS-DMA fp64 kernel; other dtypes / layouts / alignments take the next best tile
    if constexpr (sizeof(T) == 8 && AL == 1 && MODE != MODE_RESID) {
      if (glds_ok(a)) return launch_glds<MODE>(a, s);
    }
    if constexpr (sizeof(T) == 4 && AL == 1 && MODE != MODE_RESID) {
      if (glds32_ok(a)) return launch_glds32<MODE>(a, s);
    }
    v = fallback;
  }
  switch (v) {
    case 1: return launch_cfg<T, AL, MODE, CfgNarrow>(a, s);
    case 6: return launch_cfg<T, AL, MODE, CfgSquarePf>(a, s);
    case 9: return launch_cfg<T, AL, MODE, CfgBigPf>(a, s);
    default: return launch_cfg<T, AL, MODE, CfgBig>(a, s);
  }
}

static void fill_extra(GemmArgs& a, const GemmExtra* ex) {
  constexpr int64_t kNone = -(int64_t(1) << 62);
  a.zc0 = ex ? ex->zc0 : 0;
  a.zc1 = ex ? ex->zc1 : 0;
  a.zh = ex ? ex->zh : 0;
  for (int z = 0; z < GemmExtra::kMaxZeroRows; ++z) a.zr[z] = (ex && z < ex->nzr) ? ex->zr[z] : kNone;
  a.latency = ex ? ex->latency : false;
  a.lat_wide = ex ? ex->lat_wide : false;
  a.lat_reg = ex ? ex->lat_reg : false;
  a.c_overlap = glds_covl();
  a.tneg = ex ? ex->tneg : nullptr;
  a.ldt = ex ? ex->ldtneg : 0;
  a.tncols = (ex && ex->tneg_cols > 0) ? ex->tneg_cols : (int64_t(1) << 62);
  a.pred = ex ? ex->owner_phys : nullptr;
  a.pred_p = ex ? ex->owner_p : 1;
  a.pred_k = ex ? ex->owner_k : 0;
  a.dense = ex ? ex->dense : false;
  a.build = ex ? ex->glds_build : 0;
  a.tile = ex ? ex->glds_tile : 0;
  a.c_nt = ex ? ex->c_nt : -1;
  a.rsel_m = ex ? ex->rsel_m : 0;
  a.cin = ex ? ex->c_in : nullptr;
  a.skc0 = ex ? ex->skip_c0 : 0;
  a.skc1 = ex ? ex->skip_c1 : 0;
  if (a.skc1 > a.skc0 && (a.skc0 % 128 != 0 || a.skc1 % 128 != 0))
    throw Error(Status::BadArgs, "gemm: skip columns must be multiples of 128");
  a.ldcin = ex ? ex->ldc_in : 0;
  for (int w = 0; w < GemmExtra::kRselWords; ++w) a.rsel[w] = ex ? ex->rsel[w] : 0;
}

void gemm(DType dt, int op, int a_kmajor, int64_t M, int64_t N, int64_t K, const void* A,
          int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, hipStream_t s,
          const GemmExtra* ex) {
  if (M <= 0 || N <= 0) return;
  GemmArgs a{};
  a.M = M; a.N = N; a.K = K; a.A = A; a.lda = lda; a.B = B; a.ldb = ldb; a.C = C; a.ldc = ldc;
  fill_extra(a, ex);
  if (a.tneg && a.ldt * 128 * (dt == DType::F64 ? 8 : 4) >= kRecords)
    throw Error(Status::BadArgs, "gemm: -C^T leading dimension too large for 32-bit buffer offsets");
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

void gemm_batch(DType dt, const GemmDesc* d, int n, hipStream_t s) {
  using CF = CfgSmall;
  // the register-fed tile (GemmExtra::lat_reg on every product, fp64, offsets within 32 bits)
  static const bool lat_batch = !getenv("GJ_LAT_BATCH") || std::atoi(getenv("GJ_LAT_BATCH")) != 0;
  bool lat = lat_batch && dt == DType::F64 && n > 0;
  for (int e = 0; e < n && lat; ++e) {
    GemmArgs t{};
    t.lat_reg = d[e].ex.lat_reg;
    lat = lat_kernel(t) && d[e].lda * d[e].K * 8 < kRecords && d[e].ldb * d[e].K * 8 < kRecords &&
          d[e].ldc * 128 * 8 < kRecords;
  }
  const int64_t TBM = lat ? 128 : CF::BM, TBN = lat ? 32 : CF::BN;
  GemmBatch b{};
  int tiles = 0;
  auto flush = [&]() {
    if (b.n == 0) return;
    for (int k = b.n; k < kMaxBatch; ++k) b.start[k] = tiles;
    if (lat)
      hipLaunchKernelGGL(gemm_lat_batch_f64, dim3((unsigned)tiles), dim3(256), 0, s, b);
    else if (dt == DType::F64)
      hipLaunchKernelGGL((gemm_batch_kernel<double, CF>), dim3((unsigned)tiles), dim3(CF::NT), 0, s, b);
    else
      hipLaunchKernelGGL((gemm_batch_kernel<float, CF>), dim3((unsigned)tiles), dim3(CF::NT), 0, s, b);
    b = GemmBatch{};
    tiles = 0;
  };
  for (int e = 0; e < n; ++e) {
    const GemmDesc& g = d[e];
    if (g.M <= 0 || g.N <= 0) continue;
    GemmArgs& a = b.a[b.n];
    a = GemmArgs{};
    a.M = g.M; a.N = g.N; a.K = g.K; a.A = g.A; a.lda = g.lda; a.B = g.B; a.ldb = g.ldb; a.C = g.C;
    a.ldc = g.ldc;
    fill_extra(a, &g.ex);
    if (g.op == GemmOp::Store) {  // every input column masked: C enters as 0 and is never read
      a.zc0 = 0;
      a.zc1 = g.N;
    }
    a.tiles_m = (int)((g.M + TBM - 1) / TBM);
    a.tiles_n = (int)((g.N + TBN - 1) / TBN);
    b.start[b.n++] = tiles;
    tiles += a.tiles_m * a.tiles_n;
    if (b.n == kMaxBatch) flush();
  }
  flush();
}

int residual_nparts(int64_t N) { return (int)(((N + CfgBig::BN - 1) / CfgBig::BN) * CfgBig::WN); }

void residual_partial(DType dt, int64_t M, int64_t N, int64_t K, const void* A, int64_t lda,
                      const void* B, int64_t ldb, int64_t n_real, int64_t blk_m, int64_t p,
                      int64_t k, double* partial, hipStream_t s) {
  if (M <= 0 || N <= 0) return;
  GemmArgs a{};
  a.M = M; a.N = N; a.K = K; a.A = A; a.lda = lda; a.B = B; a.ldb = ldb; a.C = nullptr; a.ldc = 0;
  fill_extra(a, nullptr);
  a.n_real = n_real; a.blk_m = blk_m; a.p = p; a.k = k; a.partial = partial;
  a.nparts = residual_nparts(N);
  if (dt == DType::F64)
    launch<double, 0, MODE_RESID>(a, s);
  else
    launch<float, 0, MODE_RESID>(a, s);
}

}  // namespace kern
}  // namespace gj
