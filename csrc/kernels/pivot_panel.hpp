// Pivot-wave panel factorisation shared by the candidate-block inverse kernels (gfx950):
// blockinv_mfma.hip (m <= 128, block in registers) and blockinv_big.hip (m <= 256, block in an
// L2-resident fragment image).  One wave factors a 16-column panel of 64 x RPL rows in registers.
#pragma once

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <utility>

#include "wave_ops.hpp"

namespace gj {
namespace kern {

// ---- pivot wave, software-pipelined panel factorisation (16 steps, rows lane + 64 s) ----------
// Step j's chain: argmax of column j -> pivot value (v_readlane) -> 1/pivot -> multipliers u ->
// column j+1 updated.  The rest of step j (v_readlane of the pivot row, the rank-1 update of the
// other 14 columns) is independent of that chain until step j+1 reads the pivot row, so it is
// issued in the latency gaps: the pivot-row reads between the reciprocal's dependent ops, the
// update FMAs between the stages of step j+1's wave-wide max (the order is pinned with
// sched_barrier: a single in-order wave only hides latency with independent work placed
// between the dependent instructions).
#define GJ_SB() __builtin_amdgcn_sched_barrier(0)
// GJ_PP_PIN: pin every pending-update FMA result and every wave-max stage (empty volatile asm on the
// register): IR-level code motion otherwise sinks the FMAs below the whole argmax, which then runs
// with an s_nop in each DPP hazard slot instead of the interleaved update
#ifndef GJ_PP_PIN
#define GJ_PP_PIN 1
#endif
template <typename X>
__device__ __forceinline__ void pp_pin(X& x) {
  if constexpr (GJ_PP_PIN) asm volatile("" : "+v"(x));
}

#ifdef GJ_BI_PROBE_STEPS  // per-step shader-clock stamps of workgroup 0 (bench/blockinv_mfma_probe.hip)
extern __device__ unsigned long long g_bim_probe[1024];
#define GJ_PP_PROBE(slot)                                                                     \
  do {                                                                                        \
    if (blockIdx.x == 0 && lane == 0) g_bim_probe[(slot)] = __builtin_amdgcn_s_memtime();     \
  } while (0)
#else
#define GJ_PP_PROBE(slot) \
  do {                    \
  } while (0)
#endif

// Column kk of the pending update of step PJ at list position e: column PJ+2 first, then the
// others in order (PJ, PJ+1 excluded); -1 past the end.
__host__ __device__ constexpr int pend_col(int pj, int e) {
  int cnt = 0;
  if (pj + 2 < 16) {
    if (e == 0) return pj + 2;
    cnt = 1;
  }
  for (int kk = 0; kk < 16; ++kk) {
    if (kk == pj || kk == pj + 1 || kk == pj + 2) continue;
    if (cnt == e) return kk;
    ++cnt;
  }
  return -1;
}
// Position e of the pivot-row read list of step J (every column but J and J+1); -1 past the end.
__host__ __device__ constexpr int read_col(int j, int e) {
  int cnt = 0;
  for (int kk = 0; kk < 16; ++kk) {
    if (kk == j || kk == j + 1) continue;
    if (cnt == e) return kk;
    ++cnt;
  }
  return -1;
}

// Pivot choice = the reference's scan exactly (main.cpp:756-763, with its physical row swaps): the
// largest |value| (64-bit magnitude keys), and among equal magnitudes the row at the lowest CURRENT
// position, where positions follow the swaps the reference would have made (step k swaps the pivot
// row into position k).  pos[s] = current position of row lane + 64 s; kept across panels.
template <typename T, int RPL>
struct PivotPanel {
  T (&W)[RPL][16];
  uint64_t (&keymask)[RPL];
  int (&pos)[RPL];
  int (&rr)[16];
  bool& sing;
  const int lane, c0, m;
  const double thresh;
  T up[RPL];  // multipliers of the previous step (its update is still pending)
  T rvp[16];  // the previous step's pivot row (wave-uniform)
  T rv[16];   // this step's pivot row
  // singular-step flag, OR-ed per step and pinned in a VGPR: left to the compiler, the 16 steps'
  // comparisons were sunk to the end of the panel, every step's pivot value kept live until then
  // (SGPR spills to VGPR lanes: ~100 v_readlane / v_writelane per panel)
  uint32_t singv = 0;

  __device__ __forceinline__ PivotPanel(T (&W_)[RPL][16], uint64_t (&km)[RPL], int (&pos_)[RPL], int (&rr_)[16],
                                        bool& sg, int lane_, int c0_, int m_, double th)
      : W(W_), keymask(km), pos(pos_), rr(rr_), sing(sg), lane(lane_), c0(c0_), m(m_), thresh(th) {}

  template <int PJ, int COL>
  __device__ __forceinline__ void upd() {
    if constexpr (COL >= 0) {
#pragma unroll
      for (int s = 0; s < RPL; ++s) {
        W[s][COL] = __builtin_fma(up[s], rvp[COL], W[s][COL]);
        pp_pin(W[s][COL]);
      }
    }
  }
  // chunk C (0..6) of the pending update of step PJ: two columns; chunk 6 also stores column PJ
  template <int PJ, int C>
  __device__ __forceinline__ void work() {
    if constexpr (PJ >= 0) {
      upd<PJ, pend_col(PJ, 2 * C)>();
      upd<PJ, pend_col(PJ, 2 * C + 1)>();
      if constexpr (C == 6) {
#pragma unroll
        for (int s = 0; s < RPL; ++s) W[s][PJ] = up[s];
      }
    }
  }
  template <int S, int J, int E0, int E1>
  __device__ __forceinline__ void reads(int rl) {
    if constexpr (E0 < E1 && read_col(J, E0) >= 0) {
      rv[read_col(J, E0)] = readlane_t(W[S][read_col(J, E0)], rl);
      reads<S, J, E0 + 1, E1>(rl);
    }
  }
  template <int S, int J>
  __device__ __forceinline__ void chain(int rl, T& piv, T& nx, T& inv) {
    piv = readlane_t(W[S][J], rl);
    if constexpr (J + 1 < 16) nx = readlane_t(W[S][J + 1], rl);
    else nx = T(0);
    if constexpr (sizeof(T) == 8) {
      inv = __builtin_amdgcn_rcp(piv);
      GJ_SB();
      reads<S, J, 0, 4>(rl);
      GJ_SB();
      T t = __builtin_fma(-piv, inv, T(1));
      GJ_SB();
      reads<S, J, 4, 7>(rl);
      GJ_SB();
      inv = __builtin_fma(inv, t, inv);
      GJ_SB();
      reads<S, J, 7, 10>(rl);
      GJ_SB();
      t = __builtin_fma(-piv, inv, T(1));
      GJ_SB();
      reads<S, J, 10, 12>(rl);
      GJ_SB();
      inv = __builtin_fma(inv, t, inv);
      GJ_SB();
      reads<S, J, 12, 15>(rl);  // (15 columns at J = 15)
    } else {
      inv = T(1) / piv;
      reads<S, J, 0, 15>(rl);
    }
  }

  // chain<S, J> for the row slot S = rs of the pivot row (wave-uniform branch)
  template <int S, int J>
  __device__ __forceinline__ void chain_sel(int rs, int rl, T& piv, T& nx, T& inv) {
    if constexpr (S + 1 < RPL) {
      if (rs != S) {
        chain_sel<S + 1, J>(rs, rl, piv, nx, inv);
        return;
      }
    }
    chain<S, J>(rl, piv, nx, inv);
  }

  template <int J>
  __device__ __forceinline__ void step() {
    constexpr int PJ = J - 1;
    GJ_PP_PROBE(9 + 24 * (c0 / 16) + J);
    // argmax of column J (exact: see wave_pivot_row_u64), step J-1's update in its gaps
    uint64_t key[RPL];
    uint32_t v = 0;
#pragma unroll
    for (int s = 0; s < RPL; ++s) {
      key[s] = __builtin_bit_cast(uint64_t, (double)W[s][J]) & keymask[s];
      v = umax32(v, (uint32_t)(key[s] >> 32));
    }
    work<PJ, 0>();
    v = umax32(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, true));
    pp_pin(v);
    GJ_SB();
    work<PJ, 1>();
    v = umax32(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, true));
    pp_pin(v);
    GJ_SB();
    work<PJ, 2>();
    v = umax32(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, true));
    pp_pin(v);
    GJ_SB();
    work<PJ, 3>();
    v = umax32(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, true));
    pp_pin(v);
    GJ_SB();
    work<PJ, 4>();
    {
      const auto p = __builtin_amdgcn_permlane16_swap(v, v, false, false);
      v = umax32(p[0], p[1]);
      pp_pin(v);
    }
    GJ_SB();
    work<PJ, 5>();
    {
      const auto p = __builtin_amdgcn_permlane32_swap(v, v, false, false);
      v = umax32(p[0], p[1]);
    }
    GJ_SB();
    work<PJ, 6>();
    const uint32_t mh = v;
    uint64_t bal[RPL];
    int cnt = 0;
#pragma unroll
    for (int s = 0; s < RPL; ++s) {
      bal[s] = __builtin_amdgcn_ballot_w64((uint32_t)(key[s] >> 32) == mh);
      cnt += __builtin_popcountll(bal[s]);
    }
    bool none = false;
    if (cnt > 1) {  // tie in the high word (or all zero): compare the low words of the tied rows
      uint32_t ml = 0;
#pragma unroll
      for (int s = 0; s < RPL; ++s) ml = umax32(ml, (uint32_t)(key[s] >> 32) == mh ? (uint32_t)key[s] : 0u);
      ml = wave_max_u32(ml);
#pragma unroll
      for (int s = 0; s < RPL; ++s)
        bal[s] = __builtin_amdgcn_ballot_w64((uint32_t)(key[s] >> 32) == mh && (uint32_t)key[s] == ml);
      none = (mh == 0 && ml == 0);
    }
    int r = 0;
    if (cnt > 1 && !none) {  // exact magnitude tie (rare): the lowest current position wins
      uint32_t pm = 0xFFFFFFFFu;
#pragma unroll
      for (int s = 0; s < RPL; ++s) pm = ((bal[s] >> lane) & 1) && (uint32_t)pos[s] < pm ? (uint32_t)pos[s] : pm;
      pm = ~wave_max_u32(~pm);
#pragma unroll
      for (int s = 0; s < RPL; ++s) bal[s] = __builtin_amdgcn_ballot_w64(((bal[s] >> lane) & 1) && (uint32_t)pos[s] == pm);
    }
    {
      bool f = false;
#pragma unroll
      for (int s = 0; s < RPL; ++s)
        if (!f && bal[s]) {
          r = 64 * s + (int)__builtin_ctzll(bal[s]);
          f = true;
        }
    }
    if (none) r = c0 + J;  // nothing left to choose (singular): any in-range row
    r = __builtin_amdgcn_readfirstlane(r);
    rr[J] = r;
    const int rl = r & 63, rs = r >> 6;
#pragma unroll
    for (int s = 0; s < RPL; ++s)
      if (lane + 64 * s == r) keymask[s] = 0ull;
    {  // the reference's swap of step c0 + J: the pivot row <-> the row at position c0 + J
      int pv = pos[0];
#pragma unroll
      for (int s = 1; s < RPL; ++s) pv = (rs == s) ? pos[s] : pv;
      const int pr = __builtin_amdgcn_readlane(pv, rl);
#pragma unroll
      for (int s = 0; s < RPL; ++s)
        pos[s] = (lane + 64 * s == r) ? c0 + J : (pos[s] == c0 + J ? pr : pos[s]);
    }
    // pivot value, next column's entry, reciprocal; the pivot-row reads in its gaps
    T piv, nx, inv;
    chain_sel<0, J>(rs, rl, piv, nx, inv);  // rs is wave-uniform
    singv |= ((c0 + J < m) && (none || !(fabs((double)piv) >= thresh))) ? 1u : 0u;
    asm volatile("" : "+v"(singv));
    T u[RPL];
#pragma unroll
    for (int s = 0; s < RPL; ++s) u[s] = (lane + 64 * s == r) ? inv - T(1) : -W[s][J] * inv;
    if constexpr (J + 1 < 16) {
#pragma unroll
      for (int s = 0; s < RPL; ++s) W[s][J + 1] = __builtin_fma(u[s], nx, W[s][J + 1]);
    }
#pragma unroll
    for (int s = 0; s < RPL; ++s) up[s] = u[s];
#pragma unroll
    for (int kk = 0; kk < 16; ++kk)
      if (kk != J && kk != J + 1) rvp[kk] = rv[kk];
  }

  template <int... J>
  __device__ __forceinline__ void run(std::integer_sequence<int, J...>) {
    (step<J>(), ...);
    sing = sing || (singv != 0);
    // the last step's update (no next argmax to hide it in)
#pragma unroll
    for (int c = 0; c < 15; ++c) {
#pragma unroll
      for (int s = 0; s < RPL; ++s) W[s][c] = __builtin_fma(up[s], rvp[c], W[s][c]);
    }
#pragma unroll
    for (int s = 0; s < RPL; ++s) W[s][15] = up[s];
  }
};

template <typename T, int RPL>
__device__ __forceinline__ void pivot_panel_il(T (&W)[RPL][16], uint64_t (&keymask)[RPL], int (&pos)[RPL], int lane,
                                               int c0, int m, double thresh, int (&rr)[16], bool& sing) {
  PivotPanel<T, RPL> pp(W, keymask, pos, rr, sing, lane, c0, m, thresh);
  pp.run(std::make_integer_sequence<int, 16>{});
}

}  // namespace kern
}  // namespace gj
