// Wave-level (64-lane) register exchanges shared by the block-inverse kernels (gfx950).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace gj {
namespace kern {

// 64-bit DPP move: two 32-bit v_mov_b32_dpp with the same control.
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

// Wave-wide max of a double, result in every lane, no LDS: DPP quad/row permutes inside each
// 16-lane row, then v_permlane16_swap / v_permlane32_swap (gfx950) across rows.  Exact (fmax
// returns one of its operands), so the result can be compared for equality with the inputs.
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

// Wave-wide max of a uint32 (DPP inside rows, permlane swaps across rows), result in every lane.
__device__ __forceinline__ uint32_t umax32(uint32_t a, uint32_t b) { return a > b ? a : b; }
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
  v = umax32(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, true));
  v = umax32(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, true));
  v = umax32(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, true));
  v = umax32(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, true));
  {
    const auto p = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    v = umax32(p[0], p[1]);
  }
  {
    const auto p = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    v = umax32(p[0], p[1]);
  }
  return v;
}

// Exact partial-pivot choice over 64 x RPL rows (row = lane + 64 s) on 64-bit magnitude keys:
// the largest |value|, the LOWEST row among equal magnitudes (the reference's strict '>' scan,
// main.cpp:756-763).  key[s] = bits of |value| (non-negative doubles order like their bit
// patterns), 0 for rows that may not be chosen.  Fast path: a 32-bit max of the high words
// (exponent + 20 mantissa bits); only when two rows tie there is the low word compared.  Returns
// the row (wave-uniform); *none = every key is 0 (nothing to choose, or only zeros: singular).
template <int RPL>
__device__ __forceinline__ int wave_pivot_row_u64(const uint64_t (&key)[RPL], bool& none) {
  uint32_t mh = 0;
#pragma unroll
  for (int s = 0; s < RPL; ++s) mh = umax32(mh, (uint32_t)(key[s] >> 32));
  mh = wave_max_u32(mh);
  uint64_t bal[RPL];
  int cnt = 0;
#pragma unroll
  for (int s = 0; s < RPL; ++s) {
    bal[s] = __builtin_amdgcn_ballot_w64((uint32_t)(key[s] >> 32) == mh);
    cnt += __builtin_popcountll(bal[s]);
  }
  if (cnt > 1) {  // tie in the high word (or all zero): compare the low words of the tied rows
    uint32_t ml = 0;
#pragma unroll
    for (int s = 0; s < RPL; ++s) ml = umax32(ml, (uint32_t)(key[s] >> 32) == mh ? (uint32_t)key[s] : 0u);
    ml = wave_max_u32(ml);
#pragma unroll
    for (int s = 0; s < RPL; ++s)
      bal[s] = __builtin_amdgcn_ballot_w64((uint32_t)(key[s] >> 32) == mh && (uint32_t)key[s] == ml);
    none = (mh == 0 && ml == 0);
  } else {
    none = false;
  }
#pragma unroll
  for (int s = 0; s < RPL; ++s)
    if (bal[s]) return 64 * s + (int)__builtin_ctzll(bal[s]);
  return 0;
}

// Uniform-lane read of a 32/64-bit value into scalar registers.
template <typename T>
__device__ __forceinline__ T readlane_t(T v, int lane) {
  if constexpr (sizeof(T) == 8) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, lane);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), lane);
    return __builtin_bit_cast(T, ((uint64_t)hi << 32) | lo);
  } else {
    return __builtin_bit_cast(T, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), lane));
  }
}

// Exact partial-pivot choice over 64 x RPL candidate rows (row = lane + 64 s): the largest
// magnitude, the LOWEST row among equal magnitudes — the reference's strict '>' scan
// (main.cpp:756-763).  a[s] >= 0 is the candidate's |value|, -1 for rows that may not be chosen
// (already pivots, padding, NaN).  Returns the row (wave-uniform) and the max magnitude.
template <int RPL>
__device__ __forceinline__ int wave_pivot_row(const double (&a)[RPL], double& mx_out) {
  double mx = a[0];
#pragma unroll
  for (int s = 1; s < RPL; ++s) mx = fmax(mx, a[s]);
  mx = wave_max_f64(mx);
  mx_out = mx;
#pragma unroll
  for (int s = 0; s < RPL; ++s) {
    const uint64_t bal = __builtin_amdgcn_ballot_w64(a[s] == mx);
    if (bal) return 64 * s + (int)__builtin_ctzll(bal);
  }
  return 0;  // unreachable: mx is one of the a[s]
}

// 1/x: v_rcp_f64 + two Newton steps for doubles (the IEEE division is a 10-op dependent chain on
// the pivot path), plain division for floats.
template <typename T>
__device__ __forceinline__ T fast_recip(T x) {
  if constexpr (sizeof(T) == 8) {
    T inv = __builtin_amdgcn_rcp(x);
    inv = __builtin_fma(inv, __builtin_fma(-x, inv, T(1)), inv);
    inv = __builtin_fma(inv, __builtin_fma(-x, inv, T(1)), inv);
    return inv;
  } else {
    return T(1) / x;
  }
}

// The candidate of this workgroup when the launch covers only the LIVE candidates (grid = this
// rank's count of local block rows that have not served as a pivot row, Device::block_inverse
// nlive): the blockIdx.x-th local block b < nblk with used[b p + k] == 0, or -1 past the last.
// Every wave computes it (uniform, no barrier); the used flags are read 256 at a time so the
// loads of a pass are in flight together (one pass for the 256 blocks of N = 32768 at p = 1).
// Reference: only rows >= t are candidates (main.cpp:1028-1039); a dispatched dead workgroup
// would hold a whole CU's LDS and wave slots until it exits.
__device__ __forceinline__ int live_block(const int32_t* __restrict__ used, int nblk, int64_t p, int64_t k) {
  const int want = (int)blockIdx.x;
  const int lane = (int)(threadIdx.x & 63);
  int base = 0;
  for (int b0 = 0; b0 < nblk; b0 += 256) {
    bool lv[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int b = b0 + 64 * s + lane;
      lv[s] = b < nblk && used[(int64_t)b * p + k] == 0;
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const uint64_t bal = __ballot(lv[s]);
      const int cnt = __popcll(bal);
      if (want < base + cnt) {
        const int below = __popcll(bal & ((1ull << lane) - 1ull));
        const uint64_t hit = __ballot(lv[s] && below == want - base);
        return b0 + 64 * s + __ffsll((unsigned long long)hit) - 1;
      }
      base += cnt;
    }
  }
  return -1;
}

}  // namespace kern
}  // namespace gj
