// Matrix generators shared by the host and device executors (bitwise identical on both).
//
// Reference: f(i,j) = |i-j| (default) or 1/(i+j+1) under -DHILBERT, f_i = identity
// (main.cpp:47-64).  `random` is a counter-based (stateless) uniform [-1, 1) generator so any rank
// can produce any element without communication — the synthetic dense system of the benchmark.
#pragma once

#include <cmath>

#include "gj/common.hpp"
#include "gj/device.hpp"

namespace gj {

GJ_HD inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// Term of 32-bit word `w` at word index `idx` of a hashed buffer (Device::hash_rows): the hash is
// the wrapping sum of the terms, so it is independent of the order the words are visited in.
GJ_HD inline uint64_t hash_term(uint32_t w, uint64_t idx) {
  return splitmix64(((uint64_t)w << 32) ^ (idx * 0xD1B54A32D192ED03ull) ^ 0x5851F42D4C957F2Dull);
}

// Element (i, j) of the padded matrix A' = diag(A, I) (i, j < npad).
GJ_HD inline double gen_value(int kind, uint64_t seed, int64_t n, int64_t i, int64_t j) {
  if (i >= n || j >= n) return (i == j) ? 1.0 : 0.0;
  switch (kind) {
    case 0: {  // AbsDiff
      const int64_t d = i - j;
      return (double)(d < 0 ? -d : d);
    }
    case 1:  // Hilbert
      return 1.0 / (double)(i + j + 1);
    case 2:  // Identity
      return (i == j) ? 1.0 : 0.0;
    case 3:    // Random uniform [-1, 1)
    case 5: {  // RandomShifted: + sqrt(n) on the diagonal
      const uint64_t h = splitmix64(seed * 0x2545F4914F6CDD1Dull ^ ((uint64_t)i << 32) ^ (uint64_t)j);
      const double u = (double)(h >> 11) * (2.0 / 9007199254740992.0) - 1.0;
      return (kind == 5 && i == j) ? u + sqrt((double)n) : u;
    }
    default:  // Zero
      return 0.0;
  }
}

}  // namespace gj
