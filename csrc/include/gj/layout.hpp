// Block-row-cyclic data layout (64-bit everywhere).
//
// Parity with the reference's layout math:
//   num_block_rows  main.cpp:124-127   Nr = ceil(n/m)
//   rows_p_process  main.cpp:95-116    block rows owned by rank k
//   find_sender     main.cpp:521-532   owner of the last block row = (Nr-1) mod p
//   local_to_global main.cpp:118-123   local row i -> ((i/m)*p + k)*m + i%m
// The reference keeps these in `int` and overflows once a rank owns >= 2^31 elements
// (main.cpp:366); here every size is int64_t.
//
// MI355X design choice: the matrix is padded to npad = Nr*m with A' = diag(A, I) so every kernel
// sees whole m x m blocks.  The padded last block row is singular in every block
// column < Nr-1, which reproduces the reference's "exclude the short last block row from the pivot
// search until the last step" rule (main.cpp:967-970, :1031-1032) without special cases.
#pragma once

#include "gj/common.hpp"

namespace gj {

GJ_HD inline int64_t num_block_rows(int64_t n, int64_t m) { return (n + m - 1) / m; }

GJ_HD inline int64_t rows_owned(int64_t Nr, int64_t p, int64_t k) {
  return Nr / p + (k < Nr % p ? 1 : 0);
}

GJ_HD inline int64_t last_owner(int64_t Nr, int64_t p) { return (Nr - 1) % p; }

struct Layout {
  int64_t n = 0;       // matrix order
  int64_t m = 0;       // block size
  int64_t p = 1;       // number of ranks
  int64_t k = 0;       // this rank
  int64_t Nr = 0;      // block rows
  int64_t npad = 0;    // padded order Nr*m (leading dimension of every panel)
  int64_t l_h = 0;     // height of the last (possibly short) block row
  int64_t nblk = 0;    // block rows owned by this rank
  int64_t max_nblk = 0;  // max over ranks (= ceil(Nr/p))
  int64_t rows = 0;    // scalar rows owned by this rank (nblk*m, padded)

  static Layout make(int64_t n, int64_t m, int64_t p, int64_t k) {
    Layout L;
    L.n = n;
    L.m = m;
    L.p = p;
    L.k = k;
    L.Nr = num_block_rows(n, m);
    L.npad = L.Nr * m;
    L.l_h = n - (L.Nr - 1) * m;
    L.nblk = rows_owned(L.Nr, p, k);
    L.max_nblk = (L.Nr + p - 1) / p;
    L.rows = L.nblk * m;
    return L;
  }

  GJ_HD int64_t owner(int64_t I) const { return I % p; }
  GJ_HD int64_t local_block(int64_t I) const { return I / p; }
  GJ_HD int64_t global_block(int64_t local_b) const { return local_b * p + k; }
  GJ_HD int64_t global_row(int64_t local_row) const {
    return ((local_row / m) * p + k) * m + local_row % m;
  }
};

}  // namespace gj
