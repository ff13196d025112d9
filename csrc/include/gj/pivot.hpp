// Pivot record and the deterministic global pivot rule.
//
// Reference: struct PivotMin (main.cpp:35-42) reduced with the non-commutative user op
// pivot_op/pivot_func (main.cpp:729-744, registered at :1023-1024, used at :1074).  RCCL has no
// user-defined reductions, so every rank all-gathers the p local records (32 B each) and applies
// `pivot_better` in the same order -> identical result on every GPU without a second round trip.
//
// Selection rule (SURVEY.md §3.4, §4.3.4 [measured on the reference]):
//   minimise ||inv(candidate)||_inf over non-singular candidates;
//   exact ties -> the larger rank, then the smaller local row,
// where rank / local row refer to the *logical* block-row position (the reference physically swaps
// block rows, main.cpp:1100-1131; this framework does not move rows but tracks the logical position
// of every physical block row, so the tie rule is reproduced exactly).
#pragma once

#include <cmath>

#include "gj/common.hpp"

namespace gj {

struct alignas(16) PivotRec {
  double score;      // ||inv(block)||_inf
  int32_t logical;   // logical block-row position of the candidate
  int32_t phys;      // physical (storage) global block row
  int32_t valid;     // non-singular (reference: non_sing)
  int32_t pad_;
};
static_assert(sizeof(PivotRec) == 32, "PivotRec must be 32 bytes");

// Result of the global selection, mirrored to pinned host memory every step.
struct alignas(16) PivotResult {
  int32_t found;     // 0 => "singular matrix"
  int32_t phys;      // chosen physical global block row s_t
  int32_t owner;     // rank that stores s_t (= s_t mod p)
  int32_t logical;   // logical position the row had before the swap
  double score;
  int32_t step;
  int32_t pad_;
};
static_assert(sizeof(PivotResult) == 32, "PivotResult must be 32 bytes");

// true iff candidate a is strictly preferred over b.
GJ_HD inline bool pivot_better(const PivotRec& a, const PivotRec& b, int32_t p) {
  if (!a.valid) return false;
  if (!b.valid) return true;
  if (a.score != b.score) return a.score < b.score;
  const int32_t ra = a.logical % p, rb = b.logical % p;
  if (ra != rb) return ra > rb;
  return (a.logical / p) < (b.logical / p);
}

GJ_HD inline PivotRec pivot_invalid() {
  PivotRec r;
  r.score = 0.0;
  r.logical = -1;
  r.phys = -1;
  r.valid = 0;
  r.pad_ = 0;
  return r;
}

// Book-keeping after step t selected physical row s (identical on every rank):
// the reference swaps the contents of logical positions t and pos[s].
//   pos[phys]     : logical position of a physical block row
//   phys_at[L]    : physical block row at logical position L
//   used[phys]    : already served as a pivot row
//   seq[t]        : pivot physical row of step t
GJ_HD inline void pivot_commit(int32_t t, int32_t s, int32_t* pos, int32_t* phys_at, int32_t* used,
                               int32_t* seq) {
  const int32_t q = phys_at[t];
  const int32_t ls = pos[s];
  pos[q] = ls;
  phys_at[ls] = q;
  pos[s] = t;
  phys_at[t] = s;
  used[s] = 1;
  seq[t] = s;
}

// Pivot selection fused into the candidate-inverse launch (Device::block_inverse_select): the
// batch's last workgroup to finish (counted on *done, which it resets to 0) runs the local argmin
// (p > 1: -> *rec, the record the all-gather sends) or, with one rank, the whole selection and
// book-keeping (-> *rec, *out and the pinned host mirror), so the pivot chain loses a launch.
struct PivotSelectArgs {
  int32_t* done = nullptr;   // device counter, 0 between launches
  int32_t t = 0;             // step
  const int32_t* pos = nullptr;
  int32_t* pos_w = nullptr;  // (p == 1: book-keeping arrays, written)
  int32_t* phys_at = nullptr;
  int32_t* used_w = nullptr;
  int32_t* seq = nullptr;
  PivotRec* rec = nullptr;
  PivotResult* out = nullptr;       // p == 1 only
  PivotResult* host_out = nullptr;  // p == 1 only
  int32_t single = 0;               // 1: p == 1, the full selection
  int32_t sysfence = 0;             // host_out publication: 1 = system-scope fences (set by the launcher)
};

}  // namespace gj
