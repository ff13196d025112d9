// Device side of the pivot selection (gfx950): the one-wave local argmin, the book-keeping of the
// winner, and the tail that runs both inside the candidate-inverse launch (PivotSelectArgs).
// Reference: the local candidate scan main.cpp:1039-1066, pivot_op main.cpp:729-744.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "gj/pivot.hpp"

namespace gj {
namespace kern {

// Shuffle-tree argmin of one record per lane (every lane returns the winner).
__device__ inline PivotRec pivot_wave_best(PivotRec best, int32_t p) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    PivotRec o;
    o.score = __shfl_xor(best.score, off, 64);
    o.logical = __shfl_xor(best.logical, off, 64);
    o.phys = __shfl_xor(best.phys, off, 64);
    o.valid = __shfl_xor(best.valid, off, 64);
    o.pad_ = 0;
    if (pivot_better(o, best, p)) best = o;
  }
  return best;
}

// One wave: each lane scans every 64th candidate, then a 6-step shuffle tree (no LDS, no
// workgroup barrier).  pivot_better is a strict total order on valid records (distinct logical
// rows), so the tree shape cannot change the winner.
__device__ inline PivotRec pivot_local_wave(const double* scores, const int32_t* valid, const int32_t* used,
                                            const int32_t* pos, int64_t nblk, int64_t p, int64_t k) {
  const int lane = (int)(threadIdx.x & 63);
  PivotRec best = pivot_invalid();
  for (int64_t b = lane; b < nblk; b += 64) {
    const int64_t g = b * p + k;
    if (used[g] || !valid[b]) continue;
    PivotRec c;
    c.score = scores[b];
    c.logical = pos[g];
    c.phys = (int32_t)g;
    c.valid = 1;
    c.pad_ = 0;
    if (pivot_better(c, best, (int32_t)p)) best = c;
  }
  return pivot_wave_best(best, (int32_t)p);
}

// Every record of one all-gather (one per rank): lane q holds record q, then the same tree.  All
// loads are issued at once; the former one-thread loop waited for each record in turn.
__device__ inline PivotRec pivot_gathered_wave(const PivotRec* recs, int32_t p) {
  PivotRec best = pivot_invalid();
  for (int32_t q = (int32_t)(threadIdx.x & 63); q < p; q += 64) {
    const PivotRec c = recs[q];
    if (pivot_better(c, best, p)) best = c;
  }
  return pivot_wave_best(best, p);
}

// The host mirror lives in coherent pinned memory (hipHostMallocCoherent: not cached in L2).
// Default publication: every field as a relaxed SYSTEM-scope atomic store (written through, no
// L2 involvement), a wait for their completion, then `step` the same way -- the host polls `step`
// and then reads the rest.  A system-scope fence (sysfence = 1, GJ_HOST_FENCE=1) also writes back
// every dirty L2 line of this XCD -- the trailing update's C tiles -- and cost the p > 1 chain's
// pivot_global launch ~15 us per step (profiles/host_fence_r5.md).
template <typename V>
__device__ inline void sys_store(V* p, V v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Winner of the gathered records -> book-keeping, *out, and the host mirror (one thread).
__device__ inline void pivot_finish(PivotRec best, int32_t p, int32_t t, int32_t* pos, int32_t* phys_at,
                                    int32_t* used, int32_t* seq, PivotResult* out, PivotResult* host_out,
                                    int sysfence) {
  PivotResult r;
  r.step = t;
  r.pad_ = 0;
  if (best.valid) {
    r.found = 1;
    r.phys = best.phys;
    r.owner = best.phys % p;
    r.logical = best.logical;
    r.score = best.score;
    pivot_commit(t, best.phys, pos, phys_at, used, seq);
  } else {
    seq[t] = -1;  // the step's owner-predicated launches (enqueued ahead) stay no-ops on every rank
    r.found = 0;
    r.phys = -1;
    r.owner = -1;
    r.logical = -1;
    r.score = 0.0;
  }
  *out = r;
  if (host_out && !sysfence) {
    sys_store(&host_out->found, r.found);
    sys_store(&host_out->phys, r.phys);
    sys_store(&host_out->owner, r.owner);
    sys_store(&host_out->logical, r.logical);
    sys_store(reinterpret_cast<long long*>(&host_out->score), __double_as_longlong(r.score));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the fields are written before `step`
    sys_store(&host_out->step, r.step);
  } else if (host_out) {  // the host polls `step`: every other field first, then a system-scope fence
    volatile PivotResult* h = host_out;
    h->found = r.found;
    h->phys = r.phys;
    h->owner = r.owner;
    h->logical = r.logical;
    h->score = r.score;
    __threadfence_system();
    h->step = r.step;
    __threadfence_system();
  }
}

// Called by exactly ONE whole wave of every workgroup of a candidate-inverse launch, after its
// lane 0 wrote scores[b] / valid[b].  Release fence + counter; the workgroup that brings the count
// to gridDim.x sees every record (acquire fence) and runs the selection, then re-arms the counter.
__device__ inline void select_tail(const PivotSelectArgs& a, const double* scores, const int32_t* valid,
                                   const int32_t* used, int64_t nblk, int64_t p, int64_t k) {
  if (a.done == nullptr) return;
  const int lane = (int)(threadIdx.x & 63);
  __threadfence();
  int32_t old = 0;
  if (lane == 0) old = atomicAdd(a.done, 1);
  old = __shfl(old, 0, 64);
  if (old != (int32_t)gridDim.x - 1) return;
  __threadfence();
  const PivotRec best = pivot_local_wave(scores, valid, used, a.pos, nblk, p, k);
  if (lane != 0) return;
  *a.rec = best;
  if (a.single) pivot_finish(best, 1, a.t, a.pos_w, a.phys_at, a.used_w, a.seq, a.out, a.host_out, a.sysfence);
  *a.done = 0;
}

}  // namespace kern
}  // namespace gj
