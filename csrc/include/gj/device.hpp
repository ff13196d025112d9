// Device abstraction used by the solver engine.
//
// Two implementations exist:
//   * HipDevice  (csrc/runtime/hip_device.hip)  — the product path: hand-written gfx950 kernels,
//     three HIP streams (MAIN/SIDE/COMM) with priorities, event-based ordering.
//   * HostDevice (csrc/runtime/host_device.cpp) — a plain C++ reference executor with identical
//     semantics.  It is only ever selected explicitly (`--device cpu`, CPU tests, the reference's
//     "512x512 single rank on CPU" plumbing config); a GPU run never falls back to it.
//
// Every op takes a stream role (S_MAIN/S_SIDE/S_COMM); the host device executes synchronously.
#pragma once

#include <memory>
#include <string>

#include "gj/common.hpp"
#include "gj/layout.hpp"
#include "gj/pivot.hpp"

namespace gj {

// Matrix generators (reference f / f_i, main.cpp:47-64, plus a seeded random dense generator for
// the synthetic benchmark system).
// RandomShifted: Random + sqrt(n) on the diagonal (well conditioned at any n: where fp32 solves
// and their refinement are meaningful, BASELINE.md "fp32").
enum class GenKind : int { AbsDiff = 0, Hilbert = 1, Identity = 2, Random = 3, Zero = 4, RandomShifted = 5 };

struct GenSpec {
  GenKind kind = GenKind::AbsDiff;
  uint64_t seed = 0;
};

// C (+)= A * B.  A is M x K and is stored either row-major (A[i*lda + k]) or "K-major"
// (At[k*lda + i], the layout the solver keeps its multiplier panel in).
enum class GemmOp : int { Acc = 0, Store = 1 };
enum class ALayout : int { RowMajor = 0, KMajor = 1 };

// Elimination extras of GemmOp::Acc: C enters as 0 in the columns [zc0, zc1) (the pivot block
// columns of the current panel) and in the row blocks [zr[i], zr[i] + zh) (its pivot rows).
struct GemmExtra {
  static constexpr int kMaxZeroRows = 8;  // = the deepest panel (SolveOptions::depth <= 8)
  int64_t zc0 = 0, zc1 = 0;
  int nzr = 0;
  int64_t zr[kMaxZeroRows] = {};
  int64_t zh = 0;
  // Few-tile GEMM on the panel-factorisation critical path: prefer small tiles (more workgroups,
  // shorter K loop per workgroup) over the throughput tiles of the trailing update.
  bool latency = false;
  // latency launch of >= 1024 rows: the LDS-DMA kernel (128 x 64 tiles, 4 per CU) instead of the
  // small tile -- the pivot chain's column updates when they run on reserved CUs (Engine::lat_wide_)
  bool lat_wide = false;
  // latency launch on CUs reserved for the chain: the register-fed small fp64 kernel (every operand
  // fragment loaded straight into registers, two 32-deep K chunks in flight; Engine::lat_reg_)
  bool lat_reg = false;
  // Also write the result transposed and negated, tneg[c*ldtneg + r] = -C[r][c], for the output
  // columns c < tneg_cols (0 = all): the K-major multiplier panel of the next pivot search, fused
  // into the column update that produces it (one launch fewer on the pivot chain).
  void* tneg = nullptr;
  int64_t ldtneg = 0;
  int64_t tneg_cols = 0;
  // Output columns [skip_c0, skip_c1) are neither read nor written (nor are those columns of B):
  // one launch for a chunk whose middle columns another stream updates (the trailing update around
  // the look-ahead columns).  GPU: whole tiles, so both bounds multiples of Device::skip_align().
  int64_t skip_c0 = 0, skip_c1 = 0;
  // Owner-predicated launch (the host-free pivot chain at p > 1): the GEMM does nothing unless this
  // rank owns the pivot g = *owner_phys (g % owner_p == owner_k) -- read on the device.
  const int32_t* owner_phys = nullptr;
  int64_t owner_p = 1, owner_k = 0;
  // Trailing-update residency: 5 LDS-DMA workgroups per CU instead of 4 (a 96-VGPR build).  Faster
  // when the pivot chain has CUs of its own (a CU reservation), slower when it must share them
  // (profiles/gemm_stall_r4.md).
  bool dense = false;
  // This launch's LDS-DMA build (stages * 10 + waves-per-SIMD bound: 23 | 25 | 33), 0 = by `dense`:
  // the owner's chunk-pass normalisations under a CU reservation (Engine::chunk_build_)
  int glds_build = 0;
  // This launch's LDS-DMA tile width (64 | 128), 0 = the device's hint (Device::set_gemm_tile_hint)
  int glds_tile = 0;
  // fp64 LDS-DMA kernel: C read (bit 0) / written (bit 1) with the non-temporal cache policy, for C
  // that nothing reads again soon (MAIN's trailing update: Engine::main_cnt_); -1 = GJ_GLDS_CNT / 0
  int c_nt = -1;
  // Row-block selection (the pivot-chain / deferred split of a panel's column updates, Engine):
  // only the row blocks b (height rsel_m, b < 64 kRselWords) whose bit b of rsel is set take part;
  // M counts the selected rows ((set bits) * rsel_m) and the i-th block of M is the i-th set bit.
  // Rows of A (K-major), C and tneg are addressed through the map; zero rows stay physical.
  // rsel_m = 0: off.  The GPU path needs the tile height to divide rsel_m (64 | rsel_m).
  // GemmOp::Acc reading its input from another array: C = C_in (+ masks) + A B, C_in with its own
  // leading dimension (the owner's pivot-row normalisation, X row -> temp, without a separate copy)
  const void* c_in = nullptr;
  int64_t ldc_in = 0;
  static constexpr int kRselWords = 8;
  uint64_t rsel[kRselWords] = {};
  int64_t rsel_m = 0;
  int64_t rsel_count() const {
    int64_t c = 0;
    for (int w = 0; w < kRselWords; ++w) c += __builtin_popcountll(rsel[w]);
    return c;
  }
  // physical row of selected row i (i < rsel_count() * rsel_m)
  int64_t rsel_row(int64_t i) const {
    int64_t bl = i / rsel_m;
    const int64_t off = i - bl * rsel_m;
    for (int w = 0; w < kRselWords; ++w) {
      uint64_t x = rsel[w];
      const int c = __builtin_popcountll(x);
      if (bl < c) {
        for (; bl > 0; --bl) x &= x - 1;
        return (64 * w + __builtin_ctzll(x)) * rsel_m + off;
      }
      bl -= c;
    }
    return -1;
  }
};

// Owner-side piece work fused into Device::owner_edits (all optional; w = 0 / eye = null: none):
// the pivot row's later panel columns moved out of X, dst[r*ldd + c] = X[(row0+r)*ldx + col0 + c],
// then zeroed in X (r < m, c < w; the next column updates need them as 0), and the m x m identity
// written at eye (ld ld_eye) -- the pivot's own block of the piece GEMM's B, so H_t lands in the
// piece without a separate copy (H I = H exactly).
struct PieceMove {
  void* dst = nullptr;
  int64_t ldd = 0;
  void* X = nullptr;
  int64_t ldx = 0;
  int64_t col0 = 0;
  int64_t w = 0;
  void* eye = nullptr;
  int64_t ld_eye = 0;
};

// One product of a batched small-GEMM launch (Device::gemm_batch): C (+)= A B, A K-major.
struct GemmDesc {
  GemmOp op = GemmOp::Acc;
  int64_t M = 0, N = 0, K = 0;
  const void* A = nullptr;
  int64_t lda = 0;
  const void* B = nullptr;
  int64_t ldb = 0;
  void* C = nullptr;
  int64_t ldc = 0;
  GemmExtra ex;
};

class Device {
 public:
  virtual ~Device() = default;
  virtual bool on_gpu() const = 0;
  virtual std::string describe() const = 0;
  virtual int device_index() const { return -1; }

  // ---- memory ----
  virtual void* alloc(size_t bytes) = 0;
  virtual void release(void* p) = 0;
  virtual void* alloc_pinned(size_t bytes) = 0;
  // Fine-grained (coherent) pinned host memory: kernels store into it and the host polls it.
  virtual void* alloc_pinned_coherent(size_t bytes) { return alloc_pinned(bytes); }
  virtual void release_pinned(void* p) = 0;
  virtual size_t free_memory() const = 0;
  virtual void memset0(void* p, size_t bytes, int s) = 0;
  virtual void memset2d(void* p, size_t pitch, size_t width_bytes, size_t height, int s) = 0;
  virtual void copy(void* dst, const void* src, size_t bytes, int s) = 0;
  virtual void copy2d(void* dst, size_t dpitch, const void* src, size_t spitch, size_t width_bytes,
                      size_t height, int s) = 0;

  // ---- ordering ----
  virtual int create_event(bool timing = false) = 0;
  virtual void record(int ev, int s) = 0;
  virtual void wait(int s, int ev) = 0;
  virtual void sync_event(int ev) = 0;
  virtual bool query_event(int ev) = 0;  // true once all work before the record has completed
  virtual void sync_stream(int s) = 0;
  virtual void sync_all() = 0;
  // Non-blocking: true once everything enqueued on stream s has completed (Comm::drain polls it so
  // that a host wait behind a collective can notice a dead peer).  Synchronous devices: always true.
  virtual bool stream_idle(int s) { sync_stream(s); return true; }
  virtual float event_ms(int ev_start, int ev_end) = 0;
  virtual void* native_stream(int s) = 0;  // hipStream_t (nullptr on host)
  // Cross-device ordering points (the asynchronous virtual-rank transport, AsyncLoopbackComm):
  // mark(s) enqueues a marker on stream s and returns a handle that completes when everything
  // enqueued on s before it has; wait_mark(s, h) makes stream s wait for a handle from ANY device
  // of the same kind in this process (HIP: an event, so the same GPU or peer GPUs; host: a fence).
  // A null handle means "already complete".  Devices that execute synchronously return null.
  virtual std::shared_ptr<void> mark(int s) { (void)s; return nullptr; }
  virtual void wait_mark(int s, const std::shared_ptr<void>& h) { (void)s; (void)h; }
  // Timing / scheduling probes: keep stream s busy for `us` microseconds on `nwg` workgroups
  // (nwg = 1: a pure delay, e.g. per-rank start jitter; more: the CU footprint of a transfer in the
  // single-GPU communication-cost model of ShadowComm).  No-op where it has no meaning.
  virtual void occupy(int s, int nwg, double us, int lds_bytes = 0) {
    (void)s; (void)nwg; (void)us; (void)lds_bytes;
  }
  // Zero `bytes` at p on stream s with `nwg` workgroups of an RCCL channel's footprint (the data a
  // synthetic peer "sends" in ShadowComm's cost model, written with the CU footprint of the
  // receiving channel kernels rather than a full-chip fill kernel).  Default: memset0.
  virtual void zero_channels(void* p, size_t bytes, int s, int nwg, int lds_bytes) {
    (void)nwg; (void)lds_bytes;
    memset0(p, bytes, s);
  }
  // Keep the MAIN (trailing-update) stream off `n` CUs so the latency-critical SIDE/COMM kernels
  // always find idle CUs (the first n bits of the CU mask; n = 32 is one CU per shader engine).
  // Returns the number of CUs actually reserved.  Call while the device is idle.
  virtual int reserve_cus(int n) { (void)n; return 0; }
  // alignment (columns) of GemmExtra::skip_c0 / skip_c1 this device honours
  virtual int64_t skip_align() const { return 1; }

  // ---- schedule-checking hooks (RaceCheckDevice, gj/race_check.hpp; no-ops elsewhere) ----
  // Where the caller is (read at every op for reports): its step counter and phase name.
  virtual void trace_context(const int64_t* step, const char* const* phase) { (void)step; (void)phase; }
  // Name of an allocation in reports.
  virtual void label(const void* p, const char* name) { (void)p; (void)name; }
  // The host thread reads / writes host-visible memory directly (pinned staging, polled records).
  virtual void host_access(const void* p, size_t bytes, bool write) { (void)p; (void)bytes; (void)write; }
  // The host observed the record at p that a device op published (pivot_global's host_out): it
  // now knows everything that op was ordered after.
  virtual void host_acquire(const void* p, size_t bytes) { (void)p; (void)bytes; }
  // Host-thread ordering across devices (LoopbackComm's rendezvous): a handle of everything this
  // device's host has observed, and joining a peer's handle into it.
  virtual std::shared_ptr<void> host_mark() { return nullptr; }
  virtual void host_wait_mark(const std::shared_ptr<void>& h) { (void)h; }

  // ---- kernels ----
  // X (layout.rows x npad, ld npad) := A' restricted to this rank's block rows.
  virtual void generate(DType dt, void* X, const Layout& L, GenSpec g, int s) = 0;
  // generate() and out[0] = row_abs_max() of the result (a device may fuse the two passes; the
  // HIP device does, one read of the matrix less)
  virtual void generate_norm(DType dt, void* X, const Layout& L, GenSpec g, double* out, int s) {
    generate(dt, X, L, g, s);
    row_abs_max(dt, X, L.npad, L, out, s);
  }
  // X[r][c] := src[r][c] (doubles, ld src_ld) for r < rows, c < cols (dtype conversion).
  virtual void upload_convert(DType dt, void* X, int64_t ldx, const double* src_dev, int64_t src_ld,
                              int64_t rows, int64_t cols, int s) = 0;
  // dst[r*ldd + c] := (double)X[r*ldx + c] for r < rows, c < cols (X of dtype dt, device memory).
  virtual void widen(DType dt, double* dst, int64_t ldd, const void* X, int64_t ldx, int64_t rows,
                     int64_t cols, int s) = 0;
  // Lt[c*ldl + r] = -X[r*ldx + col0 + c]  for r < rows, c < m   (multiplier panel, K-major).
  virtual void extract_neg_t(DType dt, void* Lt, int64_t ldl, const void* X, int64_t ldx,
                             int64_t rows, int64_t col0, int64_t m, int s) = 0;
  // A[i*ld + i] += alpha, i < nd.
  virtual void add_diag(DType dt, void* A, int64_t ld, int64_t nd, double alpha, int s) = 0;
  // For every local block row b with used[global(b)] == 0: W = -(Lt block b)^T = X[b, col-block],
  // compute inv(W) by Gauss-Jordan with partial pivoting (reference inverse_block, main.cpp:746-820),
  // write it transposed to inv_t[b*m*m + j*m + i] = inv(W)[i][j], its inf-norm to scores[b]
  // (block_norm, main.cpp:669-683), and valid[b] (0 when singular: |pivot| < thresh).
  // nlive = the number of local blocks with used == 0 (the caller knows every earlier pivot):
  // devices launch one workgroup per LIVE candidate only, so no used block is dispatched (its
  // workgroup would hold a whole CU's LDS / wave slots for nothing); scores / valid of used blocks
  // are then left as they were (every consumer skips used blocks).  nlive < 0: all nblk.
  virtual void block_inverse(DType dt, const void* Lt, int64_t ldl, void* inv_t, double* scores,
                             int32_t* valid, const int32_t* used, const Layout& L, double thresh, int64_t nlive,
                             int s) = 0;
  // block_inverse with the pivot selection run by the launch's last workgroup (PivotSelectArgs:
  // p > 1 the local argmin -> *sel.rec, like pivot_local; p == 1 the whole pivot_select_single).
  // Returns false, having enqueued nothing, where the device or the kernel family it would use
  // cannot fuse them; the caller then runs block_inverse and the selection as separate launches.
  virtual bool block_inverse_select(DType dt, const void* Lt, int64_t ldl, void* inv_t, double* scores,
                                    int32_t* valid, const int32_t* used, const Layout& L, double thresh, int64_t nlive,
                                    const PivotSelectArgs& sel, int s) {
    (void)dt; (void)Lt; (void)ldl; (void)inv_t; (void)scores; (void)valid; (void)used; (void)L;
    (void)thresh; (void)sel; (void)s;
    return false;
  }
  // Kernel family for the following block_inverse calls (-1 = the process default; 5 = the
  // co-resident form, which the engine picks where its pivot chain waits for whole CUs).  Devices
  // with a single implementation ignore it.
  virtual void set_block_inverse_hint(int variant) { (void)variant; }
  // Tile width of the fp64 LDS-DMA trailing-update kernel for launches that do not name one
  // (GemmExtra::glds_tile): 128 by default, 64 where CUs are reserved for the pivot chain (Engine)
  virtual void set_gemm_tile_hint(int bn) { (void)bn; }
  // Device scratch the candidate-inverse kernel family `variant` needs for layout L (bytes), and
  // its allocation ahead of the first block_inverse call.
  virtual size_t block_inverse_scratch_bytes(DType dt, const Layout& L, int variant) const {
    (void)dt; (void)L; (void)variant;
    return 0;
  }
  virtual void prepare_block_inverse(DType dt, const Layout& L, int variant) { (void)dt; (void)L; (void)variant; }
  // Partial pivoting (SolveOptions::pivot = Partial, `--pivot partial`).  Every local candidate
  // W_b (as in block_inverse) gets scores[b] = -max|W_b| and valid[b] = (max|W_b| >= thresh), so the
  // common argmin (pivot_local) picks this rank's largest-magnitude candidate; its block alone is
  // then copied out (gather_candidate: sel = K-major m x m, ld m; -I for an invalid record),
  // inverted by block_inverse on a one-block layout, and commit_candidate stores that inverse in
  // the candidate's slot of inv_t and clears rec->valid when the block is singular or, growth > 0,
  // when its growth estimate ||inv||_inf * max|W| (score1[0] * -rec->score) exceeds growth.
  virtual void candidate_maxabs(DType dt, const void* Lt, int64_t ldl, double* scores, int32_t* valid,
                                const int32_t* used, const Layout& L, double thresh, int s) = 0;
  virtual void gather_candidate(DType dt, void* sel, const void* Lt, int64_t ldl, const PivotRec* rec,
                                const Layout& L, int s) = 0;
  virtual void commit_candidate(DType dt, void* inv_t, const void* inv1, const int32_t* valid1, const double* score1, double growth, PivotRec* rec,
                                const Layout& L, int s) = 0;
  // Local argmin over this rank's candidates -> *out.
  virtual void pivot_local(const double* scores, const int32_t* valid, const int32_t* used,
                           const int32_t* pos, const Layout& L, PivotRec* out, int s) = 0;
  // Global selection over p records + book-keeping (pivot_commit) -> *out, and the same record to
  // host_out (pinned host memory the host polls: its `step` field is written last, after a
  // system-scope fence) when host_out != nullptr.
  virtual void pivot_global(const PivotRec* recs, int32_t p, int32_t t, int32_t* pos,
                            int32_t* phys_at, int32_t* used, int32_t* seq, PivotResult* out,
                            PivotResult* host_out, int s) = 0;
  // One rank (p == 1): pivot_local + pivot_global as one launch (the record all-gather is skipped
  // there, so the two were back to back on the pivot chain).  Default: the two calls.
  virtual void pivot_select_single(const double* scores, const int32_t* valid, const Layout& L,
                                   int32_t t, int32_t* pos, int32_t* phys_at, int32_t* used,
                                   int32_t* seq, PivotRec* rec, PivotResult* out,
                                   PivotResult* host_out, int s) {
    pivot_local(scores, valid, used, pos, L, rec, s);
    pivot_global(rec, 1, t, pos, phys_at, used, seq, out, host_out, s);
  }
  // Owner-side edits of a pivot step, fused (one launch).  The pivot is read on the device: g =
  // *phys (the step's entry of the pivot sequence, written by the selection), and the launch does
  // nothing unless g % p == k (this rank owns it), so the host can enqueue it before it has seen
  // the pivot.  For the pivot's local block row b = g / p (rows row0 = b m .. of the K-major
  // multiplier panel At, ld ldl): save the multipliers of the panel's earlier steps,
  // lrow[kk*m + c] = At[kk*ldl + row0 + c] for kk < j*m, set those rows of At to [0 .. 0 | I] over
  // the first (j+1)*m K-rows (identity in segment j), and copy the block's inverse:
  // ht[e] = inv[b*m*m + e], e < m*m.
  // mv: the PieceMove work of the same pivot, in the same launch.
  virtual void owner_edits(DType dt, void* At, int64_t ldl, const int32_t* phys, int64_t p, int64_t k,
                           int64_t j, int64_t m, void* lrow, void* ht, const void* inv, const PieceMove& mv,
                           int s) = 0;
  // Take the pivot row's piece (device-addressed like owner_edits): for g = *phys owned here (else
  // nothing), local rows row0 = (g / p) m .. + m:  dst[r*ldd + c] = X[(row0 + r)*ldx + col0 + c],
  // then X[row0 + r][col0 + c] = 0, for r < m, c < w.  The panel's later columns of a pivot row
  // enter the next column updates as 0 (the sweep's zero-row rule) without a zero-row mask.
  virtual void take_rows(DType dt, void* dst, int64_t ldd, void* X, int64_t ldx, const int32_t* phys, int64_t p,
                         int64_t k, int64_t col0, int64_t w, int64_t m, int s) = 0;
  // dst[i] = sum over q < nslices of src[q*count + i], in q order (identical on every rank).
  virtual void sum_slices(DType dt, void* dst, const void* src, int64_t count, int64_t nslices, int s) = 0;
  // buf[0 .. count) = 0 unless this rank owns the pivot g = *phys (g % p == k): the non-owners'
  // share of a root-agnostic exchange (an all-reduce sum carries the owner's values).
  virtual void zero_unless_owner(DType dt, void* buf, int64_t count, const int32_t* phys, int64_t p, int64_t k,
                                 int s) = 0;
  virtual void h_block(DType dt, void* R, int64_t ldr, const void* Ht, int64_t m, int s) = 0;
  virtual void gemm(DType dt, GemmOp op, ALayout al, int64_t M, int64_t N, int64_t K, const void* A,
                    int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int s,
                    const GemmExtra& ex = GemmExtra()) = 0;
  // Independent small K-major GEMMs (the panel-piece products of one pivot step) as one launch
  // where the device can; the default issues them one by one.
  virtual void gemm_batch(DType dt, const GemmDesc* d, int n, int s) {
    for (int i = 0; i < n; ++i) {
      GemmExtra ex = d[i].ex;
      ex.latency = true;
      gemm(dt, d[i].op, ALayout::KMajor, d[i].M, d[i].N, d[i].K, d[i].A, d[i].lda, d[i].B, d[i].ldb,
           d[i].C, d[i].ldc, s, ex);
    }
  }
  // Finalisation gather: dst[(dst_blk[b]*m + r)*ldd + c*m + j] = X[(b*m + r)*ldx + colsrc[c]*m + j]
  // for local block b < nblk, destination column block c < Nr.
  virtual void permute_blocks(DType dt, void* dst, int64_t ldd, const void* X, int64_t ldx,
                              int64_t nblk, int64_t m, int64_t Nr, const int32_t* dst_blk,
                              const int32_t* colsrc, int s) = 0;
  // Consumption-point verification (GJ_VERIFY, Engine): a position-dependent 64-bit hash of the
  // bytes [r*ld_bytes, r*ld_bytes + width_bytes) of rows r < rows at `base` (width a multiple of 4),
  // as kHashParts partial sums that add (mod 2^64) to the hash of those bytes (gen.hpp hash_term) --
  // enqueued on the stream that consumes the buffer, right before its consumer, so it sees what the
  // consumer saw.
  static constexpr int kHashParts = 64;
  virtual void hash_rows(const void* base, int64_t ld_bytes, int64_t width_bytes, int64_t rows,
                         uint64_t* parts, int s) = 0;
  // out[0] = max over local real rows of sum_{j<n} |X[r][j]|  (reference norm(), main.cpp:643-667).
  virtual void row_abs_max(DType dt, const void* X, int64_t ldx, const Layout& L, double* out,
                           int s) = 0;
  // out[0] = max over local real rows r of sum_{j<n} |X[r][j] - delta(global(r), j)|
  virtual void row_abs_max_minus_i(DType dt, const void* X, int64_t ldx, const Layout& L, double* out,
                                   int s) = 0;
  // out[0] = max over local real rows r of sum_{j<n} |(A_loc * Full)[r][j] - delta(global(r), j)|
  // (matrix_mult_matrix + minus_i + norm, main.cpp:534-667, fused).  A_loc row-major ld npad,
  // Full = the whole inverse in natural row order (npad x npad).
  virtual void residual(DType dt, const void* A, const void* Full, const Layout& L, double* out,
                        int s) = 0;
};

}  // namespace gj
