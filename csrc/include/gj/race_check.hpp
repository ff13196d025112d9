// Happens-before race checker for the engine's stream schedule.
//
// The reference is race-free by construction: every step is a sequence of blocking MPI calls
// (main.cpp:1074 MPI_Allreduce, :1097 MPI_Bcast, :1118-1131 Send/Recv).  The MI355X engine replaces
// that with three streams per rank, events between them, stream-ordered collectives and a host
// thread that polls pinned memory, so its correctness rests on an ordering argument.  This checker
// makes that argument mechanical instead of relying on a jittered run happening to expose a bug.
//
// RaceCheckDevice wraps any Device (host, asynchronous host, HIP).  Every op it forwards declares
// the byte regions it reads and writes (`MemRegion`: `height` rows of `width` bytes, `pitch` apart,
// so column blocks of a row-major panel are exact, not bounding boxes).  HbChecker keeps one vector
// clock per agent -- the MAIN / SIDE / COMM streams and the host thread of every wrapped device --
// and derives happens-before purely from the enqueue order, exactly as the HIP / RCCL contracts
// define it:
//   * program order on a stream; an op enqueued by the host is ordered after everything that host
//     has observed (its clock is joined into the stream's at every enqueue);
//   * record(ev, s) snapshots s's clock into ev; wait(s, ev) joins the latest snapshot (the
//     hipStreamWaitEvent rule: the record issued last before the wait);
//   * mark / wait_mark carry a clock across devices (the virtual-rank collectives of
//     AsyncLoopbackComm are built from them, so cross-rank ordering is modelled as the transport
//     provides it: receivers after the root's mark, the root's reuse after the receivers' marks);
//   * host synchronisation (sync_stream, sync_all, sync_event, a true stream_idle / query_event)
//     joins into the host clock; host_acquire() joins the clock of the op that released a pinned
//     record the host polls (the engine's per-step pivot result).
// Two accesses to overlapping bytes, at least one a write, neither ordered before the other, are a
// race: reported with the buffer (engine label + rank), both ops, their streams, and the solver
// step / phase each was enqueued in.  The result does not depend on timing: a schedule with a
// missing edge is reported on every run, whether or not the interleaving that breaks it happens.
//
// Scope: memory allocated through the wrapped devices (the engine's panels and work space, pinned
// host buffers); foreign pointers (torch tensors, host vectors) are not tracked.  RcclComm issues
// its collectives on native streams the checker cannot see, so checked runs use the in-process
// transports (SelfComm, LoopbackComm, AsyncLoopbackComm).
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "gj/device.hpp"

namespace gj {

struct MemRegion {
  const char* base = nullptr;
  int64_t pitch = 0;   // bytes between row starts (ignored when height == 1)
  int64_t width = 0;   // bytes per row
  int64_t height = 0;  // rows
};

// Exact geometry helpers (exposed for tests).
bool regions_overlap(const MemRegion& a, const MemRegion& b);
bool region_covers(const MemRegion& big, const MemRegion& small);

class HbChecker {
 public:
  struct Access {
    MemRegion r;
    bool write = false;
    const char* operand = "";
  };
  using Clock = std::vector<uint32_t>;

  explicit HbChecker(size_t max_reports = 32) : max_reports_(max_reports) {}

  int add_device(const std::string& name);
  // Everything below is called by RaceCheckDevice with the stream role s (kNumStreams = host).
  void op(int dev, int s, const std::string& what, const std::vector<Access>& acc, int64_t step,
          const char* phase);
  Clock snapshot(int dev, int s);                   // record / mark
  void stream_join(int dev, int s, const Clock& c);  // wait / wait_mark
  void host_join(int dev, const Clock& c);           // sync_event / true query
  void host_sync(int dev, int s);                    // sync_stream / true stream_idle (s < 0: all)
  void host_access(int dev, const MemRegion& r, bool write, const std::string& what, int64_t step,
                   const char* phase);
  void release_point(const void* p, int dev, int s);  // the op just checked on s published p
  void host_acquire(int dev, const void* p);
  void set_event(int dev, int ev, Clock c);
  Clock event(int dev, int ev);

  void add_alloc(const void* p, size_t bytes, int dev);
  void drop_alloc(const void* p);
  void label(const void* p, const std::string& name);

  std::vector<std::string> reports() const;
  int64_t races() const;
  int64_t ops() const;
  int64_t live_records() const;

 private:
  struct Rec {
    MemRegion r;
    bool write;
    int agent;
    uint32_t epoch;
    uint32_t op;       // index into ops_
    const char* operand;
  };
  struct OpInfo {
    std::string what;
    int agent;
    int64_t step;
    std::string phase;
  };
  struct Alloc {
    size_t bytes = 0;
    int dev = -1;
    std::string label;
    std::vector<Rec> recs;
  };
  int agent(int dev, int s) const { return dev * (kNumStreams + 1) + s; }
  std::string agent_name(int a) const;
  Alloc* find(const void* p);
  std::string where(const Alloc& al, const MemRegion& r) const;
  // check acc (agent a, clock c) against the live records, then record it
  void check_and_record(int a, const Clock& c, uint32_t opid, const std::vector<Access>& acc);
  void report(const Alloc& al, const Rec& old, const Access& acc, uint32_t opid);
  void maybe_prune();
  static void join(Clock& a, const Clock& b);
  static uint32_t at(const Clock& c, int i) { return i < (int)c.size() ? c[(size_t)i] : 0u; }

  mutable std::mutex mu_;
  size_t max_reports_;
  std::vector<std::string> devs_;
  std::vector<Clock> clk_;                     // per agent
  std::vector<std::vector<Clock>> ev_;          // per device, per event id
  std::map<const void*, Clock> rel_;            // host-visible release points
  std::map<uintptr_t, Alloc> allocs_;
  std::vector<OpInfo> ops_;
  std::vector<std::string> reports_;
  std::map<std::string, int> seen_;             // de-duplication of identical reports
  int64_t races_ = 0;
  uint64_t since_prune_ = 0;
};

// Device decorator: declares every op's accesses to the shared checker, then forwards it.
class RaceCheckDevice : public Device {
 public:
  RaceCheckDevice(std::unique_ptr<Device> inner, std::shared_ptr<HbChecker> hb, const std::string& name);
  ~RaceCheckDevice() override;
  Device& inner() { return *inner_; }
  HbChecker& checker() { return *hb_; }

  bool on_gpu() const override { return inner_->on_gpu(); }
  std::string describe() const override { return "race-check(" + inner_->describe() + ")"; }
  int device_index() const override { return inner_->device_index(); }

  void* alloc(size_t bytes) override;
  void release(void* p) override;
  void* alloc_pinned(size_t bytes) override;
  void* alloc_pinned_coherent(size_t bytes) override;
  void release_pinned(void* p) override;
  size_t free_memory() const override { return inner_->free_memory(); }
  void memset0(void* p, size_t bytes, int s) override;
  void memset2d(void* p, size_t pitch, size_t width_bytes, size_t height, int s) override;
  void copy(void* dst, const void* src, size_t bytes, int s) override;
  void copy2d(void* dst, size_t dpitch, const void* src, size_t spitch, size_t width_bytes, size_t height,
              int s) override;

  int create_event(bool timing = false) override;
  void record(int ev, int s) override;
  void wait(int s, int ev) override;
  void sync_event(int ev) override;
  bool query_event(int ev) override;
  void sync_stream(int s) override;
  void sync_all() override;
  bool stream_idle(int s) override;
  float event_ms(int a, int b) override { return inner_->event_ms(a, b); }
  void* native_stream(int s) override { return inner_->native_stream(s); }
  std::shared_ptr<void> mark(int s) override;
  void wait_mark(int s, const std::shared_ptr<void>& h) override;
  void occupy(int s, int nwg, double us, int lds_bytes = 0) override;
  int reserve_cus(int n) override { return inner_->reserve_cus(n); }
  int64_t skip_align() const override { return inner_->skip_align(); }

  void trace_context(const int64_t* step, const char* const* phase) override {
    step_ = step;
    phase_ = phase;
  }
  void label(const void* p, const char* name) override;
  void host_access(const void* p, size_t bytes, bool write) override;
  void host_acquire(const void* p, size_t bytes) override;
  std::shared_ptr<void> host_mark() override;
  void host_wait_mark(const std::shared_ptr<void>& h) override;

  void generate(DType dt, void* X, const Layout& L, GenSpec g, int s) override;
  void upload_convert(DType dt, void* X, int64_t ldx, const double* src_dev, int64_t src_ld, int64_t rows,
                      int64_t cols, int s) override;
  void widen(DType dt, double* dst, int64_t ldd, const void* X, int64_t ldx, int64_t rows, int64_t cols,
             int s) override;
  void extract_neg_t(DType dt, void* Lt, int64_t ldl, const void* X, int64_t ldx, int64_t rows, int64_t col0,
                     int64_t m, int s) override;
  void add_diag(DType dt, void* A, int64_t ld, int64_t nd, double alpha, int s) override;
  void block_inverse(DType dt, const void* Lt, int64_t ldl, void* inv_t, double* scores, int32_t* valid,
                     const int32_t* used, const Layout& L, double thresh, int64_t nlive, int s) override;
  bool block_inverse_select(DType dt, const void* Lt, int64_t ldl, void* inv_t, double* scores,
                            int32_t* valid, const int32_t* used, const Layout& L, double thresh, int64_t nlive,
                            const PivotSelectArgs& sel, int s) override;
  void set_block_inverse_hint(int variant) override { inner_->set_block_inverse_hint(variant); }
  void set_gemm_tile_hint(int bn) override { inner_->set_gemm_tile_hint(bn); }
  size_t block_inverse_scratch_bytes(DType dt, const Layout& L, int variant) const override {
    return inner_->block_inverse_scratch_bytes(dt, L, variant);
  }
  void prepare_block_inverse(DType dt, const Layout& L, int variant) override {
    inner_->prepare_block_inverse(dt, L, variant);
  }
  void candidate_maxabs(DType dt, const void* Lt, int64_t ldl, double* scores, int32_t* valid,
                        const int32_t* used, const Layout& L, double thresh, int s) override;
  void gather_candidate(DType dt, void* sel, const void* Lt, int64_t ldl, const PivotRec* rec, const Layout& L,
                        int s) override;
  void commit_candidate(DType dt, void* inv_t, const void* inv1, const int32_t* valid1, const double* score1, double growth, PivotRec* rec,
                        const Layout& L, int s) override;
  void pivot_local(const double* scores, const int32_t* valid, const int32_t* used, const int32_t* pos,
                   const Layout& L, PivotRec* out, int s) override;
  void pivot_global(const PivotRec* recs, int32_t p, int32_t t, int32_t* pos, int32_t* phys_at, int32_t* used,
                    int32_t* seq, PivotResult* out, PivotResult* host_out, int s) override;
  void pivot_select_single(const double* scores, const int32_t* valid, const Layout& L, int32_t t, int32_t* pos,
                           int32_t* phys_at, int32_t* used, int32_t* seq, PivotRec* rec, PivotResult* out,
                           PivotResult* host_out, int s) override;
  void owner_edits(DType dt, void* At, int64_t ldl, const int32_t* phys, int64_t p, int64_t k, int64_t j,
                   int64_t m, void* lrow, void* ht, const void* inv, const PieceMove& mv, int s) override;
  void take_rows(DType dt, void* dst, int64_t ldd, void* X, int64_t ldx, const int32_t* phys, int64_t p, int64_t k,
                 int64_t col0, int64_t w, int64_t m, int s) override;
  void sum_slices(DType dt, void* dst, const void* src, int64_t count, int64_t nslices, int s) override;
  void zero_unless_owner(DType dt, void* buf, int64_t count, const int32_t* phys, int64_t p, int64_t k,
                         int s) override;
  void h_block(DType dt, void* R, int64_t ldr, const void* Ht, int64_t m, int s) override;
  void gemm(DType dt, GemmOp op, ALayout al, int64_t M, int64_t N, int64_t K, const void* A, int64_t lda,
            const void* B, int64_t ldb, void* C, int64_t ldc, int s, const GemmExtra& ex = GemmExtra()) override;
  void gemm_batch(DType dt, const GemmDesc* d, int n, int s) override;
  void permute_blocks(DType dt, void* dst, int64_t ldd, const void* X, int64_t ldx, int64_t nblk, int64_t m,
                      int64_t Nr, const int32_t* dst_blk, const int32_t* colsrc, int s) override;
  void hash_rows(const void* base, int64_t ld_bytes, int64_t width_bytes, int64_t rows, uint64_t* parts,
                 int s) override;
  void row_abs_max(DType dt, const void* X, int64_t ldx, const Layout& L, double* out, int s) override;
  void row_abs_max_minus_i(DType dt, const void* X, int64_t ldx, const Layout& L, double* out, int s) override;
  void residual(DType dt, const void* A, const void* Full, const Layout& L, double* out, int s) override;

 private:
  using Acc = HbChecker::Access;
  void check(int s, const std::string& what, const std::vector<Acc>& acc);
  int64_t cur_step() const { return step_ ? *step_ : -1; }
  const char* cur_phase() const { return (phase_ && *phase_) ? *phase_ : ""; }

  std::unique_ptr<Device> inner_;
  std::shared_ptr<HbChecker> hb_;
  int id_;
  const int64_t* step_ = nullptr;
  const char* const* phase_ = nullptr;
};

}  // namespace gj
