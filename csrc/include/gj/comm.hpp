// Communication abstraction (replaces the reference's direct MPI calls).
//
// Implementations:
//   * RcclComm     (csrc/runtime/rccl_comm.cpp)  — one RCCL communicator per stream role, over xGMI.
//   * LoopbackComm (csrc/runtime/loopback_comm.cpp) — p "virtual ranks" as threads of one process
//     (host or one GPU); used by the CLI's --device cpu mode and by multi-rank tests on a 1-GPU box.
//   * PyComm       (csrc/python/module.cpp)      — trampolines into torch.distributed (gloo) so the
//     multi-process path is testable on CPU.
//
// All collective calls are stream-ordered w.r.t. the Device stream role they are issued on, and
// every rank issues them in the same program order (SPMD), exactly like the reference's blocking MPI.
#pragma once

#include <string>
#include <vector>

#include "gj/device.hpp"

namespace gj {

struct P2POp {
  void* ptr;
  size_t bytes;
  int peer;
  bool send;
};

struct BcastOp {
  void* buf;
  size_t bytes;
  int root;
};

class Comm {
 public:
  virtual ~Comm() = default;
  virtual int size() const = 0;
  virtual int rank() const = 0;
  virtual std::string describe() const = 0;

  // Device-memory, stream-ordered collectives.
  virtual void allgather(Device& dev, const void* send, void* recv, size_t bytes, int s) = 0;
  virtual void bcast(Device& dev, void* buf, size_t bytes, int root, int s) = 0;
  virtual void allreduce_max(Device& dev, double* buf, size_t count, int s) = 0;
  virtual void group_p2p(Device& dev, const std::vector<P2POp>& ops, int s) = 0;
  // In-place sum of `count` elements of dtype dt over the ranks (every rank gets the same bits).
  // Default: all-gather into a scratch buffer the communicator keeps (free_scratch) + an ordered
  // device sum; RCCL uses ncclAllReduce.
  virtual void allreduce_sum(Device& dev, void* buf, size_t count, DType dt, int s);
  void free_scratch(Device& dev);
  // Several broadcasts (any roots) issued as one group: RCCL runs them concurrently, so pivot rows
  // owned by different ranks travel over different xGMI links at the same time.
  // Ops of at least direct_bcast_min() bytes take the two-round direct algorithm (bcast_direct).
  virtual void bcast_many(Device& dev, const std::vector<BcastOp>& ops, int s) {
    std::vector<BcastOp> big;
    for (const auto& o : ops)
      if (use_direct(o.bytes)) big.push_back(o);
      else bcast(dev, o.buf, o.bytes, o.root, s);
    bcast_direct(dev, big, s);
  }

  // Large-broadcast algorithm.  "ring" = the transport's own broadcast (RCCL:
  // a pipelined chain per channel, so each hop forwards the whole message).  "direct" = the root
  // sends 1/(p-1) of the message to every other rank over its own xGMI link, then the p-1 holders
  // exchange their slices (two grouped point-to-point rounds; every link carries ~2/(p-1) of the
  // message).  tune_bcast() sets it once per engine from GJ_BCAST=ring|direct|auto (default auto:
  // on a GPU transport both are timed at the real message sizes, checked for bit-exact delivery,
  // and the faster is kept on every rank) and GJ_BCAST_MIN (smallest message measured / sent direct, 64 KiB).
  // Returns the chosen algorithm's name ("ring" at p <= 2: the two coincide).
  std::string tune_bcast(Device& dev, size_t bytes);
  // Several message sizes: direct from the smallest measured size at which it wins there and at
  // every larger one (the engine passes its panel-piece and row-segment sizes).
  std::string tune_bcast(Device& dev, std::vector<size_t> sizes);
  size_t direct_bcast_min() const { return direct_min_; }
  void set_direct_bcast_min(size_t b) { direct_min_ = b; }
  const std::string& bcast_report() const { return bcast_report_; }

  // The solver step the following collectives belong to (diagnostics; the single-GPU emulation
  // ShadowComm synthesises its peers' pivot records from it).
  virtual void set_step(int64_t t) { (void)t; }

  // Host-blocking helpers (once-per-run agreement: errors, timings, residual maxima).
  virtual void barrier(Device& dev) = 0;
  virtual double host_max(Device& dev, double v) = 0;
  virtual void host_allgather(Device& dev, const void* send, void* recv, size_t bytes) = 0;

  // Failure detection: throw Error(CommError) if the transport reports an
  // asynchronous failure (a peer died, a link error); abort() tears the transport down so that
  // device-side collectives blocked on a dead peer return.
  virtual void check_health() {}
  virtual void abort() {}
  // Host wait for stream s (all streams) with failure detection: the stream is polled, the
  // transport checked every 20 ms, and after timeout() seconds the transport is aborted and
  // Error(CommError) thrown.  Every host wait that can sit behind a collective goes through here:
  // a plain hipStreamSynchronize behind a collective with a dead peer never returns.
  void drain(Device& dev, int s);
  void drain_all(Device& dev);
  void set_timeout(double seconds) { timeout_s_ = seconds; }
  double timeout() const { return timeout_s_; }

  // Diagnostics: the last collective issued on each stream role (kind, root, bytes and its
  // sequence number on that role).  Every timeout message names it, so a hang on a p-GPU node
  // says which collective each rank sat in; ranks that disagree on the sequence number show
  // which one fell behind.
  void note(int s, const char* kind, size_t bytes, int root = -1);
  std::string last_op(int s) const;

 protected:
  double timeout_s_ = 600;
  std::string last_[kNumStreams];
  uint64_t nops_[kNumStreams] = {};
  // Whether GJ_BCAST=auto measures (a GPU transport whose two algorithms differ in cost).
  virtual bool tunable() const { return false; }
  // Whether bcast_direct moves real data (false for the timing emulation, whose peers are synthetic).
  virtual bool direct_capable() const { return true; }
  bool use_direct(size_t bytes) const { return direct_min_ > 0 && size() > 2 && bytes >= direct_min_; }
  void bcast_direct(Device& dev, const std::vector<BcastOp>& ops, int s);
  size_t direct_min_ = 0;
  std::string bcast_report_;
  void* sum_scratch_[kNumStreams] = {};
  size_t sum_cap_[kNumStreams] = {};
};

// A trivial single-rank communicator.
class SelfComm : public Comm {
 public:
  int size() const override { return 1; }
  int rank() const override { return 0; }
  std::string describe() const override { return "self"; }
  void allgather(Device& dev, const void* send, void* recv, size_t bytes, int s) override {
    if (send != recv) dev.copy(recv, send, bytes, s);
  }
  void bcast(Device&, void*, size_t, int, int) override {}
  void allreduce_max(Device&, double*, size_t, int) override {}
  void allreduce_sum(Device&, void*, size_t, DType, int) override {}
  void group_p2p(Device&, const std::vector<P2POp>& ops, int) override {
    GJ_REQUIRE(ops.empty(), "SelfComm: point-to-point with a peer requested");
  }
  void barrier(Device& dev) override { dev.sync_all(); }
  double host_max(Device&, double v) override { return v; }
  void host_allgather(Device&, const void* send, void* recv, size_t bytes) override;
};

}  // namespace gj
