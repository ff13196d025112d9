// Concrete communicators (see gj/comm.hpp for the interface).
#pragma once

#include <condition_variable>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "gj/comm.hpp"

namespace gj {

// ---------------------------------------------------------------- RCCL over xGMI
// One RCCL communicator per stream role that issues collectives (SIDE: pivot records, panel-piece
// broadcasts and once-per-run maxima; COMM: pivot-row chunk broadcasts, finalisation exchange,
// residual all-gather),
// so collectives of different roles can never be reordered against each other across ranks.
class RcclComm : public Comm {
 public:
  static constexpr int kIdBytes = 128;
  static std::string unique_id();  // opaque bytes (kIdBytes)
  // ids: one unique id per communicator (2); every rank passes the same ids.
  // one_comm (every rank passes the same value): the SIDE and COMM roles share ONE communicator
  // (ids[0]; ids[1] unused).  RCCL runs a communicator's kernels one after another in issue order,
  // and every rank issues its collectives in the same program order with every cross-stream edge
  // an event that points back in that order, so no cross-rank wait cycle can form however the
  // streams share hardware queues: the schedule for processes with fewer than kMinHwQueues
  // hardware queues (the SIDE collectives then queue behind the chunk broadcasts issued before
  // them: slower, never stuck).  With two communicators each needs its own queue (README
  // "Progress of the two communicators"); that condition is the launcher's to check, since only
  // it knows the count HIP really initialised with (parallel/dist.py agree_comm_mode).
  RcclComm(const std::vector<std::string>& ids, int nranks, int rank, int device, bool one_comm = false);
  bool one_comm() const { return one_comm_; }
  ~RcclComm() override;
  int size() const override { return n_; }
  int rank() const override { return r_; }
  std::string describe() const override;

  void allgather(Device& dev, const void* send, void* recv, size_t bytes, int s) override;
  void bcast(Device& dev, void* buf, size_t bytes, int root, int s) override;
  void bcast_many(Device& dev, const std::vector<BcastOp>& ops, int s) override;
  void allreduce_max(Device& dev, double* buf, size_t count, int s) override;
  void allreduce_sum(Device& dev, void* buf, size_t count, DType dt, int s) override;
  void group_p2p(Device& dev, const std::vector<P2POp>& ops, int s) override;
  void barrier(Device& dev) override;
  double host_max(Device& dev, double v) override;
  void host_allgather(Device& dev, const void* send, void* recv, size_t bytes) override;
  void check_health() override;
  void abort() override;

 protected:
  bool tunable() const override { return true; }

 private:
  void* comm_for(int s) const;
  int n_ = 1, r_ = 0, device_ = 0;
  bool one_comm_ = false;
  void* comms_[2] = {nullptr, nullptr};  // ncclComm_t
  void* dbuf_ = nullptr;                 // small device scratch for host helpers
  size_t dbuf_sz_ = 0;
};

// ---------------------------------------------------------------- in-process virtual ranks
// p ranks = p threads of one process sharing a LoopbackHub.  Each collective synchronises the
// issuing stream, meets the other ranks at a barrier and copies between their buffers (device
// peer copies for HipDevice, memcpy for HostDevice).  Used by `gj --device cpu -p N` and by the
// multi-rank tests that run on a single GPU.
class LoopbackHub {
 public:
  explicit LoopbackHub(int p);
  int size() const { return p_; }
  // Rendezvous of all ranks; throws Error(CommError) once any rank has called fail() (a rank that
  // died must not leave its peers blocked forever).
  void arrive_and_wait();
  void fail(const std::string& why);
  bool failed() const;
  // published pointers / values
  std::vector<const void*> ptr;
  std::vector<double> val;
  std::vector<std::vector<P2POp>> p2p;  // per source rank
  std::vector<std::string> sig;          // per rank: signature of the collective being entered
  // AsyncLoopbackComm: per rank, the marker at which its stream reached the collective and the
  // marker after its own copies (Device::mark handles)
  std::vector<std::shared_ptr<void>> mk, done;

 private:
  int p_;
  mutable std::mutex mu_;
  std::condition_variable cv_;
  int count_ = 0;
  long gen_ = 0;
  bool failed_ = false;
  std::string why_;
};

class LoopbackComm : public Comm {
 public:
  LoopbackComm(std::shared_ptr<LoopbackHub> hub, int rank) : hub_(std::move(hub)), r_(rank) {}
  int size() const override { return hub_->size(); }
  int rank() const override { return r_; }
  std::string describe() const override { return "loopback(" + std::to_string(size()) + ")"; }

  void allgather(Device& dev, const void* send, void* recv, size_t bytes, int s) override;
  void bcast(Device& dev, void* buf, size_t bytes, int root, int s) override;
  void allreduce_max(Device& dev, double* buf, size_t count, int s) override;
  void group_p2p(Device& dev, const std::vector<P2POp>& ops, int s) override;
  void barrier(Device& dev) override;
  double host_max(Device& dev, double v) override;
  void host_allgather(Device& dev, const void* send, void* recv, size_t bytes) override;

 private:
  // SPMD consistency check: every rank must enter the same collective (kind,
  // size, root, stream role) at the same point of its program, as RCCL requires; a divergence
  // throws on every rank instead of silently exchanging the wrong buffers.
  void enter(const std::string& signature);
  void meet(Device& dev);
  std::shared_ptr<LoopbackHub> hub_;
  int r_;
  uint64_t meets_ = 0;
};

// ---------------------------------------------------------------- asynchronous virtual ranks
// p ranks as threads of one process (one GPU, several GPUs, or AsyncHostDevice on the CPU) whose
// collectives are STREAM-ORDERED, like RCCL's: no stream is ever drained.  A collective records a
// marker on the issuing stream (Device::mark); after a host rendezvous that exchanges buffer
// pointers and markers, every rank's stream waits on its peers' markers (Device::wait_mark) and
// copies on its own stream, then the owners of read buffers wait for the readers' "done" markers
// before their stream may overwrite them.  The host threads only meet to swap pointers, so COMM
// broadcasts really race MAIN GEMMs through events, as on 8 GPUs.  jitter_us > 0 delays each
// rank's arrival at random (a device-side delay on the stream and a host-side one), so the ranks
// reach every collective in a different order on every run.
class AsyncLoopbackComm : public Comm {
 public:
  AsyncLoopbackComm(std::shared_ptr<LoopbackHub> hub, int rank, double jitter_us = 0.0,
                    uint64_t seed = 0);
  int size() const override { return hub_->size(); }
  int rank() const override { return r_; }
  std::string describe() const override;

  void allgather(Device& dev, const void* send, void* recv, size_t bytes, int s) override;
  void bcast(Device& dev, void* buf, size_t bytes, int root, int s) override;
  void allreduce_max(Device& dev, double* buf, size_t count, int s) override;
  void group_p2p(Device& dev, const std::vector<P2POp>& ops, int s) override;
  void barrier(Device& dev) override;
  double host_max(Device& dev, double v) override;
  void host_allgather(Device& dev, const void* send, void* recv, size_t bytes) override;
  void check_health() override;
  void abort() override;

 private:
  void jitter(Device& dev, int s);
  // publish (signature, pointer, marker[, sends]) and meet; throws on an SPMD mismatch
  void enter(const std::string& signature, const void* p, std::shared_ptr<void> mk,
             const std::vector<P2POp>* sends = nullptr);
  std::shared_ptr<LoopbackHub> hub_;
  int r_;
  double jitter_us_;
  uint64_t rng_;
  bool drop_root_wait_ = false;  // GJ_TEST_DROP_WAIT=bcast_root (tests)
};

}  // namespace gj

namespace gj {

// ---------------------------------------------------------------- critical-path emulation
// Rank 0 of a p-rank job, alone on one device: lets a 1-GPU box time the per-rank critical path
// of a p-GPU solve (1/p of the rows, every step's pivot search / panel pieces / chunk pipeline,
// the full-width trailing update) without p GPUs.  Peers are synthetic: at step t the pivot is
// rank 0's own best candidate when t % p == 0, otherwise block row t (owned by rank t % p) with
// a winning score; rows "received" from peers are zeros.  The inverse is meaningless; only the
// timing is.
//
// Communication-cost model (CostModel, off when bw_gbs <= 0): every collective occupies its
// stream for  lat_us + bytes / bandwidth  on `channels` workgroups of a spin kernel of RCCL's
// footprint (256 threads, lds_kib of LDS), so a transfer both takes time on its stream AND
// competes with the trailing-update GEMM for CUs, as RCCL's channel workgroups do.  Bandwidth is
// the per-link bandwidth: a ring broadcast delivers the whole message to every rank at the rate of
// its slowest hop (one link); a group of point-to-point transfers (the direct broadcast's two
// rounds, the final block exchange) takes as long as its busiest link.
struct CostModel {
  double bw_gbs = 0;     // broadcast / point-to-point algorithm bandwidth, GB/s (0 = free comm)
  double lat_us = 0;     // per-collective latency (launch + handshake), us
  int channels = 16;     // workgroups a collective holds while it runs
  // LDS per channel workgroup: rcclGenericKernel<2, false> of a p = 2 solve declares 19 744 B
  // (256 threads, 140 VGPRs, which the spin kernel reproduces; profiles/rccl_footprint_r5.md)
  int lds_kib = 20;
  // The direct broadcast (Comm::bcast_direct: root -> 1/(p-1) slices over p-1 links, then the
  // slice exchange) is modelled as its two point-to-point rounds, each costing lat_us plus the
  // busiest link's bytes / bw_gbs (every peer pair has its own xGMI link).  Off: ring only.
  bool direct = false;
};

class ShadowComm : public Comm {
 public:
  explicit ShadowComm(int p, CostModel cm = CostModel()) : p_(p), cm_(cm) {}
  ~ShadowComm() override;
  int size() const override { return p_; }
  int rank() const override { return 0; }
  std::string describe() const override;
  void allgather(Device& dev, const void* send, void* recv, size_t bytes, int s) override;
  void bcast(Device& dev, void* buf, size_t bytes, int root, int s) override;
  void bcast_many(Device& dev, const std::vector<BcastOp>& ops, int s) override;
  void allreduce_max(Device&, double*, size_t, int) override {}
  // ring all-reduce cost (2 (p-1)/p of the bytes over one link); the synthetic peers add zeros
  void allreduce_sum(Device& dev, void* buf, size_t count, DType dt, int s) override;
  void group_p2p(Device& dev, const std::vector<P2POp>& ops, int s) override;
  void barrier(Device& dev) override { dev.sync_all(); }
  double host_max(Device&, double v) override { return v; }
  void host_allgather(Device& dev, const void* send, void* recv, size_t bytes) override;
  void reset() { step_ = 0; }
  void set_step(int64_t t) override { step_ = t; }
  const CostModel& cost_model() const { return cm_; }
  double modelled_us() const { return modelled_us_; }  // total modelled transfer time issued

 protected:
  bool direct_capable() const override { return cm_.direct; }

 private:
  void cost(Device& dev, size_t bytes, int links, int s);
  void receive_zeros(Device& dev, void* buf, size_t bytes, int s);
  int p_;
  CostModel cm_;
  int64_t step_ = 0;
  double modelled_us_ = 0;
  // the synthetic peers' pivot records, staged in pinned memory: a ring of kSlots steps, so the
  // record copy of step t never waits for the host (the engine's own wait for step t's pivot
  // orders it before slot t is reused, kSlots steps later) -- a real all-gather has no host sync
  static constexpr int kSlots = 8;
  char* pin_ = nullptr;      // hipHostMalloc'd (GPU device) or malloc'd (host device)
  bool pin_hip_ = false;
  size_t pin_bytes_ = 0;
};

}  // namespace gj
