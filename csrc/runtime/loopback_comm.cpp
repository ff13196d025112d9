// LoopbackComm: p virtual ranks as threads of one process (host memory or one/several GPUs).
// Semantics match RcclComm: every rank calls the same collectives in the same order; a collective
// first drains the issuing stream so it observes all work enqueued before it (stream ordering).
#include <algorithm>
#include <cstring>

#include "gj/comms.hpp"

namespace gj {

LoopbackHub::LoopbackHub(int p) : ptr(p, nullptr), val(p, 0.0), p2p(p), sig(p), mk(p), done(p), p_(p) {}

void LoopbackHub::arrive_and_wait() {
  std::unique_lock<std::mutex> lk(mu_);
  if (failed_) throw Error(Status::CommError, "peer rank failed: " + why_);
  const long g = gen_;
  if (++count_ == p_) {
    count_ = 0;
    ++gen_;
    cv_.notify_all();
  } else {
    cv_.wait(lk, [&] { return gen_ != g || failed_; });
    if (gen_ == g) throw Error(Status::CommError, "peer rank failed: " + why_);
  }
}

void LoopbackHub::fail(const std::string& why) {
  std::lock_guard<std::mutex> lk(mu_);
  if (!failed_) {
    failed_ = true;
    why_ = why;
  }
  cv_.notify_all();
}

bool LoopbackHub::failed() const {
  std::lock_guard<std::mutex> lk(mu_);
  return failed_;
}

void LoopbackComm::enter(const std::string& signature) {
  hub_->sig[r_] = signature;
  hub_->arrive_and_wait();
  for (int q = 0; q < size(); ++q)
    if (hub_->sig[q] != hub_->sig[0])
      throw Error(Status::CommError, "collective mismatch: rank " + std::to_string(q) + " entered " +
                                         hub_->sig[q] + " while rank 0 entered " + hub_->sig[0]);
}

// Rendezvous that also carries the host threads' ordering (Device::host_mark): after it, every
// rank's host has observed what every peer's host had observed when it arrived (the streams each
// drained before).  Only the schedule checker (RaceCheckDevice) looks at the marks.
// Consecutive meets alternate between two slot vectors: a rank writes its slot of meet k + 2 only
// after the rendezvous of meet k + 1, which every rank reaches only once it has read meet k's.
void LoopbackComm::meet(Device& dev) {
  auto& slot = (meets_++ & 1) ? hub_->done : hub_->mk;
  slot[r_] = dev.host_mark();
  hub_->arrive_and_wait();
  for (int q = 0; q < size(); ++q)
    if (q != r_) dev.host_wait_mark(slot[q]);
}

static std::string sig(const char* kind, size_t bytes, int root, int s) {
  return std::string(kind) + "(" + std::to_string(bytes) + " B, root " + std::to_string(root) +
         ", stream " + std::to_string(s) + ")";
}

void LoopbackComm::allgather(Device& dev, const void* send, void* recv, size_t bytes, int s) {
  dev.sync_stream(s);
  enter(sig("allgather", bytes, -1, s));
  hub_->ptr[r_] = send;
  meet(dev);
  for (int q = 0; q < size(); ++q)
    dev.copy(static_cast<char*>(recv) + (size_t)q * bytes, hub_->ptr[q], bytes, s);
  dev.sync_stream(s);
  meet(dev);
}

void LoopbackComm::bcast(Device& dev, void* buf, size_t bytes, int root, int s) {
  dev.sync_stream(s);
  enter(sig("bcast", bytes, root, s));
  hub_->ptr[r_] = buf;
  meet(dev);
  if (r_ != root) dev.copy(buf, hub_->ptr[root], bytes, s);
  dev.sync_stream(s);
  meet(dev);
}

void LoopbackComm::allreduce_max(Device& dev, double* buf, size_t count, int s) {
  dev.sync_stream(s);
  enter(sig("allreduce_max", count * sizeof(double), -1, s));
  std::vector<double> mine(count), tmp(count);
  dev.copy(mine.data(), buf, count * sizeof(double), s);
  dev.sync_stream(s);
  hub_->ptr[r_] = mine.data();
  hub_->arrive_and_wait();
  for (int q = 0; q < size(); ++q) {
    const double* o = static_cast<const double*>(hub_->ptr[q]);
    for (size_t i = 0; i < count; ++i) tmp[i] = (q == 0) ? o[i] : std::max(tmp[i], o[i]);
  }
  hub_->arrive_and_wait();
  dev.copy(buf, tmp.data(), count * sizeof(double), s);
  dev.sync_stream(s);
}

void LoopbackComm::group_p2p(Device& dev, const std::vector<P2POp>& ops, int s) {
  dev.sync_stream(s);
  enter(sig("group_p2p", 0, -1, s));
  auto& mine = hub_->p2p[r_];
  mine.clear();
  for (const auto& op : ops)
    if (op.send) mine.push_back(op);
  meet(dev);
  // receives from peer q match q's sends to me in issue order (NCCL p2p semantics)
  std::vector<size_t> cursor(size(), 0);
  for (const auto& op : ops) {
    if (op.send) continue;
    const auto& theirs = hub_->p2p[op.peer];
    size_t& c = cursor[op.peer];
    while (c < theirs.size() && theirs[c].peer != r_) ++c;
    GJ_REQUIRE(c < theirs.size(), "loopback p2p: unmatched receive");
    GJ_REQUIRE(theirs[c].bytes == op.bytes, "loopback p2p: size mismatch");
    dev.copy(op.ptr, theirs[c].ptr, op.bytes, s);
    ++c;
  }
  dev.sync_stream(s);
  meet(dev);
}

void LoopbackComm::barrier(Device& dev) {
  dev.sync_all();
  meet(dev);
}

double LoopbackComm::host_max(Device&, double v) {
  enter("host_max");
  hub_->val[r_] = v;
  hub_->arrive_and_wait();
  double m = hub_->val[0];
  for (int q = 1; q < size(); ++q) m = std::max(m, hub_->val[q]);
  hub_->arrive_and_wait();
  return m;
}

void LoopbackComm::host_allgather(Device&, const void* send, void* recv, size_t bytes) {
  enter(sig("host_allgather", bytes, -1, -1));
  hub_->ptr[r_] = send;
  hub_->arrive_and_wait();
  for (int q = 0; q < size(); ++q)
    std::memcpy(static_cast<char*>(recv) + (size_t)q * bytes, hub_->ptr[q], bytes);
  hub_->arrive_and_wait();
}

}  // namespace gj
