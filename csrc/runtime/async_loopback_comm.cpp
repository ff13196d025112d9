// AsyncLoopbackComm: stream-ordered collectives between virtual ranks (see gj/comms.hpp).
//
// Every collective follows the RCCL contract the engine relies on: it is
// enqueued on one stream of every rank in the same program order, it starts on a rank's stream
// only after everything enqueued there before it, and what a rank enqueues after it runs only
// once the collective is complete for that rank.  No host thread ever waits for a stream here.
#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "gj/comms.hpp"

namespace gj {

namespace {
uint64_t splitmix(uint64_t& x) {
  uint64_t z = (x += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
std::string sig(const char* kind, size_t bytes, int root, int s) {
  return std::string(kind) + "(" + std::to_string(bytes) + " B, root " + std::to_string(root) +
         ", stream " + std::to_string(s) + ")";
}
}  // namespace

AsyncLoopbackComm::AsyncLoopbackComm(std::shared_ptr<LoopbackHub> hub, int rank, double jitter_us,
                                     uint64_t seed)
    : hub_(std::move(hub)), r_(rank), jitter_us_(jitter_us), rng_(seed * 1000003ull + (uint64_t)rank + 1) {
  // GJ_TEST_DROP_WAIT=bcast_root: broadcast receivers copy without waiting for the root's marker (a
  // planted cross-rank hazard for the schedule checker's tests)
  if (const char* e = std::getenv("GJ_TEST_DROP_WAIT"))
    drop_root_wait_ = (std::string(",") + e + ",").find(",bcast_root,") != std::string::npos;
}

std::string AsyncLoopbackComm::describe() const {
  return "async-loopback(" + std::to_string(size()) +
         (jitter_us_ > 0 ? ", jitter " + std::to_string((int)jitter_us_) + " us" : "") + ")";
}

// Random arrival skew: half the collectives start behind a device-side delay on the issuing
// stream, and the host thread itself dawdles a little before it publishes.
void AsyncLoopbackComm::jitter(Device& dev, int s) {
  if (!(jitter_us_ > 0)) return;
  const uint64_t x = splitmix(rng_);
  const double u = (double)(x >> 11) * (1.0 / 9007199254740992.0);
  if (x & 1) dev.occupy(s, 1, u * jitter_us_);
  if (x & 2) std::this_thread::sleep_for(std::chrono::duration<double, std::micro>(0.25 * u * jitter_us_));
}

void AsyncLoopbackComm::enter(const std::string& signature, const void* p, std::shared_ptr<void> mk,
                              const std::vector<P2POp>* sends) {
  hub_->sig[r_] = signature;
  hub_->ptr[r_] = p;
  hub_->mk[r_] = std::move(mk);
  if (sends) hub_->p2p[r_] = *sends;
  hub_->arrive_and_wait();
  for (int q = 0; q < size(); ++q)
    if (hub_->sig[q] != hub_->sig[0]) {
      const std::string msg = "collective mismatch: rank " + std::to_string(q) + " entered " + hub_->sig[q] +
                              " while rank 0 entered " + hub_->sig[0];
      hub_->fail(msg);
      throw Error(Status::CommError, msg);
    }
}

void AsyncLoopbackComm::bcast(Device& dev, void* buf, size_t bytes, int root, int s) {
  jitter(dev, s);
  enter(sig("bcast", bytes, root, s), buf, dev.mark(s));
  if (r_ != root) {
    if (!drop_root_wait_) dev.wait_mark(s, hub_->mk[root]);
    dev.copy(buf, hub_->ptr[root], bytes, s);
    hub_->done[r_] = dev.mark(s);
  }
  hub_->arrive_and_wait();
  if (r_ == root)
    for (int q = 0; q < size(); ++q)
      if (q != root) dev.wait_mark(s, hub_->done[q]);  // the root's buffer is read until then
}

void AsyncLoopbackComm::allgather(Device& dev, const void* send, void* recv, size_t bytes, int s) {
  jitter(dev, s);
  enter(sig("allgather", bytes, -1, s), send, dev.mark(s));
  char* out = static_cast<char*>(recv);
  for (int q = 0; q < size(); ++q) {
    if (q != r_) dev.wait_mark(s, hub_->mk[q]);
    dev.copy(out + (size_t)q * bytes, hub_->ptr[q], bytes, s);
  }
  hub_->done[r_] = dev.mark(s);
  hub_->arrive_and_wait();
  for (int q = 0; q < size(); ++q)
    if (q != r_) dev.wait_mark(s, hub_->done[q]);
}

void AsyncLoopbackComm::group_p2p(Device& dev, const std::vector<P2POp>& ops, int s) {
  jitter(dev, s);
  std::vector<P2POp> sends;
  for (const auto& op : ops)
    if (op.send) sends.push_back(op);
  enter(sig("group_p2p", 0, -1, s), nullptr, dev.mark(s), &sends);
  // receives from peer q match q's sends to me in issue order (NCCL p2p semantics)
  std::vector<size_t> cursor(size(), 0);
  std::vector<char> waited(size(), 0);
  for (const auto& op : ops) {
    if (op.send) continue;
    const auto& theirs = hub_->p2p[op.peer];
    size_t& c = cursor[op.peer];
    while (c < theirs.size() && theirs[c].peer != r_) ++c;
    GJ_REQUIRE(c < theirs.size(), "async loopback p2p: unmatched receive");
    GJ_REQUIRE(theirs[c].bytes == op.bytes, "async loopback p2p: size mismatch");
    if (!waited[op.peer]) {
      dev.wait_mark(s, hub_->mk[op.peer]);
      waited[op.peer] = 1;
    }
    dev.copy(op.ptr, theirs[c].ptr, op.bytes, s);
    ++c;
  }
  hub_->done[r_] = dev.mark(s);
  hub_->arrive_and_wait();
  std::vector<char> sent(size(), 0);
  for (const auto& op : sends)
    if (!sent[op.peer]) {
      dev.wait_mark(s, hub_->done[op.peer]);  // my send buffers are read until then
      sent[op.peer] = 1;
    }
}

// Scalar maxima are once-per-run agreements (the engine uses host_max); a synchronous fallback
// keeps the interface complete.
void AsyncLoopbackComm::allreduce_max(Device& dev, double* buf, size_t count, int s) {
  dev.sync_stream(s);
  std::vector<double> mine(count), tmp(count);
  dev.copy(mine.data(), buf, count * sizeof(double), s);
  dev.sync_stream(s);
  enter(sig("allreduce_max", count * sizeof(double), -1, s), mine.data(), nullptr);
  for (int q = 0; q < size(); ++q) {
    const double* o = static_cast<const double*>(hub_->ptr[q]);
    for (size_t i = 0; i < count; ++i) tmp[i] = (q == 0) ? o[i] : std::max(tmp[i], o[i]);
  }
  hub_->arrive_and_wait();
  dev.copy(buf, tmp.data(), count * sizeof(double), s);
  dev.sync_stream(s);
}

void AsyncLoopbackComm::barrier(Device& dev) {
  dev.sync_all();
  hub_->arrive_and_wait();
}

double AsyncLoopbackComm::host_max(Device&, double v) {
  hub_->sig[r_] = "host_max";
  hub_->val[r_] = v;
  hub_->arrive_and_wait();
  for (int q = 0; q < size(); ++q)
    if (hub_->sig[q] != "host_max") {
      const std::string msg = "collective mismatch: rank " + std::to_string(q) + " entered " + hub_->sig[q] +
                              " while this rank entered host_max";
      hub_->fail(msg);
      throw Error(Status::CommError, msg);
    }
  double m = hub_->val[0];
  for (int q = 1; q < size(); ++q) m = std::max(m, hub_->val[q]);
  hub_->arrive_and_wait();
  return m;
}

void AsyncLoopbackComm::host_allgather(Device&, const void* send, void* recv, size_t bytes) {
  enter(sig("host_allgather", bytes, -1, -1), send, nullptr);
  for (int q = 0; q < size(); ++q)
    std::memcpy(static_cast<char*>(recv) + (size_t)q * bytes, hub_->ptr[q], bytes);
  hub_->arrive_and_wait();
}

void AsyncLoopbackComm::check_health() {
  if (hub_->failed()) throw Error(Status::CommError, "a peer rank failed");
}

void AsyncLoopbackComm::abort() { hub_->fail("aborted by rank " + std::to_string(r_)); }

}  // namespace gj
