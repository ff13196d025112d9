// ShadowComm: see gj/comms.hpp.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <limits>

#include "gj/comms.hpp"
#include "gj/pivot.hpp"

namespace gj {

std::string ShadowComm::describe() const {
  std::string d = "shadow(" + std::to_string(p_);
  if (cm_.bw_gbs > 0)
    d += ", cost model " + std::to_string(cm_.bw_gbs) + " GB/s per link + " + std::to_string(cm_.lat_us) +
         " us on " + std::to_string(cm_.channels) + " workgroups" + (cm_.direct ? ", direct broadcast" : "");
  return d + ")";
}

void ShadowComm::cost(Device& dev, size_t bytes, int links, int s) {
  if (!(cm_.bw_gbs > 0)) return;
  const double us = cm_.lat_us + (double)bytes / (cm_.bw_gbs * 1e3 * std::max(1, links));
  modelled_us_ += us;
  dev.occupy(s, cm_.channels, us, cm_.lds_kib << 10);
}

void ShadowComm::group_p2p(Device& dev, const std::vector<P2POp>& ops, int s) {
  // one link per peer and direction (fully connected xGMI): the busiest link bounds the group
  if (ops.empty()) return;
  std::vector<size_t> out((size_t)p_, 0), in((size_t)p_, 0);
  for (const auto& o : ops) (o.send ? out : in)[(size_t)o.peer] += o.bytes;
  size_t busiest = 0;
  for (int q = 0; q < p_; ++q) busiest = std::max({busiest, out[q], in[q]});
  cost(dev, busiest, 1, s);
}

// What the synthetic peers broadcast arrives as zeros, one memset per message as in the ring path
// (bcast): the direct path's receives used to keep whatever the buffer held -- uninitialised on
// first use, an intermittent "singular matrix" of the emulated rank (tests/test_shadow_model.py).
void ShadowComm::bcast_many(Device& dev, const std::vector<BcastOp>& ops, int s) {
  Comm::bcast_many(dev, ops, s);
  for (const auto& o : ops)
    if (use_direct(o.bytes) && o.root != 0) receive_zeros(dev, o.buf, o.bytes, s);
}

// Under the cost model the channel workgroups that model the transfer also write its bytes (zeros,
// 16 workgroups of the RCCL channel footprint: the receive side of a real transfer, not a full-chip
// fill kernel on the CUs the pivot chain needs); comm-free, a plain memset.
void ShadowComm::receive_zeros(Device& dev, void* buf, size_t bytes, int s) {
  if (cm_.bw_gbs > 0) dev.zero_channels(buf, bytes, s, cm_.channels, cm_.lds_kib << 10);
  else dev.memset0(buf, bytes, s);
}

ShadowComm::~ShadowComm() {
  if (!pin_) return;
  if (pin_hip_) (void)hipHostFree(pin_);
  else std::free(pin_);
}

void ShadowComm::allgather(Device& dev, const void* send, void* recv, size_t bytes, int s) {
  cost(dev, bytes * (p_ - 1), 1, s);
  dev.copy(recv, send, bytes, s);  // slot 0 = own contribution
  if (bytes != sizeof(PivotRec)) {  // residual/corner gathers: replicate rank 0
    for (int q = 1; q < p_; ++q) dev.copy(static_cast<char*>(recv) + q * bytes, send, bytes, s);
    return;
  }
  // the engine's step (Comm::set_step): a --pivot partial fallback's second exchange of a step
  // must see the same synthetic winner as its first
  const int64_t t = step_;
  const size_t slot = (size_t)p_ * bytes;
  if (!pin_ || pin_hip_ != dev.on_gpu() || pin_bytes_ < kSlots * slot) {
    dev.sync_all();
    if (pin_) {
      if (pin_hip_) (void)hipHostFree(pin_);
      else std::free(pin_);
      pin_ = nullptr;
    }
    pin_hip_ = dev.on_gpu();
    pin_bytes_ = kSlots * slot;
    if (pin_hip_) {
      void* p = nullptr;
      if (hipHostMalloc(&p, pin_bytes_, hipHostMallocDefault) != hipSuccess)
        throw Error(Status::NoMemory, "ShadowComm: pinned record ring");
      pin_ = static_cast<char*>(p);
    } else {
      pin_ = static_cast<char*>(std::malloc(pin_bytes_));
    }
  }
  auto* recs = reinterpret_cast<PivotRec*>(pin_ + (size_t)(t % kSlots) * slot);
  for (int q = 1; q < p_; ++q) recs[q] = pivot_invalid();
  const int q = (int)(t % p_);
  if (q != 0) {
    // strictly better than any real record under both rules (MinInvNorm scores ||inv|| >= 0,
    // Partial scores -max|W| < 0)
    recs[q].score = -std::numeric_limits<double>::max();
    recs[q].logical = (int32_t)t;
    recs[q].phys = (int32_t)t;
    recs[q].valid = 1;
  }
  dev.copy(static_cast<char*>(recv) + bytes, reinterpret_cast<char*>(recs) + bytes, (p_ - 1) * bytes, s);
}

void ShadowComm::allreduce_sum(Device& dev, void*, size_t count, DType dt, int s) {
  cost(dev, 2 * count * dtype_size(dt) * (size_t)(p_ - 1) / (size_t)p_, 1, s);
}

void ShadowComm::bcast(Device& dev, void* buf, size_t bytes, int root, int s) {
  if (use_direct(bytes)) return bcast_many(dev, {BcastOp{buf, bytes, root}}, s);
  cost(dev, bytes, 1, s);
  if (root != 0) receive_zeros(dev, buf, bytes, s);
}

void ShadowComm::host_allgather(Device&, const void* send, void* recv, size_t bytes) {
  for (int q = 0; q < p_; ++q) std::memcpy(static_cast<char*>(recv) + q * bytes, send, bytes);
}

}  // namespace gj
