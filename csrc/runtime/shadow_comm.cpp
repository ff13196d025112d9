// ShadowComm: see gj/comms.hpp.
#include <cstring>

#include "gj/comms.hpp"
#include "gj/pivot.hpp"

namespace gj {

void ShadowComm::allgather(Device& dev, const void* send, void* recv, size_t bytes, int s) {
  dev.copy(recv, send, bytes, s);  // slot 0 = own contribution
  if (bytes != sizeof(PivotRec)) {  // residual/corner gathers: replicate rank 0
    for (int q = 1; q < p_; ++q) dev.copy(static_cast<char*>(recv) + q * bytes, send, bytes, s);
    return;
  }
  const int64_t t = step_++;
  host_.assign((size_t)p_ * bytes, 0);
  auto* recs = reinterpret_cast<PivotRec*>(host_.data());
  for (int q = 1; q < p_; ++q) recs[q] = pivot_invalid();
  const int q = (int)(t % p_);
  if (q != 0) {
    recs[q].score = 0.0;  // strictly better than any real ||inv||
    recs[q].logical = (int32_t)t;
    recs[q].phys = (int32_t)t;
    recs[q].valid = 1;
  }
  dev.copy(static_cast<char*>(recv) + bytes, host_.data() + bytes, (p_ - 1) * bytes, s);
  dev.sync_stream(s);  // host_ is reused by the next step
}

void ShadowComm::bcast(Device& dev, void* buf, size_t bytes, int root, int s) {
  if (root != 0) dev.memset0(buf, bytes, s);
}

void ShadowComm::host_allgather(Device&, const void* send, void* recv, size_t bytes) {
  for (int q = 0; q < p_; ++q) std::memcpy(static_cast<char*>(recv) + q * bytes, send, bytes);
}

}  // namespace gj
