// Transport-independent parts of Comm: the direct (scatter + exchange) broadcast and its tuner
// ("benchmark both against ncclBroadcast").  The reference has one broadcast,
// MPI_Bcast of the packed pivot row (main.cpp:1093-1097); on xGMI every GPU pair has its own link,
// so a chain that forwards the whole row hop by hop leaves most links idle.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "gj/comm.hpp"

namespace gj {

namespace {

// Slice of the message held by rank j after round 1: the p-1 non-root ranks split it in 256-byte
// aligned pieces (the last ones may be short or empty).
void direct_slice(size_t bytes, int p, int root, int j, size_t& off, size_t& len) {
  const int idx = j < root ? j : j - 1;
  size_t q = (bytes + (size_t)(p - 2)) / (size_t)(p - 1);
  q = (q + 255) & ~size_t(255);
  off = std::min(bytes, q * (size_t)idx);
  len = std::min(bytes, off + q) - off;
}

size_t env_size(const char* name, size_t dflt) {
  const char* e = std::getenv(name);
  if (!e || !*e) return dflt;
  char* end = nullptr;
  const unsigned long long v = std::strtoull(e, &end, 10);
  GJ_REQUIRE(end && *end == '\0', std::string(name) + " must be a byte count");
  return (size_t)v;
}

}  // namespace

void Comm::bcast_direct(Device& dev, const std::vector<BcastOp>& ops, int s) {
  if (ops.empty()) return;
  const int p = size(), me = rank();
  std::vector<P2POp> ph;
  // round 1: the root hands slice j to rank j (p-1 links out of the root in parallel)
  for (const auto& o : ops)
    for (int j = 0; j < p; ++j) {
      if (j == o.root || (me != o.root && me != j)) continue;
      size_t off, len;
      direct_slice(o.bytes, p, o.root, j, off, len);
      if (len == 0) continue;
      char* b = static_cast<char*>(o.buf) + off;
      ph.push_back(me == o.root ? P2POp{b, len, j, true} : P2POp{b, len, o.root, false});
    }
  group_p2p(dev, ph, s);
  // round 2: every non-root rank sends its slice to the other non-root ranks and receives theirs
  // (per peer pair, sends and receives are issued in op order on both sides, so they match)
  ph.clear();
  for (const auto& o : ops) {
    if (me == o.root) continue;
    size_t off, len;
    direct_slice(o.bytes, p, o.root, me, off, len);
    char* b = static_cast<char*>(o.buf);
    for (int k = 0; k < p; ++k) {
      if (k == me || k == o.root) continue;
      size_t ko, kl;
      direct_slice(o.bytes, p, o.root, k, ko, kl);
      if (len) ph.push_back(P2POp{b + off, len, k, true});
      if (kl) ph.push_back(P2POp{b + ko, kl, k, false});
    }
  }
  group_p2p(dev, ph, s);
}

void Comm::note(int s, const char* kind, size_t bytes, int root) {
  if (s < 0 || s >= kNumStreams) return;
  char buf[160];
  if (root >= 0)
    std::snprintf(buf, sizeof buf, "#%llu %s root=%d bytes=%zu", (unsigned long long)++nops_[s], kind, root, bytes);
  else
    std::snprintf(buf, sizeof buf, "#%llu %s bytes=%zu", (unsigned long long)++nops_[s], kind, bytes);
  last_[s] = buf;
}

std::string Comm::last_op(int s) const {
  static const char* names[kNumStreams] = {"MAIN", "SIDE", "COMM"};
  if (s < 0 || s >= kNumStreams) return "?";
  return std::string(names[s]) + " stream, last collective " + (last_[s].empty() ? "none" : last_[s]);
}

void Comm::drain(Device& dev, int s) {
  if (size() == 1 || !dev.on_gpu()) {
    dev.sync_stream(s);
    return;
  }
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  auto next = t0 + std::chrono::milliseconds(20);
  int spins = 0;
  while (!dev.stream_idle(s)) {
    if (++spins > 64) std::this_thread::sleep_for(std::chrono::microseconds(50));
    const auto t = clk::now();
    if (t < next) continue;
    check_health();
    if (std::chrono::duration<double>(t - t0).count() > timeout_s_) {
      abort();
      throw Error(Status::CommError, "timed out after " + std::to_string(timeout_s_) +
                                         " s waiting for the " + last_op(s) +
                                         " (peer failure or hang)");
    }
    next = t + std::chrono::milliseconds(20);
  }
}

void Comm::drain_all(Device& dev) {
  for (int s = 0; s < kNumStreams; ++s) drain(dev, s);
}

std::string Comm::tune_bcast(Device& dev, size_t bytes) { return tune_bcast(dev, std::vector<size_t>{bytes}); }

std::string Comm::tune_bcast(Device& dev, std::vector<size_t> sizes) {
  const char* e = std::getenv("GJ_BCAST");
  const std::string mode = (e && *e) ? e : "auto";
  GJ_REQUIRE(mode == "auto" || mode == "ring" || mode == "direct", "GJ_BCAST must be ring|direct|auto");
  size_t mn = std::max<size_t>(1, env_size("GJ_BCAST_MIN", size_t(64) << 10));
  direct_min_ = 0;
  if (size() <= 2) {  // the two algorithms coincide
    bcast_report_ = "ring";
    return "ring";
  }
  // Every rank reads its own environment: a rank sending direct while a peer sends ring would hang
  // both, so the mode and the threshold are agreed first (a mismatch is an error on every rank).
  const double code = mode == "ring" ? 0.0 : mode == "direct" ? 1.0 : 2.0;
  const double lo_code = -host_max(dev, -code), hi_code = host_max(dev, code);
  const double lo_mn = -host_max(dev, -(double)mn), hi_mn = host_max(dev, (double)mn);
  if (lo_code != hi_code || lo_mn != hi_mn)
    throw Error(Status::BadArgs, "GJ_BCAST / GJ_BCAST_MIN differ between ranks");
  if (mode == "ring" || !direct_capable()) {
    bcast_report_ = direct_capable() ? "ring" : "ring (transport has no point-to-point path)";
    return "ring";
  }
  if (mode == "direct") {
    direct_min_ = mn;
    bcast_report_ = "direct (GJ_BCAST)";
    return "direct";
  }
  std::sort(sizes.begin(), sizes.end());
  sizes.erase(std::unique(sizes.begin(), sizes.end()), sizes.end());
  sizes.erase(std::remove_if(sizes.begin(), sizes.end(), [&](size_t b) { return b < mn; }), sizes.end());
  if (!tunable() || !dev.on_gpu() || sizes.empty()) {
    bcast_report_ = "ring";
    return "ring";
  }
  // Measure both at the engine's message sizes on the COMM stream, roots rotating.
  const int p = size(), me = rank();
  const int s = S_COMM;
  const size_t maxb = sizes.back();
  void* buf = dev.alloc(maxb);
  // bit-exact delivery check of the direct path on BOTH communicators (COMM carries the row
  // segments, SIDE the panel pieces; root 1, so the root's own slice index is skipped)
  std::vector<uint32_t> pat(maxb / 4 + 1), got(maxb / 4 + 1);
  for (size_t i = 0; i < pat.size(); ++i) pat[i] = (uint32_t)(i * 2654435761u) ^ 0x5bd1e995u;
  const int vroot = 1 % p;
  bool ok_local = true;
  for (int cs : {S_COMM, S_SIDE}) {
    if (me == vroot) dev.copy(buf, pat.data(), maxb, cs);
    else dev.memset0(buf, maxb, cs);
    drain(dev, cs);
    bcast_direct(dev, {BcastOp{buf, maxb, vroot}}, cs);
    dev.copy(got.data(), buf, maxb, cs);
    drain(dev, cs);
    ok_local = ok_local && std::memcmp(got.data(), pat.data(), maxb) == 0;
  }
  const bool ok = host_max(dev, ok_local ? 0.0 : 1.0) == 0.0;
  // One timed round = p broadcasts (every rank the root once), the max over ranks of its mean per
  // broadcast.  The two algorithms alternate round by round (a drifting clock or a busy link hits
  // both), kRounds rounds each after 2 warm-ups; the decision uses the MEDIANS, and the report
  // carries median, min and max of both (2p samples decided the p = 8 pick, whose wrong
  // choice costs 72 % under the model).
  constexpr int kRounds = 7;
  auto round_ms = [&](bool direct, size_t bytes) {
    auto run = [&](int it) {
      const BcastOp o{buf, bytes, it % p};
      if (direct) bcast_direct(dev, {o}, s);
      else bcast(dev, o.buf, o.bytes, o.root, s);
    };
    drain(dev, s);
    host_max(dev, 0.0);  // barrier
    const auto t0 = std::chrono::steady_clock::now();
    for (int it = 0; it < p; ++it) run(it);
    drain(dev, s);
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() / p;
    return host_max(dev, ms);
  };
  struct Stat { double med = -1, lo = -1, hi = -1; };
  auto stat = [](std::vector<double> v) {
    Stat r;
    if (v.empty()) return r;
    std::sort(v.begin(), v.end());
    r.med = v[v.size() / 2];
    r.lo = v.front();
    r.hi = v.back();
    return r;
  };
  // direct from the smallest measured size at which it wins at that and every larger size
  std::string detail;
  size_t thr = 0;
  bool wins_above = true;
  std::vector<bool> win(sizes.size());
  std::vector<Stat> tr(sizes.size()), td(sizes.size());
  for (size_t i = 0; i < sizes.size(); ++i) {
    for (int w = 0; w < 2; ++w) {  // warm-ups of both
      round_ms(false, sizes[i]);
      if (ok) round_ms(true, sizes[i]);
    }
    std::vector<double> vr, vd;
    for (int r = 0; r < kRounds; ++r) {
      vr.push_back(round_ms(false, sizes[i]));
      if (ok) vd.push_back(round_ms(true, sizes[i]));
    }
    tr[i] = stat(vr);
    td[i] = stat(vd);
    win[i] = ok && td[i].med < 0.95 * tr[i].med;
  }
  for (size_t i = sizes.size(); i-- > 0;) {
    wins_above = wins_above && win[i];
    if (wins_above) thr = sizes[i];
  }
  dev.release(buf);
  direct_min_ = thr;
  for (size_t i = 0; i < sizes.size(); ++i) {
    char line[256];
    std::snprintf(line, sizeof line,
                  "%s%zu B: ring %.3f ms [%.3f-%.3f], direct %.3f ms [%.3f-%.3f] (median [min-max] of %d rounds)",
                  i ? "; " : "", sizes[i], tr[i].med, tr[i].lo, tr[i].hi, td[i].med, td[i].lo, td[i].hi, kRounds);
    detail += line;
  }
  const std::string choice = thr == 0 ? "ring" : (thr == sizes.front() ? "direct" : "direct from " + std::to_string(thr) + " B");
  bcast_report_ = choice + " (auto: " + detail + (ok ? "" : "; direct FAILED check") + ")";
  return thr == 0 ? "ring" : "direct";
}

// Generic sum: every rank's contribution gathered (stream-ordered, the transport's all-gather), then
// summed in rank order on the device, so every rank computes the same bits.  The scratch is kept
// per stream role (the engine frees it, free_scratch) -- freeing per call would synchronise.
void Comm::allreduce_sum(Device& dev, void* buf, size_t count, DType dt, int s) {
  if (size() == 1 || count == 0) return;
  const size_t bytes = count * dtype_size(dt), need = bytes * (size_t)size();
  if (sum_cap_[s] < need) {
    if (sum_scratch_[s]) {
      dev.sync_all();
      dev.release(sum_scratch_[s]);
    }
    sum_scratch_[s] = dev.alloc(need);
    sum_cap_[s] = need;
    dev.label(sum_scratch_[s], "comm sum scratch");
  }
  allgather(dev, buf, sum_scratch_[s], bytes, s);
  dev.sum_slices(dt, buf, sum_scratch_[s], (int64_t)count, size(), s);
}

void Comm::free_scratch(Device& dev) {
  for (int s = 0; s < kNumStreams; ++s)
    if (sum_scratch_[s]) {
      dev.release(sum_scratch_[s]);
      sum_scratch_[s] = nullptr;
      sum_cap_[s] = 0;
    }
}

}  // namespace gj
