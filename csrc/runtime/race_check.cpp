// Happens-before race checker (see gj/race_check.hpp).
#include "gj/race_check.hpp"

#include <algorithm>
#include <cstdio>
#include <sstream>

namespace gj {

// ---------------------------------------------------------------- geometry
namespace {

int64_t floor_div(int64_t a, int64_t b) {  // b > 0
  const int64_t q = a / b;
  return (a % b != 0 && a < 0) ? q - 1 : q;
}

int64_t lo_of(const MemRegion& r) { return (int64_t)(uintptr_t)r.base; }
bool contiguous(const MemRegion& r) { return r.height <= 1 || r.width >= r.pitch; }
int64_t hi_of(const MemRegion& r) {  // one past the last byte
  return lo_of(r) + (r.height <= 1 ? r.width : (r.height - 1) * r.pitch + r.width);
}
bool empty(const MemRegion& r) { return r.width <= 0 || r.height <= 0; }

// [lo, hi) against the rows of a non-contiguous region
bool span_vs_rows(int64_t lo, int64_t hi, const MemRegion& b) {
  const int64_t B = lo_of(b), p = b.pitch, w = b.width;
  int64_t rmax = floor_div(hi - B - 1, p);      // B + r p < hi
  int64_t rmin = floor_div(lo - B - w, p) + 1;  // B + r p + w > lo
  rmin = std::max<int64_t>(rmin, 0);
  rmax = std::min<int64_t>(rmax, b.height - 1);
  return rmin <= rmax;
}

}  // namespace

bool regions_overlap(const MemRegion& a, const MemRegion& b) {
  if (empty(a) || empty(b)) return false;
  if (!(lo_of(a) < hi_of(b) && lo_of(b) < hi_of(a))) return false;  // bounding spans
  if (contiguous(a)) return contiguous(b) ? true : span_vs_rows(lo_of(a), hi_of(a), b);
  if (contiguous(b)) return span_vs_rows(lo_of(b), hi_of(b), a);
  if (a.pitch == b.pitch) {
    // b's row rb sits in a's frame at row q + rb, bytes [rd, rd + wb), spilling into the next row
    // when rd + wb > pitch (both widths are below the pitch here)
    const int64_t p = a.pitch, d = lo_of(b) - lo_of(a);
    const int64_t q = floor_div(d, p), rd = d - q * p;
    auto rows_meet = [&](int64_t r0, int64_t r1) { return std::max<int64_t>(r0, 0) <= std::min<int64_t>(r1, a.height - 1); };
    if (rd < a.width && rows_meet(q, q + b.height - 1)) return true;
    if (rd + b.width > p && rows_meet(q + 1, q + b.height)) return true;
    return false;
  }
  const MemRegion& s = a.height <= b.height ? a : b;  // walk the shorter one's rows
  const MemRegion& o = a.height <= b.height ? b : a;
  for (int64_t r = 0; r < s.height; ++r) {
    const int64_t lo = lo_of(s) + r * s.pitch;
    if (span_vs_rows(lo, lo + s.width, o)) return true;
  }
  return false;
}

bool region_covers(const MemRegion& big, const MemRegion& small) {
  if (empty(small)) return true;
  if (empty(big)) return false;
  const int64_t slo = lo_of(small), shi = hi_of(small);
  if (contiguous(big)) return lo_of(big) <= slo && shi <= hi_of(big);
  const int64_t p = big.pitch;
  if (contiguous(small)) {  // inside one row of big
    const int64_t r = floor_div(slo - lo_of(big), p), c = slo - lo_of(big) - r * p;
    return r >= 0 && r < big.height && c + (shi - slo) <= big.width;
  }
  if (small.pitch != p) return false;
  const int64_t d = slo - lo_of(big);
  const int64_t q = floor_div(d, p), rd = d - q * p;
  return q >= 0 && q + small.height <= big.height && rd + small.width <= big.width;
}

// ---------------------------------------------------------------- checker
void HbChecker::join(Clock& a, const Clock& b) {
  if (a.size() < b.size()) a.resize(b.size(), 0u);
  for (size_t i = 0; i < b.size(); ++i) a[i] = std::max(a[i], b[i]);
}

int HbChecker::add_device(const std::string& name) {
  std::lock_guard<std::mutex> lk(mu_);
  devs_.push_back(name);
  clk_.resize(devs_.size() * (kNumStreams + 1));
  ev_.resize(devs_.size());
  return (int)devs_.size() - 1;
}

std::string HbChecker::agent_name(int a) const {
  static const char* roles[kNumStreams + 1] = {"MAIN", "SIDE", "COMM", "host"};
  const int d = a / (kNumStreams + 1), s = a % (kNumStreams + 1);
  return devs_.at((size_t)d) + " " + roles[s];
}

HbChecker::Alloc* HbChecker::find(const void* p) {
  const uintptr_t x = (uintptr_t)p;
  auto it = allocs_.upper_bound(x);
  if (it == allocs_.begin()) return nullptr;
  --it;
  if (x >= it->first + std::max<size_t>(it->second.bytes, 1)) return nullptr;
  return &it->second;
}

std::string HbChecker::where(const Alloc& al, const MemRegion& r) const {
  std::ostringstream o;
  uintptr_t base = 0;
  for (const auto& kv : allocs_)
    if (&kv.second == &al) base = kv.first;
  o << (al.label.empty() ? std::string("buffer") : al.label) << "@" << devs_.at((size_t)al.dev) << " +"
    << ((uintptr_t)r.base - base);
  if (r.height > 1) o << " (" << r.height << " rows x " << r.width << " B, pitch " << r.pitch << ")";
  else o << " (" << r.width << " B)";
  return o.str();
}

void HbChecker::report(const Alloc& al, const Rec& old, const Access& acc, uint32_t opid) {
  ++races_;
  const OpInfo& a = ops_[old.op];
  const OpInfo& b = ops_[opid];
  std::ostringstream key;
  key << al.label << "|" << a.what << "|" << old.operand << "|" << b.what << "|" << acc.operand << "|" << a.phase
      << "|" << b.phase;
  if (seen_[key.str()]++ > 0 || reports_.size() >= max_reports_) return;
  std::ostringstream o;
  o << "unordered " << (old.write ? "write" : "read") << "/" << (acc.write ? "write" : "read") << " on "
    << where(al, acc.r) << ": " << a.what << " [" << old.operand << "] on " << agent_name(a.agent) << " (step "
    << a.step << ", " << (a.phase.empty() ? "-" : a.phase) << ") vs " << b.what << " [" << acc.operand << "] on "
    << agent_name(b.agent) << " (step " << b.step << ", " << (b.phase.empty() ? "-" : b.phase)
    << "): no happens-before edge between them";
  reports_.push_back(o.str());
}

void HbChecker::check_and_record(int a, const Clock& c, uint32_t opid, const std::vector<Access>& acc_in) {
  std::vector<Access> acc = acc_in;
  std::vector<Alloc*> where_(acc.size(), nullptr);
  for (size_t i = 0; i < acc.size(); ++i) {
    Access& x = acc[i];
    if (x.r.base == nullptr) continue;
    Alloc* al = find(x.r.base);
    where_[i] = al;
    if (!al) continue;  // untracked memory
    // extents the op could not know (device-addressed rows): to the end of the allocation
    uintptr_t abase = 0;
    for (auto it = allocs_.upper_bound((uintptr_t)x.r.base); it != allocs_.begin();) {
      --it;
      abase = it->first;
      break;
    }
    const int64_t left = (int64_t)(abase + al->bytes) - (int64_t)(uintptr_t)x.r.base;
    if (x.r.width < 0) {
      x.r.width = left;
      x.r.pitch = left;
      x.r.height = 1;
    } else if (x.r.height < 0) {
      x.r.height = x.r.pitch > 0 && left >= x.r.width ? (left - x.r.width) / x.r.pitch + 1 : 1;
    }
    if (empty(x.r)) {
      where_[i] = nullptr;
      continue;
    }
    for (const Rec& r : al->recs) {
      if (!(r.write || x.write)) continue;
      if (at(c, r.agent) >= r.epoch) continue;  // ordered before this op
      if (regions_overlap(r.r, x.r)) report(*al, r, x, opid);
    }
  }
  const uint32_t epoch = at(c, a);
  for (size_t i = 0; i < acc.size(); ++i) {
    Alloc* al = where_[i];
    if (!al) continue;
    const Access& x = acc[i];
    // a record this access covers and is ordered after can no longer be the first half of a race
    // that this one would not also report (a write is only superseded by a write)
    auto& v = al->recs;
    v.erase(std::remove_if(v.begin(), v.end(),
                           [&](const Rec& r) {
                             return (x.write || !r.write) && at(c, r.agent) >= r.epoch && region_covers(x.r, r.r);
                           }),
            v.end());
    v.push_back(Rec{x.r, x.write, a, epoch, opid, x.operand});
  }
}

void HbChecker::maybe_prune() {
  if (++since_prune_ < 256) return;
  since_prune_ = 0;
  // records every agent has already seen can never race again
  Clock floor;
  bool first = true;
  for (const Clock& c : clk_) {
    if (first) {
      floor = c;
      first = false;
      continue;
    }
    if (floor.size() > c.size()) floor.resize(c.size());
    for (size_t i = 0; i < floor.size(); ++i) floor[i] = std::min(floor[i], c[i]);
  }
  for (auto& kv : allocs_) {
    auto& v = kv.second.recs;
    v.erase(std::remove_if(v.begin(), v.end(), [&](const Rec& r) { return at(floor, r.agent) >= r.epoch; }), v.end());
  }
}

void HbChecker::op(int dev, int s, const std::string& what, const std::vector<Access>& acc, int64_t step,
                   const char* phase) {
  std::lock_guard<std::mutex> lk(mu_);
  const int a = agent(dev, s);
  Clock& c = clk_[(size_t)a];
  join(c, clk_[(size_t)agent(dev, kNumStreams)]);  // enqueued by the host: after all it has seen
  if (c.size() <= (size_t)a) c.resize((size_t)a + 1, 0u);
  c[(size_t)a] += 1;
  const uint32_t opid = (uint32_t)ops_.size();
  ops_.push_back(OpInfo{what, a, step, phase ? phase : ""});
  check_and_record(a, c, opid, acc);
  maybe_prune();
}

void HbChecker::host_access(int dev, const MemRegion& r, bool write, const std::string& what, int64_t step,
                            const char* phase) {
  std::vector<Access> acc{Access{r, write, write ? "host write" : "host read"}};
  op(dev, kNumStreams, what, acc, step, phase);
}

HbChecker::Clock HbChecker::snapshot(int dev, int s) {
  std::lock_guard<std::mutex> lk(mu_);
  Clock& c = clk_[(size_t)agent(dev, s)];
  join(c, clk_[(size_t)agent(dev, kNumStreams)]);
  return c;
}

void HbChecker::stream_join(int dev, int s, const Clock& x) {
  std::lock_guard<std::mutex> lk(mu_);
  Clock& c = clk_[(size_t)agent(dev, s)];
  join(c, clk_[(size_t)agent(dev, kNumStreams)]);
  join(c, x);
}

void HbChecker::host_join(int dev, const Clock& x) {
  std::lock_guard<std::mutex> lk(mu_);
  join(clk_[(size_t)agent(dev, kNumStreams)], x);
}

void HbChecker::host_sync(int dev, int s) {
  std::lock_guard<std::mutex> lk(mu_);
  Clock& h = clk_[(size_t)agent(dev, kNumStreams)];
  for (int r = 0; r < kNumStreams; ++r)
    if (s < 0 || r == s) join(h, clk_[(size_t)agent(dev, r)]);
}

void HbChecker::release_point(const void* p, int dev, int s) {
  std::lock_guard<std::mutex> lk(mu_);
  rel_[p] = clk_[(size_t)agent(dev, s)];
}

void HbChecker::host_acquire(int dev, const void* p) {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = rel_.find(p);
  if (it != rel_.end()) join(clk_[(size_t)agent(dev, kNumStreams)], it->second);
}

void HbChecker::set_event(int dev, int ev, Clock c) {
  std::lock_guard<std::mutex> lk(mu_);
  auto& v = ev_[(size_t)dev];
  if ((int)v.size() <= ev) v.resize((size_t)ev + 1);
  v[(size_t)ev] = std::move(c);
}

HbChecker::Clock HbChecker::event(int dev, int ev) {
  std::lock_guard<std::mutex> lk(mu_);
  const auto& v = ev_[(size_t)dev];
  return ev < (int)v.size() ? v[(size_t)ev] : Clock();
}

void HbChecker::add_alloc(const void* p, size_t bytes, int dev) {
  std::lock_guard<std::mutex> lk(mu_);
  Alloc& a = allocs_[(uintptr_t)p];
  a = Alloc();
  a.bytes = bytes;
  a.dev = dev;
}

void HbChecker::drop_alloc(const void* p) {
  std::lock_guard<std::mutex> lk(mu_);
  auto a = allocs_.find((uintptr_t)p);
  if (a == allocs_.end()) return;
  const uintptr_t lo = a->first, hi = a->first + std::max<size_t>(a->second.bytes, 1);
  allocs_.erase(a);
  for (auto it = rel_.begin(); it != rel_.end();)
    it = ((uintptr_t)it->first >= lo && (uintptr_t)it->first < hi) ? rel_.erase(it) : std::next(it);
}

void HbChecker::label(const void* p, const std::string& name) {
  std::lock_guard<std::mutex> lk(mu_);
  if (Alloc* a = find(p)) a->label = name;
}

std::vector<std::string> HbChecker::reports() const {
  std::lock_guard<std::mutex> lk(mu_);
  return reports_;
}
int64_t HbChecker::races() const {
  std::lock_guard<std::mutex> lk(mu_);
  return races_;
}
int64_t HbChecker::ops() const {
  std::lock_guard<std::mutex> lk(mu_);
  return (int64_t)ops_.size();
}
int64_t HbChecker::live_records() const {
  std::lock_guard<std::mutex> lk(mu_);
  int64_t n = 0;
  for (const auto& kv : allocs_) n += (int64_t)kv.second.recs.size();
  return n;
}

// ---------------------------------------------------------------- the device decorator
namespace {

struct MarkBox {
  std::shared_ptr<void> inner;
  HbChecker::Clock clock;
};

MemRegion span(const void* p, int64_t bytes) {
  MemRegion r;
  r.base = static_cast<const char*>(p);
  r.pitch = bytes;
  r.width = bytes;
  r.height = p && bytes > 0 ? 1 : 0;
  return r;
}
// rows x width elements, ld elements apart (bytes = es each)
MemRegion rect(const void* p, int64_t ld, int64_t width, int64_t rows, int64_t es) {
  MemRegion r;
  r.base = static_cast<const char*>(p);
  r.pitch = ld * es;
  r.width = width * es;
  r.height = p ? rows : 0;
  if (r.height == 1) r.pitch = r.width;
  return r;
}
using Acc = HbChecker::Access;
Acc R(MemRegion r, const char* n) { return Acc{r, false, n}; }
Acc W(MemRegion r, const char* n) { return Acc{r, true, n}; }

std::string gemm_name(const char* k, GemmOp op, int64_t M, int64_t N, int64_t K) {
  return std::string(k) + (op == GemmOp::Acc ? " C+=AB " : " C=AB ") + std::to_string(M) + "x" +
         std::to_string(N) + "x" + std::to_string(K);
}

void gemm_acc(std::vector<Acc>& a, DType dt, GemmOp op, ALayout al, int64_t M, int64_t N, int64_t K,
              const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, const GemmExtra& ex) {
  const int64_t es = (int64_t)dtype_size(dt);
  if (M <= 0 || N <= 0) return;
  if (ex.rsel_m > 0) {  // row-block selection: the selected blocks' rows of A, C and tneg only
    const int64_t h = ex.rsel_m, cols = ex.tneg ? (ex.tneg_cols > 0 ? std::min(ex.tneg_cols, N) : N) : 0;
    if (K > 0) a.push_back(R(rect(B, ldb, N, K, es), "B"));
    for (int64_t i = 0; i < M; i += h) {
      const int64_t r = ex.rsel_row(i);
      if (K > 0)
        a.push_back(R(al == ALayout::KMajor ? rect(static_cast<const char*>(A) + r * es, lda, h, K, es)
                                            : rect(static_cast<const char*>(A) + r * lda * es, lda, K, h, es),
                      "A"));
      a.push_back(W(rect(static_cast<char*>(C) + r * ldc * es, ldc, N, h, es), "C"));
      if (ex.c_in)
        a.push_back(R(rect(static_cast<const char*>(ex.c_in) + r * ex.ldc_in * es, ex.ldc_in, N, h, es), "C_in"));
      if (ex.tneg) a.push_back(W(rect(static_cast<char*>(ex.tneg) + r * es, ex.ldtneg, h, cols, es), "tneg"));
    }
    if (ex.owner_phys) a.push_back(R(span(ex.owner_phys, 4), "owner"));
    return;
  }
  // column ranges touched: [0, N) minus GemmExtra::skip_c0 / skip_c1
  int64_t cr0[2] = {0, 0}, cr1[2] = {N, 0};
  int ncr = 1;
  if (ex.skip_c1 > ex.skip_c0) {
    cr1[0] = std::min(N, ex.skip_c0);
    cr0[1] = ex.skip_c1;
    cr1[1] = N;
    ncr = 2;
  }
  if (K > 0) a.push_back(R(al == ALayout::KMajor ? rect(A, lda, M, K, es) : rect(A, lda, K, M, es), "A"));
  (void)op;  // C += AB reads C too; a write of the same bytes already conflicts with any access
  for (int z = 0; z < ncr; ++z) {
    const int64_t w = cr1[z] - cr0[z];
    if (w <= 0) continue;
    if (K > 0) a.push_back(R(rect(static_cast<const char*>(B) + cr0[z] * es, ldb, w, K, es), "B"));
    a.push_back(W(rect(static_cast<char*>(C) + cr0[z] * es, ldc, w, M, es), "C"));
    if (ex.c_in) a.push_back(R(rect(static_cast<const char*>(ex.c_in) + cr0[z] * es, ex.ldc_in, w, M, es), "C_in"));
  }
  if (ex.tneg) {
    const int64_t cols = ex.tneg_cols > 0 ? std::min(ex.tneg_cols, N) : N;
    a.push_back(W(rect(ex.tneg, ex.ldtneg, M, cols, es), "tneg"));
  }
  if (ex.owner_phys) a.push_back(R(span(ex.owner_phys, 4), "owner"));
}

}  // namespace

RaceCheckDevice::RaceCheckDevice(std::unique_ptr<Device> inner, std::shared_ptr<HbChecker> hb,
                                 const std::string& name)
    : inner_(std::move(inner)), hb_(std::move(hb)) {
  id_ = hb_->add_device(name);
}

RaceCheckDevice::~RaceCheckDevice() = default;

void RaceCheckDevice::check(int s, const std::string& what, const std::vector<Acc>& acc) {
  hb_->op(id_, s, what, acc, cur_step(), cur_phase());
}

void* RaceCheckDevice::alloc(size_t bytes) {
  void* p = inner_->alloc(bytes);
  hb_->add_alloc(p, bytes, id_);
  return p;
}
void RaceCheckDevice::release(void* p) {
  hb_->host_sync(id_, -1);  // HIP: hipFree synchronises; host: the queues drain first
  hb_->drop_alloc(p);
  inner_->release(p);
}
void* RaceCheckDevice::alloc_pinned(size_t bytes) {
  void* p = inner_->alloc_pinned(bytes);
  hb_->add_alloc(p, bytes, id_);
  return p;
}
void* RaceCheckDevice::alloc_pinned_coherent(size_t bytes) {
  void* p = inner_->alloc_pinned_coherent(bytes);
  hb_->add_alloc(p, bytes, id_);
  return p;
}
void RaceCheckDevice::release_pinned(void* p) {
  hb_->host_sync(id_, -1);
  hb_->drop_alloc(p);
  inner_->release_pinned(p);
}
void RaceCheckDevice::memset0(void* p, size_t bytes, int s) {
  check(s, "memset", {W(span(p, (int64_t)bytes), "dst")});
  inner_->memset0(p, bytes, s);
}
void RaceCheckDevice::memset2d(void* p, size_t pitch, size_t w, size_t h, int s) {
  check(s, "memset2d", {W(rect(p, (int64_t)pitch, (int64_t)w, (int64_t)h, 1), "dst")});
  inner_->memset2d(p, pitch, w, h, s);
}
void RaceCheckDevice::copy(void* dst, const void* src, size_t bytes, int s) {
  if (dst != src) check(s, "copy", {R(span(src, (int64_t)bytes), "src"), W(span(dst, (int64_t)bytes), "dst")});
  inner_->copy(dst, src, bytes, s);
}
void RaceCheckDevice::copy2d(void* dst, size_t dpitch, const void* src, size_t spitch, size_t w, size_t h, int s) {
  check(s, "copy2d", {R(rect(src, (int64_t)spitch, (int64_t)w, (int64_t)h, 1), "src"),
                      W(rect(dst, (int64_t)dpitch, (int64_t)w, (int64_t)h, 1), "dst")});
  inner_->copy2d(dst, dpitch, src, spitch, w, h, s);
}

int RaceCheckDevice::create_event(bool timing) { return inner_->create_event(timing); }
void RaceCheckDevice::record(int ev, int s) {
  hb_->set_event(id_, ev, hb_->snapshot(id_, s));
  inner_->record(ev, s);
}
void RaceCheckDevice::wait(int s, int ev) {
  hb_->stream_join(id_, s, hb_->event(id_, ev));
  inner_->wait(s, ev);
}
void RaceCheckDevice::sync_event(int ev) {
  inner_->sync_event(ev);
  hb_->host_join(id_, hb_->event(id_, ev));
}
bool RaceCheckDevice::query_event(int ev) {
  const bool done = inner_->query_event(ev);
  if (done) hb_->host_join(id_, hb_->event(id_, ev));
  return done;
}
void RaceCheckDevice::sync_stream(int s) {
  inner_->sync_stream(s);
  hb_->host_sync(id_, s);
}
void RaceCheckDevice::sync_all() {
  inner_->sync_all();
  hb_->host_sync(id_, -1);
}
bool RaceCheckDevice::stream_idle(int s) {
  const bool idle = inner_->stream_idle(s);
  if (idle) hb_->host_sync(id_, s);
  return idle;
}
std::shared_ptr<void> RaceCheckDevice::mark(int s) {
  auto box = std::make_shared<MarkBox>();
  box->clock = hb_->snapshot(id_, s);
  box->inner = inner_->mark(s);
  return box;
}
void RaceCheckDevice::wait_mark(int s, const std::shared_ptr<void>& h) {
  if (!h) return;
  auto box = std::static_pointer_cast<MarkBox>(h);
  hb_->stream_join(id_, s, box->clock);
  inner_->wait_mark(s, box->inner);
}
void RaceCheckDevice::occupy(int s, int nwg, double us, int lds_bytes) {
  check(s, "occupy", {});
  inner_->occupy(s, nwg, us, lds_bytes);
}

void RaceCheckDevice::label(const void* p, const char* name) { hb_->label(p, name); }
void RaceCheckDevice::host_access(const void* p, size_t bytes, bool write) {
  hb_->host_access(id_, span(p, (int64_t)bytes), write, write ? "host store" : "host load", cur_step(),
                   cur_phase());
}
void RaceCheckDevice::host_acquire(const void* p, size_t bytes) {
  hb_->host_acquire(id_, p);
  hb_->host_access(id_, span(p, (int64_t)bytes), false, "host poll", cur_step(), cur_phase());
}

std::shared_ptr<void> RaceCheckDevice::host_mark() {
  auto box = std::make_shared<MarkBox>();
  box->clock = hb_->snapshot(id_, kNumStreams);
  return box;
}
void RaceCheckDevice::host_wait_mark(const std::shared_ptr<void>& h) {
  if (h) hb_->host_join(id_, std::static_pointer_cast<MarkBox>(h)->clock);
}

void RaceCheckDevice::generate(DType dt, void* X, const Layout& L, GenSpec g, int s) {
  check(s, "generate", {W(rect(X, L.npad, L.npad, L.rows, (int64_t)dtype_size(dt)), "X")});
  inner_->generate(dt, X, L, g, s);
}
void RaceCheckDevice::upload_convert(DType dt, void* X, int64_t ldx, const double* src, int64_t src_ld,
                                     int64_t rows, int64_t cols, int s) {
  check(s, "upload_convert",
        {R(rect(src, src_ld, cols, rows, 8), "src"), W(rect(X, ldx, cols, rows, (int64_t)dtype_size(dt)), "X")});
  inner_->upload_convert(dt, X, ldx, src, src_ld, rows, cols, s);
}
void RaceCheckDevice::widen(DType dt, double* dst, int64_t ldd, const void* X, int64_t ldx, int64_t rows,
                            int64_t cols, int s) {
  check(s, "widen", {R(rect(X, ldx, cols, rows, (int64_t)dtype_size(dt)), "X"), W(rect(dst, ldd, cols, rows, 8), "dst")});
  inner_->widen(dt, dst, ldd, X, ldx, rows, cols, s);
}
void RaceCheckDevice::extract_neg_t(DType dt, void* Lt, int64_t ldl, const void* X, int64_t ldx, int64_t rows,
                                    int64_t col0, int64_t m, int s) {
  const int64_t es = (int64_t)dtype_size(dt);
  check(s, "extract_neg_t",
        {R(rect(static_cast<const char*>(X) + col0 * es, ldx, m, rows, es), "X"), W(rect(Lt, ldl, rows, m, es), "Lt")});
  inner_->extract_neg_t(dt, Lt, ldl, X, ldx, rows, col0, m, s);
}
void RaceCheckDevice::add_diag(DType dt, void* A, int64_t ld, int64_t nd, double alpha, int s) {
  check(s, "add_diag", {W(rect(A, ld + 1, 1, nd, (int64_t)dtype_size(dt)), "A")});
  inner_->add_diag(dt, A, ld, nd, alpha, s);
}

namespace {
void inverse_acc(std::vector<Acc>& a, DType dt, const void* Lt, int64_t ldl, void* inv_t, double* scores,
                 int32_t* valid, const int32_t* used, const Layout& L) {
  const int64_t es = (int64_t)dtype_size(dt);
  a.push_back(R(rect(Lt, ldl, L.rows, L.m, es), "Lt"));
  a.push_back(R(span(used, (int64_t)sizeof(int32_t) * L.Nr), "used"));
  a.push_back(W(span(inv_t, L.nblk * L.m * L.m * es), "inv"));
  a.push_back(W(span(scores, (int64_t)sizeof(double) * L.nblk), "scores"));
  a.push_back(W(span(valid, (int64_t)sizeof(int32_t) * L.nblk), "valid"));
}
}  // namespace

void RaceCheckDevice::block_inverse(DType dt, const void* Lt, int64_t ldl, void* inv_t, double* scores,
                                    int32_t* valid, const int32_t* used, const Layout& L, double thresh, int64_t nlive, int s) {
  std::vector<Acc> a;
  inverse_acc(a, dt, Lt, ldl, inv_t, scores, valid, used, L);
  check(s, "block_inverse", a);
  inner_->block_inverse(dt, Lt, ldl, inv_t, scores, valid, used, L, thresh, nlive, s);
}
bool RaceCheckDevice::block_inverse_select(DType dt, const void* Lt, int64_t ldl, void* inv_t, double* scores,
                                           int32_t* valid, const int32_t* used, const Layout& L, double thresh, int64_t nlive,
                                           const PivotSelectArgs& sel, int s) {
  if (!inner_->block_inverse_select(dt, Lt, ldl, inv_t, scores, valid, used, L, thresh, nlive, sel, s)) return false;
  std::vector<Acc> a;
  inverse_acc(a, dt, Lt, ldl, inv_t, scores, valid, used, L);
  const int64_t nr = (int64_t)sizeof(int32_t) * L.Nr;
  a.push_back(W(span(sel.done, 4), "done"));
  a.push_back(R(span(sel.pos, nr), "pos"));
  a.push_back(W(span(sel.rec, sizeof(PivotRec)), "rec"));
  if (sel.single) {
    a.push_back(W(span(sel.pos_w, nr), "pos"));
    a.push_back(W(span(sel.phys_at, nr), "phys_at"));
    a.push_back(W(span(sel.used_w, nr), "used"));
    a.push_back(W(span(sel.seq, nr), "seq"));
    a.push_back(W(span(sel.out, sizeof(PivotResult)), "out"));
    a.push_back(W(span(sel.host_out, sizeof(PivotResult)), "host_out"));
  }
  check(s, "block_inverse+select", a);
  if (sel.single && sel.host_out) hb_->release_point(sel.host_out, id_, s);
  return true;
}
void RaceCheckDevice::candidate_maxabs(DType dt, const void* Lt, int64_t ldl, double* scores, int32_t* valid,
                                       const int32_t* used, const Layout& L, double thresh, int s) {
  check(s, "candidate_maxabs",
        {R(rect(Lt, ldl, L.rows, L.m, (int64_t)dtype_size(dt)), "Lt"),
         R(span(used, (int64_t)sizeof(int32_t) * L.Nr), "used"), W(span(scores, 8 * L.nblk), "scores"),
         W(span(valid, 4 * L.nblk), "valid")});
  inner_->candidate_maxabs(dt, Lt, ldl, scores, valid, used, L, thresh, s);
}
void RaceCheckDevice::gather_candidate(DType dt, void* sel, const void* Lt, int64_t ldl, const PivotRec* rec,
                                       const Layout& L, int s) {
  const int64_t es = (int64_t)dtype_size(dt);
  check(s, "gather_candidate",
        {R(span(rec, sizeof(PivotRec)), "rec"), R(rect(Lt, ldl, L.rows, L.m, es), "Lt"),
         W(span(sel, L.m * L.m * es), "sel")});
  inner_->gather_candidate(dt, sel, Lt, ldl, rec, L, s);
}
void RaceCheckDevice::commit_candidate(DType dt, void* inv_t, const void* inv1, const int32_t* valid1, const double* score1, double growth,
                                       PivotRec* rec, const Layout& L, int s) {
  const int64_t es = (int64_t)dtype_size(dt);
  check(s, "commit_candidate",
        {R(span(inv1, L.m * L.m * es), "inv1"), R(span(valid1, 4), "valid1"), R(span(score1, 8), "score1"),
         W(span(rec, sizeof(PivotRec)), "rec"),
         W(span(inv_t, L.nblk * L.m * L.m * es), "inv")});
  inner_->commit_candidate(dt, inv_t, inv1, valid1, score1, growth, rec, L, s);
}
void RaceCheckDevice::pivot_local(const double* scores, const int32_t* valid, const int32_t* used, const int32_t* pos,
                                  const Layout& L, PivotRec* out, int s) {
  const int64_t nr = (int64_t)sizeof(int32_t) * L.Nr;
  check(s, "pivot_local",
        {R(span(scores, 8 * L.nblk), "scores"), R(span(valid, 4 * L.nblk), "valid"), R(span(used, nr), "used"),
         R(span(pos, nr), "pos"), W(span(out, sizeof(PivotRec)), "rec")});
  inner_->pivot_local(scores, valid, used, pos, L, out, s);
}
void RaceCheckDevice::pivot_global(const PivotRec* recs, int32_t p, int32_t t, int32_t* pos, int32_t* phys_at,
                                   int32_t* used, int32_t* seq, PivotResult* out, PivotResult* host_out, int s) {
  // the book-keeping arrays are Nr long; this call does not know Nr: one element per step is
  // enough to order the accesses (every access to them is whole-array or this one)
  std::vector<Acc> a{R(span(recs, (int64_t)sizeof(PivotRec) * p), "recs"), W(span(pos, 4), "pos"),
                     W(span(phys_at, 4), "phys_at"), W(span(used, 4), "used"), W(span(seq, 4), "seq"),
                     W(span(out, sizeof(PivotResult)), "out")};
  if (host_out) a.push_back(W(span(host_out, sizeof(PivotResult)), "host_out"));
  check(s, "pivot_global", a);
  inner_->pivot_global(recs, p, t, pos, phys_at, used, seq, out, host_out, s);
  if (host_out) hb_->release_point(host_out, id_, s);
}
void RaceCheckDevice::pivot_select_single(const double* scores, const int32_t* valid, const Layout& L, int32_t t,
                                          int32_t* pos, int32_t* phys_at, int32_t* used, int32_t* seq,
                                          PivotRec* rec, PivotResult* out, PivotResult* host_out, int s) {
  const int64_t nr = (int64_t)sizeof(int32_t) * L.Nr;
  std::vector<Acc> a{R(span(scores, 8 * L.nblk), "scores"), R(span(valid, 4 * L.nblk), "valid"),
                     W(span(pos, nr), "pos"), W(span(phys_at, nr), "phys_at"), W(span(used, nr), "used"),
                     W(span(seq, nr), "seq"), W(span(rec, sizeof(PivotRec)), "rec"),
                     W(span(out, sizeof(PivotResult)), "out")};
  if (host_out) a.push_back(W(span(host_out, sizeof(PivotResult)), "host_out"));
  check(s, "pivot_select_single", a);
  inner_->pivot_select_single(scores, valid, L, t, pos, phys_at, used, seq, rec, out, host_out, s);
  if (host_out) hb_->release_point(host_out, id_, s);
}
void RaceCheckDevice::owner_edits(DType dt, void* At, int64_t ldl, const int32_t* phys, int64_t p, int64_t k,
                                  int64_t j, int64_t m, void* lrow, void* ht, const void* inv, const PieceMove& mv,
                                  int s) {
  const int64_t es = (int64_t)dtype_size(dt);
  // the pivot's rows are chosen on the device: every row of the first (j + 1) m K-rows, every block
  // of the inverses, the piece's column range of every row of X (height / width -1: to the end of
  // the allocation)
  std::vector<Acc> a{R(span(phys, 4), "phys"), W(rect(At, ldl, ldl, (j + 1) * m, es), "At rows"),
                     W(span(ht, m * m * es), "Ht"), R(MemRegion{static_cast<const char*>(inv), -1, -1, 1}, "inv")};
  if (j > 0) a.push_back(W(span(lrow, j * m * m * es), "Lrow"));
  if (mv.w > 0) {
    MemRegion xr = rect(static_cast<char*>(mv.X) + mv.col0 * es, mv.ldx, mv.w, 2, es);
    xr.height = -1;
    a.push_back(W(xr, "X piece"));
    a.push_back(W(rect(mv.dst, mv.ldd, mv.w, m, es), "piece"));
  }
  if (mv.eye) a.push_back(W(rect(mv.eye, mv.ld_eye, m, m, es), "eye"));
  check(s, "owner_edits", a);
  inner_->owner_edits(dt, At, ldl, phys, p, k, j, m, lrow, ht, inv, mv, s);
}
void RaceCheckDevice::take_rows(DType dt, void* dst, int64_t ldd, void* X, int64_t ldx, const int32_t* phys,
                                int64_t p, int64_t k, int64_t col0, int64_t w, int64_t m, int s) {
  const int64_t es = (int64_t)dtype_size(dt);
  MemRegion xr = rect(static_cast<char*>(X) + col0 * es, ldx, w, 1, es);
  xr.pitch = ldx * es;
  xr.height = -1;  // rows of the pivot chosen on the device: the column range of every row
  check(s, "take_rows", {R(span(phys, 4), "phys"), W(xr, "X piece"), W(rect(dst, ldd, w, m, es), "dst")});
  inner_->take_rows(dt, dst, ldd, X, ldx, phys, p, k, col0, w, m, s);
}
void RaceCheckDevice::sum_slices(DType dt, void* dst, const void* src, int64_t count, int64_t nslices, int s) {
  const int64_t es = (int64_t)dtype_size(dt);
  check(s, "sum_slices", {R(span(src, count * nslices * es), "slices"), W(span(dst, count * es), "dst")});
  inner_->sum_slices(dt, dst, src, count, nslices, s);
}
void RaceCheckDevice::zero_unless_owner(DType dt, void* buf, int64_t count, const int32_t* phys, int64_t p,
                                        int64_t k, int s) {
  check(s, "zero_unless_owner", {R(span(phys, 4), "phys"), W(span(buf, count * (int64_t)dtype_size(dt)), "buf")});
  inner_->zero_unless_owner(dt, buf, count, phys, p, k, s);
}
void RaceCheckDevice::h_block(DType dt, void* Rp, int64_t ldr, const void* Ht, int64_t m, int s) {
  const int64_t es = (int64_t)dtype_size(dt);
  check(s, "h_block", {R(span(Ht, m * m * es), "Ht"), W(rect(Rp, ldr, m, m, es), "R")});
  inner_->h_block(dt, Rp, ldr, Ht, m, s);
}
void RaceCheckDevice::gemm(DType dt, GemmOp op, ALayout al, int64_t M, int64_t N, int64_t K, const void* A,
                           int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int s, const GemmExtra& ex) {
  std::vector<Acc> a;
  gemm_acc(a, dt, op, al, M, N, K, A, lda, B, ldb, C, ldc, ex);
  check(s, gemm_name("gemm", op, M, N, K), a);
  inner_->gemm(dt, op, al, M, N, K, A, lda, B, ldb, C, ldc, s, ex);
}
void RaceCheckDevice::gemm_batch(DType dt, const GemmDesc* d, int n, int s) {
  std::vector<Acc> a;
  for (int i = 0; i < n; ++i)
    gemm_acc(a, dt, d[i].op, ALayout::KMajor, d[i].M, d[i].N, d[i].K, d[i].A, d[i].lda, d[i].B, d[i].ldb, d[i].C,
             d[i].ldc, d[i].ex);
  check(s, "gemm_batch x" + std::to_string(n), a);
  inner_->gemm_batch(dt, d, n, s);
}
void RaceCheckDevice::permute_blocks(DType dt, void* dst, int64_t ldd, const void* X, int64_t ldx, int64_t nblk,
                                     int64_t m, int64_t Nr, const int32_t* dst_blk, const int32_t* colsrc, int s) {
  const int64_t es = (int64_t)dtype_size(dt);
  // destination rows follow dst_blk (device data): the whole destination panel
  check(s, "permute_blocks",
        {R(rect(X, ldx, Nr * m, nblk * m, es), "X"), R(span(dst_blk, 4 * nblk), "dst_blk"),
         R(span(colsrc, 4 * Nr), "colsrc"), W(rect(dst, ldd, Nr * m, nblk * m, es), "dst")});
  inner_->permute_blocks(dt, dst, ldd, X, ldx, nblk, m, Nr, dst_blk, colsrc, s);
}
void RaceCheckDevice::hash_rows(const void* base, int64_t ld_bytes, int64_t width_bytes, int64_t rows,
                                uint64_t* parts, int s) {
  check(s, "hash_rows", {R(rect(base, ld_bytes, width_bytes, rows, 1), "buffer"),
                         W(span(parts, sizeof(uint64_t) * kHashParts), "parts")});
  inner_->hash_rows(base, ld_bytes, width_bytes, rows, parts, s);
}

void RaceCheckDevice::row_abs_max(DType dt, const void* X, int64_t ldx, const Layout& L, double* out, int s) {
  check(s, "row_abs_max", {R(rect(X, ldx, L.n, L.rows, (int64_t)dtype_size(dt)), "X"), W(span(out, 8), "out")});
  inner_->row_abs_max(dt, X, ldx, L, out, s);
}
void RaceCheckDevice::row_abs_max_minus_i(DType dt, const void* X, int64_t ldx, const Layout& L, double* out,
                                          int s) {
  check(s, "row_abs_max_minus_i",
        {R(rect(X, ldx, L.n, L.rows, (int64_t)dtype_size(dt)), "X"), W(span(out, 8), "out")});
  inner_->row_abs_max_minus_i(dt, X, ldx, L, out, s);
}
void RaceCheckDevice::residual(DType dt, const void* A, const void* Full, const Layout& L, double* out, int s) {
  const int64_t es = (int64_t)dtype_size(dt);
  check(s, "residual",
        {R(rect(A, L.npad, L.npad, L.rows, es), "A"), R(span(Full, L.npad * L.npad * es), "inverse"),
         W(span(out, 8), "out")});
  inner_->residual(dt, A, Full, L, out, s);
}

}  // namespace gj
