// AsyncHostDevice: HostDevice's ops on per-stream worker threads (see gj/async_host_device.hpp).
#include "gj/async_host_device.hpp"

#include <atomic>
#include <chrono>
#include <cstring>

namespace gj {

void AsyncHostDevice::Fence::signal() {
  std::lock_guard<std::mutex> lk(mu);
  done = true;
  t_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
  cv.notify_all();
}

bool AsyncHostDevice::Fence::wait_for(double seconds) {
  std::unique_lock<std::mutex> lk(mu);
  return cv.wait_for(lk, std::chrono::duration<double>(seconds), [&] { return done; });
}

AsyncHostDevice::AsyncHostDevice(int nthreads, double jitter_us, uint64_t seed, double wait_timeout_s)
    : inner_(nthreads), jitter_us_(jitter_us), wait_timeout_s_(wait_timeout_s) {
  for (int s = 0; s < kNumStreams; ++s) {
    w_[s].rng.seed(seed * 0x9E3779B97F4A7C15ull + (uint64_t)s * 7919u + 1u);
    w_[s].th = std::thread([this, s] { run(s); });
  }
}

AsyncHostDevice::~AsyncHostDevice() {
  for (auto& w : w_) {
    std::lock_guard<std::mutex> lk(w.mu);
    w.stop = true;
    w.cv.notify_all();
  }
  for (auto& w : w_)
    if (w.th.joinable()) w.th.join();
}

std::string AsyncHostDevice::describe() const {
  return "host-async(" + inner_.describe() + (jitter_us_ > 0 ? ", jitter " + std::to_string((int)jitter_us_) + " us" : "") + ")";
}

void AsyncHostDevice::check_stream(int s) const {
  GJ_REQUIRE(s >= 0 && s < kNumStreams, "bad stream role");
}

void AsyncHostDevice::fail(std::exception_ptr e) {
  std::lock_guard<std::mutex> lk(err_mu_);
  if (!err_) err_ = e;
}

void AsyncHostDevice::rethrow() {
  std::exception_ptr e;
  {
    std::lock_guard<std::mutex> lk(err_mu_);
    e = err_;
  }
  if (e) std::rethrow_exception(e);
}

// Worker loop: ops run in queue order; after the first failure (any stream of this device) the
// remaining ops are skipped, except markers and fences, which still signal so that no other stream
// or host wait hangs on a failed one (a copy behind a timed-out wait_mark must not read a peer
// buffer that is not ready).
void AsyncHostDevice::run(int s) {
  Worker& w = w_[s];
  std::uniform_real_distribution<double> U(0.0, 1.0);
  for (;;) {
    Op op;
    {
      std::unique_lock<std::mutex> lk(w.mu);
      w.cv.wait(lk, [&] { return w.stop || !w.q.empty(); });
      if (w.q.empty()) return;
      op = std::move(w.q.front());
      w.q.pop_front();
    }
    bool failed;
    {
      std::lock_guard<std::mutex> lk(err_mu_);
      failed = (bool)err_;
    }
    if (failed && !op.signal) continue;  // a failed device runs nothing but its signals
    std::function<void()>& f = op.f;
    if (jitter_us_ > 0 && U(w.rng) < 0.25)
      std::this_thread::sleep_for(std::chrono::duration<double, std::micro>(U(w.rng) * jitter_us_));
    try {
      f();
    } catch (...) {
      fail(std::current_exception());
    }
  }
}

void AsyncHostDevice::enqueue(int s, std::function<void()> f, bool signal) {
  check_stream(s);
  rethrow();
  Worker& w = w_[s];
  std::lock_guard<std::mutex> lk(w.mu);
  w.q.push_back(Op{std::move(f), signal});
  w.cv.notify_one();
}

// ---- memory: releases wait for the queues (an op may still use the buffer)
void AsyncHostDevice::release(void* p) {
  for (int s = 0; s < kNumStreams; ++s) {
    auto f = std::make_shared<Fence>();
    enqueue(s, [f] { f->signal(); }, true);
    f->wait_for(1e9);
  }
  inner_.release(p);
}
void AsyncHostDevice::release_pinned(void* p) {
  for (int s = 0; s < kNumStreams; ++s) {
    auto f = std::make_shared<Fence>();
    enqueue(s, [f] { f->signal(); }, true);
    f->wait_for(1e9);
  }
  inner_.release_pinned(p);
}
void AsyncHostDevice::memset0(void* p, size_t bytes, int s) {
  enqueue(s, [=] { inner_.memset0(p, bytes, s); });
}
void AsyncHostDevice::memset2d(void* p, size_t pitch, size_t w, size_t h, int s) {
  enqueue(s, [=] { inner_.memset2d(p, pitch, w, h, s); });
}
// Copies read their source when they run (like hipMemcpyAsync from pinned memory): callers that
// pass pageable/stack memory synchronise before reusing it, as on the GPU.
void AsyncHostDevice::copy(void* dst, const void* src, size_t bytes, int s) {
  enqueue(s, [=] { inner_.copy(dst, src, bytes, s); });
}
void AsyncHostDevice::copy2d(void* dst, size_t dpitch, const void* src, size_t spitch, size_t w,
                             size_t h, int s) {
  enqueue(s, [=] { inner_.copy2d(dst, dpitch, src, spitch, w, h, s); });
}

// ---- ordering
int AsyncHostDevice::create_event(bool) {
  std::lock_guard<std::mutex> lk(ev_mu_);
  ev_last_.push_back(nullptr);
  return (int)ev_last_.size() - 1;
}
void AsyncHostDevice::record(int ev, int s) {
  auto f = std::make_shared<Fence>();
  {
    std::lock_guard<std::mutex> lk(ev_mu_);
    ev_last_.at(ev) = f;
  }
  enqueue(s, [f] { f->signal(); }, true);
}
// Like hipStreamWaitEvent: waits for the record issued last before this call (none: no wait).
void AsyncHostDevice::wait(int s, int ev) {
  std::shared_ptr<Fence> f;
  {
    std::lock_guard<std::mutex> lk(ev_mu_);
    f = ev_last_.at(ev);
  }
  if (f) wait_mark(s, f);
}
void AsyncHostDevice::sync_event(int ev) {
  std::shared_ptr<Fence> f;
  {
    std::lock_guard<std::mutex> lk(ev_mu_);
    f = ev_last_.at(ev);
  }
  if (f && !f->wait_for(wait_timeout_s_)) throw Error(Status::CommError, "host-async: event wait timed out");
  rethrow();
}
bool AsyncHostDevice::query_event(int ev) {
  std::shared_ptr<Fence> f;
  {
    std::lock_guard<std::mutex> lk(ev_mu_);
    f = ev_last_.at(ev);
  }
  if (!f) return true;
  std::lock_guard<std::mutex> lk(f->mu);
  return f->done;
}
void AsyncHostDevice::sync_stream(int s) {
  auto f = std::make_shared<Fence>();
  enqueue(s, [f] { f->signal(); }, true);
  if (!f->wait_for(wait_timeout_s_ * 4)) throw Error(Status::CommError, "host-async: stream synchronisation timed out");
  rethrow();
}
void AsyncHostDevice::sync_all() {
  for (int s = 0; s < kNumStreams; ++s) sync_stream(s);
}
float AsyncHostDevice::event_ms(int a, int b) {
  std::shared_ptr<Fence> fa, fb;
  {
    std::lock_guard<std::mutex> lk(ev_mu_);
    fa = ev_last_.at(a);
    fb = ev_last_.at(b);
  }
  if (!fa || !fb) return 0.f;
  fa->wait_for(wait_timeout_s_);
  fb->wait_for(wait_timeout_s_);
  return (float)(fb->t_ms - fa->t_ms);
}
std::shared_ptr<void> AsyncHostDevice::mark(int s) {
  auto f = std::make_shared<Fence>();
  enqueue(s, [f] { f->signal(); }, true);
  return f;
}
void AsyncHostDevice::wait_mark(int s, const std::shared_ptr<void>& h) {
  if (!h) return;
  auto f = std::static_pointer_cast<Fence>(h);
  const double to = wait_timeout_s_;
  enqueue(s, [f, to] {
    if (!f->wait_for(to))
      throw Error(Status::CommError, "host-async: a stream waited " + std::to_string((int)to) +
                                         " s for an event (missing collective on a peer, or a dependency cycle)");
  });
}
void AsyncHostDevice::occupy(int s, int, double us, int) {
  if (us > 0) enqueue(s, [us] { std::this_thread::sleep_for(std::chrono::duration<double, std::micro>(us)); });
}

// ---- kernels (arguments captured by value; pointers refer to buffers the engine keeps alive)
void AsyncHostDevice::generate(DType dt, void* X, const Layout& L, GenSpec g, int s) {
  enqueue(s, [=] { inner_.generate(dt, X, L, g, s); });
}
void AsyncHostDevice::widen(DType dt, double* dst, int64_t ldd, const void* X, int64_t ldx, int64_t rows,
                            int64_t cols, int s) {
  enqueue(s, [=] { inner_.widen(dt, dst, ldd, X, ldx, rows, cols, s); });
}
void AsyncHostDevice::upload_convert(DType dt, void* X, int64_t ldx, const double* src, int64_t src_ld,
                                     int64_t rows, int64_t cols, int s) {
  enqueue(s, [=] { inner_.upload_convert(dt, X, ldx, src, src_ld, rows, cols, s); });
}
void AsyncHostDevice::extract_neg_t(DType dt, void* Lt, int64_t ldl, const void* X, int64_t ldx,
                                    int64_t rows, int64_t col0, int64_t m, int s) {
  enqueue(s, [=] { inner_.extract_neg_t(dt, Lt, ldl, X, ldx, rows, col0, m, s); });
}
void AsyncHostDevice::add_diag(DType dt, void* A, int64_t ld, int64_t nd, double alpha, int s) {
  enqueue(s, [=] { inner_.add_diag(dt, A, ld, nd, alpha, s); });
}
void AsyncHostDevice::block_inverse(DType dt, const void* Lt, int64_t ldl, void* inv_t, double* scores,
                                    int32_t* valid, const int32_t* used, const Layout& L,
                                    double thresh, int64_t nlive, int s) {
  enqueue(s, [=] { inner_.block_inverse(dt, Lt, ldl, inv_t, scores, valid, used, L, thresh, nlive, s); });
}
bool AsyncHostDevice::block_inverse_select(DType dt, const void* Lt, int64_t ldl, void* inv_t, double* scores,
                                           int32_t* valid, const int32_t* used, const Layout& L, double thresh, int64_t nlive,
                                           const PivotSelectArgs& sel, int s) {
  if (L.m <= 16 || L.m > 128 || L.nblk <= 0) return false;  // = HostDevice's range
  enqueue(s, [=] {
    inner_.block_inverse(dt, Lt, ldl, inv_t, scores, valid, used, L, thresh, nlive, s);
    inner_.pivot_local(scores, valid, used, sel.pos, L, sel.rec, s);
    if (sel.single) pivot_global_now(sel.rec, 1, sel.t, sel.pos_w, sel.phys_at, sel.used_w, sel.seq, sel.out,
                                     sel.host_out, s);
  });
  return true;
}
void AsyncHostDevice::candidate_maxabs(DType dt, const void* Lt, int64_t ldl, double* scores, int32_t* valid,
                                       const int32_t* used, const Layout& L, double thresh, int s) {
  enqueue(s, [=] { inner_.candidate_maxabs(dt, Lt, ldl, scores, valid, used, L, thresh, s); });
}
void AsyncHostDevice::gather_candidate(DType dt, void* sel, const void* Lt, int64_t ldl, const PivotRec* rec,
                                       const Layout& L, int s) {
  enqueue(s, [=] { inner_.gather_candidate(dt, sel, Lt, ldl, rec, L, s); });
}
void AsyncHostDevice::commit_candidate(DType dt, void* inv_t, const void* inv1, const int32_t* valid1, const double* score1, double growth,
                                       PivotRec* rec, const Layout& L, int s) {
  enqueue(s, [=] { inner_.commit_candidate(dt, inv_t, inv1, valid1, score1, growth, rec, L, s); });
}
void AsyncHostDevice::pivot_local(const double* scores, const int32_t* valid, const int32_t* used,
                                  const int32_t* pos, const Layout& L, PivotRec* out, int s) {
  enqueue(s, [=] { inner_.pivot_local(scores, valid, used, pos, L, out, s); });
}
// The host polls host_out->step: every other field is written first, then a release fence, then
// the step (the GPU kernel's protocol, pivot_global_kernel).
void AsyncHostDevice::pivot_global(const PivotRec* recs, int32_t p, int32_t t, int32_t* pos,
                                   int32_t* phys_at, int32_t* used, int32_t* seq, PivotResult* out,
                                   PivotResult* host_out, int s) {
  enqueue(s, [=] { pivot_global_now(recs, p, t, pos, phys_at, used, seq, out, host_out, s); });
}
void AsyncHostDevice::pivot_global_now(const PivotRec* recs, int32_t p, int32_t t, int32_t* pos, int32_t* phys_at,
                                       int32_t* used, int32_t* seq, PivotResult* out, PivotResult* host_out,
                                       int s) {
  inner_.pivot_global(recs, p, t, pos, phys_at, used, seq, out, nullptr, s);
  if (host_out) {
    PivotResult r = *out;
    const int32_t step = r.step;
    r.step = -1;
    std::memcpy(static_cast<void*>(host_out), &r, sizeof(r));
    std::atomic_thread_fence(std::memory_order_release);
    *reinterpret_cast<volatile int32_t*>(&host_out->step) = step;
  }
}
void AsyncHostDevice::owner_edits(DType dt, void* At, int64_t ldl, const int32_t* phys, int64_t p, int64_t k,
                                  int64_t j, int64_t m, void* lrow, void* ht, const void* inv, const PieceMove& mv,
                                  int s) {
  enqueue(s, [=] { inner_.owner_edits(dt, At, ldl, phys, p, k, j, m, lrow, ht, inv, mv, s); });
}
void AsyncHostDevice::take_rows(DType dt, void* dst, int64_t ldd, void* X, int64_t ldx, const int32_t* phys,
                                int64_t p, int64_t k, int64_t col0, int64_t w, int64_t m, int s) {
  enqueue(s, [=] { inner_.take_rows(dt, dst, ldd, X, ldx, phys, p, k, col0, w, m, s); });
}
void AsyncHostDevice::sum_slices(DType dt, void* dst, const void* src, int64_t count, int64_t nslices, int s) {
  enqueue(s, [=] { inner_.sum_slices(dt, dst, src, count, nslices, s); });
}
void AsyncHostDevice::zero_unless_owner(DType dt, void* buf, int64_t count, const int32_t* phys, int64_t p, int64_t k,
                                        int s) {
  enqueue(s, [=] { inner_.zero_unless_owner(dt, buf, count, phys, p, k, s); });
}
void AsyncHostDevice::h_block(DType dt, void* R, int64_t ldr, const void* Ht, int64_t m, int s) {
  enqueue(s, [=] { inner_.h_block(dt, R, ldr, Ht, m, s); });
}
void AsyncHostDevice::gemm(DType dt, GemmOp op, ALayout al, int64_t M, int64_t N, int64_t K,
                           const void* A, int64_t lda, const void* B, int64_t ldb, void* C,
                           int64_t ldc, int s, const GemmExtra& ex) {
  enqueue(s, [=] { inner_.gemm(dt, op, al, M, N, K, A, lda, B, ldb, C, ldc, s, ex); });
}
void AsyncHostDevice::permute_blocks(DType dt, void* dst, int64_t ldd, const void* X, int64_t ldx,
                                     int64_t nblk, int64_t m, int64_t Nr, const int32_t* dst_blk,
                                     const int32_t* colsrc, int s) {
  enqueue(s, [=] { inner_.permute_blocks(dt, dst, ldd, X, ldx, nblk, m, Nr, dst_blk, colsrc, s); });
}
void AsyncHostDevice::row_abs_max_minus_i(DType dt, const void* X, int64_t ldx, const Layout& L, double* out,
                                          int s) {
  enqueue(s, [=] { inner_.row_abs_max_minus_i(dt, X, ldx, L, out, s); });
}
void AsyncHostDevice::hash_rows(const void* base, int64_t ld_bytes, int64_t width_bytes, int64_t rows,
                                uint64_t* parts, int s) {
  enqueue(s, [=] { inner_.hash_rows(base, ld_bytes, width_bytes, rows, parts, s); });
}

void AsyncHostDevice::row_abs_max(DType dt, const void* X, int64_t ldx, const Layout& L, double* out,
                                  int s) {
  enqueue(s, [=] { inner_.row_abs_max(dt, X, ldx, L, out, s); });
}
void AsyncHostDevice::residual(DType dt, const void* A, const void* Full, const Layout& L,
                               double* out, int s) {
  enqueue(s, [=] { inner_.residual(dt, A, Full, L, out, s); });
}

}  // namespace gj
