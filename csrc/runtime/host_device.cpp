// HostDevice: plain C++ reference executor of the Device interface.
//
// Used for `gj --device cpu` (the reference's CPU-only "plumbing" configuration), for CPU tests of
// the distributed protocol, and as an oracle.  It is never chosen implicitly for a GPU run.
// Streams/events are no-ops: every op completes before it returns.
#include <chrono>
#include "gj/host_device.hpp"

#include <algorithm>
#include <type_traits>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "gj/gen.hpp"

namespace gj {

namespace {

template <typename F>
void parallel_for(int64_t n, int nthreads, F f) {
  if (n <= 0) return;
  int nt = (int)std::min<int64_t>(nthreads, n);
  if (nt <= 1) {
    for (int64_t i = 0; i < n; ++i) f(i);
    return;
  }
  std::vector<std::thread> th;
  th.reserve(nt);
  for (int w = 0; w < nt; ++w)
    th.emplace_back([=, &f] {
      for (int64_t i = w; i < n; i += nt) f(i);
    });
  for (auto& t : th) t.join();
}

template <typename T>
T* tp(void* p) {
  return static_cast<T*>(p);
}
template <typename T>
const T* tp(const void* p) {
  return static_cast<const T*>(p);
}

template <typename T>
void gemm_t(GemmOp op, ALayout al, int64_t M, int64_t N, int64_t K, const T* A, int64_t lda,
            const T* B, int64_t ldb, T* C, int64_t ldc, int nthreads, const GemmExtra& ex) {
  if (ex.owner_phys) {  // owner-predicated (GemmExtra::owner_phys)
    const int64_t g = *ex.owner_phys;
    if (g < 0 || g % ex.owner_p != ex.owner_k) return;
  }
  parallel_for(M, nthreads, [&](int64_t il) {
    const int64_t i = ex.rsel_m > 0 ? ex.rsel_row(il) : il;  // GemmExtra::rsel: physical row
    bool zrow = false;
    for (int z = 0; z < ex.nzr; ++z) zrow |= (i >= ex.zr[z] && i < ex.zr[z] + ex.zh);
    std::vector<double> acc(N, 0.0);
    for (int64_t k = 0; k < K; ++k) {
      const double a = (al == ALayout::RowMajor) ? (double)A[i * lda + k] : (double)A[k * lda + i];
      if (a == 0.0) continue;
      const T* b = B + k * ldb;
      for (int64_t j = 0; j < N; ++j)
        if (!(j >= ex.skip_c0 && j < ex.skip_c1)) acc[j] += a * (double)b[j];
    }
    T* c = C + i * ldc;
    const T* ci = ex.c_in ? static_cast<const T*>(ex.c_in) + i * ex.ldc_in : c;  // GemmExtra::c_in
    const auto skip = [&](int64_t j) { return j >= ex.skip_c0 && j < ex.skip_c1; };  // GemmExtra::skip_c0/c1
    if (op == GemmOp::Acc) {
      for (int64_t j = 0; j < N; ++j)
        if (!skip(j)) c[j] = (T)((zrow || (j >= ex.zc0 && j < ex.zc1) ? 0.0 : (double)ci[j]) + acc[j]);
    } else {
      for (int64_t j = 0; j < N; ++j)
        if (!skip(j)) c[j] = (T)acc[j];
    }
    if (ex.tneg) {
      const int64_t nt = ex.tneg_cols > 0 ? std::min(ex.tneg_cols, N) : N;
      for (int64_t j = 0; j < nt; ++j)
        if (!skip(j)) static_cast<T*>(ex.tneg)[j * ex.ldtneg + i] = -c[j];
    }
  });
}

// In-place Gauss-Jordan sweep on W (m x m, row-major) with partial pivoting over not-yet-used rows.
// Returns false when singular (|pivot| < thresh).  prow[k] = pivot row of column k.
template <typename T>
bool sweep_inverse(std::vector<double>& W, int64_t m, double thresh, std::vector<int64_t>& prow) {
  std::vector<char> used(m, 0);
  for (int64_t k = 0; k < m; ++k) {
    int64_t r = -1;
    double best = -1.0;
    for (int64_t i = 0; i < m; ++i)
      if (!used[i] && std::fabs(W[i * m + k]) > best) {
        best = std::fabs(W[i * m + k]);
        r = i;
      }
    if (!(best >= thresh)) return false;  // also catches NaN
    used[r] = 1;
    prow[k] = r;
    const double inv = 1.0 / W[r * m + k];
    for (int64_t j = 0; j < m; ++j) W[r * m + j] *= inv;
    W[r * m + k] = inv;
    for (int64_t i = 0; i < m; ++i) {
      if (i == r) continue;
      const double f = W[i * m + k];
      if (f == 0.0) continue;
      for (int64_t j = 0; j < m; ++j) W[i * m + j] -= f * W[r * m + j];
      W[i * m + k] = -f * inv;
    }
  }
  return true;
}

}  // namespace

HostDevice::HostDevice(int nthreads) {
  nthreads_ = nthreads > 0 ? nthreads : (int)std::max(1u, std::thread::hardware_concurrency());
}

std::string HostDevice::describe() const {
  return "host(" + std::to_string(nthreads_) + " threads)";
}

void* HostDevice::alloc(size_t bytes) {
  void* p = nullptr;
  if (posix_memalign(&p, 64, std::max<size_t>(bytes, 64)) != 0 || !p)
    throw Error(Status::NoMemory, "host allocation failed");
  return p;
}
void HostDevice::release(void* p) { std::free(p); }
void* HostDevice::alloc_pinned(size_t bytes) { return alloc(bytes); }
void HostDevice::release_pinned(void* p) { std::free(p); }
size_t HostDevice::free_memory() const { return ~size_t(0); }
void HostDevice::memset0(void* p, size_t bytes, int) { std::memset(p, 0, bytes); }
void HostDevice::memset2d(void* p, size_t pitch, size_t w, size_t h, int) {
  for (size_t r = 0; r < h; ++r) std::memset(static_cast<char*>(p) + r * pitch, 0, w);
}
void HostDevice::copy(void* dst, const void* src, size_t bytes, int) {
  if (dst != src) std::memmove(dst, src, bytes);
}
void HostDevice::copy2d(void* dst, size_t dpitch, const void* src, size_t spitch, size_t w, size_t h,
                        int) {
  for (size_t r = 0; r < h; ++r)
    std::memmove(static_cast<char*>(dst) + r * dpitch, static_cast<const char*>(src) + r * spitch, w);
}

// Events carry the host time at which they were recorded (all work before them is complete).
int HostDevice::create_event(bool) {
  ev_time_.push_back(0.0);
  return nev_++;
}
void HostDevice::record(int ev, int) {
  ev_time_[ev] = std::chrono::duration<double, std::milli>(
                     std::chrono::steady_clock::now().time_since_epoch()).count();
}
void HostDevice::wait(int, int) {}
void HostDevice::sync_event(int) {}
void HostDevice::sync_stream(int) {}
void HostDevice::sync_all() {}
float HostDevice::event_ms(int a, int b) { return (float)(ev_time_[b] - ev_time_[a]); }

void HostDevice::generate(DType dt, void* X, const Layout& L, GenSpec g, int) {
  parallel_for(L.rows, nthreads_, [&](int64_t r) {
    const int64_t gr = L.global_row(r);
    for (int64_t j = 0; j < L.npad; ++j) {
      const double v = gen_value((int)g.kind, g.seed, L.n, gr, j);
      if (dt == DType::F64)
        tp<double>(X)[r * L.npad + j] = v;
      else
        tp<float>(X)[r * L.npad + j] = (float)v;
    }
  });
}

void HostDevice::widen(DType dt, double* dst, int64_t ldd, const void* X, int64_t ldx, int64_t rows,
                       int64_t cols, int) {
  for (int64_t r = 0; r < rows; ++r)
    for (int64_t j = 0; j < cols; ++j)
      dst[r * ldd + j] = dt == DType::F64 ? tp<double>(X)[r * ldx + j] : (double)tp<float>(X)[r * ldx + j];
}

void HostDevice::upload_convert(DType dt, void* X, int64_t ldx, const double* src, int64_t src_ld,
                                int64_t rows, int64_t cols, int) {
  for (int64_t r = 0; r < rows; ++r)
    for (int64_t j = 0; j < cols; ++j) {
      if (dt == DType::F64)
        tp<double>(X)[r * ldx + j] = src[r * src_ld + j];
      else
        tp<float>(X)[r * ldx + j] = (float)src[r * src_ld + j];
    }
}

void HostDevice::extract_neg_t(DType dt, void* Lt, int64_t ldl, const void* X, int64_t ldx,
                               int64_t rows, int64_t col0, int64_t m, int) {
  for (int64_t r = 0; r < rows; ++r)
    for (int64_t c = 0; c < m; ++c) {
      if (dt == DType::F64)
        tp<double>(Lt)[c * ldl + r] = -tp<double>(X)[r * ldx + col0 + c];
      else
        tp<float>(Lt)[c * ldl + r] = -tp<float>(X)[r * ldx + col0 + c];
    }
}

void HostDevice::add_diag(DType dt, void* A, int64_t ld, int64_t nd, double alpha, int) {
  for (int64_t i = 0; i < nd; ++i) {
    if (dt == DType::F64)
      tp<double>(A)[i * ld + i] += alpha;
    else
      tp<float>(A)[i * ld + i] += (float)alpha;
  }
}

void HostDevice::block_inverse(DType dt, const void* Lt, int64_t ldl, void* inv_t, double* scores,
                               int32_t* valid, const int32_t* used, const Layout& L, double thresh, int64_t nlive,
                               int) {
  const int64_t m = L.m;
  parallel_for(L.nblk, nthreads_, [&](int64_t b) {
    const int64_t g = L.global_block(b);
    if (used[g]) {
      valid[b] = 0;
      scores[b] = 0;
      return;
    }
    std::vector<double> W(m * m);
    for (int64_t i = 0; i < m; ++i)
      for (int64_t j = 0; j < m; ++j)
        W[i * m + j] = (dt == DType::F64) ? -tp<double>(Lt)[j * ldl + b * m + i]
                                          : -(double)tp<float>(Lt)[j * ldl + b * m + i];
    std::vector<int64_t> prow(m);
    const bool ok = sweep_inverse<double>(W, m, thresh, prow);
    if (!ok) {
      valid[b] = 0;
      scores[b] = 0;
      return;
    }
    double sc = 0.0;
    for (int64_t i = 0; i < m; ++i) {
      double s = 0.0;
      for (int64_t j = 0; j < m; ++j) s += std::fabs(W[i * m + j]);
      sc = std::max(sc, s);
    }
    valid[b] = std::isfinite(sc) ? 1 : 0;
    scores[b] = sc;
    // Y[k][prow[u]] = W[prow[k]][u]; inv_t[j*m + i] = Y[i][j]
    for (int64_t k = 0; k < m; ++k)
      for (int64_t u = 0; u < m; ++u) {
        const double y = W[prow[k] * m + u];
        const int64_t idx = b * m * m + prow[u] * m + k;
        if (dt == DType::F64)
          tp<double>(inv_t)[idx] = y;
        else
          tp<float>(inv_t)[idx] = (float)y;
      }
  });
}

// The fused candidate-inverse + selection launch of the GPU (Device::block_inverse_select), for the
// same kernel family range (16 < m <= 128), so the CPU executes the GPU's op sequence.
bool HostDevice::block_inverse_select(DType dt, const void* Lt, int64_t ldl, void* inv_t, double* scores,
                                      int32_t* valid, const int32_t* used, const Layout& L, double thresh, int64_t nlive,
                                      const PivotSelectArgs& sel, int s) {
  if (L.m <= 16 || L.m > 128 || L.nblk <= 0) return false;
  block_inverse(dt, Lt, ldl, inv_t, scores, valid, used, L, thresh, nlive, s);
  pivot_local(scores, valid, used, sel.pos, L, sel.rec, s);
  if (sel.single)
    pivot_global(sel.rec, 1, sel.t, sel.pos_w, sel.phys_at, sel.used_w, sel.seq, sel.out, sel.host_out, s);
  return true;
}

void HostDevice::candidate_maxabs(DType dt, const void* Lt, int64_t ldl, double* scores, int32_t* valid,
                                  const int32_t* used, const Layout& L, double thresh, int) {
  const int64_t m = L.m;
  for (int64_t b = 0; b < L.nblk; ++b) {
    if (used[L.global_block(b)]) {
      valid[b] = 0;
      scores[b] = 0;
      continue;
    }
    double mx = 0.0;
    for (int64_t c = 0; c < m; ++c)
      for (int64_t i = 0; i < m; ++i) {
        const int64_t idx = c * ldl + b * m + i;
        const double v = dt == DType::F64 ? tp<double>(Lt)[idx] : (double)tp<float>(Lt)[idx];
        mx = std::max(mx, std::fabs(v));
      }
    scores[b] = -mx;
    valid[b] = (mx >= thresh && std::isfinite(mx)) ? 1 : 0;
  }
}

void HostDevice::gather_candidate(DType dt, void* sel, const void* Lt, int64_t ldl, const PivotRec* rec,
                                  const Layout& L, int) {
  const int64_t m = L.m;
  const bool ok = rec->valid != 0;
  const int64_t b = ok ? rec->phys / L.p : 0;
  for (int64_t c = 0; c < m; ++c)
    for (int64_t i = 0; i < m; ++i) {
      const int64_t src = c * ldl + b * m + i, dst = c * m + i;
      if (dt == DType::F64)
        tp<double>(sel)[dst] = ok ? tp<double>(Lt)[src] : (c == i ? -1.0 : 0.0);
      else
        tp<float>(sel)[dst] = ok ? tp<float>(Lt)[src] : (c == i ? -1.0f : 0.0f);
    }
}

void HostDevice::commit_candidate(DType dt, void* inv_t, const void* inv1, const int32_t* valid1, const double* score1, double growth, PivotRec* rec,
                                  const Layout& L, int) {
  // growth guard: ||inv(W)||_inf * max|W| (score1 * -rec->score) above the bound counts as singular
  if (!rec->valid || !valid1[0] || (growth > 0 && !(score1[0] * -rec->score <= growth))) {
    rec->valid = 0;
    return;
  }
  const size_t blk = (size_t)L.m * L.m * dtype_size(dt);
  std::memcpy(static_cast<char*>(inv_t) + (size_t)(rec->phys / L.p) * blk, inv1, blk);
}

void HostDevice::pivot_local(const double* scores, const int32_t* valid, const int32_t* used,
                             const int32_t* pos, const Layout& L, PivotRec* out, int) {
  PivotRec best = pivot_invalid();
  for (int64_t b = 0; b < L.nblk; ++b) {
    const int64_t g = L.global_block(b);
    if (used[g] || !valid[b]) continue;
    PivotRec c;
    c.score = scores[b];
    c.logical = pos[g];
    c.phys = (int32_t)g;
    c.valid = 1;
    c.pad_ = 0;
    if (pivot_better(c, best, (int32_t)L.p)) best = c;
  }
  *out = best;
}

void HostDevice::pivot_global(const PivotRec* recs, int32_t p, int32_t t, int32_t* pos,
                              int32_t* phys_at, int32_t* used, int32_t* seq, PivotResult* out,
                              PivotResult* host_out, int) {
  PivotRec best = pivot_invalid();
  for (int32_t q = 0; q < p; ++q)
    if (pivot_better(recs[q], best, p)) best = recs[q];
  PivotResult r{};
  r.step = t;
  if (best.valid) {
    r.found = 1;
    r.phys = best.phys;
    r.owner = best.phys % p;
    r.logical = best.logical;
    r.score = best.score;
    pivot_commit(t, best.phys, pos, phys_at, used, seq);
  } else {
    seq[t] = -1;  // as the GPU kernel: the step's owner-predicated launches stay no-ops
    r.found = 0;
    r.phys = -1;
    r.owner = -1;
    r.logical = -1;
  }
  *out = r;
  if (host_out) *host_out = r;
}

void HostDevice::owner_edits(DType dt, void* At, int64_t ldl, const int32_t* phys, int64_t p, int64_t k,
                             int64_t j, int64_t m, void* lrow, void* ht, const void* inv, const PieceMove& mv,
                             int s) {
  const int64_t g = *phys;
  if (g < 0 || g % p != k) return;
  if (mv.w > 0) take_rows(dt, mv.dst, mv.ldd, mv.X, mv.ldx, phys, p, k, mv.col0, mv.w, m, s);
  if (mv.eye) {
    const size_t es = dtype_size(dt);
    for (int64_t r = 0; r < m; ++r)
      for (int64_t c = 0; c < m; ++c) {
        char* e = static_cast<char*>(mv.eye) + (r * mv.ld_eye + c) * (int64_t)es;
        if (dt == DType::F64) *reinterpret_cast<double*>(e) = r == c ? 1.0 : 0.0;
        else *reinterpret_cast<float*>(e) = r == c ? 1.0f : 0.0f;
      }
  }
  const int64_t row0 = (g / p) * m;
  auto run = [&](auto* a, auto* lr, auto* h, const auto* iv) {
    using T = std::remove_pointer_t<decltype(a)>;
    for (int64_t kk = 0; kk < (j + 1) * m; ++kk)
      for (int64_t c = 0; c < m; ++c) {
        T& x = a[kk * ldl + row0 + c];
        if (kk < j * m) lr[kk * m + c] = x;
        x = (kk - j * m == c) ? T(1) : T(0);
      }
    for (int64_t e = 0; e < m * m; ++e) h[e] = iv[(g / p) * m * m + e];
  };
  if (dt == DType::F64)
    run(static_cast<double*>(At), static_cast<double*>(lrow), static_cast<double*>(ht), static_cast<const double*>(inv));
  else
    run(static_cast<float*>(At), static_cast<float*>(lrow), static_cast<float*>(ht), static_cast<const float*>(inv));
}

void HostDevice::take_rows(DType dt, void* dst, int64_t ldd, void* X, int64_t ldx, const int32_t* phys, int64_t p,
                           int64_t k, int64_t col0, int64_t w, int64_t m, int) {
  const int64_t g = *phys;
  if (g < 0 || g % p != k || w <= 0) return;
  const size_t es = dtype_size(dt);
  const int64_t row0 = (g / p) * m;
  for (int64_t r = 0; r < m; ++r) {
    char* src = static_cast<char*>(X) + ((row0 + r) * ldx + col0) * (int64_t)es;
    std::memcpy(static_cast<char*>(dst) + r * ldd * (int64_t)es, src, (size_t)w * es);
    std::memset(src, 0, (size_t)w * es);
  }
}

void HostDevice::sum_slices(DType dt, void* dst, const void* src, int64_t count, int64_t nslices, int) {
  auto run = [&](auto* d, const auto* x) {
    using T = std::remove_pointer_t<decltype(d)>;
    for (int64_t i = 0; i < count; ++i) {
      T acc = x[i];
      for (int64_t q = 1; q < nslices; ++q) acc += x[q * count + i];
      d[i] = acc;
    }
  };
  if (dt == DType::F64) run(static_cast<double*>(dst), static_cast<const double*>(src));
  else run(static_cast<float*>(dst), static_cast<const float*>(src));
}

void HostDevice::zero_unless_owner(DType dt, void* buf, int64_t count, const int32_t* phys, int64_t p, int64_t k,
                                   int) {
  const int64_t g = *phys;
  if (g >= 0 && g % p == k) return;
  std::memset(buf, 0, (size_t)count * dtype_size(dt));
}

void HostDevice::h_block(DType dt, void* R, int64_t ldr, const void* Ht, int64_t m, int) {
  for (int64_t i = 0; i < m; ++i)
    for (int64_t j = 0; j < m; ++j) {
      if (dt == DType::F64)
        tp<double>(R)[i * ldr + j] = tp<double>(Ht)[j * m + i];
      else
        tp<float>(R)[i * ldr + j] = tp<float>(Ht)[j * m + i];
    }
}

void HostDevice::gemm(DType dt, GemmOp op, ALayout al, int64_t M, int64_t N, int64_t K,
                      const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc,
                      int, const GemmExtra& ex) {
  if (M <= 0 || N <= 0) return;
  if (dt == DType::F64)
    gemm_t<double>(op, al, M, N, K, tp<double>(A), lda, tp<double>(B), ldb, tp<double>(C), ldc,
                   nthreads_, ex);
  else
    gemm_t<float>(op, al, M, N, K, tp<float>(A), lda, tp<float>(B), ldb, tp<float>(C), ldc,
                  nthreads_, ex);
}

void HostDevice::permute_blocks(DType dt, void* dst, int64_t ldd, const void* X, int64_t ldx,
                                int64_t nblk, int64_t m, int64_t Nr, const int32_t* dst_blk,
                                const int32_t* colsrc, int) {
  const size_t es = dtype_size(dt);
  parallel_for(nblk * m, nthreads_, [&](int64_t row) {
    const int64_t b = row / m, r = row % m;
    char* d = static_cast<char*>(dst) + ((int64_t)dst_blk[b] * m + r) * ldd * es;
    const char* s = static_cast<const char*>(X) + (b * m + r) * ldx * es;
    for (int64_t c = 0; c < Nr; ++c)
      std::memcpy(d + c * m * es, s + (int64_t)colsrc[c] * m * es, m * es);
  });
}

void HostDevice::row_abs_max_minus_i(DType dt, const void* X, int64_t ldx, const Layout& L, double* out,
                                     int) {
  double mx = 0.0;
  for (int64_t r = 0; r < L.rows; ++r) {
    const int64_t gr = L.global_row(r);
    if (gr >= L.n) continue;
    double s = 0.0;
    for (int64_t j = 0; j < L.n; ++j) {
      const double v = dt == DType::F64 ? tp<double>(X)[r * ldx + j] : (double)tp<float>(X)[r * ldx + j];
      s += std::fabs(v - (j == gr ? 1.0 : 0.0));
    }
    mx = std::max(mx, s);
  }
  out[0] = mx;
}

void HostDevice::hash_rows(const void* base, int64_t ld_bytes, int64_t width_bytes, int64_t rows,
                           uint64_t* parts, int) {
  const int64_t ww = width_bytes / 4;
  uint64_t h = 0;
  for (int64_t r = 0; r < rows; ++r)
    for (int64_t w = 0; w < ww; ++w) {
      uint32_t v;
      std::memcpy(&v, static_cast<const char*>(base) + r * ld_bytes + 4 * w, 4);
      h += hash_term(v, (uint64_t)(r * ww + w));
    }
  parts[0] = h;
  for (int g = 1; g < kHashParts; ++g) parts[g] = 0;
}

void HostDevice::row_abs_max(DType dt, const void* X, int64_t ldx, const Layout& L, double* out,
                             int) {
  double mx = 0.0;
  for (int64_t r = 0; r < L.rows; ++r) {
    if (L.global_row(r) >= L.n) continue;
    double s = 0.0;
    for (int64_t j = 0; j < L.n; ++j)
      s += std::fabs(dt == DType::F64 ? tp<double>(X)[r * ldx + j] : (double)tp<float>(X)[r * ldx + j]);
    mx = std::max(mx, s);
  }
  out[0] = mx;
}

void HostDevice::residual(DType dt, const void* A, const void* Full, const Layout& L, double* out,
                          int) {
  const int64_t np = L.npad;
  std::vector<double> rowres(L.rows, 0.0);
  parallel_for(L.rows, nthreads_, [&](int64_t r) {
    const int64_t gr = L.global_row(r);
    if (gr >= L.n) return;
    std::vector<double> acc(L.n, 0.0);
    for (int64_t k = 0; k < L.n; ++k) {
      const double a = dt == DType::F64 ? tp<double>(A)[r * np + k] : (double)tp<float>(A)[r * np + k];
      if (a == 0.0) continue;
      for (int64_t j = 0; j < L.n; ++j)
        acc[j] += a * (dt == DType::F64 ? tp<double>(Full)[k * np + j]
                                        : (double)tp<float>(Full)[k * np + j]);
    }
    double s = 0.0;
    for (int64_t j = 0; j < L.n; ++j) s += std::fabs(acc[j] - (j == gr ? 1.0 : 0.0));
    rowres[r] = s;
  });
  double mx = 0.0;
  for (double v : rowres) mx = std::max(mx, v);
  out[0] = mx;
}

}  // namespace gj
