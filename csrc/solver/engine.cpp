// Distributed Gauss-Jordan engine — see gj/engine.hpp for the design summary.
//
// Reference parity map (main.cpp line numbers):
//   norm()              :643-667  -> norm_inf() (global max instead of the local strip norm)
//   pivot search        :1039-1066 -> select(): Device::block_inverse + pivot_local
//   MPI_Allreduce(piv)  :1074     -> Comm::allgather of 32-B records + Device::pivot_global
//   singular exit       :1075-1083 -> Status::Singular on every rank at the same step
//   gather_row + Bcast  :1093-1097 -> normalize_and_bcast(): owner normalises, chunked broadcast
//   row swap            :1100-1131 -> none per step (logical bookkeeping) + finalize() once
//   normalise (replicated on all ranks) :1132-1159 -> once, on the owner, as an MFMA GEMM
//   eliminate           :1165-1194 -> Device::gemm(Acc) over every local row, chunked by columns
#include "gj/engine.hpp"

#include <algorithm>
#include <chrono>
#include <cstring>

namespace gj {

namespace {
double now_s() {
  using clk = std::chrono::steady_clock;
  return std::chrono::duration<double>(clk::now().time_since_epoch()).count();
}
}  // namespace

Engine::Engine(Device& dev, Comm& comm, int64_t n, int64_t m, const SolveOptions& opt)
    : dev_(dev), comm_(comm), opt_(opt) {
  GJ_REQUIRE(n > 0 && m > 0, "n and m must be positive");
  L_ = Layout::make(n, m, comm.size(), comm.rank());
  GJ_REQUIRE(L_.Nr < (int64_t(1) << 31), "too many block rows");

  // Column chunk plan: fixed partition of the Nr block columns.
  int64_t target_cols = opt_.chunk_cols;
  if (target_cols <= 0) target_cols = std::max<int64_t>(2048, (L_.npad + 7) / 8);
  int64_t cw = std::max<int64_t>(1, target_cols / m);
  for (int64_t b = 0; b < L_.Nr; b += cw) {
    cb0_.push_back(b);
    cb1_.push_back(std::min(L_.Nr, b + cw));
  }
  chunk_of_.resize(L_.Nr);
  for (size_t c = 0; c < cb0_.size(); ++c)
    for (int64_t b = cb0_[c]; b < cb1_[c]; ++b) chunk_of_[b] = (int64_t)c;

  alloc_buffers();
}

Engine::~Engine() { free_buffers(); }

int64_t Engine::real_local_rows() const {
  if (L_.nblk == 0) return 0;
  const int64_t last_global_block = L_.global_block(L_.nblk - 1);
  return L_.rows - (last_global_block == L_.Nr - 1 ? (L_.m - L_.l_h) : 0);
}

void Engine::alloc_buffers() {
  const int64_t m = L_.m, rows = std::max<int64_t>(L_.rows, 1), npad = L_.npad;
  const size_t es = esz();
  const size_t panel = (size_t)rows * npad * es;
  const size_t need = 2 * panel + 2 * (size_t)m * rows * es + 2 * (size_t)m * npad * es +
                      (size_t)std::max<int64_t>(L_.nblk, 1) * m * m * es;
  if (dev_.on_gpu()) {
    size_t avail = dev_.free_memory();
    if (need + (64u << 20) > avail)
      throw Error(Status::NoMemory, "not enough device memory: need " + std::to_string(need) +
                                        " bytes, have " + std::to_string(avail));
  }
  X_ = dev_.alloc(panel);
  out_ = dev_.alloc(panel);
  for (int i = 0; i < 2; ++i) {
    Lt_[i] = dev_.alloc((size_t)m * rows * es);
    R_[i] = dev_.alloc((size_t)m * npad * es);
    Ht_[i] = dev_.alloc((size_t)m * m * es);
  }
  inv_ = dev_.alloc((size_t)std::max<int64_t>(L_.nblk, 1) * m * m * es);
  scores_ = static_cast<double*>(dev_.alloc(sizeof(double) * std::max<int64_t>(L_.nblk, 1)));
  valid_ = static_cast<int32_t*>(dev_.alloc(sizeof(int32_t) * std::max<int64_t>(L_.nblk, 1)));
  pos_ = static_cast<int32_t*>(dev_.alloc(sizeof(int32_t) * L_.Nr));
  phys_at_ = static_cast<int32_t*>(dev_.alloc(sizeof(int32_t) * L_.Nr));
  used_ = static_cast<int32_t*>(dev_.alloc(sizeof(int32_t) * L_.Nr));
  seq_ = static_cast<int32_t*>(dev_.alloc(sizeof(int32_t) * L_.Nr));
  myrec_ = static_cast<PivotRec*>(dev_.alloc(sizeof(PivotRec)));
  recs_ = static_cast<PivotRec*>(dev_.alloc(sizeof(PivotRec) * L_.p));
  piv_dev_ = static_cast<PivotResult*>(dev_.alloc(sizeof(PivotResult)));
  dscratch_ = static_cast<double*>(dev_.alloc(sizeof(double) * 64));
  ihost_len_ = std::max<int64_t>(L_.Nr, 16) * 2 + 16;
  iscratch_ = static_cast<int32_t*>(dev_.alloc(sizeof(int32_t) * ihost_len_));
  piv_host_ = static_cast<PivotResult*>(dev_.alloc_pinned(sizeof(PivotResult) * 2));
  ihost_ = static_cast<int32_t*>(dev_.alloc_pinned(sizeof(int32_t) * ihost_len_));
  dhost_ = static_cast<double*>(dev_.alloc_pinned(sizeof(double) * 64));

  ev_L_ = dev_.create_event();
  ev_main_ = dev_.create_event();
  ev_comm_ = dev_.create_event();
  for (int i = 0; i < 2; ++i) {
    ev_sel_[i] = dev_.create_event();
    ev_adj_[i] = dev_.create_event();
    for (size_t c = 0; c < cb0_.size(); ++c) ev_b_[i].push_back(dev_.create_event());
  }
  for (size_t c = 0; c < cb0_.size(); ++c) ev_c_.push_back(dev_.create_event());
}

void Engine::free_buffers() {
  void* dptrs[] = {X_, out_, Lt_[0], Lt_[1], R_[0], R_[1], Ht_[0], Ht_[1], inv_, scores_, valid_,
                   pos_, phys_at_, used_, seq_, myrec_, recs_, piv_dev_, dscratch_, iscratch_};
  for (void* p : dptrs)
    if (p) dev_.release(p);
  if (piv_host_) dev_.release_pinned(piv_host_);
  if (ihost_) dev_.release_pinned(ihost_);
  if (dhost_) dev_.release_pinned(dhost_);
}

void Engine::dbg_sync() {
  if (opt_.sync_debug) dev_.sync_all();
}

// ---------------------------------------------------------------- input
void Engine::generate(GenSpec g) {
  dev_.generate(opt_.dtype, X_, L_, g, S_MAIN);
  dev_.sync_stream(S_MAIN);
  solved_ = false;
}

void Engine::upload_local_rows(const double* host, int64_t ld) {
  GenSpec z;
  z.kind = GenKind::Zero;  // zero + identity on the padded diagonal
  dev_.generate(opt_.dtype, X_, L_, z, S_MAIN);
  const int64_t real = real_local_rows();
  const int64_t n = L_.n;
  if (real > 0) {
    // stream the rows through a bounded staging buffer (<= 256 MiB)
    const int64_t rows_per = std::max<int64_t>(1, (int64_t(256) << 20) / (n * 8));
    const int64_t chunk = std::min(rows_per, real);
    double* stage = static_cast<double*>(dev_.alloc(sizeof(double) * chunk * n));
    for (int64_t r0 = 0; r0 < real; r0 += chunk) {
      const int64_t nr = std::min(chunk, real - r0);
      dev_.copy2d(stage, n * 8, host + r0 * ld, ld * 8, n * 8, nr, S_MAIN);
      dev_.upload_convert(opt_.dtype, elem(X_, r0 * L_.npad), L_.npad, stage, n, nr, n, S_MAIN);
      dev_.sync_stream(S_MAIN);
    }
    dev_.release(stage);
  }
  dev_.sync_stream(S_MAIN);
  solved_ = false;
}

double Engine::norm_inf() {
  dev_.row_abs_max(opt_.dtype, X_, L_.npad, L_, dscratch_, S_MAIN);
  dev_.copy(dhost_, dscratch_, sizeof(double), S_MAIN);
  dev_.sync_stream(S_MAIN);
  return comm_.host_max(dev_, dhost_[0]);
}

// ---------------------------------------------------------------- pivot search (SIDE stream)
void Engine::select(int64_t t) {
  const int par = (int)(t & 1);
  const double thresh = opt_.eps * norm_a_;
  if (L_.nblk > 0)
    dev_.block_inverse(opt_.dtype, Lt_[par], L_.rows, inv_, scores_, valid_, used_, L_, thresh,
                       S_SIDE);
  dev_.pivot_local(scores_, valid_, used_, pos_, L_, myrec_, S_SIDE);
  comm_.allgather(dev_, myrec_, recs_, sizeof(PivotRec), S_SIDE);
  dev_.pivot_global(recs_, (int32_t)L_.p, (int32_t)t, pos_, phys_at_, used_, seq_, piv_dev_, S_SIDE);
  dev_.copy(&piv_host_[par], piv_dev_, sizeof(PivotResult), S_SIDE);
  dev_.record(ev_sel_[par], S_SIDE);
  dbg_sync();
}

// Owner of the pivot row: keep H = inv(P) (transposed) for the normalisation of step t.
void Engine::post_select(int64_t t, const PivotResult& r) {
  const int par = (int)(t & 1);
  if (r.owner == L_.k) {
    const int64_t sl = r.phys / L_.p;  // local block index of s_t
    const int64_t m = L_.m;
    dev_.copy(Ht_[par], elem(inv_, sl * m * m), (size_t)m * m * esz(), S_SIDE);
  }
  dev_.record(ev_adj_[par], S_SIDE);
  dbg_sync();
}

// COMM stream: chunk by chunk, the owner forms R_t = H * X[s_t, :] (block t -> H) and every rank
// takes part in the broadcast of that chunk.
void Engine::normalize_and_bcast(int64_t t, const PivotResult& r, bool wait_main) {
  const int par = (int)(t & 1);
  const int64_t m = L_.m;
  const bool owner = (r.owner == L_.k);
  const int64_t C = (int64_t)cb0_.size();
  const int64_t start = chunk_of_[t];
  dev_.wait(S_COMM, ev_adj_[par]);
  for (int64_t i = 0; i < C; ++i) {
    const int64_t c = (start + i) % C;
    const int64_t c0 = cb0_[c] * m, c1 = cb1_[c] * m, W = c1 - c0;
    void* Rc = elem(R_[par], m * c0);
    if (owner) {
      if (wait_main) dev_.wait(S_COMM, ev_c_[c]);
      const int64_t sl = r.phys / L_.p;
      dev_.gemm(opt_.dtype, GemmOp::Store, ALayout::KMajor, m, W, m, Ht_[par], m,
                elem(X_, sl * m * L_.npad + c0), L_.npad, Rc, W, S_COMM);
      if (t >= cb0_[c] && t < cb1_[c])
        dev_.h_block(opt_.dtype, elem(Rc, t * m - c0), W, Ht_[par], m, S_COMM);
    }
    comm_.bcast(dev_, Rc, (size_t)m * W * esz(), r.owner, S_COMM);
    dev_.record(ev_b_[par][c], S_COMM);
  }
  dbg_sync();
}

// ---------------------------------------------------------------- solve
SolveStats Engine::solve() {
  GJ_REQUIRE(!solved_, "solve(): input panel already consumed; load the matrix again");
  SolveStats st;
  const int64_t m = L_.m, Nr = L_.Nr, rows = L_.rows, npad = L_.npad;
  const int64_t C = (int64_t)cb0_.size();

  comm_.barrier(dev_);
  const double t_begin = now_s();

  norm_a_ = norm_inf();
  if (std::fabs(norm_a_) < opt_.eps) {  // reference main.cpp:782 second clause
    st.status = Status::Singular;
    st.singular_step = 0;
    st.seconds = now_s() - t_begin;
    solved_ = true;
    return st;
  }

  // book-keeping arrays: pos = phys_at = identity, used = 0
  for (int64_t i = 0; i < Nr; ++i) ihost_[i] = (int32_t)i;
  dev_.copy(pos_, ihost_, sizeof(int32_t) * Nr, S_SIDE);
  dev_.copy(phys_at_, ihost_, sizeof(int32_t) * Nr, S_SIDE);
  dev_.memset0(used_, sizeof(int32_t) * Nr, S_SIDE);
  dev_.memset0(seq_, sizeof(int32_t) * Nr, S_SIDE);
  dev_.sync_stream(S_SIDE);

  st.pivots.assign(Nr, -1);
  double host_wait = 0;

  // ---- prologue: step 0 selection and broadcast
  if (rows > 0) dev_.extract_neg_t(opt_.dtype, Lt_[0], rows, X_, npad, rows, 0, m, S_MAIN);
  dev_.record(ev_L_, S_MAIN);
  dev_.wait(S_SIDE, ev_L_);
  select(0);
  {
    const double w0 = now_s();
    dev_.sync_event(ev_sel_[0]);
    host_wait += now_s() - w0;
  }
  PivotResult r = piv_host_[0];
  PivotResult piv[2];
  piv[0] = r;
  if (!r.found) {
    dev_.sync_all();
    st.status = Status::Singular;
    st.singular_step = 0;
    st.seconds = now_s() - t_begin;
    solved_ = true;
    return st;
  }
  st.pivots[0] = r.phys;
  if (r.owner == L_.k) st.bcast_bytes += double(m) * npad * esz();
  post_select(0, r);
  normalize_and_bcast(0, r, /*wait_main=*/false);

  // ---- main loop
  for (int64_t t = 0; t < Nr; ++t) {
    const int cur = (int)(t & 1), nx = cur ^ 1;
    const bool has_next = (t + 1 < Nr);
    dev_.wait(S_MAIN, ev_adj_[cur]);
    // Step t on every local row i:  X[i, :] += (-L_i) R_t, except
    //   * block column t enters as 0:   X[i, t] = -L_i H            (no I + H cancellation)
    //   * the pivot rows s_t are overwritten with R_t (owner only).
    const int64_t pr0 = (piv[cur].owner == L_.k) ? (piv[cur].phys / L_.p) * m : -1;
    const int64_t tz0 = t * m, tz1 = tz0 + m;

    if (has_next) {
      // (a) look-ahead column block t+1 first
      const int64_t b = t + 1, cb = chunk_of_[b];
      const int64_t c0 = cb0_[cb] * m, W = (cb1_[cb] - cb0_[cb]) * m;
      dev_.wait(S_MAIN, ev_b_[cur][cb]);
      if (rows > 0) {
        dev_.gemm(opt_.dtype, GemmOp::Acc, ALayout::KMajor, rows, m, m, Lt_[cur], rows,
                  elem(R_[cur], m * c0 + (b * m - c0)), W, elem(X_, b * m), npad, S_MAIN, 0, 0, pr0);
        dev_.extract_neg_t(opt_.dtype, Lt_[nx], rows, X_, npad, rows, b * m, m, S_MAIN);
      }
      dev_.record(ev_L_, S_MAIN);
      dbg_sync();
      // (b) pivot search for step t+1 on the SIDE stream
      dev_.wait(S_SIDE, ev_L_);
      select(t + 1);
    }

    // (c) the rest of step t's update, chunk by chunk
    const int64_t start = has_next ? chunk_of_[t + 1] : 0;
    for (int64_t i = 0; i < C; ++i) {
      const int64_t c = (start + i) % C;
      const int64_t c0 = cb0_[c] * m, c1 = cb1_[c] * m, W = c1 - c0;
      dev_.wait(S_MAIN, ev_b_[cur][c]);
      int64_t ra[2], rb[2], nr = 0;
      if (has_next && (t + 1) >= cb0_[c] && (t + 1) < cb1_[c]) {
        const int64_t x0 = (t + 1) * m, x1 = x0 + m;
        if (x0 > c0) { ra[nr] = c0; rb[nr] = x0; ++nr; }
        if (c1 > x1) { ra[nr] = x1; rb[nr] = c1; ++nr; }
      } else {
        ra[0] = c0; rb[0] = c1; nr = 1;
      }
      if (rows > 0)
        for (int64_t q = 0; q < nr; ++q)
          dev_.gemm(opt_.dtype, GemmOp::Acc, ALayout::KMajor, rows, rb[q] - ra[q], m, Lt_[cur], rows,
                    elem(R_[cur], m * c0 + (ra[q] - c0)), W, elem(X_, ra[q]), npad, S_MAIN,
                    tz0 - ra[q], tz1 - ra[q], pr0);
      dev_.record(ev_c_[c], S_MAIN);
    }
    dbg_sync();

    if (has_next) {
      // (d) wait (host) for the pivot of step t+1 — normally long finished behind (c)
      const double w0 = now_s();
      dev_.sync_event(ev_sel_[nx]);
      host_wait += now_s() - w0;
      r = piv_host_[nx];
      piv[nx] = r;
      if (!r.found) {
        dev_.sync_all();
        st.status = Status::Singular;
        st.singular_step = t + 1;
        st.host_wait_ms = host_wait * 1e3;
        st.seconds = now_s() - t_begin;
        solved_ = true;
        return st;
      }
      st.pivots[t + 1] = r.phys;
      if (r.owner == L_.k) st.bcast_bytes += double(m) * npad * esz();
      post_select(t + 1, r);
      normalize_and_bcast(t + 1, r, /*wait_main=*/true);
    }
  }

  finalize(st.pivots);
  dev_.sync_all();
  const double t_end = now_s();
  for (int64_t t = 0; t < Nr; ++t)
    if (st.pivots[t] != t) st.offdiag_pivots++;
  st.host_wait_ms = host_wait * 1e3;
  st.seconds = t_end - t_begin;
  solved_ = true;
  return st;
}

// inv(A)[t, block s_u] = X[s_t, block u]  (derivation: SURVEY-style sweep bookkeeping; verified
// against numpy in tests/test_host_engine.py).  Row block t belongs on rank t mod p, slot t div p.
void Engine::finalize(const std::vector<int32_t>& seq) {
  const int64_t m = L_.m, Nr = L_.Nr, p = L_.p, k = L_.k, npad = L_.npad;
  std::vector<int32_t> step_of(Nr);
  for (int64_t t = 0; t < Nr; ++t) step_of[seq[t]] = (int32_t)t;
  // colsrc[c] = u with seq[u] == c ; dst_blk[b] = destination slot
  int32_t* colsrc = ihost_;
  int32_t* dstblk = ihost_ + Nr;
  for (int64_t u = 0; u < Nr; ++u) colsrc[seq[u]] = (int32_t)u;
  for (int64_t b = 0; b < L_.nblk; ++b) {
    const int64_t g = L_.global_block(b);
    const int64_t t = step_of[g];
    dstblk[b] = (p == 1) ? (int32_t)t : (int32_t)b;  // p>1: column-permute in local order first
  }
  dev_.copy(iscratch_, ihost_, sizeof(int32_t) * (Nr + std::max<int64_t>(L_.nblk, 1)), S_MAIN);
  if (L_.nblk > 0)
    dev_.permute_blocks(opt_.dtype, out_, npad, X_, npad, L_.nblk, m, Nr, iscratch_ + Nr, iscratch_,
                        S_MAIN);
  if (p == 1) {
    dev_.sync_stream(S_MAIN);
    return;
  }
  // p > 1: move every block row to its owner; receive straight into the (now free) X panel.
  dev_.record(ev_main_, S_MAIN);
  dev_.wait(S_COMM, ev_main_);
  std::vector<P2POp> ops;
  const size_t blk_bytes = (size_t)m * npad * esz();
  for (int64_t g = 0; g < Nr; ++g) {
    const int64_t src = g % p;
    const int64_t t = step_of[g];
    const int64_t dst = t % p;
    if (src == k && dst == k) {
      dev_.copy(elem(X_, (t / p) * m * npad), elem(out_, (g / p) * m * npad), blk_bytes, S_COMM);
    } else if (src == k) {
      ops.push_back(P2POp{elem(out_, (g / p) * m * npad), blk_bytes, (int)dst, true});
    } else if (dst == k) {
      ops.push_back(P2POp{elem(X_, (t / p) * m * npad), blk_bytes, (int)src, false});
    }
  }
  comm_.group_p2p(dev_, ops, S_COMM);
  dev_.sync_stream(S_COMM);
  std::swap(X_, out_);
}

// ---------------------------------------------------------------- output
void Engine::download_local_rows(double* host, int64_t ld) {
  const int64_t real = real_local_rows(), n = L_.n;
  if (real == 0) return;
  const size_t es = esz();
  const int64_t rows_per = std::max<int64_t>(1, (int64_t(128) << 20) / (n * (int64_t)es));
  void* stage = dev_.alloc_pinned(std::min(rows_per, real) * n * es);
  for (int64_t r0 = 0; r0 < real; r0 += rows_per) {
    const int64_t nr = std::min(rows_per, real - r0);
    dev_.copy2d(stage, n * es, elem(out_, r0 * L_.npad), L_.npad * es, n * es, nr, S_MAIN);
    dev_.sync_stream(S_MAIN);
    for (int64_t r = 0; r < nr; ++r)
      for (int64_t j = 0; j < n; ++j)
        host[(r0 + r) * ld + j] = (opt_.dtype == DType::F64)
                                      ? static_cast<double*>(stage)[r * n + j]
                                      : (double)static_cast<float*>(stage)[r * n + j];
  }
  dev_.release_pinned(stage);
}

std::vector<double> Engine::corner(int nm, int which) {
  const int64_t m = L_.m;
  std::vector<double> mine((size_t)nm * nm + nm, 0.0);  // values + row mask
  void* src = (which == 0) ? X_ : out_;
  const size_t es = esz();
  void* stage = dev_.alloc_pinned((size_t)nm * es + 16);
  for (int64_t b = 0; b < L_.nblk; ++b) {
    const int64_t g = L_.global_block(b);
    for (int64_t r = 0; r < m; ++r) {
      const int64_t gr = g * m + r;
      if (gr >= nm) continue;
      dev_.copy(stage, elem(src, (b * m + r) * L_.npad), (size_t)nm * es, S_MAIN);
      dev_.sync_stream(S_MAIN);
      for (int j = 0; j < nm; ++j)
        mine[gr * nm + j] = (opt_.dtype == DType::F64) ? static_cast<double*>(stage)[j]
                                                       : (double)static_cast<float*>(stage)[j];
      mine[(size_t)nm * nm + gr] = 1.0;
    }
  }
  dev_.release_pinned(stage);
  const size_t sz = mine.size();
  std::vector<double> all(sz * L_.p);
  comm_.host_allgather(dev_, mine.data(), all.data(), sz * sizeof(double));
  std::vector<double> res((size_t)nm * nm, 0.0);
  for (int64_t q = 0; q < L_.p; ++q) {
    const double* part = all.data() + q * sz;
    for (int r = 0; r < nm; ++r)
      if (part[(size_t)nm * nm + r] != 0.0)
        for (int j = 0; j < nm; ++j) res[(size_t)r * nm + j] = part[(size_t)r * nm + j];
  }
  return res;
}

double Engine::residual_common() {
  const int64_t m = L_.m, p = L_.p, npad = L_.npad;
  const size_t es = esz();
  void* full = out_;
  void* gath = nullptr;
  if (p > 1) {
    const size_t per = (size_t)L_.max_nblk * m * npad * es;
    full = dev_.alloc((size_t)npad * npad * es);
    gath = dev_.alloc(per * p);
    void* send = out_;
    void* tmp = nullptr;
    if (L_.nblk < L_.max_nblk) {  // pad the send buffer to the common size
      tmp = dev_.alloc(per);
      dev_.memset0(tmp, per, S_COMM);
      if (L_.nblk > 0) dev_.copy(tmp, out_, (size_t)L_.rows * npad * es, S_COMM);
      send = tmp;
    }
    comm_.allgather(dev_, send, gath, per, S_COMM);
    for (int64_t q = 0; q < p; ++q) {
      const int64_t nb = rows_owned(L_.Nr, p, q);
      for (int64_t j = 0; j < nb; ++j)
        dev_.copy(elem(full, (j * p + q) * m * npad),
                  static_cast<char*>(gath) + q * per + (size_t)j * m * npad * es,
                  (size_t)m * npad * es, S_COMM);
    }
    dev_.sync_stream(S_COMM);
    if (tmp) dev_.release(tmp);
    dev_.release(gath);
  }
  double local = 0.0;
  if (L_.nblk > 0) {
    dev_.residual(opt_.dtype, X_, full, L_, dscratch_, S_MAIN);
    dev_.copy(dhost_, dscratch_, sizeof(double), S_MAIN);
    dev_.sync_stream(S_MAIN);
    local = dhost_[0];
  }
  if (p > 1) dev_.release(full);
  return comm_.host_max(dev_, local);
}

double Engine::residual_generated(GenSpec g) {
  GJ_REQUIRE(solved_, "residual: solve() first");
  dev_.generate(opt_.dtype, X_, L_, g, S_MAIN);
  dev_.sync_stream(S_MAIN);
  return residual_common();
}

double Engine::residual_rows(const double* host, int64_t ld) {
  GJ_REQUIRE(solved_, "residual: solve() first");
  upload_local_rows(host, ld);
  solved_ = true;
  return residual_common();
}

void SelfComm::host_allgather(Device&, const void* send, void* recv, size_t bytes) {
  if (send != recv) std::memcpy(recv, send, bytes);
}

[[noreturn]] void fail(const char* file, int line, const std::string& msg) {
  throw Error(Status::BadArgs, std::string(file) + ":" + std::to_string(line) + ": " + msg);
}

}  // namespace gj
