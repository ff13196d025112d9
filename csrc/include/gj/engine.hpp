// Distributed block Gauss-Jordan inversion engine (one instance per rank / GPU).
//
// Semantics: the reference's Jordan() (main.cpp:953-1204) with the pivot-row bug at main.cpp:1095
// fixed: block pivoting by the minimum inf-norm of the candidate block's inverse,
// ties -> larger rank, then smaller local row.  Mechanics are MI355X-native:
//
//   * The local panel X holds only the block rows this rank owns (block-row-cyclic, main.cpp:118-123)
//     and is inverted IN PLACE (Gauss-Jordan "sweep" form): 2n^3 flops instead of the reference's
//     3n^3 (it eliminates the full-width B = I part every step, main.cpp:1176-1193).
//   * Rows are never swapped; the pivot of step t is tracked as a physical block row s_t and the
//     result is permuted once at the end (finalize).  A row swap therefore costs nothing per step.
//   * Step t is ONE rank-m update of every local row:  X += Lt^T * R_t  with
//        Lt  = -X[:, block t]  (K-major multiplier panel; the owner of s_t adds I to its block),
//        R_t = H * X[s_t, :]  with block t replaced by I + H,  H = inv(X[s_t, block t]).
//     That folds normalisation, the pivot-row write-back and the pivot-column update into the same
//     MFMA GEMM (no special rows or columns in the hot kernel).
//   * Look-ahead: column block t+1 is updated first; the SIDE stream runs the pivot search for step
//     t+1 (batched block inverses + RCCL all-gather of 32-B records + deterministic argmin) while the
//     MAIN stream runs the rest of step t's update; the COMM stream normalises and broadcasts the
//     next pivot row chunk by chunk as soon as each column chunk of step t is finished.
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "gj/comm.hpp"
#include "gj/device.hpp"

namespace gj {

struct SolveOptions {
  DType dtype = DType::F64;
  int64_t chunk_cols = 0;   // pipelining granularity of the pivot-row broadcast (0 = auto)
  double eps = kDefaultEps;
  bool sync_debug = false;  // synchronise every stream after every phase (race screening)
  bool profile = false;     // per-phase timing (adds synchronisation)
};

struct PhaseTimes {
  double select_ms = 0;     // pivot search + exchange (host-visible wait)
  double total_ms = 0;
};

struct SolveStats {
  Status status = Status::Ok;
  int64_t singular_step = -1;
  double seconds = 0;            // this rank's wall time of solve() (device-synchronised)
  double host_wait_ms = 0;       // time the host spent blocked on pivot results
  std::vector<int32_t> pivots;   // physical pivot block row of every step
  int64_t offdiag_pivots = 0;    // steps whose pivot was not the "natural" row (needed a swap)
  double bcast_bytes = 0;        // bytes of pivot rows broadcast by this rank (as root)
};

class Engine {
 public:
  Engine(Device& dev, Comm& comm, int64_t n, int64_t m, const SolveOptions& opt);
  ~Engine();
  Engine(const Engine&) = delete;
  Engine& operator=(const Engine&) = delete;

  const Layout& layout() const { return L_; }
  const SolveOptions& options() const { return opt_; }
  Device& device() { return dev_; }
  Comm& comm() { return comm_; }

  // ---- input (collective only where noted) ----
  void generate(GenSpec g);
  // host: this rank's real rows, in local order, n columns (ld >= n), fp64.
  void upload_local_rows(const double* host, int64_t ld);
  // The input panel as it is right now (dtype elements, ld npad, layout().rows rows).
  void* input_panel() { return X_; }
  double norm_inf();  // collective

  // ---- solve (collective) ----
  SolveStats solve();

  // ---- output ----
  void* result_panel() { return out_; }  // local rows of inv(A), padded, ld npad
  void download_local_rows(double* host, int64_t ld);  // this rank's real rows of the result
  // Top-left nm x nm corner (collective; valid on every rank).  which: 0 = current input, 1 = result.
  std::vector<double> corner(int nm, int which);
  // ||A * inv(A) - I||_inf  (collective).  The input panel is overwritten by A again.
  double residual_generated(GenSpec g);
  double residual_rows(const double* host, int64_t ld);

  int64_t real_local_rows() const;

 private:
  void alloc_buffers();
  void free_buffers();
  void select(int64_t t);      // pivot search for column block t (SIDE stream)
  void post_select(int64_t t, const PivotResult& r);
  void normalize_and_bcast(int64_t t, const PivotResult& r, bool wait_main);
  void finalize(const std::vector<int32_t>& seq);
  double residual_common();
  void dbg_sync();
  size_t esz() const { return dtype_size(opt_.dtype); }
  char* elem(void* base, int64_t off) const { return static_cast<char*>(base) + off * (int64_t)esz(); }

  Device& dev_;
  Comm& comm_;
  SolveOptions opt_;
  Layout L_;
  double norm_a_ = -1;

  // chunk plan (block-column ranges)
  std::vector<int64_t> cb0_, cb1_;   // in blocks
  std::vector<int64_t> chunk_of_;    // block -> chunk

  // device buffers
  void* X_ = nullptr;       // input / working panel
  void* out_ = nullptr;     // result panel
  void* Lt_[2] = {nullptr, nullptr};
  void* R_[2] = {nullptr, nullptr};
  void* Ht_[2] = {nullptr, nullptr};
  void* inv_ = nullptr;
  double* scores_ = nullptr;
  int32_t* valid_ = nullptr;
  int32_t* pos_ = nullptr;
  int32_t* phys_at_ = nullptr;
  int32_t* used_ = nullptr;
  int32_t* seq_ = nullptr;
  PivotRec* myrec_ = nullptr;
  PivotRec* recs_ = nullptr;
  PivotResult* piv_dev_ = nullptr;
  double* dscratch_ = nullptr;
  int32_t* iscratch_ = nullptr;
  // pinned host
  PivotResult* piv_host_ = nullptr;
  int32_t* ihost_ = nullptr;
  double* dhost_ = nullptr;
  int64_t ihost_len_ = 0;

  // events
  int ev_L_ = -1, ev_sel_[2] = {-1, -1}, ev_adj_[2] = {-1, -1}, ev_main_ = -1, ev_comm_ = -1;
  std::vector<int> ev_c_;        // per chunk: MAIN finished step t's chunk
  std::vector<int> ev_b_[2];     // per chunk: R chunk broadcast complete
  bool solved_ = false;
};

}  // namespace gj
