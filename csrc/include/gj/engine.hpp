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
//   * Step t eliminates block column t from every row with the multipliers L_i = -X[i, t] and the
//     normalised pivot row R_t = H * X[s_t, :], H = inv(X[s_t, t]).  The exact (cancellation-free)
//     sweep form is used: column t enters the update as 0 (so X[i,t] becomes L_i H), the pivot row
//     enters as 0 with its multiplier row edited to "I" at its own position (so it becomes R_t).
//   * Depth-d panels: d consecutive steps are fused into ONE trailing update
//        X += [L_t0 .. L_t0+d-1] * [R_t0 ; .. ; R_t0+d-1]        (K = d*m, MFMA GEMM)
//     The panel's own d columns and d pivot rows are produced by narrow side updates ("panel
//     pieces", d*m x d*m) so that the big GEMM needs only zero-column / zero-row masks (GemmExtra)
//     and no special rows inside the hot kernel.  d = 4 gives K = 512 at m = 128.
//   * Look-ahead (three HIP streams): MAIN runs the big update of panel u; SIDE (high priority)
//     first forms and broadcasts panel u's pivot rows over the next panel's columns (look-ahead
//     rows), updates those columns, then runs the next panel's pivot searches (batched in-register
//     block inverses + RCCL all-gather of 32-B PivotRec + deterministic argmin on device) and the
//     narrow edits; COMM normalises panel u's pivot rows over the rest of the columns and
//     broadcasts them chunk by chunk (one event per chunk) so MAIN's update can start on chunk 0
//     while chunk k is in flight.  Every cross-stream edge is checked by RaceCheckDevice.
#pragma once

#include <algorithm>
#include <memory>
#include <string>
#include <vector>

#include "gj/comm.hpp"
#include "gj/device.hpp"

namespace gj {

// Pivot rule of every step.
//   MinInvNorm: the reference's rule (main.cpp:1039-1066): invert every candidate block, take the
//               smallest ||inv||_inf (ties -> larger rank, then smaller local row).
//   Partial:    block partial pivoting, a faster alternative: each rank takes its candidate with
//               the largest-magnitude entry and inverts that block alone; among the ranks' records
//               whose block is invertible the largest magnitude wins (same tie rule).  When every
//               rank's choice is singular, that step falls back to the MinInvNorm search.  One
//               candidate inverse per rank and step instead of one per candidate.
enum class PivotRule : int { MinInvNorm = 0, Partial = 1 };

struct SolveOptions {
  DType dtype = DType::F64;
  int64_t chunk_cols = 0;   // pipelining granularity of the pivot-row broadcast (0 = auto)
  int depth = 0;            // elimination steps fused per trailing update (K = depth*m), 1..8;
                            // 0 = auto: 2 up to N = 8192 on one rank (pivot-chain-bound); 8 on ranks of
                            // <= 4096 rows of a p > 1 job with N > 16384 (p = 8 at N = 32768);
                            // else 4 (profiles/small_n_sweep.md, profiles/depth_pgt1.md)
  double eps = kDefaultEps;
  PivotRule pivot = PivotRule::MinInvNorm;
  // PivotRule::Partial: a rank's candidate whose growth estimate ||inv(W)||_inf * max|W| exceeds
  // this is treated as singular (another rank's, or the full MinInvNorm search, takes the step), so
  // partial pivoting cannot silently accept a near-singular block.  0: no guard; < 0 (default): by
  // dtype, min(1e8, 0.01 / eps) -- 1e8 for fp64, 8.4e4 for fp32 (a dtype-blind 1e8
  // accepted fp32 blocks whose inverse has no correct digit; the estimate can understate
  // cond_inf by up to m, hence the margin below 1 / eps).
  double pivot_growth = -1;
  double pivot_growth_bound() const {
    if (pivot_growth >= 0) return pivot_growth;
    const double e = dtype == DType::F64 ? 2.220446049250313e-16 : 1.1920928955078125e-07;
    return std::min(1e8, 0.01 / e);
  }
  bool sync_debug = false;  // synchronise every stream after every phase (race screening)
  bool profile = false;     // per-phase device timers (HIP events) + roctx ranges
  // Consumption-point verification (also GJ_VERIFY=1): every broadcast buffer is hashed on the
  // stream that consumes it, right before its consumer (MAIN: each Rb chunk segment; SIDE: each
  // panel piece, look-ahead row segment, gathered pivot records and the pivot sequence; COMM: the
  // last piece).  After the solve the hashes are all-gathered and compared with the root's; the
  // first mismatch (in step order) fails the solve on every rank with Status::VerifyFailed, naming
  // step, phase, buffer, root, the differing receivers and the consuming stream.
  bool verify = false;
  double comm_timeout_s = 600;  // a host wait on a pivot longer than this is a peer failure
  int reserve_cus = -1;     // CUs kept free of the trailing update for the pivot path (-1 = auto)
};

// Device time per phase (sum over the solve; phases on different streams overlap in time).
enum Phase : int {
  PH_COLUMN = 0,   // SIDE: next pivot column brought up to date + transposed multipliers
  PH_PIVOT,        // SIDE: batched candidate inverses + local argmin
  PH_EXCHANGE,     // SIDE: pivot record all-gather + global argmin + 32-B readback
  PH_EDITS,        // SIDE: owner-side multiplier / H edits
  PH_PIECES,       // SIDE: panel piece (fused owner kernel) + its broadcast
  PH_NORMALISE,    // COMM: owner normalises its pivot rows chunk by chunk (GEMM)
  PH_BCAST,        // COMM: pivot-row chunk broadcasts
  PH_UPDATE,       // MAIN: depth-d trailing update (the MFMA GEMM)
  PH_FINALIZE,     // COMM: final block permutation + exchange
  kNumPhases
};
const char* phase_name(int ph);

struct SolveStats {
  Status status = Status::Ok;
  int64_t singular_step = -1;
  double seconds = 0;            // this rank's wall time of solve() (device-synchronised)
  double host_wait_ms = 0;       // time the host spent blocked on pivot results
  std::vector<int32_t> pivots;   // physical pivot block row of every step
  int64_t offdiag_pivots = 0;    // steps whose pivot was not the "natural" row (needed a swap)
  int64_t pivot_fallbacks = 0;   // PivotRule::Partial: steps that needed the MinInvNorm search
  double bcast_bytes = 0;        // bytes of pivot rows broadcast by this rank (as root)
  // payload bytes of the collectives this rank took part in (p > 1), by kind: the algorithm
  // bandwidth is bytes / the phase time of that kind (bench.py "comm_bandwidth")
  enum CommKind : int { CK_ROWS = 0, CK_PIECES, CK_RECORDS, kNumCommKinds };
  double comm_bytes[kNumCommKinds] = {};
  int64_t comm_calls[kNumCommKinds] = {};
  bool profiled = false;
  double phase_ms[kNumPhases] = {};   // SolveOptions::profile only
  int64_t phase_calls[kNumPhases] = {};
};

// Result of Engine::solve_rhs.
struct RhsResult {
  double residual = 0;           // ||b - A x||_inf (fp64) of the returned x
  double backward_error = 0;     // ||b - A x|| / (||A|| ||x|| + ||b||), inf-norms
  std::vector<double> history;   // ||b - A x_k||_inf / ||b||_inf for k = 0 (x = X b), 1, ...
  int steps = 0;                 // refinement steps applied
  bool converged = false;        // backward error <= tol
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
  // Device-resident I/O: this rank's real rows as a device array of the engine dtype (ld >= n
  // elements), copied device-to-device (e.g. straight from / into a torch CUDA tensor).
  void upload_rows_device(const void* src, int64_t ld);
  void download_rows_device(void* dst, int64_t ld);
  // This rank's rows of a matrix file (text / .bin, read_matrix_rows): collective, every rank
  // parses only its own rows.  Returns Ok, CannotOpen or CannotRead (the same on every rank).
  Status load_file(const std::string& path, int nthreads = 0);
  // The input panel as it is right now (dtype elements, ld npad, layout().rows rows).
  // A raw pointer into X: whoever writes through it changes the input behind generate()'s cached
  // row norm, so handing it out drops that cache (a stale ||A|| in the singular test).
  void* input_panel() {
    local_norm_valid_ = false;
    solved_ = false;
    return X_;
  }
  double norm_inf();  // collective

  // ---- solve (collective) ----
  SolveStats solve();
  // Per-phase device timers for the following solves (SolveOptions::profile), switchable between
  // solves: bench.py times its steps unprofiled, then profiles one extra untimed solve.
  void set_profile(bool on) { opt_.profile = on; }

  // ---- output ----
  void* result_panel() { return out_; }  // local rows of inv(A), padded, ld npad
  void download_local_rows(double* host, int64_t ld);  // this rank's real rows of the result
  // Top-left nm x nm corner (collective; valid on every rank).  which: 0 = current input, 1 = result.
  std::vector<double> corner(int nm, int which);
  // ||A * inv(A) - I||_inf  (collective).  The input panel is overwritten by A again.
  double residual_generated(GenSpec g);
  double residual_rows(const double* host, int64_t ld);
  // Re-reads the file (reference main.cpp:463-484); *status = Ok / CannotOpen / CannotRead.
  double residual_file(const std::string& path, int nthreads = 0, Status* status = nullptr);

  // ---- A x = b (BASELINE config 1; SURVEY.md §5.6 --rhs) ----
  // x = inv(A) b from the result panel: one MFMA GEMV per rank + all-gather (collective).
  // b and x are full n-vectors on every rank.
  void apply_inverse(const double* b, double* x);
  // ||A x - b||_inf with the input panel currently holding A (after generate/upload; collective).
  double axb_residual(const double* x, const double* b);
  // A x = b with iterative refinement, the residual always in fp64 (A from `gen` or from this
  // rank's fp64 rows `host_rows`, ld): x_0 = inv(A) b, x_{k+1} = x_k + inv(A) (b - A x_k).
  // Collective; b and x are full n-vectors on every rank.
  RhsResult solve_rhs(const double* b, double* x, const GenSpec* gen, const double* host_rows, int64_t ld,
                      int max_refine, double tol);
  // The same with this rank's real rows of A as an fp64 DEVICE array (ld >= n elements), e.g. a
  // torch CUDA tensor: copied device-to-device, never through the host.
  RhsResult solve_rhs_device(const double* b, double* x, const void* dev_rows_f64, int64_t ld, int max_refine,
                             double tol);
  // Precision of the last residual: true = fp64 (always for fp64 solves; fp32 solves when it fits).
  bool residual_fp64() const { return last_residual_fp64_; }
  // ||A||_inf of the last solve's input (the reference's norm, taken at solve start) and
  // ||inv(A)||_inf of its result (collective): the scale of the normalised residual
  // ||A inv(A) - I|| / (||A|| ||inv(A)|| eps) that utils/metrics.py gates on.
  double input_norm_inf() const { return norm_a_; }
  double result_norm_inf();

  int64_t real_local_rows() const;
  int depth() const { return d_; }  // elimination steps per panel (after the auto choice)
  // What the auto policies chose on this rank (bench.py / --json report them).
  struct Policy {
    int depth = 0;
    int64_t chunk_cols = 0;       // widest pivot-row chunk (columns)
    int nchunks = 0;
    int reserve_cus = 0;          // CUs kept off the trailing-update stream
    std::string block_inverse;    // candidate-inverse kernel
    bool comm_small_tiles = false;
    bool dense_gemm = false;      // trailing update at 5 workgroups per CU
    bool la_side = true;          // look-ahead rows on SIDE (else COMM)
    std::string pivot;            // "block-min-inv-norm" | "partial"
    std::string fault_injection;  // active GJ_TEST_* knobs ("" in every normal run)
    // every GJ_* variable set in this process's environment when the engine was built ("NAME=value"):
    // a stray schedule override is visible in every record
    std::vector<std::string> env_overrides;
    int gemm_tile = 128;          // fp64 LDS-DMA trailing-update tile width (64 | 128)
    int split = 0;                // chain / deferred split of the column updates (split_: 0, 1, 2)
    bool lat_wide = false;        // chain column updates on the LDS-DMA kernel (lat_wide_)
    bool skip_cols = false;       // one MAIN launch per chunk around the look-ahead columns (skip_cols_)
    bool lat_reg = false;         // the chain's latency GEMMs on the register-fed kernel (lat_reg_)
    bool chunk_skip = false;      // one chunk-pass launch per step around the panel columns (chunk_skip_)
    int first_depth = 0;          // steps of the first panel (f_)
    int main_cnt = 0;             // MAIN's C tile non-temporal: loads (1) / stores (2) (main_cnt_)
  };
  Policy policy() const;
  const std::string& bcast_algo() const { return bcast_algo_; }  // "ring" | "direct"

 private:
  static constexpr int kMaxDepth = GemmExtra::kMaxZeroRows;
  // pinned pivot-result slots: one per step of a panel in flight (the host-free chain of one rank
  // enqueues a whole panel's steps before it reads any result)
  static constexpr int kPivSlots = 2 * kMaxDepth;
  static int hslot(int64_t t) { return (int)(t % kPivSlots); }
  // The reference pivot rule: the pivot chain is enqueued a panel at a time, every owner-side
  // launch reading the pivot from device memory, the host reading the results after it (no host
  // round trip per step).  One rank always; p > 1 with host_free_multi_ (GJ_HOST_FREE), where the
  // panel piece travels by a root-agnostic all-reduce (non-owners contribute zeros) because a
  // broadcast needs its root on the host.
  bool host_free_chain() const {
    return opt_.pivot == PivotRule::MinInvNorm && !opt_.sync_debug && (L_.p == 1 || host_free_multi_);
  }
  bool host_free_multi_ = false;
  // 0 = ok, 1 = the work space does not fit, 2 = the matrix panels do not fit (why: the reason)
  int alloc_buffers(std::string& why);
  void alloc_work(int64_t wmax);
  void free_work();     // everything but the matrix panels
  void label_work();    // buffer names for schedule-check reports
  void free_buffers();
  // Pivot search for step t on the multiplier segment Lt (SIDE stream); result -> piv_host_[hslot(t)].
  void select(int64_t t, const void* Lt, bool full = false);
  // Panel factorisation (pivot searches of its q steps, panel pieces, then the chunk pipeline of
  // the normalised pivot rows).  Returns false when the matrix is singular.
  void begin_panel(int64_t v);
  bool factor_panel(int64_t v, SolveStats& st, double& host_wait);
  bool await_step(int64_t v, int64_t j, SolveStats& st, double& host_wait, PivotResult& r);
  void lookahead_rows(int64_t v, bool wait_main);
  void chunk_pipeline(int64_t v, bool wait_main);
  void lookahead_update(int64_t u);
  void big_update(int64_t u);
  void finalize(const std::vector<int32_t>& seq);
  SolveStats solve_steps();
  RhsResult solve_rhs_impl(const double* b, double* x, const GenSpec* gen, const double* host_rows,
                           const void* dev_rows, int64_t ld, int max_refine, double tol);
  // GJ_VERIFY (SolveOptions::verify): hash slots of a panel, (d*C + 3d + 1) + 3 (2d + 2) of them:
  //   [chunk c][step j] Rb segment at MAIN's chunk update | pp[j] panel piece at its first consumer
  //   | la[j] look-ahead row segment at the look-ahead update | recs[j] gathered pivot records |
  //   seq (the panel's pivot sequence, after its last step)
  //   | rank-local hand-overs (round 6), per buffer group g (VLocal) at three points: P where the
  //   producing stream (SIDE) finished writing it, C right before its consumer on another stream
  //   reads it, E right after that consumer's last read.  C != P: the consumer read it before it was
  //   produced (a missing wait, or a write not yet visible: the event release); E != P: it was
  //   rewritten while the consumer still read it (a missing wait of the next writer).  Compared on
  //   the rank itself, no root involved.
  enum VKind { V_RB = 0, V_PP, V_LA, V_RECS, V_SEQ, V_LP, V_LC, V_LE };
  // groups: 0 = the multiplier panel At[v % 3] (SIDE -> MAIN's trailing update), 1 = the panel pieces
  // PP[v & 1], 2 .. 1+d = Lrow[v & 1][j], 2+d .. 1+2d = Ht[v & 1][j] (SIDE -> COMM's chunk pass)
  int vlocal_groups() const { return 2 * d_ + 2; }
  struct VRegion {
    const void* base = nullptr;
    int64_t ld = 0, width = 0, rows = 0;
    std::string name;
  };
  VRegion vlocal_region(int64_t v, int g) const;
  void vlocal_hash(int64_t v, VKind point, bool at_group, int s);  // the groups of one consumer
  bool vlocal_on() const { return vparts_ && split_ == 0; }  // split_ moves At writes off SIDE
  int vslot(VKind k, int64_t j, int64_t c = 0) const;
  int vslots() const { return (int)(d_ * (int64_t)cb0_.size() + 3 * d_ + 1 + 3 * vlocal_groups()); }
  void vhash(int64_t v, int slot, const void* base, int64_t ld_bytes, int64_t width_bytes, int64_t rows, int s);
  void verify_hashes(const SolveStats& st);
  double residual_common(const void* A, bool wide);
  double residual_streamed(const void* A, bool wide);
  bool residual_wide();
  size_t residual_fp64_bytes() const;
  void upload_rows_into(void* P, DType dt, const double* host, int64_t ld);
  Status read_file_rows(const std::string& path, int nthreads, std::vector<double>& rows);
  void dbg_sync();
  // Host wait for the pivot result of `step` (pinned slot par) with failure detection
  // (Comm::check_health + timeout).
  void wait_pivot(int par, int64_t step, double& host_wait);
  // profiling: begin() records a timing event on stream s, end() closes the interval
  int prof_begin(int s);
  void prof_end(int phase, int ev0, int s);
  int prof_event();
  void prof_collect(SolveStats& st);
  size_t esz() const { return dtype_size(opt_.dtype); }
  char* elem(void* base, int64_t off) const { return static_cast<char*>(base) + off * (int64_t)esz(); }
  // panel 0 is f_ steps deep (a shorter prologue before MAIN's first update), every later one d_
  int64_t panel_t0(int64_t v) const { return v == 0 ? 0 : f_ + (v - 1) * d_; }
  int64_t panel_q(int64_t v) const { return std::min<int64_t>(v == 0 ? f_ : d_, L_.Nr - panel_t0(v)); }
  int64_t npanels() const { return L_.Nr <= f_ ? 1 : 1 + (L_.Nr - f_ + d_ - 1) / d_; }
  int64_t panel_of(int64_t t) const { return t < f_ ? 0 : 1 + (t - f_) / d_; }
  bool panel_boundary(int64_t b) const { return b == 0 || b >= L_.Nr || (b >= f_ && (b - f_) % d_ == 0); }
  // chunk c of the stacked-rows buffer: (d*m) x W block, ld W
  char* rb_chunk(int par, int64_t c) const {
    return elem(Rb_[par], (int64_t)d_ * L_.m * cb0_[c] * L_.m);
  }
  int64_t chunk_w(int64_t c) const { return (cb1_[c] - cb0_[c]) * L_.m; }
  GemmExtra pivot_rows_extra(int par, int64_t nsteps) const;  // this rank's pivot rows of a panel

  Device& dev_;
  Comm& comm_;
  SolveOptions opt_;
  Layout L_;
  int d_ = 1;
  int f_ = 1;  // depth of the first panel (GJ_FIRST_DEPTH; default d_)
  int main_cnt_ = 0;  // GemmExtra::c_nt of MAIN's trailing-update launches
  int main_split_ = 0;  // GJ_MAIN_SPLIT: MAIN's chunk launches in two column halves (1 first, 2 all)
  std::string bcast_algo_ = "ring";
  bool comm_small_tiles_ = false;  // COMM chunk-normalisation GEMMs on the small latency tile
  int bi_hint_ = -1;               // candidate-inverse kernel family (Device::set_block_inverse_hint)
  int reserved_cus_ = 0;
  bool dense_gemm_ = false;        // trailing update at 5 workgroups per CU (GemmExtra::dense)
  bool la_side_ = true;            // look-ahead rows on SIDE (else COMM); GJ_LA_SIDE overrides
  // Chain / deferred split of a panel's column updates (GJ_SPLIT, profiles/split_r5.md): the
  // look-ahead update and the in-panel column updates on the pivot chain (SIDE) cover only the local
  // block rows that are still pivot candidates when the panel starts (chain_sel_); the rows already
  // used as pivot rows (defer_sel_) get the same updates later -- they are needed only by MAIN's
  // trailing update: 1 = on COMM ahead of the panel's chunk pass, 2 = on MAIN ahead of the panel's
  // trailing update.  Bit-identical results (same products, same k order per row).  Needs 64 | m
  // and <= 512 local blocks (GemmExtra::rsel).
  int split_ = 0;
  // the pivot chain's column updates (rows x m x j m) on the LDS-DMA kernel instead of the 64 x 32
  // latency tile (GemmExtra::lat_wide): on when CUs are reserved for the chain at p = 1
  bool lat_wide_ = false;
  // MAIN's chunk update as one launch around the look-ahead columns (GemmExtra::skip_c0/c1) instead
  // of one launch per side: on under a CU reservation (GJ_SKIP_COLS=0/1 overrides)
  bool skip_cols_ = false;
  // the same for the chunk pass's normalisation GEMMs around the panel / next-panel columns
  // (follows skip_cols_; GJ_CHUNK_SKIP=0/1 overrides)
  bool chunk_skip_ = false;
  // the chain's latency GEMMs on the register-fed small fp64 kernel (GemmExtra::lat_reg): on under
  // a CU reservation (GJ_LAT_REG=0/1 overrides)
  bool lat_reg_ = false;
  int chunk_build_ = 0;  // LDS-DMA build of the chunk pass's GEMMs (GemmExtra::glds_build; 0 = auto)
  int chunk_tile_ = 0;   // ... and their tile width (GemmExtra::glds_tile; 0 = gemm_tile_; A/B runs)
  int gemm_tile_ = 128;  // LDS-DMA tile width of this engine's launches (Device::set_gemm_tile_hint)
  std::vector<char> used_local_;       // local blocks used as pivot rows so far (host copy)
  double comm_bytes_[SolveStats::kNumCommKinds] = {};  // per solve, -> SolveStats::comm_bytes
  int64_t comm_calls_[SolveStats::kNumCommKinds] = {};
  void count_comm(int kind, double bytes) {
    if (L_.p > 1) comm_bytes_[kind] += bytes, comm_calls_[kind] += 1;
  }
  GemmExtra chain_sel_[2], defer_sel_[2];  // by panel parity; rsel_m == 0: panel without a split
  void deferred_updates(int64_t v, int stream);
  double norm_a_ = -1;
  double local_norm_ = 0;           // this rank's ||X||_inf part, computed by generate()
  bool local_norm_valid_ = false;   // X unchanged since generate()
  bool step_events_ = false;  // GJ_STEP_EVENTS=1: SIDE records ev_edit_ / ev_pp_ after every step

  // chunk plan (block-column ranges, multiples of d_ blocks so a panel never straddles chunks)
  std::vector<int64_t> cb0_, cb1_;
  std::vector<int64_t> chunk_of_;    // block -> chunk

  // device buffers
  void* X_ = nullptr;       // input / working panel
  void* out_ = nullptr;     // result panel
  // stacked K-major multipliers of a panel, (d*m) x rows, by panel index mod 3 (panel u's chunks
  // read theirs while the look-ahead of panel u writes panel u+1's and SIDE edits them)
  void* At_[3] = {nullptr, nullptr, nullptr};
  void* Rb_[2] = {nullptr, nullptr};   // stacked normalised pivot rows, chunk-major (d*m) x npad
  void* PP_[2] = {nullptr, nullptr};   // panel pieces: R_t restricted to the panel's columns, (d*m) x (d*m)
  // look-ahead rows: a panel's normalised pivot rows restricted to the NEXT panel's block columns,
  // (q*m) x (qn*m), step-major; formed and broadcast ahead of the first chunk so that the next
  // panel's look-ahead update (and with it the next pivot chain) does not wait for a whole chunk
  void* LA_[2] = {nullptr, nullptr};
  void* T2_ = nullptr;                 // LA temp when LA runs on SIDE, m x (d*m)
  void* Lrow_[2][kMaxDepth] = {};      // multipliers of pivot row s_t for earlier panel steps, K-major
  void* Ht_[2][kMaxDepth] = {};        // H_t^T
  void* T_ = nullptr;                  // row-update temp, m x Wmax
  void* RP_ = nullptr;                 // panel-piece temp, m x (d*m)
  void* inv_ = nullptr;
  // PivotRule::Partial: the chosen candidate (K-major m x m), its inverse, score / validity, a zero
  // "used" flag, and the one-block layout the inverse runs on
  void* sel_ = nullptr;
  void* inv1_ = nullptr;
  double* score1_ = nullptr;
  int32_t* valid1_ = nullptr;
  int32_t* used1_ = nullptr;
  Layout L1_;
  double* scores_ = nullptr;
  int32_t* valid_ = nullptr;
  int32_t* pos_ = nullptr;
  int32_t* phys_at_ = nullptr;
  int32_t* used_ = nullptr;
  int32_t* seq_ = nullptr;
  PivotRec* myrec_ = nullptr;
  int32_t* sel_done_ = nullptr;  // workgroup counter of the fused candidate-inverse + selection launch
  PivotRec* recs_ = nullptr;
  PivotResult* piv_dev_ = nullptr;
  double* dscratch_ = nullptr;
  uint64_t* vparts_ = nullptr;  // GJ_VERIFY: npanels x vslots x Device::kHashParts partial hashes
  int32_t* iscratch_ = nullptr;
  // pinned host
  PivotResult* piv_host_ = nullptr;
  int32_t* ihost_ = nullptr;
  double* dhost_ = nullptr;
  int64_t ihost_len_ = 0;
  PivotResult piv_[2][kMaxDepth];      // pivots of the panels in flight (by panel parity)
  int64_t live_ = 0;                   // local block rows not yet used as a pivot row (candidates)

  // events
  int ev_L_ = -1, ev_main_ = -1, ev_edit_[2] = {-1, -1};
  int ev_pp_[2][kMaxDepth] = {};
  int ev_la_[2] = {-1, -1};            // LA_[par] formed and broadcast (COMM)
  int ev_cp_[2] = {-1, -1};            // chunk pass of a panel of that parity done (COMM)
  int ev_def_[2] = {-1, -1};           // split_ == 2: MAIN's deferred updates of that panel done
  std::vector<int> ev_c_;        // per chunk: MAIN finished the panel update of that chunk
  std::vector<int> ev_b_[2];     // per chunk: all stacked rows of that chunk broadcast
  std::vector<int> pev_pool_;    // profiling events (timing enabled), reused across solves
  size_t pev_next_ = 0;
  struct PMark { int phase, ev0, ev1; };
  std::vector<PMark> pmarks_;
  bool solved_ = false;
  // The work space did not fit on some rank (agreed at construction): solve() reports
  // Status::NoBlockMemory, the reference's "not enough memory for block" (main.cpp:428-436).
  bool block_mem_fail_ = false;
  bool last_residual_fp64_ = true;
  std::string block_mem_why_;
  // where the solve is (named by communication-failure messages)
  int64_t cur_step_ = -1;
  const char* cur_phase_ = "setup";
  std::string fault_injection_;  // active GJ_TEST_* knobs (announced, reported in policy())
  std::vector<std::string> env_overrides_;  // GJ_* variables at construction (policy())
  int64_t hang_step_ = -1;  // GJ_TEST_HANG (fault injection)
  int64_t corrupt_step_ = -1;  // GJ_TEST_CORRUPT (a wrong inverse on purpose)
  bool corrupt_unprofiled_ = false;  // ... only in solves without the phase timers
  // GJ_TEST_DROP_WAIT=<name>[,<name>]: leave out one ordering edge of the schedule (a planted
  // hazard the happens-before checker must report; tests only): "cp" the SIDE wait for the chunk
  // pass two panels back, "edit" MAIN's wait for the owner edits, "b" MAIN's wait for a chunk's
  // broadcast, "x" the chunk pass's exclusion of the next panel's columns
  std::string drop_wait_;
  bool dropped(const char* name) const {
    return !drop_wait_.empty() && drop_wait_.find(std::string(",") + name + ",") != std::string::npos;
  }
};

}  // namespace gj
