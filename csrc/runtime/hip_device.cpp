// HipDevice: HIP runtime side of the MI355X backend — streams, events, HBM allocation and kernel
// dispatch into csrc/kernels/*.hip.
//
// Streams: MAIN (trailing update, normal priority), SIDE (look-ahead pivot search, highest
// priority) and COMM (normalise + broadcast, highest priority).  All three are non-blocking w.r.t.
// the legacy default stream.  Nothing in the step loop ever calls hipDeviceSynchronize; the host
// only blocks on the 32-byte pivot result of the SIDE stream.
#include "gj/hip_device.hpp"

#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "../kernels/kernels.hpp"

namespace gj {

#define HIP_OK(expr)                                                                         \
  do {                                                                                       \
    hipError_t e_ = (expr);                                                                  \
    if (e_ != hipSuccess)                                                                    \
      throw Error(e_ == hipErrorOutOfMemory ? Status::NoMemory : Status::CommError,          \
                  std::string("HIP error ") + hipGetErrorString(e_) + " at " + __FILE__ + ":" + \
                      std::to_string(__LINE__) + " (" #expr ")");                            \
  } while (0)

static inline hipStream_t hs(void* p) { return static_cast<hipStream_t>(p); }

HipDevice::HipDevice(int device_index) : dev_(device_index) {
  int ndev = 0;
  HIP_OK(hipGetDeviceCount(&ndev));
  GJ_REQUIRE(device_index >= 0 && device_index < ndev, "HIP device index out of range");
  activate();
  int lo = 0, hi = 0;
  HIP_OK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  for (int s = 0; s < kNumStreams; ++s) {
    hipStream_t st;
    const int prio = (s == S_MAIN) ? lo : hi;
    HIP_OK(hipStreamCreateWithPriority(&st, hipStreamNonBlocking, prio));
    streams_[s] = st;
  }
}

HipDevice::~HipDevice() {
  activate();
  (void)hipDeviceSynchronize();
  for (void* e : events_) (void)hipEventDestroy(static_cast<hipEvent_t>(e));
  for (void* s : streams_)
    if (s) (void)hipStreamDestroy(hs(s));
  for (void* p : scratch_)
    if (p) (void)hipFree(p);
}

void HipDevice::activate() const { (void)hipSetDevice(dev_); }

int HipDevice::reserve_cus(int n) {
  if (n == reserved_) return reserved_;
  activate();
  hipDeviceProp_t prop;
  HIP_OK(hipGetDeviceProperties(&prop, dev_));
  const int ncu = prop.multiProcessorCount;
  n = std::max(0, std::min(n, ncu / 2));
  for (int role : {S_MAIN}) {
    HIP_OK(hipStreamSynchronize(hs(streams_[role])));
    HIP_OK(hipStreamDestroy(hs(streams_[role])));
    hipStream_t st;
    if (n == 0) {
      int lo = 0, hi = 0;
      HIP_OK(hipDeviceGetStreamPriorityRange(&lo, &hi));
      HIP_OK(hipStreamCreateWithPriority(&st, hipStreamNonBlocking, lo));
    } else {
      std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
      for (int c = 0; c < ncu; ++c) mask[c / 32] |= 1u << (c % 32);
      // the first n bits: bit i is a CU of XCC i % 8, shader engine (i / 8) % 4, so n = 32 takes
      // one CU from every shader engine (bench/cu_mask_probe.hip, profiles/cu_reserve_sweep.md)
      for (int i = 0; i < n; ++i) mask[i / 32] &= ~(1u << (i % 32));
      HIP_OK(hipExtStreamCreateWithCUMask(&st, (uint32_t)mask.size(), mask.data()));
    }
    streams_[role] = st;
  }
  reserved_ = n;
  return n;
}

std::string HipDevice::describe() const {
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev_) != hipSuccess) return "hip:" + std::to_string(dev_);
  return std::string("hip:") + std::to_string(dev_) + " " + prop.gcnArchName + " (" +
         std::to_string(prop.multiProcessorCount) + " CUs, " +
         std::to_string(prop.totalGlobalMem >> 30) + " GiB)";
}

void* HipDevice::alloc(size_t bytes) {
  activate();
  void* p = nullptr;
  HIP_OK(hipMalloc(&p, bytes ? bytes : 64));
  return p;
}
void HipDevice::release(void* p) {
  activate();
  (void)hipFree(p);
}
void* HipDevice::alloc_pinned(size_t bytes) {
  void* p = nullptr;
  HIP_OK(hipHostMalloc(&p, bytes ? bytes : 64, hipHostMallocDefault));
  return p;
}
void* HipDevice::alloc_pinned_coherent(size_t bytes) {
  void* p = nullptr;
  HIP_OK(hipHostMalloc(&p, bytes ? bytes : 64, hipHostMallocCoherent));
  return p;
}
void HipDevice::release_pinned(void* p) { (void)hipHostFree(p); }
size_t HipDevice::free_memory() const {
  activate();
  size_t fr = 0, tot = 0;
  if (hipMemGetInfo(&fr, &tot) != hipSuccess) return 0;
  return fr;
}
void HipDevice::memset0(void* p, size_t bytes, int s) {
  if (bytes) HIP_OK(hipMemsetAsync(p, 0, bytes, hs(streams_[s])));
}
void HipDevice::memset2d(void* p, size_t pitch, size_t w, size_t h, int s) {
  if (w && h) HIP_OK(hipMemset2DAsync(p, pitch, 0, w, h, hs(streams_[s])));
}
void HipDevice::copy(void* dst, const void* src, size_t bytes, int s) {
  if (bytes && dst != src)
    HIP_OK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, hs(streams_[s])));
}
void HipDevice::copy2d(void* dst, size_t dpitch, const void* src, size_t spitch, size_t w, size_t h,
                       int s) {
  if (w && h) HIP_OK(hipMemcpy2DAsync(dst, dpitch, src, spitch, w, h, hipMemcpyDefault, hs(streams_[s])));
}

// Ordering events (never synchronised by the host: it waits on streams or polls pinned memory).
// GJ_EVENT_RELEASE=device records them with a device-scope release instead of HIP's default
// system-scope one: even at N = 8192 (profiles/host_fence_r5.md).  Dropping the release altogether
// (hipEventDisableSystemFence) was 1.2 % faster at N = 8192 but returned a wrong inverse in the
// p = 8 async-virtual-rank golden test: `none` exists only as fault injection, to reproduce that
// failure under GJ_VERIFY (announced on stderr and in the engine policy's fault_injection;
// profiles/verify_r6.md).
static unsigned event_release_flags() {
  static const unsigned f = [] {
    const char* e = std::getenv("GJ_EVENT_RELEASE");
    const std::string v = e ? e : "";
    if (v == "device") return (unsigned)hipEventReleaseToDevice;
    if (v == "none") {
      std::fprintf(stderr, "gj: WARNING: FAULT INJECTION ACTIVE (GJ_EVENT_RELEASE=none): ordering events "
                           "carry no release fence; cross-stream hand-overs may read stale data\n");
      return (unsigned)hipEventDisableSystemFence;
    }
    if (v.empty() || v == "system") return 0u;
    throw Error(Status::BadArgs, "GJ_EVENT_RELEASE must be device or system (none: fault injection only)");
  }();
  return f;
}

int HipDevice::create_event(bool timing) {
  activate();
  hipEvent_t e;
  HIP_OK(hipEventCreateWithFlags(&e, timing ? hipEventDefault : (hipEventDisableTiming | event_release_flags())));
  events_.push_back(e);
  return (int)events_.size() - 1;
}
void HipDevice::record(int ev, int s) {
  HIP_OK(hipEventRecord(static_cast<hipEvent_t>(events_[ev]), hs(streams_[s])));
}
void HipDevice::wait(int s, int ev) {
  HIP_OK(hipStreamWaitEvent(hs(streams_[s]), static_cast<hipEvent_t>(events_[ev]), 0));
}
void HipDevice::sync_event(int ev) { HIP_OK(hipEventSynchronize(static_cast<hipEvent_t>(events_[ev]))); }
bool HipDevice::query_event(int ev) {
  const hipError_t e = hipEventQuery(static_cast<hipEvent_t>(events_[ev]));
  if (e == hipErrorNotReady) return false;
  HIP_OK(e);
  return true;
}
void HipDevice::sync_stream(int s) { HIP_OK(hipStreamSynchronize(hs(streams_[s]))); }
bool HipDevice::stream_idle(int s) {
  const hipError_t e = hipStreamQuery(hs(streams_[s]));
  if (e == hipErrorNotReady) return false;
  HIP_OK(e);
  return true;
}
void HipDevice::sync_all() {
  for (int s = 0; s < kNumStreams; ++s) sync_stream(s);
}
float HipDevice::event_ms(int a, int b) {
  float ms = 0.f;
  HIP_OK(hipEventElapsedTime(&ms, static_cast<hipEvent_t>(events_[a]), static_cast<hipEvent_t>(events_[b])));
  return ms;
}
void* HipDevice::native_stream(int s) { return streams_[s]; }
static void check_launch();
// A marker is an event of its own (recorded once): other devices' streams wait on it by handle.
std::shared_ptr<void> HipDevice::mark(int s) {
  activate();
  hipEvent_t e;
  HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  HIP_OK(hipEventRecord(e, hs(streams_[s])));
  return std::shared_ptr<void>(static_cast<void*>(e), [](void* p) { (void)hipEventDestroy(static_cast<hipEvent_t>(p)); });
}
void HipDevice::wait_mark(int s, const std::shared_ptr<void>& h) {
  if (h) HIP_OK(hipStreamWaitEvent(hs(streams_[s]), static_cast<hipEvent_t>(h.get()), 0));
}
void HipDevice::occupy(int s, int nwg, double us, int lds_bytes) {
  kern::spin(nwg, us, hs(streams_[s]), lds_bytes);
  check_launch();
}
void HipDevice::zero_channels(void* p, size_t bytes, int s, int nwg, int lds_bytes) {
  if (!bytes) return;
  kern::zero_channels(p, bytes, nwg, lds_bytes, hs(streams_[s]));
  check_launch();
}

void* HipDevice::scratch(size_t bytes, int slot) {
  if (bytes > scratch_sz_[slot]) {
    activate();
    sync_all();
    if (scratch_[slot]) (void)hipFree(scratch_[slot]);
    scratch_[slot] = nullptr;
    HIP_OK(hipMalloc(&scratch_[slot], bytes));
    scratch_sz_[slot] = bytes;
  }
  return scratch_[slot];
}

static void check_launch() {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw Error(Status::CommError, std::string("kernel launch failed: ") + hipGetErrorString(e));
}

void HipDevice::generate(DType dt, void* X, const Layout& L, GenSpec g, int s) {
  kern::generate(dt, X, L, (int)g.kind, g.seed, hs(streams_[s]));
  check_launch();
}
void HipDevice::generate_norm(DType dt, void* X, const Layout& L, GenSpec g, double* out, int s) {
  kern::generate_norm(dt, X, L, (int)g.kind, g.seed, out, hs(streams_[s]));
  check_launch();
}
void HipDevice::widen(DType dt, double* dst, int64_t ldd, const void* X, int64_t ldx, int64_t rows,
                      int64_t cols, int s) {
  kern::widen(dt, dst, ldd, X, ldx, rows, cols, hs(streams_[s]));
  check_launch();
}
void HipDevice::upload_convert(DType dt, void* X, int64_t ldx, const double* src, int64_t src_ld,
                               int64_t rows, int64_t cols, int s) {
  kern::upload_convert(dt, X, ldx, src, src_ld, rows, cols, hs(streams_[s]));
  check_launch();
}
void HipDevice::extract_neg_t(DType dt, void* Lt, int64_t ldl, const void* X, int64_t ldx,
                              int64_t rows, int64_t col0, int64_t m, int s) {
  kern::extract_neg_t(dt, Lt, ldl, X, ldx, rows, col0, m, hs(streams_[s]));
  check_launch();
}
void HipDevice::add_diag(DType dt, void* A, int64_t ld, int64_t nd, double alpha, int s) {
  kern::add_diag(dt, A, ld, nd, alpha, hs(streams_[s]));
  check_launch();
}
size_t HipDevice::block_inverse_scratch_bytes(DType dt, const Layout& L, int variant) const {
  const size_t b1 = kern::block_inverse_scratch_bytes(dt, L, variant);
  return b1 ? b1 + kern::block_inverse_iscratch_bytes(L) : 0;
}
void HipDevice::prepare_block_inverse(DType dt, const Layout& L, int variant) {
  const size_t b1 = kern::block_inverse_scratch_bytes(dt, L, variant);
  if (!b1) return;
  scratch(b1, 0);
  scratch(kern::block_inverse_iscratch_bytes(L), 1);
}
void HipDevice::block_inverse(DType dt, const void* Lt, int64_t ldl, void* inv_t, double* scores,
                              int32_t* valid, const int32_t* used, const Layout& L, double thresh, int64_t nlive,
                              int s) {
  void* sc = nullptr;
  int* isc = nullptr;
  const int variant = bi_hint_;  // one read: the scratch must match the kernel that is launched
  const size_t b1 = kern::block_inverse_scratch_bytes(dt, L, variant);
  if (b1) {
    sc = scratch(b1, 0);
    isc = static_cast<int*>(scratch(kern::block_inverse_iscratch_bytes(L), 1));
  }
  kern::block_inverse(dt, Lt, ldl, inv_t, scores, valid, used, L, thresh, nlive, hs(streams_[s]), sc, isc, variant);
  check_launch();
}
bool HipDevice::block_inverse_select(DType dt, const void* Lt, int64_t ldl, void* inv_t, double* scores,
                                     int32_t* valid, const int32_t* used, const Layout& L, double thresh, int64_t nlive,
                                     const PivotSelectArgs& sel, int s) {
  const int variant = bi_hint_;
  const size_t b1 = kern::block_inverse_scratch_bytes(dt, L, variant);
  void* sc = b1 ? scratch(b1, 0) : nullptr;
  if (!kern::block_inverse_select(dt, Lt, ldl, inv_t, scores, valid, used, L, thresh, nlive, hs(streams_[s]), sel,
                                  variant, sc))
    return false;
  check_launch();
  return true;
}
void HipDevice::candidate_maxabs(DType dt, const void* Lt, int64_t ldl, double* scores, int32_t* valid,
                                 const int32_t* used, const Layout& L, double thresh, int s) {
  kern::candidate_maxabs(dt, Lt, ldl, scores, valid, used, L, thresh, hs(streams_[s]));
  check_launch();
}
void HipDevice::gather_candidate(DType dt, void* sel, const void* Lt, int64_t ldl, const PivotRec* rec,
                                 const Layout& L, int s) {
  kern::gather_candidate(dt, sel, Lt, ldl, rec, L, hs(streams_[s]));
  check_launch();
}
void HipDevice::commit_candidate(DType dt, void* inv_t, const void* inv1, const int32_t* valid1, const double* score1, double growth, PivotRec* rec,
                                 const Layout& L, int s) {
  kern::commit_candidate(dt, inv_t, inv1, valid1, score1, growth, rec, L, hs(streams_[s]));
  check_launch();
}
void HipDevice::pivot_local(const double* scores, const int32_t* valid, const int32_t* used,
                            const int32_t* pos, const Layout& L, PivotRec* out, int s) {
  kern::pivot_local(scores, valid, used, pos, L, out, hs(streams_[s]));
  check_launch();
}
void HipDevice::pivot_select_single(const double* scores, const int32_t* valid, const Layout& L,
                                    int32_t t, int32_t* pos, int32_t* phys_at, int32_t* used,
                                    int32_t* seq, PivotRec* rec, PivotResult* out,
                                    PivotResult* host_out, int s) {
  kern::pivot_select_single(scores, valid, L, t, pos, phys_at, used, seq, rec, out, host_out,
                            hs(streams_[s]));
  check_launch();
}
void HipDevice::pivot_global(const PivotRec* recs, int32_t p, int32_t t, int32_t* pos,
                             int32_t* phys_at, int32_t* used, int32_t* seq, PivotResult* out,
                             PivotResult* host_out, int s) {
  kern::pivot_global(recs, p, t, pos, phys_at, used, seq, out, host_out, hs(streams_[s]));
  check_launch();
}
void HipDevice::owner_edits(DType dt, void* At, int64_t ldl, const int32_t* phys, int64_t p, int64_t k, int64_t j,
                            int64_t m, void* lrow, void* ht, const void* inv, const PieceMove& mv, int s) {
  kern::owner_edits(dt, At, ldl, phys, p, k, j, m, lrow, ht, inv, mv, hs(streams_[s]));
  check_launch();
}
void HipDevice::take_rows(DType dt, void* dst, int64_t ldd, void* X, int64_t ldx, const int32_t* phys, int64_t p,
                          int64_t k, int64_t col0, int64_t w, int64_t m, int s) {
  kern::take_rows(dt, dst, ldd, X, ldx, phys, p, k, col0, w, m, hs(streams_[s]));
  check_launch();
}
void HipDevice::sum_slices(DType dt, void* dst, const void* src, int64_t count, int64_t nslices, int s) {
  kern::sum_slices(dt, dst, src, count, nslices, hs(streams_[s]));
  check_launch();
}
void HipDevice::zero_unless_owner(DType dt, void* buf, int64_t count, const int32_t* phys, int64_t p, int64_t k,
                                  int s) {
  kern::zero_unless_owner(dt, buf, count, phys, p, k, hs(streams_[s]));
  check_launch();
}
void HipDevice::h_block(DType dt, void* R, int64_t ldr, const void* Ht, int64_t m, int s) {
  kern::h_block(dt, R, ldr, Ht, m, hs(streams_[s]));
  check_launch();
}
void HipDevice::gemm(DType dt, GemmOp op, ALayout al, int64_t M, int64_t N, int64_t K, const void* A,
                     int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int s,
                     const GemmExtra& ex) {
  const GemmExtra* e = &ex;
  GemmExtra hinted;
  if (!ex.glds_tile && tile_hint_) {
    hinted = ex;
    hinted.glds_tile = tile_hint_;
    e = &hinted;
  }
  kern::gemm(dt, op == GemmOp::Acc ? 0 : 1, al == ALayout::KMajor ? 1 : 0, M, N, K, A, lda, B, ldb,
             C, ldc, hs(streams_[s]), e);
  check_launch();
}
void HipDevice::gemm_batch(DType dt, const GemmDesc* d, int n, int s) {
  if (n <= 0) return;
  kern::gemm_batch(dt, d, n, hs(streams_[s]));
  check_launch();
}
void HipDevice::permute_blocks(DType dt, void* dst, int64_t ldd, const void* X, int64_t ldx,
                               int64_t nblk, int64_t m, int64_t Nr, const int32_t* dst_blk,
                               const int32_t* colsrc, int s) {
  kern::permute_blocks(dt, dst, ldd, X, ldx, nblk, m, Nr, dst_blk, colsrc, hs(streams_[s]));
  check_launch();
}
void HipDevice::row_abs_max_minus_i(DType dt, const void* X, int64_t ldx, const Layout& L, double* out,
                                    int s) {
  kern::row_abs_max(dt, X, ldx, L, out, hs(streams_[s]), true);
  check_launch();
}
void HipDevice::hash_rows(const void* base, int64_t ld_bytes, int64_t width_bytes, int64_t rows, uint64_t* parts,
                          int s) {
  kern::hash_rows(base, ld_bytes, width_bytes, rows, parts, kHashParts, hs(streams_[s]));
}

void HipDevice::row_abs_max(DType dt, const void* X, int64_t ldx, const Layout& L, double* out,
                            int s) {
  kern::row_abs_max(dt, X, ldx, L, out, hs(streams_[s]));
  check_launch();
}
void HipDevice::residual(DType dt, const void* A, const void* Full, const Layout& L, double* out,
                         int s) {
  const int nparts = kern::residual_nparts(L.npad);
  double* partial = static_cast<double*>(scratch(sizeof(double) * (size_t)L.rows * nparts, 0));
  kern::residual_partial(dt, L.rows, L.npad, L.npad, A, L.npad, Full, L.npad, L.n, L.m, L.p, L.k,
                         partial, hs(streams_[s]));
  check_launch();
  kern::residual_reduce(partial, nparts, L, out, hs(streams_[s]));
  check_launch();
}

}  // namespace gj
