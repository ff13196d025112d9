// Distributed Gauss-Jordan engine — see gj/engine.hpp for the design summary.
//
// Reference parity map (main.cpp line numbers):
//   norm()              :643-667  -> norm_inf() (global max instead of the local strip norm)
//   pivot search        :1039-1066 -> select(): Device::block_inverse + pivot_local
//   MPI_Allreduce(piv)  :1074     -> Comm::allgather of 32-B records + Device::pivot_global
//   singular exit       :1075-1083 -> Status::Singular on every rank at the same step
//   gather_row + Bcast  :1093-1097 -> chunk_pipeline(): owner normalises, chunked broadcast
//   row swap            :1100-1131 -> none per step (logical bookkeeping) + finalize() once
//   normalise (replicated on all ranks) :1132-1159 -> once, on the owner, as an MFMA GEMM
//   eliminate           :1165-1194 -> big_update(): one MFMA GEMM of depth d*m per panel of d steps
//
// Panel algebra (steps t0..t0+q-1 of panel v, sequential semantics of the in-place sweep):
//   L_t = -X^(t)[:, t],  R_t = H_t X^(t)[s_t, :] with R_t[t] := H_t,  H_t = inv(X^(t)[s_t, t])
//   X^(t+1)[i, c] = X^(t)[i, c] + L_t[i] R_t[c]   (c != t, i != s_t)
//   X^(t+1)[i, t] = L_t[i] H_t ,  X^(t+1)[s_t, :] = R_t
// Unrolled over the panel this is ONE update  X += [L_t0 .. L_t1] [R_t0; ..; R_t1]  provided
//   * the panel's own block columns enter as 0 and R_t'[t] := 0 for t' < t inside the panel,
//   * the panel's pivot rows enter as 0 and their multiplier rows become [0 .. 0, I, L_t'' ..],
// which is exactly what the GEMM extras (zero columns / zero rows) and the owner-side edits do.
// Nothing cancels (no I + H tricks), so the numerics match the step-by-step reference.
#include "gj/engine.hpp"

#include "gj/io.hpp"
#include "../kernels/kernels.hpp"

#include <rocprofiler-sdk-roctx/roctx.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include <unistd.h>  // environ
#include <thread>

namespace gj {

namespace {
double now_s() {
  using clk = std::chrono::steady_clock;
  return std::chrono::duration<double>(clk::now().time_since_epoch()).count();
}
}  // namespace

namespace {
// `var`=<rank>:<tag>[,<rank>:<tag>...]: whether the list names (rank, tag).  Fault injection for
// the failure-agreement tests:
//   GJ_TEST_ALLOC_FAIL  tag = matrix | block | residual | residual_stream | residual64: that rank's
//                       allocation of that stage fails;
//   GJ_TEST_HANG        tag = a step number: that rank never issues the pivot exchange of that
//                       step (a rank stuck in, or dead before, a collective);
//   GJ_TEST_CORRUPT     tag = a step number: that rank zeroes its copy of the step's normalised
//                       pivot row in the first chunk it updates (a wrong inverse that must fail
//                       the residual check, bench.py / --check-residual).
bool injected(const char* var, int rank, const std::string& tag) {
  const char* e = std::getenv(var);
  if (!e || !*e) return false;
  const std::string all = e;
  size_t b = 0;
  while (b <= all.size()) {
    const size_t end = std::min(all.find(',', b), all.size());
    const std::string v = all.substr(b, end - b);
    const size_t c = v.find(':');
    if (c != std::string::npos && std::atoi(v.substr(0, c).c_str()) == rank && v.substr(c + 1) == tag) return true;
    b = end + 1;
  }
  return false;
}
bool injected_alloc_fail(int rank, const char* stage) { return injected("GJ_TEST_ALLOC_FAIL", rank, stage); }
// `var`=<rank>:<step>[,...]: the step named for this rank (-1: none).
int64_t injected_step(const char* var, int rank) {
  const char* e = std::getenv(var);
  if (!e || !*e) return -1;
  const std::string all = e;
  for (size_t b = 0; b <= all.size();) {
    const size_t end = std::min(all.find(',', b), all.size());
    const std::string v = all.substr(b, end - b);
    const size_t c = v.find(':');
    if (c != std::string::npos && std::atoi(v.substr(0, c).c_str()) == rank) return std::atoll(v.substr(c + 1).c_str());
    b = end + 1;
  }
  return -1;
}
}  // namespace

Engine::Engine(Device& dev, Comm& comm, int64_t n, int64_t m, const SolveOptions& opt)
    : dev_(dev), comm_(comm), opt_(opt) {
  GJ_REQUIRE(n > 0 && m > 0, "n and m must be positive");
  if (const char* e = std::getenv("GJ_VERIFY")) opt_.verify = opt_.verify || std::atoi(e) != 0;
  if (const char* e = std::getenv("GJ_STEP_EVENTS")) step_events_ = std::atoi(e) != 0;
  L_ = Layout::make(n, m, comm.size(), comm.rank());
  GJ_REQUIRE(L_.Nr < (int64_t(1) << 31), "too many block rows");
  // auto depth: profiles/small_n_sweep.md (N=8192: depth 2 34.6 vs 35.9 ms; N=16384: 4 wins), and
  // 8 on ranks of <= 4096 rows of a large matrix (p = 8 at N = 32768: K = 1024 halves the panel
  // boundaries the pivot chain must hide behind a short trailing update; emulated under the
  // communication-cost model 0.167 vs 0.177 s, while depth 6 / 8 lose at p = 1 / 2 / 4 and at
  // N = 16384: profiles/depth_pgt1.md)
  const bool small_rank = L_.p > 1 && L_.max_nblk * L_.m <= 4096;
  // Depth 2 on p > 1 ranks of <= 2048 rows (p = 8 at N = 16384) is 0.0382 vs 0.0408 s per emulated
  // rank under the direct 50 GB/s model (profiles/depth_pgt1.md), but it is the configuration of
  // the round-3 wrong inverse (p = 8, depth 2, async ranks), whose cause is not localised
  // (profiles/verify_r6.md): p > 1 keeps depth 4 by default; --depth 2 selects it explicitly.
  // (One GPU at N = 32768, depth 8 with the co-resident candidate inverse: 0.9 % faster on one box,
  // 0.5-0.8 % slower on another, same-box A/Bs of round 4 -- not adopted, profiles/rocprof_n32768_r4.md.)
  const int want = opt_.depth > 0 ? opt_.depth
                   : (L_.p == 1 && L_.npad <= 8192) ? 2
                   : (small_rank && L_.npad > 16384) ? 8 : 4;
  d_ = (int)std::max<int64_t>(1, std::min<int64_t>({(int64_t)want, (int64_t)kMaxDepth, L_.Nr}));
  f_ = d_;
  if (const char* e = std::getenv("GJ_FIRST_DEPTH"))
    if (std::atoi(e) > 0) f_ = (int)std::min<int64_t>({(int64_t)std::atoi(e), (int64_t)d_, L_.Nr});

  // Column chunk plan: fixed partition of the Nr block columns into runs of a multiple of d blocks.
  int64_t target_cols = opt_.chunk_cols;
  // 8192 columns: measured 2-4 % faster than 4096 / 16384 in the p = 2, 4, 8 critical-path
  // emulation at N = 32768 (fewer GEMM tails per panel, still 4 chunks to pipeline the broadcast)
  if (target_cols <= 0)
    target_cols = std::max<int64_t>((L_.npad + 7) / 8, std::min<int64_t>(8192, (L_.npad + 1) / 2));
  int64_t cw = std::max<int64_t>(1, target_cols / m);
  cw = ((cw + d_ - 1) / d_) * d_;
  // (chunk boundaries sit on panel boundaries: with a shallower first panel, at f_ + k d_ -- the
  // first chunk f_ blocks wider)
  if (const char* e = std::getenv("GJ_CHUNK_PLAN")) {
    // explicit plan for A/B runs: comma-separated block counts, each a multiple of d, summing to Nr
    int64_t b = 0;
    for (const char* s = e; *s;) {
      char* end = nullptr;
      const int64_t w = std::strtoll(s, &end, 10);
      GJ_REQUIRE(end != s && w > 0 && panel_boundary(b + w),
                 "GJ_CHUNK_PLAN: block counts must end on panel boundaries (multiples of the depth)");
      cb0_.push_back(b);
      cb1_.push_back(b + w);
      b += w;
      s = (*end == ',') ? end + 1 : end;
      GJ_REQUIRE(*end == ',' || *end == 0, "GJ_CHUNK_PLAN: expected a comma-separated list");
    }
    GJ_REQUIRE(b == L_.Nr, "GJ_CHUNK_PLAN: block counts must sum to the number of block columns");
  } else {
    for (int64_t b = 0; b < L_.Nr;) {
      const int64_t e = std::min(L_.Nr, b == 0 ? cw + (f_ < d_ ? f_ : 0) : b + cw);
      cb0_.push_back(b);
      cb1_.push_back(e);
      b = e;
    }
  }
  chunk_of_.resize(L_.Nr);
  for (size_t c = 0; c < cb0_.size(); ++c)
    for (int64_t b = cb0_[c]; b < cb1_[c]; ++b) chunk_of_[b] = (int64_t)c;

  // CU reservation for the latency-bound panel factorisation (GJ_RESERVE_CUS overrides).
  int rc = opt_.reserve_cus;
  if (const char* e = std::getenv("GJ_RESERVE_CUS")) rc = std::atoi(e);
  // auto: up to N = 16384 the pivot chain is the critical path and its block inverses only start
  // on a CU no trailing-update workgroup occupies, so keep 32 CUs (1/8 of the chip) off the MAIN
  // stream -- the first 32 mask bits, i.e. one CU of every shader engine (bits interleave XCCs, then
  // SEs: bench/cu_mask_probe.hip), since a launch's workgroups are split evenly over the 32 SEs and
  // an unbalanced mask makes the smallest SE the straggler (profiles/cu_reserve_sweep.md):
  // N=8192 p=1 -12 %, emulated p=2/4/8 at N=16384 -10/-16/-14 %.  At N=32768 the GEMM is the
  // critical path and the mask costs 4-10 % (profiles/cu_reserve_sweep.md) -- except on ranks
  // with <= 4096 rows (p = 8 at N = 32768), where the pivot chain and the RCCL workgroups of its
  // collectives need the free CUs: under the communication-cost model p = 8 is 6.6 % faster with
  // the reservation at 100 GB/s, p = 2 / 4 are 9 / 6 % slower (profiles/cu_reserve_pgt1.md).
  if (rc < 0) rc = (dev_.on_gpu() && (L_.npad <= 16384 || small_rank)) ? 32 : 0;
  reserved_cus_ = dev_.reserve_cus(rc);
  // (round 5, peeled loop: at N <= 8192 on one GPU the 3-stage 4-per-CU build is faster even under
  // the reservation, 25.06 vs 25.43 ms; N = 16384 keeps 5 per CU, 153.9 vs 156.1 ms,
  // profiles/gemm_peel_r5.md)
  dense_gemm_ = reserved_cus_ > 0 && !(L_.p == 1 && L_.npad <= 8192);
  // The 128 x 128 trailing-update tile (3 per CU) on ranks of more than 8192 rows without a CU
  // reservation, where the GEMM is the critical path (N = 32768: 1120 -> 1083.5 ms on one box;
  // emulated p = 2: even); the 128 x 64 tile (4 per CU) elsewhere: under a reservation (N = 8192:
  // 22.7 vs 23.5 ms) and on the 8192-row ranks of p = 4 at N = 32768 (emulated 0.2735 vs 0.2911 s
  // comm-free), whose pivot chain needs the slots (profiles/gemm_tile128_r6.md)
  gemm_tile_ = (reserved_cus_ == 0 && L_.max_nblk * L_.m > 8192) ? 128 : 64;
  dev_.set_gemm_tile_hint(gemm_tile_);
  if (const char* e = std::getenv("GJ_DENSE_GEMM")) dense_gemm_ = std::atoi(e) != 0;
  // (Rounds 2-5) candidate inverses on ranks whose trailing update holds every CU (p > 1 without a
  // reservation: the 16384- and 8192-row ranks of N = 32768) took the co-resident 4-wave form, which starts in
  // the slot one retiring trailing-update workgroup frees instead of waiting for a whole CU: the
  // p = 4 rank spends 616 of its 1154 us per step in a block inverse that alone takes ~100 us
  // (profiles/rocprof_emu4_r2.md).  Rank-0 emulation at N = 32768, 100 GB/s model: p = 2 0.585 ->
  // 0.576 s, p = 4 0.312 -> 0.299 s; on one GPU (and under the reservation) the register form stays
  // (N = 32768: 1152.7 vs 1161.0 ms, profiles/blockinv_coresident.md).  GJ_BI_CORESIDENT=0/1
  // overrides; an explicit process-wide GJ_BI_VARIANT wins.
  {
    const bool fits = opt_.dtype == DType::F64 && L_.m > 32 && L_.m <= 128;
    // Round 6, on the 2-stage 128 x 128 / 3-stage 128 x 64 trailing-update tiles: the register form
    // is faster on those ranks too (scripts/runs/r6_emuco.sh, emulated N = 32768, two repetitions:
    // p = 2 0.5305 / 0.5313 -> 0.5258 / 0.5275 s comm-free, p = 4 0.2740 / 0.2741 -> 0.2717 / 0.2721
    // s, direct 50 GB/s 0.2866 / 0.2873 -> 0.2776 / 0.2776 s; one GPU, profiles/blockinv_coresident.md):
    // the co-resident form is opt-in (GJ_BI_CORESIDENT=1).
    bool co = false;
    if (const char* e = std::getenv("GJ_BI_CORESIDENT")) co = std::atoi(e) != 0;
    if (std::getenv("GJ_BI_VARIANT")) co = false;
    bi_hint_ = (co && fits) ? 5 : -1;
    // (Measured round 4: the co-resident form only for steps whose live candidates outnumber the
    // reserved CUs -- two per CU, one round instead of two -- N = 8192 25.72 -> 27.36 ms: slower.)
  }

  comm_.set_timeout(opt_.comm_timeout_s);
  // Fault injection (tests only) must never pass for a normal run: every active knob is announced
  // on stderr once per engine and reported in the policy (bench.py / --json carry it).
  for (const char* var : {"GJ_TEST_ALLOC_FAIL", "GJ_TEST_HANG", "GJ_TEST_CORRUPT", "GJ_TEST_DROP_WAIT"})
    if (const char* e = std::getenv(var))
      if (*e) {
        if (!fault_injection_.empty()) fault_injection_ += " ";
        fault_injection_ += std::string(var) + "=" + e;
      }
  if (const char* e = std::getenv("GJ_EVENT_RELEASE"))
    if (std::string(e) == "none") fault_injection_ += std::string(fault_injection_.empty() ? "" : " ") + "GJ_EVENT_RELEASE=none";
  if (!fault_injection_.empty())
    std::fprintf(stderr, "gj: rank %d: WARNING: FAULT INJECTION ACTIVE (%s): results of this run are "
                         "deliberately wrong, hung or failed\n",
                 (int)L_.k, fault_injection_.c_str());
  for (char** e = environ; e && *e; ++e)
    if (std::strncmp(*e, "GJ_", 3) == 0) env_overrides_.push_back(*e);
  std::sort(env_overrides_.begin(), env_overrides_.end());
  hang_step_ = injected_step("GJ_TEST_HANG", L_.k);
  corrupt_step_ = injected_step("GJ_TEST_CORRUPT", L_.k);
  // "<rank>:<step>:unprofiled": only solves without the phase timers are corrupted (the bench's
  // timed solves, not its untimed profiled one -- tests that the gate checks a timed solve)
  if (const char* e = std::getenv("GJ_TEST_CORRUPT")) corrupt_unprofiled_ = std::strstr(e, ":unprofiled") != nullptr;
  if (const char* e = std::getenv("GJ_TEST_DROP_WAIT")) drop_wait_ = std::string(",") + e + ",";
  dev_.trace_context(&cur_step_, &cur_phase_);  // names the step / phase in schedule-check reports
  // Allocation, agreed on every rank BEFORE any other collective (reference main.cpp:366-381 and
  // :428-436): 2 = this rank's matrix panels do not fit ("Not enough memory!", thrown on every
  // rank), 1 = the elimination work space does not ("not enough memory for block", reported by
  // solve() on every rank), 0 = ok.  With Nr % p != 0 the low ranks own one more block row, so near
  // the HBM limit a single rank can fail alone; its peers must not run on into the broadcast tuner.
  std::string why;
  const int mine = alloc_buffers(why);
  const int agreed = (int)comm_.host_max(dev_, (double)mine);
  if (agreed == 2) {
    free_buffers();
    throw Error(Status::NoMemory, mine == 2 ? why : "not enough device memory on a peer rank");
  }
  if (agreed == 1) {
    free_work();
    block_mem_fail_ = true;
    block_mem_why_ = mine == 1 ? why : "not enough device memory for the work space on a peer rank";
  }
  // Broadcast algorithm for the panel pieces (m x d*m) and the pivot-row segments (m x chunk width):
  // ring or direct, measured here
  // on a GPU transport at p > 2 (Comm::tune_bcast; every rank takes the same decision).
  if (!block_mem_fail_) {
    int64_t wmax = 0;
    for (size_t c = 0; c < cb0_.size(); ++c) wmax = std::max(wmax, chunk_w((int64_t)c));
    const size_t pp_bytes = (size_t)L_.m * d_ * L_.m * esz();  // panel piece (SIDE, pivot chain)
    bcast_algo_ = comm_.tune_bcast(dev_, std::vector<size_t>{pp_bytes, (size_t)L_.m * wmax * esz()});
  }
  // (One trailing-update stream: two alternating ones were measured slower, N=32768 1283 vs 1167 ms,
  // p=8 emulation 0.191 vs 0.166 s -- concurrent GEMMs interleave their tiles, lose L2 locality and
  // crowd out the pivot path -- and were removed in round 3.)
  // COMM chunk-normalisation GEMMs (m x chunk width x m) on the small 64x32 latency tile: 4x the
  // workgroups of the 128x64 tile.  Round 2 (profiles/small_n_sweep.md): N = 8192 30.2 -> 29.3 ms,
  // N = 16384 +1.1 %, N = 32768 +0.7 %.  Round 4, with the look-ahead rows on SIDE the chunk pass
  // is off the pivot chain at every size: N = 8192 25.80 / 25.74 (small) vs 25.66 / 25.56 ms,
  // N = 16384 even (scripts/runs/r4_cst.sh) -- off by default; GJ_COMM_SMALL_TILES=1 turns it on.
  comm_small_tiles_ = false;
  // Look-ahead rows on SIDE, right behind the panel pieces, at every p (GJ_LA_SIDE=0 puts them on
  // COMM at p = 1, round 3's one-rank choice): with the host-free pivot chain, COMM's queue (the
  // previous panel's chunk pass, waiting for MAIN) is what held them back.  Round 4, same box,
  // two repetitions: N = 8192 26.71 / 26.73 -> 25.73 / 25.80 ms; N = 16384 and 32768 neutral.
  la_side_ = true;
  if (const char* e = std::getenv("GJ_LA_SIDE")) la_side_ = std::atoi(e) != 0;
  if (const char* e = std::getenv("GJ_HOST_FREE")) host_free_multi_ = std::atoi(e) != 0;
  if (const char* e = std::getenv("GJ_COMM_SMALL_TILES")) comm_small_tiles_ = std::atoi(e) != 0;
  // Measured round 5 (scripts/runs/r5_ab.sh, one box, two repetitions), deferred half on COMM (1):
  // N = 8192 25.35 / 25.49 -> 25.90 / 25.96 ms, N = 16384 159.6 / 160.7 -> 158.9 / 158.5, N = 32768
  // 1130 / 1131 -> 1139 / 1139 ms, emulated p = 4 at N = 16384 (direct 50 GB/s) 0.0515 -> 0.0586 s:
  // it delays COMM's chunk pass and runs on the same reserved CUs as the chain.  GJ_SPLIT=2 puts it
  // on MAIN instead (profiles/split_r5.md).
  // Chain column updates on the LDS-DMA kernel where the chain has reserved CUs at p = 1
  // (scripts/runs/r5_split2.sh / r5_latglds.sh, one box, two repetitions): N = 8192 24.58 / 24.55 ->
  // 24.38 / 24.34 ms, N = 16384 152.2 / 152.0 -> 152.4 / 152.1; without a reservation (N = 32768)
  // 1100.1 / 1100.2 -> 1105.6 / 1101.4 ms, emulated p = 4 / 8 even.  GJ_LAT_GLDS=0/1 overrides.
  // One launch around the look-ahead columns (MAIN) and around the panel / next-panel columns (the
  // chunk pass) where CUs are reserved for the chain (scripts/runs/r5_skip.sh, r5_skip2.sh): N = 8192
  // 24.20 -> 23.61 ms, N = 16384 151.5 -> 150.3 ms, emulated p = 8 at N = 16384 -3 %; without a
  // reservation (N = 32768) the MAIN merge measured +0.1-0.3 % and the chunk-pass merge +1.5 %.
  // Round 6, 128 x 128 tile (3 per CU, twice the work per tile: a split chunk's two launch tails
  // cost more): the MAIN merge at N = 32768 1078.2 / 1079.5 -> 1076.3 / 1075.5 ms, same box,
  // alternating (scripts/runs/r6_skip128.sh) -- on wherever that tile runs; the chunk-pass merge
  // stays with the reservation.
  // MAIN's trailing update streams its C tile (read and written once per panel) with the
  // non-temporal cache policy, loads and stores (GemmExtra::c_nt; GJ_MAIN_CNT=<bits> overrides):
  // N = 32768 1129.9 / 1129.6 -> 1111.7 / 1109.8 ms with every LDS-DMA launch streaming (one box,
  // scripts/runs/r6_cnt.sh); MAIN's launches only, another box: N = 8192 23.04 -> 22.86 ms, 16384
  // 149.2 -> 147.9 ms, 32768 1070.1 -> 1057.8 ms (scripts/runs/r6_cnt2.sh, profiles/gemm_cache_policy_r6.md)
  main_cnt_ = 3;
  if (const char* e = std::getenv("GJ_MAIN_CNT")) main_cnt_ = std::atoi(e) & 3;
  if (const char* e = std::getenv("GJ_MAIN_SPLIT")) main_split_ = std::atoi(e);
  skip_cols_ = reserved_cus_ > 0 || gemm_tile_ == 128;
  if (const char* e = std::getenv("GJ_SKIP_COLS")) skip_cols_ = std::atoi(e) != 0;
  chunk_skip_ = reserved_cus_ > 0;
  // the chain's latency GEMMs on the register-fed small kernel where CUs are reserved for it
  // (scripts/runs/r5_latk.sh): N = 8192 23.42 -> 22.80 ms, emulated p = 8 at N = 32768 -1.5 / -3.7 %
  // (comm-free / direct 50 GB/s), p = 4 at N = 16384 -4 %; N = 16384 even
  lat_reg_ = reserved_cus_ > 0;
  if (const char* e = std::getenv("GJ_LAT_REG")) lat_reg_ = std::atoi(e) != 0;
  if (const char* e = std::getenv("GJ_CHUNK_SKIP")) chunk_skip_ = std::atoi(e) != 0;
  // (N = 16384, once the register-fed latency kernel exists: that kernel is 0.25 % faster for the
  // 16384-row column update, 149.4 -> 149.0 ms; N = 8192 keeps the LDS-DMA kernel, 22.83 vs 22.92 ms;
  // scripts/runs/r5_colupd.sh)
  lat_wide_ = reserved_cus_ > 0 && L_.p == 1 && L_.npad <= 8192;
  if (const char* e = std::getenv("GJ_LAT_GLDS")) lat_wide_ = std::atoi(e) != 0;
  // GJ_CHUNK_BUILD=23|25|33: the LDS-DMA build of the chunk pass's normalisation GEMMs (COMM).
  // Under a CU reservation MAIN fills its 224 CUs, so COMM's workgroups land on the 32 reserved
  // ones, where their LDS (40 KiB each at 3 stages) decides whether an 11-wave, 95 KiB candidate
  // inverse still fits beside them (profiles/side_latency_r5.md, profiles/chain_r6.md).
  if (const char* e = std::getenv("GJ_CHUNK_BUILD")) chunk_build_ = std::atoi(e);
  if (const char* e = std::getenv("GJ_CHUNK_TILE")) chunk_tile_ = std::atoi(e);  // 64 | 128 (A/B)
  split_ = 0;
  if (const char* e = std::getenv("GJ_SPLIT")) {
    const int v = std::atoi(e);
    if (v < 0 || v > 2) throw Error(Status::BadArgs, "GJ_SPLIT: 0 | 1 | 2");
    // The deferred updates on MAIN (2) gave intermittent wrong inverses on the GPU at p = 8
    // asynchronous ranks, depth 2 (3 of 3 standalone failures of the schedule-variant test were this
    // variant; the host executor and the happens-before checker find it race-free):
    // refused there until the GPU-only hazard is found (profiles/verify_r6.md)
    if (v == 2 && L_.p > 1 && dev_.on_gpu())
      throw Error(Status::BadArgs, "GJ_SPLIT=2 is not supported on the GPU at p > 1 (intermittent wrong "
                                   "inverse, profiles/verify_r6.md); use GJ_SPLIT=1 or 0");
    if (L_.m % 64 == 0 && L_.nblk <= 64 * GemmExtra::kRselWords && L_.nblk > 0) split_ = v;
  }

}

Engine::~Engine() {
  free_buffers();
  comm_.free_scratch(dev_);
  dev_.trace_context(nullptr, nullptr);
}

Engine::Policy Engine::policy() const {
  Policy p;
  p.depth = d_;
  p.first_depth = f_;
  p.main_cnt = main_cnt_;
  p.env_overrides = env_overrides_;
  p.gemm_tile = gemm_tile_;
  p.nchunks = (int)cb0_.size();
  for (size_t c = 0; c < cb0_.size(); ++c) p.chunk_cols = std::max(p.chunk_cols, chunk_w((int64_t)c));
  p.reserve_cus = reserved_cus_;
  p.block_inverse = dev_.on_gpu() ? kern::block_inverse_kernel_name(opt_.dtype, L_.m, bi_hint_) : "host";
  p.comm_small_tiles = comm_small_tiles_;
  p.dense_gemm = dense_gemm_;
  p.la_side = la_side_;
  p.pivot = opt_.pivot == PivotRule::Partial ? "partial" : "block-min-inv-norm";
  p.fault_injection = fault_injection_;
  p.split = split_;
  p.lat_wide = lat_wide_;
  p.skip_cols = skip_cols_;
  p.lat_reg = lat_reg_;
  p.chunk_skip = chunk_skip_;
  return p;
}

int64_t Engine::real_local_rows() const {
  if (L_.nblk == 0) return 0;
  const int64_t last_global_block = L_.global_block(L_.nblk - 1);
  return L_.rows - (last_global_block == L_.Nr - 1 ? (L_.m - L_.l_h) : 0);
}


int Engine::alloc_buffers(std::string& why) {
  const int64_t m = L_.m, rows = std::max<int64_t>(L_.rows, 1), npad = L_.npad, dm = (int64_t)d_ * m;
  const size_t es = esz();
  const size_t panel = (size_t)rows * npad * es;
  int64_t wmax = 0;
  for (size_t c = 0; c < cb0_.size(); ++c) wmax = std::max(wmax, chunk_w((int64_t)c));
  const size_t need_matrix = 2 * panel;
  const size_t need_work = 3 * (size_t)dm * rows * es + 2 * (size_t)dm * npad * es + 4 * (size_t)dm * dm * es +
                           (size_t)m * dm * es +
                           (size_t)std::max<int64_t>(L_.nblk, 1) * m * m * es + (size_t)m * wmax * es +
                           dev_.block_inverse_scratch_bytes(opt_.dtype, L_, bi_hint_);
  const size_t avail = dev_.on_gpu() ? dev_.free_memory() : SIZE_MAX;
  auto fits = [&](size_t need) { return !dev_.on_gpu() || need + (64u << 20) <= avail; };
  // stage 1: the matrix panels (the reference's a / b arrays)
  try {
    if (injected_alloc_fail(L_.k, "matrix")) throw Error(Status::NoMemory, "injected (GJ_TEST_ALLOC_FAIL)");
    if (!fits(need_matrix))
      throw Error(Status::NoMemory, "not enough device memory: the matrix panels need " +
                                        std::to_string(need_matrix) + " bytes, have " + std::to_string(avail));
    X_ = dev_.alloc(panel);
    out_ = dev_.alloc(panel);
    dev_.label(X_, "X");
    dev_.label(out_, "out");
  } catch (const Error& e) {
    if (e.status() != Status::NoMemory) throw;
    why = e.what();
    free_buffers();
    return 2;
  }
  // stage 2: the elimination work space (the reference's per-step block buffers, main.cpp:960-975)
  try {
    if (injected_alloc_fail(L_.k, "block")) throw Error(Status::NoMemory, "injected (GJ_TEST_ALLOC_FAIL)");
    if (!fits(need_matrix + need_work))
      throw Error(Status::NoMemory, "not enough device memory: the work space needs " +
                                        std::to_string(need_work) + " bytes beyond the matrix, have " +
                                        std::to_string(avail));
    alloc_work(wmax);
  } catch (const Error& e) {
    if (e.status() != Status::NoMemory) throw;
    why = e.what();
    free_work();
    return 1;
  }
  return 0;
}

void Engine::alloc_work(int64_t wmax) {
  const int64_t m = L_.m, rows = std::max<int64_t>(L_.rows, 1), npad = L_.npad, dm = (int64_t)d_ * m;
  const size_t es = esz();
  for (int i = 0; i < 3; ++i) At_[i] = dev_.alloc((size_t)dm * rows * es);
  for (int i = 0; i < 2; ++i) {
    Rb_[i] = dev_.alloc((size_t)dm * npad * es);
    PP_[i] = dev_.alloc((size_t)dm * dm * es);
    LA_[i] = dev_.alloc((size_t)dm * dm * es);
    for (int j = 0; j < d_; ++j) {
      Lrow_[i][j] = dev_.alloc((size_t)std::max<int64_t>(j, 1) * m * m * es);
      Ht_[i][j] = dev_.alloc((size_t)m * m * es);
    }
  }
  T_ = dev_.alloc((size_t)m * wmax * es);
  RP_ = dev_.alloc((size_t)m * dm * es);
  T2_ = dev_.alloc((size_t)m * dm * es);
  inv_ = dev_.alloc((size_t)std::max<int64_t>(L_.nblk, 1) * m * m * es);
  if (opt_.pivot == PivotRule::Partial) {
    L1_ = Layout::make(m, m, 1, 0);
    sel_ = dev_.alloc((size_t)m * m * es);
    inv1_ = dev_.alloc((size_t)m * m * es);
    score1_ = static_cast<double*>(dev_.alloc(sizeof(double)));
    valid1_ = static_cast<int32_t*>(dev_.alloc(sizeof(int32_t)));
    used1_ = static_cast<int32_t*>(dev_.alloc(sizeof(int32_t)));
    dev_.memset0(used1_, sizeof(int32_t), S_SIDE);
    dev_.sync_stream(S_SIDE);
  }
  // the candidate-inverse kernel's scratch, now: not lazily inside the first timed pivot search
  dev_.prepare_block_inverse(opt_.dtype, L_, bi_hint_);
  scores_ = static_cast<double*>(dev_.alloc(sizeof(double) * std::max<int64_t>(L_.nblk, 1)));
  valid_ = static_cast<int32_t*>(dev_.alloc(sizeof(int32_t) * std::max<int64_t>(L_.nblk, 1)));
  pos_ = static_cast<int32_t*>(dev_.alloc(sizeof(int32_t) * L_.Nr));
  phys_at_ = static_cast<int32_t*>(dev_.alloc(sizeof(int32_t) * L_.Nr));
  used_ = static_cast<int32_t*>(dev_.alloc(sizeof(int32_t) * L_.Nr));
  seq_ = static_cast<int32_t*>(dev_.alloc(sizeof(int32_t) * L_.Nr));
  myrec_ = static_cast<PivotRec*>(dev_.alloc(sizeof(PivotRec)));
  sel_done_ = static_cast<int32_t*>(dev_.alloc(sizeof(int32_t)));
  dev_.memset0(sel_done_, sizeof(int32_t), S_SIDE);
  dev_.sync_stream(S_SIDE);
  recs_ = static_cast<PivotRec*>(dev_.alloc(sizeof(PivotRec) * L_.p));
  piv_dev_ = static_cast<PivotResult*>(dev_.alloc(sizeof(PivotResult)));
  dscratch_ = static_cast<double*>(dev_.alloc(sizeof(double) * 64));
  if (opt_.verify)
    vparts_ = static_cast<uint64_t*>(
        dev_.alloc(sizeof(uint64_t) * Device::kHashParts * (size_t)npanels() * (size_t)vslots()));
  ihost_len_ = std::max<int64_t>(L_.Nr, 16) * 2 + 16;
  iscratch_ = static_cast<int32_t*>(dev_.alloc(sizeof(int32_t) * ihost_len_));
  piv_host_ = static_cast<PivotResult*>(dev_.alloc_pinned_coherent(sizeof(PivotResult) * kPivSlots));
  ihost_ = static_cast<int32_t*>(dev_.alloc_pinned(sizeof(int32_t) * ihost_len_));
  dhost_ = static_cast<double*>(dev_.alloc_pinned(sizeof(double) * 64));
  label_work();

  if (ev_L_ >= 0) return;  // events are the device's; created once
  ev_L_ = dev_.create_event();
  ev_main_ = dev_.create_event();
  for (int i = 0; i < 2; ++i) {
    ev_edit_[i] = dev_.create_event();
    for (int j = 0; j < kMaxDepth; ++j) ev_pp_[i][j] = dev_.create_event();
    ev_la_[i] = dev_.create_event();
    ev_cp_[i] = dev_.create_event();
    ev_def_[i] = dev_.create_event();
    for (size_t c = 0; c < cb0_.size(); ++c) ev_b_[i].push_back(dev_.create_event());
  }
  for (size_t c = 0; c < cb0_.size(); ++c) ev_c_.push_back(dev_.create_event());
}

// Buffer names in schedule-check reports (RaceCheckDevice).
void Engine::label_work() {
  static const char* at[3] = {"At[0]", "At[1]", "At[2]"};
  static const char* rb[2] = {"Rb[0]", "Rb[1]"};
  static const char* pp[2] = {"PP[0]", "PP[1]"};
  static const char* la[2] = {"LA[0]", "LA[1]"};
  for (int i = 0; i < 3; ++i) dev_.label(At_[i], at[i]);
  for (int i = 0; i < 2; ++i) {
    dev_.label(Rb_[i], rb[i]);
    dev_.label(PP_[i], pp[i]);
    dev_.label(LA_[i], la[i]);
    for (int j = 0; j < d_; ++j) {
      dev_.label(Lrow_[i][j], (std::string("Lrow[") + char('0' + i) + "][" + char('0' + j) + "]").c_str());
      dev_.label(Ht_[i][j], (std::string("Ht[") + char('0' + i) + "][" + char('0' + j) + "]").c_str());
    }
  }
  const std::pair<const void*, const char*> named[] = {
      {T_, "T"}, {RP_, "RP"}, {T2_, "T2"}, {inv_, "inv"}, {sel_, "sel"}, {inv1_, "inv1"}, {scores_, "scores"},
      {valid_, "valid"}, {pos_, "pos"}, {phys_at_, "phys_at"}, {used_, "used"}, {seq_, "seq"}, {myrec_, "myrec"},
      {sel_done_, "sel_done"}, {recs_, "recs"}, {piv_dev_, "piv_dev"}, {dscratch_, "dscratch"},
      {iscratch_, "iscratch"}, {piv_host_, "piv_host"}, {ihost_, "ihost"}, {dhost_, "dhost"},
      {vparts_, "vparts"}};
  for (const auto& nv : named)
    if (nv.first) dev_.label(nv.first, nv.second);
}

void Engine::free_work() {
  std::vector<void**> dptrs = {&T_, &T2_, &RP_, &inv_, &sel_, &inv1_, reinterpret_cast<void**>(&score1_),
                               reinterpret_cast<void**>(&valid1_), reinterpret_cast<void**>(&used1_),
                               reinterpret_cast<void**>(&scores_),
                               reinterpret_cast<void**>(&valid_), reinterpret_cast<void**>(&pos_),
                               reinterpret_cast<void**>(&phys_at_), reinterpret_cast<void**>(&used_),
                               reinterpret_cast<void**>(&seq_), reinterpret_cast<void**>(&myrec_),
                               reinterpret_cast<void**>(&sel_done_),
                               reinterpret_cast<void**>(&recs_), reinterpret_cast<void**>(&piv_dev_),
                               reinterpret_cast<void**>(&dscratch_), reinterpret_cast<void**>(&iscratch_),
                               reinterpret_cast<void**>(&vparts_)};
  for (int i = 0; i < 3; ++i) dptrs.push_back(&At_[i]);
  for (int i = 0; i < 2; ++i) {
    dptrs.push_back(&Rb_[i]);
    dptrs.push_back(&PP_[i]);
    dptrs.push_back(&LA_[i]);
    for (int j = 0; j < kMaxDepth; ++j) {
      dptrs.push_back(&Lrow_[i][j]);
      dptrs.push_back(&Ht_[i][j]);
    }
  }
  for (void** p : dptrs)
    if (*p) {
      dev_.release(*p);
      *p = nullptr;
    }
  std::vector<void**> hptrs = {reinterpret_cast<void**>(&piv_host_), reinterpret_cast<void**>(&ihost_),
                               reinterpret_cast<void**>(&dhost_)};
  for (void** p : hptrs)
    if (*p) {
      dev_.release_pinned(*p);
      *p = nullptr;
    }
}

void Engine::free_buffers() {
  free_work();
  for (void** p : {&X_, &out_})
    if (*p) {
      dev_.release(*p);
      *p = nullptr;
    }
}

void Engine::dbg_sync() {
  if (opt_.sync_debug) comm_.drain_all(dev_);
}

const char* phase_name(int ph) {
  static const char* names[kNumPhases] = {"column",    "pivot_search", "pivot_exchange",
                                          "owner_edits", "panel_pieces", "normalise_rows",
                                          "row_bcast", "trailing_update", "finalize"};
  return (ph >= 0 && ph < kNumPhases) ? names[ph] : "?";
}

// Spin on the pinned pivot record (the wait is on the critical path of small problems: polling host
// memory reacts in ~1 us where an event query took ~25), checking the communicator every 20 ms and
// giving up after comm_timeout_s: a dead peer turns into an error on every surviving rank instead
// of a hang (reference: none).
void Engine::wait_pivot(int par, int64_t step, double& host_wait) {
  const double w0 = now_s();
  double next_check = w0 + 0.02;
  int spins = 0;
  const volatile int32_t* st = &piv_host_[par].step;
  while (*st != (int32_t)step) {
    if (++spins > 2000) std::this_thread::yield();
    const double t = now_s();
    if (t >= next_check) {
      comm_.check_health();
      if (t - w0 > opt_.comm_timeout_s) {
        comm_.abort();
        throw Error(Status::CommError, "timed out after " + std::to_string(opt_.comm_timeout_s) +
                                           " s waiting for the pivot of step " + std::to_string(step) +
                                           " behind the " + comm_.last_op(S_SIDE) + " (peer failure or hang)");
      }
      next_check = t + 0.02;
    }
  }
  std::atomic_thread_fence(std::memory_order_acquire);
  dev_.host_acquire(&piv_host_[par], sizeof(PivotResult));
  host_wait += now_s() - w0;
}

int Engine::prof_event() {
  if (pev_next_ == pev_pool_.size()) pev_pool_.push_back(dev_.create_event(/*timing=*/true));
  return pev_pool_[pev_next_++];
}
int Engine::prof_begin(int s) {
  if (!opt_.profile) return -1;
  const int e = prof_event();
  dev_.record(e, s);
  return e;
}
void Engine::prof_end(int phase, int ev0, int s) {
  if (ev0 < 0) return;
  const int e = prof_event();
  dev_.record(e, s);
  pmarks_.push_back({phase, ev0, e});
}
void Engine::prof_collect(SolveStats& st) {
  if (!opt_.profile) return;
  dev_.sync_all();
  for (const auto& mk : pmarks_) {
    st.phase_ms[mk.phase] += dev_.event_ms(mk.ev0, mk.ev1);
    st.phase_calls[mk.phase] += 1;
  }
  st.profiled = true;
  pmarks_.clear();
  pev_next_ = 0;
}

namespace {
// roctx range for the host-side enqueue of a phase (visible with rocprofv3 --marker-trace)
struct Range {
  bool on;
  Range(bool enabled, const char* name) : on(enabled) {
    if (on) roctxRangePushA(name);
  }
  ~Range() {
    if (on) roctxRangePop();
  }
};
}  // namespace

// ---------------------------------------------------------------- input
void Engine::generate(GenSpec g) {
  // the local row norm comes with the generation pass (Device::generate_norm): solve() then skips
  // its own pass over the matrix (N = 32768: 1.5 ms of a 4.6 ms generate + norm)
  solved_ = false;
  static const bool fused = !std::getenv("GJ_GEN_NORM") || std::atoi(std::getenv("GJ_GEN_NORM")) != 0;
  if (!fused || block_mem_fail_ || !dscratch_ || !dhost_) {  // (no work buffers: the solve reports it)
    dev_.generate(opt_.dtype, X_, L_, g, S_MAIN);
    dev_.sync_stream(S_MAIN);
    local_norm_valid_ = false;
    return;
  }
  dev_.generate_norm(opt_.dtype, X_, L_, g, dscratch_, S_MAIN);
  dev_.copy(dhost_, dscratch_, sizeof(double), S_MAIN);
  dev_.sync_stream(S_MAIN);
  local_norm_ = dhost_[0];
  local_norm_valid_ = true;
}

void Engine::upload_local_rows(const double* host, int64_t ld) {
  upload_rows_into(X_, opt_.dtype, host, ld);
  local_norm_valid_ = false;
  solved_ = false;
}

void Engine::upload_rows_device(const void* src, int64_t ld) {
  GenSpec z;
  z.kind = GenKind::Zero;  // zero + identity on the padded diagonal
  dev_.generate(opt_.dtype, X_, L_, z, S_MAIN);
  const int64_t real = real_local_rows();
  if (real > 0)
    dev_.copy2d(X_, L_.npad * esz(), src, ld * esz(), L_.n * esz(), real, S_MAIN);
  dev_.sync_stream(S_MAIN);
  local_norm_valid_ = false;
  solved_ = false;
}

void Engine::download_rows_device(void* dst, int64_t ld) {
  const int64_t real = real_local_rows();
  if (real > 0)
    dev_.copy2d(dst, ld * esz(), out_, L_.npad * esz(), L_.n * esz(), real, S_MAIN);
  dev_.sync_stream(S_MAIN);
}

// One rank's share of a matrix file (reference read_matrix, main.cpp:209-282: there one rank parses
// everything and sends every block row to its owner; here every rank maps the file and parses
// only its own rows, so no rank holds more than its share).  Errors are agreed in the reference's
// order: "cannot open" on any rank first, then "cannot read".
Status Engine::read_file_rows(const std::string& path, int nthreads, std::vector<double>& rows) {
  std::vector<int64_t> mine;
  const int64_t real = real_local_rows();
  mine.reserve((size_t)real);
  for (int64_t r = 0; r < real; ++r) mine.push_back(L_.global_row(r));
  Status s = Status::Ok;
  if (nthreads <= 0)  // the p ranks of a node share its cores
    nthreads = (int)std::max<int64_t>(1, (int64_t)std::max(1u, std::thread::hardware_concurrency()) / L_.p);
  try {
    s = read_matrix_rows(path, L_.n, mine, rows, nthreads);
  } catch (const std::exception&) {  // bad_alloc, thread creation (system_error), ...: agreed below
    s = Status::CannotRead;
  }
  if (comm_.host_max(dev_, s == Status::CannotOpen ? 1.0 : 0.0) > 0) return Status::CannotOpen;
  if (comm_.host_max(dev_, s != Status::Ok ? 1.0 : 0.0) > 0) return Status::CannotRead;
  return Status::Ok;
}

Status Engine::load_file(const std::string& path, int nthreads) {
  std::vector<double> rows;
  const Status s = read_file_rows(path, nthreads, rows);
  if (s == Status::Ok) upload_local_rows(rows.data(), L_.n);
  return s;
}

double Engine::residual_file(const std::string& path, int nthreads, Status* status) {
  GJ_REQUIRE(solved_, "residual: solve() first");
  std::vector<double> rows;
  const Status s = read_file_rows(path, nthreads, rows);  // re-read, like main.cpp:463-484
  if (status) *status = s;
  if (s != Status::Ok) return -1.0;
  return residual_rows(rows.data(), L_.n);
}

double Engine::result_norm_inf() {
  GJ_REQUIRE(solved_, "result_norm_inf: solve() first");
  double local = 0.0;
  if (L_.nblk > 0) {
    dev_.row_abs_max(opt_.dtype, out_, L_.npad, L_, dscratch_, S_MAIN);
    dev_.copy(dhost_, dscratch_, sizeof(double), S_MAIN);
    dev_.sync_stream(S_MAIN);
    local = dhost_[0];
  }
  return comm_.host_max(dev_, local);
}

double Engine::norm_inf() {
  if (local_norm_valid_) return comm_.host_max(dev_, local_norm_);  // from generate()
  dev_.row_abs_max(opt_.dtype, X_, L_.npad, L_, dscratch_, S_MAIN);
  dev_.copy(dhost_, dscratch_, sizeof(double), S_MAIN);
  dev_.sync_stream(S_MAIN);
  return comm_.host_max(dev_, dhost_[0]);
}

// ---------------------------------------------------------------- pivot search (SIDE stream)
void Engine::select(int64_t t, const void* Lt, bool full) {
  const int par = hslot(t);
  // unused local blocks: exact at p = 1 (every step uses one), else counted as pivots arrive
  const int64_t nlive = L_.p == 1 ? L_.nblk - t : live_;
  const double thresh = opt_.eps * norm_a_;
  Range rg(opt_.profile, "gj:select");
  int pe = prof_begin(S_SIDE);
  if (opt_.pivot == PivotRule::Partial && !full) {
    // largest-magnitude local candidate, then its block alone inverted (record cleared if singular)
    if (L_.nblk > 0) dev_.candidate_maxabs(opt_.dtype, Lt, L_.rows, scores_, valid_, used_, L_, thresh, S_SIDE);
    dev_.pivot_local(scores_, valid_, used_, pos_, L_, myrec_, S_SIDE);
    dev_.gather_candidate(opt_.dtype, sel_, Lt, L_.rows, myrec_, L_, S_SIDE);
    dev_.set_block_inverse_hint(bi_hint_);
    dev_.block_inverse(opt_.dtype, sel_, L_.m, inv1_, score1_, valid1_, used1_, L1_, thresh, 1, S_SIDE);
    dev_.set_block_inverse_hint(-1);
    dev_.commit_candidate(opt_.dtype, inv_, inv1_, valid1_, score1_, opt_.pivot_growth_bound(), myrec_, L_, S_SIDE);
    prof_end(PH_PIVOT, pe, S_SIDE);
  } else {
    // The selection runs in the candidate-inverse launch's last workgroup where the kernel family
    // supports it (one launch fewer on the pivot chain per step); otherwise as its own launch.
    // One rank: the local record is the gathered set -> local argmin + book-keeping in one go; the
    // result goes straight to pinned host memory (no copy kernel), the host polls its step field.
    if (L_.p == 1) {
      dev_.host_access(&piv_host_[par].step, sizeof(int32_t), true);
      piv_host_[par].step = -1;
    }
    bool fused = false;
    if (L_.nblk > 0) {
      dev_.set_block_inverse_hint(bi_hint_);  // per call: a device may be shared with other users
      PivotSelectArgs sa;
      sa.done = sel_done_;
      sa.t = (int32_t)t;
      sa.pos = pos_;
      sa.rec = myrec_;
      if (L_.p == 1) {
        sa.single = 1;
        sa.pos_w = pos_;
        sa.phys_at = phys_at_;
        sa.used_w = used_;
        sa.seq = seq_;
        sa.out = piv_dev_;
        sa.host_out = &piv_host_[par];
      }
      fused = dev_.block_inverse_select(opt_.dtype, Lt, L_.rows, inv_, scores_, valid_, used_, L_, thresh, nlive, sa,
                                        S_SIDE);
      if (!fused) dev_.block_inverse(opt_.dtype, Lt, L_.rows, inv_, scores_, valid_, used_, L_, thresh, nlive, S_SIDE);
      dev_.set_block_inverse_hint(-1);
    }
    if (L_.p == 1) {
      if (!fused)
        dev_.pivot_select_single(scores_, valid_, L_, (int32_t)t, pos_, phys_at_, used_, seq_, myrec_,
                                 piv_dev_, &piv_host_[par], S_SIDE);
      prof_end(PH_PIVOT, pe, S_SIDE);
      dbg_sync();
      return;
    }
    if (!fused) dev_.pivot_local(scores_, valid_, used_, pos_, L_, myrec_, S_SIDE);
    prof_end(PH_PIVOT, pe, S_SIDE);
  }
  if (hang_step_ == t) {  // GJ_TEST_HANG: this rank never joins the exchange of step t
    dev_.host_access(&piv_host_[par].step, sizeof(int32_t), true);
    piv_host_[par].step = -1;
    return;
  }
  pe = prof_begin(S_SIDE);
  comm_.set_step(t);
  if (L_.p > 1) comm_.allgather(dev_, myrec_, recs_, sizeof(PivotRec), S_SIDE);
  count_comm(SolveStats::CK_RECORDS, double(sizeof(PivotRec)) * L_.p);
  dev_.host_access(&piv_host_[par].step, sizeof(int32_t), true);
  piv_host_[par].step = -1;
  dev_.pivot_global(L_.p > 1 ? recs_ : myrec_, (int32_t)L_.p, (int32_t)t, pos_, phys_at_, used_, seq_, piv_dev_,
                    &piv_host_[par], S_SIDE);
  if (vparts_ && L_.p > 1)  // the gathered records every rank just reduced identically
    vhash(panel_of(t), vslot(V_RECS, t - panel_t0(panel_of(t))), recs_, (int64_t)sizeof(PivotRec) * L_.p, (int64_t)sizeof(PivotRec) * L_.p,
          1, S_SIDE);
  prof_end(PH_EXCHANGE, pe, S_SIDE);
  dbg_sync();
}

GemmExtra Engine::pivot_rows_extra(int par, int64_t nsteps) const {
  GemmExtra ex;
  ex.zh = L_.m;
  for (int64_t j = 0; j < nsteps; ++j)
    if (piv_[par][j].owner == L_.k) ex.zr[ex.nzr++] = (piv_[par][j].phys / L_.p) * L_.m;
  return ex;
}

// The pivot search of panel v's first step, enqueued on SIDE behind the look-ahead update (event
// ev_L_: column t0 extracted into At[v % 3] segment 0; SIDE itself, or MAIN for panel 0).
void Engine::begin_panel(int64_t v) {
  cur_step_ = panel_t0(v);
  cur_phase_ = "pivot search";
  dev_.wait(S_SIDE, ev_L_);
  // this panel's steps rewrite Lrow_ / Ht_ / PP_[v & 1], which the COMM chunk pass of panel v - 2
  // reads; with the look-ahead update on SIDE nothing else orders the two (the happens-before
  // checker reports Ht / Lrow / PP conflicts without this wait: tests/test_race_check.py "cp")
  if (v >= 2 && !dropped("cp")) dev_.wait(S_SIDE, ev_cp_[v & 1]);
  select(panel_t0(v), At_[v % 3]);
}

// Pivot searches of panel v (the first one already enqueued by begin_panel); every later column
// of the panel is brought up to date on the SIDE stream from the broadcast panel pieces.  For
// every step: owner edits (Lrow save, H, multiplier rows -> [0..I]), then the panel piece
// PP_t = H_t X^(t)[s_t, panel columns] and its (small) broadcast.  The owner-side launches read
// the pivot from device memory (seq_[t]); with host_free_chain() the host enqueues all q steps and
// reads their results afterwards, otherwise it waits for each pivot (it needs the broadcast root).
bool Engine::factor_panel(int64_t v, SolveStats& st, double& host_wait) {
  const int par = (int)(v & 1);
  const int64_t m = L_.m, rows = L_.rows, npad = L_.npad, dm = (int64_t)d_ * m;
  const int64_t t0 = panel_t0(v), q = panel_q(v);
  const size_t es = esz();
  const bool ahead = host_free_chain();
  for (int64_t j = 0; j < q; ++j) {
    const int64_t t = t0 + j;
    cur_step_ = t;
    cur_phase_ = "pivot search";
    void* Lt = elem(At_[v % 3], j * m * rows);
    if (j > 0) {
      // column t after panel v-1 (look-ahead) and steps t0..t-1 of this panel; the pivot rows of
      // those steps enter as 0 without a mask: their later panel columns were moved out (take_rows)
      // (the piece and its broadcast are on SIDE already: program order covers them; the event of
      // step j-1 is only recorded with GJ_STEP_EVENTS=1)
      if (step_events_) dev_.wait(S_SIDE, ev_pp_[par][j - 1]);
      if (vparts_)  // the piece that just arrived, before its first consumer (this column update)
        vhash(v, vslot(V_PP, j - 1), elem(PP_[par], (j - 1) * m * dm), dm * (int64_t)es, dm * (int64_t)es, m,
              S_SIDE);
      const int pe = prof_begin(S_SIDE);
      if (rows > 0) {
        // the update writes the new multipliers -X[:, t]^T (segment j of At) as it stores X[:, t]:
        // one launch fewer per step (emulated p = 4, N = 16384, direct 50 GB/s: 0.0533 / 0.0538 ->
        // 0.0518 / 0.0518 s; neutral elsewhere, profiles/side_chain_r3.md)
        // (split_: the rows still candidates at the panel's start; the others in deferred_updates)
        GemmExtra ex = chain_sel_[par];
        ex.latency = true;
        ex.lat_wide = lat_wide_;
        ex.lat_reg = lat_reg_;
        ex.tneg = Lt;
        ex.ldtneg = rows;
        const int64_t M = ex.rsel_m > 0 ? ex.rsel_count() * m : rows;
        if (M > 0)
          dev_.gemm(opt_.dtype, GemmOp::Acc, ALayout::KMajor, M, m, j * m, At_[v % 3], rows,
                    elem(PP_[par], j * m), dm, elem(X_, t * m), npad, S_SIDE, ex);
      }
      prof_end(PH_COLUMN, pe, S_SIDE);
      select(t, Lt);
    }
    bool owner = true;
    int root = 0;
    if (!ahead) {
      PivotResult r;
      if (!await_step(v, j, st, host_wait, r)) return false;
      owner = (r.owner == L_.k);
      root = r.owner;
    }
    cur_phase_ = "panel piece";
    int pe = prof_begin(S_SIDE);
    if (owner) {
      // one launch: multipliers of row s_t for steps t0..t-1 -> Lrow (K-major j*m x m), H_t^T -> Ht,
      // and the multiplier rows of s_t become [0 .. 0 | I] (earlier segments 0, own segment I)
      // ... and, same launch, the pivot row's later panel columns moved into RP (they must enter the
      // panel's next column updates as 0: the sweep's pivot-row rule) and the identity block of RP
      // at the pivot's own columns (the piece GEMM then writes H_t there)
      PieceMove mv;
      if (j + 1 < q) {
        mv.dst = elem(RP_, (j + 1) * m);
        mv.ldd = dm;
        mv.X = X_;
        mv.ldx = npad;
        mv.col0 = (t0 + j + 1) * m;
        mv.w = (q - j - 1) * m;
      }
      mv.eye = elem(RP_, j * m);
      mv.ld_eye = dm;
      dev_.owner_edits(opt_.dtype, At_[v % 3], rows, seq_ + t, L_.p, L_.k, j, m, Lrow_[par][j], Ht_[par][j], inv_,
                       mv, S_SIDE);
    }
    prof_end(PH_EDITS, pe, S_SIDE);
    // Only the panel's last step is waited on from another stream (MAIN: lookahead_update; COMM /
    // MAIN: the pieces), so the earlier steps record nothing (timing even: N = 8192 22.80 vs
    // 22.85 ms, profiles/host_fence_r5.md)
    const bool rec = step_events_ || j + 1 == q;
    if (rec) dev_.record(ev_edit_[par], S_SIDE);
    dbg_sync();

    // panel piece PP_t (m x q*m, ld dm), right behind the edits on SIDE: the next step's column
    // update needs it, so the whole per-step chain stays on one stream (no cross-stream hops).
    // (A fused one-launch piece kernel was measured slower: its register/LDS footprint exceeds
    // what a retiring trailing-update workgroup frees, so it waited for CUs; small GEMMs fit.)
    pe = prof_begin(S_SIDE);
    void* pp = elem(PP_[par], j * m * dm);
    GemmExtra lat;
    lat.latency = true;
    lat.lat_reg = lat_reg_;
    if (ahead && L_.p > 1) {  // enqueued on every rank, executed by the pivot's owner only
      lat.owner_phys = seq_ + t;
      lat.owner_p = L_.p;
      lat.owner_k = L_.k;
    }
    if (owner) {
      // RP = the pivot row over the panel's columns before normalisation, in one batched launch:
      //   earlier pivot columns jc < j: the sum over steps jc..j-1 only (no input),
      //   later panel columns jc > j (contiguous): look-ahead value + all earlier steps.
      GemmDesc pr[kMaxDepth];
      int np = 0;
      for (int64_t jc = 0; jc < j; ++jc) {
        GemmDesc& g = pr[np++];
        g.op = GemmOp::Store;
        g.M = m; g.N = m; g.K = (j - jc) * m;
        g.A = elem(Lrow_[par][j], jc * m * m); g.lda = m;
        g.B = elem(PP_[par], jc * m * dm + jc * m); g.ldb = dm;
        g.C = elem(RP_, jc * m); g.ldc = dm;
      }
      if (j + 1 < q) {
        const int64_t w = (q - j - 1) * m;  // moved out of X by owner_edits above
        if (j > 0) {
          GemmDesc& g = pr[np++];
          g.op = GemmOp::Acc;
          g.M = m; g.N = w; g.K = j * m;
          g.A = Lrow_[par][j]; g.lda = m;
          g.B = elem(PP_[par], (j + 1) * m); g.ldb = dm;
          g.C = elem(RP_, (j + 1) * m); g.ldc = dm;
        }
      }
      for (int i = 0; i < np; ++i) {
        pr[i].ex.lat_reg = lat_reg_;
        pr[i].ex.owner_phys = lat.owner_phys;
        pr[i].ex.owner_p = lat.owner_p;
        pr[i].ex.owner_k = lat.owner_k;
      }
      dev_.gemm_batch(opt_.dtype, pr, np, S_SIDE);
      dev_.gemm(opt_.dtype, GemmOp::Store, ALayout::KMajor, m, q * m, m, Ht_[par][j], m, RP_, dm, pp,
                dm, S_SIDE, lat);
    }
    if (ahead && L_.p > 1) {
      // root-agnostic: every rank computed a piece, only the owner's survives the sum
      dev_.zero_unless_owner(opt_.dtype, pp, m * dm, seq_ + t, L_.p, L_.k, S_SIDE);
      comm_.allreduce_sum(dev_, pp, (size_t)m * dm, opt_.dtype, S_SIDE);
    } else {
      comm_.bcast_many(dev_, {BcastOp{pp, (size_t)m * dm * es, root}}, S_SIDE);
    }
    count_comm(SolveStats::CK_PIECES, double(m) * dm * es);
    prof_end(PH_PIECES, pe, S_SIDE);
    if (rec) dev_.record(ev_pp_[par][j], S_SIDE);
    dbg_sync();
  }
  if (vparts_)  // the panel's pivot sequence as SIDE left it (every rank must agree)
    vhash(v, vslot(V_SEQ, 0), seq_ + t0, (int64_t)sizeof(int32_t) * q, (int64_t)sizeof(int32_t) * q, 1, S_SIDE);
  if (vlocal_on()) vlocal_hash(v, V_LP, true, S_SIDE);  // what SIDE hands over to MAIN / COMM
  if (ahead) {  // the panel's pivots, in step order (the first singular step ends the solve)
    cur_phase_ = "pivot search";
    for (int64_t j = 0; j < q; ++j) {
      PivotResult r;
      if (!await_step(v, j, st, host_wait, r)) return false;
    }
  }
  return true;
}

// The host side of step t0(v) + j: wait for its pivot (pinned slot), the --pivot partial fallback,
// singular detection, book-keeping.  False when the matrix is singular at this step.
bool Engine::await_step(int64_t v, int64_t j, SolveStats& st, double& host_wait, PivotResult& r) {
  const int par = (int)(v & 1);
  const int64_t t = panel_t0(v) + j;
  cur_step_ = t;
  wait_pivot(hslot(t), t, host_wait);
  r = piv_host_[hslot(t)];
  if (!r.found && opt_.pivot == PivotRule::Partial) {
    // every rank's largest-magnitude candidate was singular: this step takes the full search
    st.pivot_fallbacks++;
    select(t, elem(At_[v % 3], j * L_.m * L_.rows), /*full=*/true);
    wait_pivot(hslot(t), t, host_wait);
    r = piv_host_[hslot(t)];
  }
  if (!r.found) {
    comm_.drain_all(dev_);
    st.status = Status::Singular;
    st.singular_step = t;
    return false;
  }
  piv_[par][j] = r;
  st.pivots[t] = r.phys;
  if (r.owner == L_.k) {
    --live_;  // this rank's block row s_t is no longer a candidate
    used_local_[(size_t)(r.phys / L_.p)] = 1;
    st.bcast_bytes += double(L_.m) * L_.npad * esz();
  }
  return true;
}

// Panel v's pivot rows over the next panel's block columns (LA_[par], step-major, ld wla), formed
// by their owners and broadcast on their own: the look-ahead update of panel v+1 needs only
// these, so the next pivot chain starts after a (q*m) x (qn*m) broadcast instead of after a whole
// chunk's.  The chunk pass broadcasts these columns again with the rest of their chunk (MAIN's
// chunk update skips them).
void Engine::lookahead_rows(int64_t v, bool wait_main) {
  const int par = (int)(v & 1);
  const int64_t m = L_.m, npad = L_.npad;
  const int64_t q = panel_q(v);
  const size_t es = esz();
  cur_phase_ = "look-ahead rows";
  if (v + 1 < npanels()) {
    const int64_t xa = panel_t0(v + 1) * m, wla = panel_q(v + 1) * m;
    // on SIDE, right behind the panel pieces, with SIDE's communicator: emulated N = 16384 p = 4 at
    // 50 GB/s per link 0.0588 -> 0.0564 s (80 % of the transfer hidden), p = 8 0.0430 -> 0.0425 s
    // (profiles/emu_direct_r3.md); one rank too since round 4 (la_side_, constructor)
    const bool la_side = la_side_;
    const int ls = la_side ? S_SIDE : S_COMM;
    void* Tl = la_side ? T2_ : T_;
    if (!la_side) dev_.wait(S_COMM, ev_pp_[par][q - 1]);  // panel pieces, Lrow, H_t (SIDE)
    if (wait_main) dev_.wait(ls, ev_c_[chunk_of_[panel_t0(v + 1)]]);
    std::vector<BcastOp> lops;
    auto lflush = [&]() {
      if (lops.empty()) return;
      const int pb = prof_begin(ls);
      for (const auto& o : lops) count_comm(SolveStats::CK_ROWS, (double)o.bytes);
      comm_.bcast_many(dev_, lops, ls);
      prof_end(PH_BCAST, pb, ls);
      lops.clear();
    };
    GemmExtra lat;
    lat.latency = true;
    lat.lat_reg = lat_reg_;
    for (int64_t j = 0; j < q; ++j) {
      const PivotResult& r = piv_[par][j];
      char* seg = elem(LA_[par], j * m * wla);
      for (const auto& o : lops)  // R_j needs the earlier steps' rows (see the chunk pass)
        if (o.root != r.owner) {
          lflush();
          break;
        }
      if (r.owner == L_.k) {
        const int pe = prof_begin(ls);
        const int64_t sl = r.phys / L_.p;
        if (j == 0) {
          dev_.gemm(opt_.dtype, GemmOp::Store, ALayout::KMajor, m, wla, m, Ht_[par][j], m,
                    elem(X_, sl * m * npad + xa), npad, seg, wla, ls, lat);
        } else {
          // Tl = X[s_t, next panel] + Lrow_t LA[earlier steps] (C_in: no separate copy launch)
          GemmExtra li = lat;
          li.c_in = elem(X_, sl * m * npad + xa);
          li.ldc_in = npad;
          dev_.gemm(opt_.dtype, GemmOp::Acc, ALayout::KMajor, m, wla, j * m, Lrow_[par][j], m, LA_[par], wla,
                    Tl, wla, ls, li);
          dev_.gemm(opt_.dtype, GemmOp::Store, ALayout::KMajor, m, wla, m, Ht_[par][j], m, Tl, wla, seg, wla,
                    ls, lat);
        }
        prof_end(PH_NORMALISE, pe, ls);
      }
      lops.push_back(BcastOp{seg, (size_t)m * wla * es, (int)r.owner});
    }
    lflush();
    dev_.record(ev_la_[par], ls);
  }
}

// COMM stream: for every column chunk (in the order MAIN will consume them) and every step of
// panel v, the owner of s_t forms R_t[chunk] = H_t (X[s_t, chunk] + Lrow_t R_prev[chunk]) outside
// the panel's columns (those come from the panel piece, later panel blocks zeroed), and the row
// segments are broadcast.  Consecutive segments with the same root go out as one RCCL group; a
// segment whose owner needs earlier segments of other roots waits for their broadcast first.
void Engine::chunk_pipeline(int64_t v, bool wait_main) {
  const int par = (int)(v & 1);
  const int64_t m = L_.m, npad = L_.npad;
  const int64_t t0 = panel_t0(v), q = panel_q(v);
  const size_t es = esz();
  const int64_t C = (int64_t)cb0_.size();
  const bool has_next = (v + 1 < npanels());
  const int64_t start = has_next ? chunk_of_[panel_t0(v + 1)] : 0;
  const int64_t pc0 = t0 * m, pc1 = (t0 + q) * m;  // panel columns
  const int64_t xn0 = has_next ? panel_t0(v + 1) * m : 0;  // the next panel's columns
  const int64_t xn1 = has_next ? (panel_t0(v + 1) + panel_q(v + 1)) * m : 0;
  dev_.wait(S_COMM, ev_pp_[par][q - 1]);  // all panel pieces, multiplier rows and H_t (SIDE)
  if (vparts_)  // the last step's piece: no column update consumes it, the chunk pass does first
    vhash(v, vslot(V_PP, q - 1), elem(PP_[par], (q - 1) * m * (int64_t)d_ * m), (int64_t)d_ * m * (int64_t)es,
          (int64_t)d_ * m * (int64_t)es, m, S_COMM);
  if (vlocal_on()) vlocal_hash(v, V_LC, false, S_COMM);  // Lrow / Ht / PP as the chunk pass reads them
  if (split_ == 1) deferred_updates(v, S_COMM);
  cur_phase_ = "pivot-row broadcast";
  for (int64_t i = 0; i < C; ++i) {
    const int64_t c = (start + i) % C;
    const int64_t c0 = cb0_[c] * m, c1 = cb1_[c] * m, W = c1 - c0;
    if (wait_main) dev_.wait(S_COMM, ev_c_[c]);
    // the chunk's columns minus the panel's own (they come from the panel pieces) and minus the next
    // panel's (the look-ahead rows carried them, MAIN's chunk pass skips them, and the look-ahead
    // update on SIDE rewrites X there while this pass runs: reading them would race it)
    int64_t ra[3], rb[3], nr = 0;
    int64_t sk0 = 0, sk1 = 0;  // or one launch over the chunk that skips the cut (GemmExtra::skip_c0/c1)
    const bool has_panel = (pc0 >= c0 && pc0 < c1);
    {
      int64_t cut0[2], cut1[2], ncut = 0;
      if (has_panel) { cut0[ncut] = pc0; cut1[ncut++] = pc1; }
      if (has_next && !dropped("x")) { cut0[ncut] = xn0; cut1[ncut++] = xn1; }
      int64_t lo_all = -1, hi_all = -1, nin = 0;
      bool contiguous = true;
      int64_t a = c0;
      for (int64_t z = 0; z < ncut; ++z) {  // the cuts are ordered (the next panel follows this one)
        const int64_t lo = std::max(cut0[z], c0), hi = std::min(cut1[z], c1);
        if (lo >= hi) continue;
        if (nin > 0 && lo != hi_all) contiguous = false;
        if (nin == 0) lo_all = lo;
        hi_all = hi;
        ++nin;
        if (lo > a) { ra[nr] = a; rb[nr] = lo; ++nr; }
        a = std::max(a, hi);
      }
      if (c1 > a) { ra[nr] = a; rb[nr] = c1; ++nr; }
      const int64_t al = dev_.skip_align();
      // (under a CU reservation only: N = 8192 24.20 -> 23.61 ms with both launches merged, but
      // N = 32768, where the chunk pass shares the CUs with the trailing update, 1069 -> 1086 ms;
      // scripts/runs/r5_skip.sh, profiles/side_chain_r5.md)
      if (nr > 1 && nin > 0 && contiguous && chunk_skip_ && (lo_all - c0) % al == 0 &&
          (hi_all - c0) % al == 0) {
        nr = 1;
        ra[0] = c0;
        rb[0] = c1;
        sk0 = lo_all - c0;
        sk1 = hi_all - c0;
      }
    }
    char* chunk = rb_chunk(par, c);
    std::vector<BcastOp> bops;
    auto flush = [&]() {
      if (bops.empty()) return;
      const int pb = prof_begin(S_COMM);
      for (const auto& o : bops) count_comm(SolveStats::CK_ROWS, (double)o.bytes);
      comm_.bcast_many(dev_, bops, S_COMM);
      prof_end(PH_BCAST, pb, S_COMM);
      bops.clear();
    };
    for (int64_t j = 0; j < q; ++j) {
      const PivotResult& r = piv_[par][j];
      char* seg = chunk + j * m * W * (int64_t)es;
      // R_j needs the segments of steps < j: the ones its owner did not form itself must have
      // arrived (the same decision on every rank: it depends only on the pivot owners)
      for (const auto& o : bops)
        if (o.root != r.owner) {
          flush();
          break;
        }
      int pe = prof_begin(S_COMM);
      if (r.owner == L_.k) {
        const int64_t sl = r.phys / L_.p;
        GemmExtra lat;
        lat.latency = comm_small_tiles_;
        lat.skip_c0 = sk0;
        lat.skip_c1 = sk1;
        lat.glds_build = chunk_build_;
        lat.glds_tile = chunk_tile_;
        for (int64_t z = 0; z < nr; ++z) {
          const int64_t a = ra[z], w = rb[z] - ra[z];
          if (j == 0) {
            dev_.gemm(opt_.dtype, GemmOp::Store, ALayout::KMajor, m, w, m, Ht_[par][j], m,
                      elem(X_, sl * m * npad + a), npad, seg + (a - c0) * (int64_t)es, W, S_COMM, lat);
          } else {
            GemmExtra li = lat;  // T = X[s_t, range] + Lrow_t R[earlier steps] (C_in: no copy launch)
            li.c_in = elem(X_, sl * m * npad + a);
            li.ldc_in = npad;
            dev_.gemm(opt_.dtype, GemmOp::Acc, ALayout::KMajor, m, w, j * m, Lrow_[par][j], m,
                      chunk + (a - c0) * (int64_t)es, W, T_, W, S_COMM, li);
            dev_.gemm(opt_.dtype, GemmOp::Store, ALayout::KMajor, m, w, m, Ht_[par][j], m, T_, W,
                      seg + (a - c0) * (int64_t)es, W, S_COMM, lat);
          }
        }
        if (has_panel) {  // panel columns: PP_t for blocks <= t, zero for later panel blocks
          char* dst = seg + (pc0 - c0) * (int64_t)es;
          dev_.copy2d(dst, W * es, elem(PP_[par], j * m * (int64_t)d_ * m), (int64_t)d_ * m * es,
                      (j + 1) * m * es, m, S_COMM);
          if (j + 1 < q)
            dev_.memset2d(dst + (j + 1) * m * (int64_t)es, W * es, (q - j - 1) * m * es, m, S_COMM);
        }
      }
      prof_end(PH_NORMALISE, pe, S_COMM);
      bops.push_back(BcastOp{seg, (size_t)m * W * es, (int)r.owner});
    }
    flush();
    if (i == 0 && corrupt_step_ >= t0 && corrupt_step_ < t0 + q &&  // GJ_TEST_CORRUPT (tests only)
        !(corrupt_unprofiled_ && opt_.profile))
      dev_.memset2d(chunk + (corrupt_step_ - t0) * m * W * (int64_t)es, W * es, W * es, m, S_COMM);
    dev_.record(ev_b_[par][c], S_COMM);
  }
  if (vlocal_on()) vlocal_hash(v, V_LE, false, S_COMM);  // ... and after its last read
  dev_.record(ev_cp_[par], S_COMM);
  dbg_sync();
}

// The split_ half that left the pivot chain: for the rows already used as pivot rows when panel v
// started, panel v-1's look-ahead update of panel v's columns (with its -X^T segment 0 of At) and
// panel v's in-panel column updates (segments 1..q-1), after the last panel piece: on COMM ahead of
// the panel's chunk pass (split_ 1) or on MAIN ahead of the panel's trailing update (split_ 2), in
// either case ahead of MAIN's trailing update, the only reader of these rows' multipliers.  The
// products and their k order are the chain's, row for row.
void Engine::deferred_updates(int64_t v, int stream) {
  const int par = (int)(v & 1);
  const GemmExtra& sel = defer_sel_[par];
  if (v == 0 || sel.rsel_m == 0 || L_.rows == 0) return;
  const int64_t cnt = sel.rsel_count();
  if (cnt == 0) return;
  const int64_t m = L_.m, rows = L_.rows, npad = L_.npad, dm = (int64_t)d_ * m, M = cnt * m;
  const int64_t q = panel_q(v), x0 = panel_t0(v) * m, qp = panel_q(v - 1);
  cur_phase_ = "deferred column updates";
  const int pe = prof_begin(stream);
  GemmExtra ex = pivot_rows_extra((int)((v - 1) & 1), qp);
  std::copy(sel.rsel, sel.rsel + GemmExtra::kRselWords, ex.rsel);
  ex.rsel_m = sel.rsel_m;
  ex.tneg = At_[v % 3];
  ex.ldtneg = rows;
  ex.tneg_cols = m;
  dev_.gemm(opt_.dtype, GemmOp::Acc, ALayout::KMajor, M, q * m, qp * m, At_[(v - 1) % 3], rows,
            LA_[(v - 1) & 1], q * m, elem(X_, x0), npad, stream, ex);
  for (int64_t j = 1; j < q; ++j) {
    GemmExtra ec = sel;
    ec.latency = true;
    ec.lat_wide = lat_wide_;
    ec.lat_reg = lat_reg_;
    ec.tneg = elem(At_[v % 3], j * m * rows);
    ec.ldtneg = rows;
    dev_.gemm(opt_.dtype, GemmOp::Acc, ALayout::KMajor, M, m, j * m, At_[v % 3], rows, elem(PP_[par], j * m), dm,
              elem(X_, x0 + j * m), npad, stream, ec);
  }
  prof_end(PH_COLUMN, pe, stream);
}

// First part of panel u's depth-q trailing update: the next panel's block columns (look-ahead), so
// its pivot search can start; big_update() then does every other chunk on MAIN.  The look-ahead
// runs on SIDE, right behind the look-ahead rows, not on MAIN: it needs only MAIN's chunk of
// panel u-1 that holds these columns (the look-ahead rows already waited for it), not the rest
// of MAIN's queue.  Measured against MAIN (scripts/ab.sh, two repetitions): N = 8192 28.6 / 29.0
// -> 27.8 / 27.9 ms, 16384 166.2 -> 163.0 ms, 32768 1137.5 -> 1135.3 ms; emulated p = 4,
// N = 16384, direct 50 GB/s 0.0551 / 0.0554 -> 0.0525 / 0.0529 s; p = 8, N = 32768 0.1670 ->
// 0.1625 s (profiles/side_chain_r3.md).  Hazards: At_[(u + 1) % 3] was last read by MAIN's
// update of panel u-2, finished before that chunk of u-1; MAIN's chunk pass of panel u skips
// these columns; Lrow_ / Ht_ / PP_ reuse is ordered by ev_cp_ (begin_panel).
void Engine::lookahead_update(int64_t u) {
  const int par = (int)(u & 1);
  const int64_t m = L_.m, rows = L_.rows, npad = L_.npad;
  const int64_t q = panel_q(u), K = q * m;
  if (!dropped("edit")) dev_.wait(S_MAIN, ev_edit_[par]);  // MAIN's chunk pass reads the edited multipliers
  if (u + 1 < npanels()) {
    const int64_t tn = panel_t0(u + 1), qn = panel_q(u + 1);
    const int ms = S_SIDE;
    const int64_t x0 = tn * m, x1 = (tn + qn) * m;
    // split_ 2: MAIN's deferred updates of panel u-1 read At_[(u-1) % 3], LA_ / PP_ of parity u-1
    // and write X and At_ rows that SIDE rewrites from here on (normally implied by the look-ahead
    // rows' wait for MAIN's chunk; explicit here)
    if (split_ == 2 && u >= 1) dev_.wait(ms, ev_def_[(u - 1) & 1]);
    const GemmExtra prows = pivot_rows_extra(par, q);
    // the look-ahead rows of panel u (lookahead_rows): N = 16384 emulated p = 4 / 8 at 50 GB/s per
    // link 0.0669 -> 0.0595 s / 0.0485 -> 0.0431 s against waiting for the whole first chunk
    // (profiles/emu_direct_r3.md)
    // split_: this update and the next panel's column updates cover the rows still candidates
    // when panel u+1 starts (every pivot of panel u is known on the host by now); the rows used
    // before get both in deferred_updates(u + 1) (COMM or MAIN)
    const int npar = (int)((u + 1) & 1);
    chain_sel_[npar] = GemmExtra{};
    defer_sel_[npar] = GemmExtra{};
    if (split_) {
      chain_sel_[npar].rsel_m = defer_sel_[npar].rsel_m = m;
      for (int64_t b = 0; b < L_.nblk; ++b)
        (used_local_[(size_t)b] ? defer_sel_[npar] : chain_sel_[npar]).rsel[b / 64] |= uint64_t(1) << (b % 64);
    }
    dev_.wait(ms, ev_la_[par]);
    if (vparts_)
      for (int64_t j = 0; j < q; ++j)
        vhash(u, vslot(V_LA, j), elem(LA_[par], j * m * (x1 - x0)), (x1 - x0) * (int64_t)esz(),
              (x1 - x0) * (int64_t)esz(), m, ms);
    const int pe = prof_begin(ms);
    if (rows > 0) {
      // the first column block's new multipliers -X[:, x0:x0+m]^T go straight into segment 0 of
      // the next panel's multiplier panel (GemmExtra::tneg, no separate extract launch; neutral to
      // -1 % in the A/B of profiles/side_chain_r3.md, one launch fewer per panel)
      GemmExtra ex = prows;
      ex.tneg = At_[(u + 1) % 3];
      ex.ldtneg = rows;
      ex.tneg_cols = m;
      std::copy(chain_sel_[npar].rsel, chain_sel_[npar].rsel + GemmExtra::kRselWords, ex.rsel);
      ex.rsel_m = chain_sel_[npar].rsel_m;
      const int64_t M = ex.rsel_m > 0 ? ex.rsel_count() * m : rows;
      if (M > 0)
        dev_.gemm(opt_.dtype, GemmOp::Acc, ALayout::KMajor, M, x1 - x0, K, At_[u % 3], rows, LA_[par],
                  x1 - x0, elem(X_, x0), npad, ms, ex);
    }
    prof_end(PH_UPDATE, pe, ms);
    dev_.record(ev_L_, ms);
    dbg_sync();
  }
}

// MAIN stream: the rest of panel u's trailing update, every chunk behind the event of its
// broadcast.  Hazards across streams: the multiplier panels are triple-buffered (At_[u % 3]);
// Rb_[par] chunk c is rewritten by the COMM stream only after ev_c_[c] of the following panel.
void Engine::big_update(int64_t u) {
  const int par = (int)(u & 1);
  void* At = At_[u % 3];
  const int64_t m = L_.m, rows = L_.rows, npad = L_.npad;
  const int64_t t0 = panel_t0(u), q = panel_q(u), K = q * m;
  const int64_t C = (int64_t)cb0_.size();
  const bool has_next = (u + 1 < npanels());
  const GemmExtra prows = pivot_rows_extra(par, q);
  const int64_t x0 = has_next ? panel_t0(u + 1) * m : -1;  // look-ahead columns (done)
  const int64_t x1 = has_next ? (panel_t0(u + 1) + panel_q(u + 1)) * m : -1;
  const int64_t start = has_next ? chunk_of_[panel_t0(u + 1)] : 0;
  const int64_t pc0 = t0 * m, pc1 = (t0 + q) * m;
  if (split_ == 2) {  // the used rows' column updates, behind the panel's last piece (SIDE)
    dev_.wait(S_MAIN, ev_pp_[par][q - 1]);
    deferred_updates(u, S_MAIN);
    dev_.record(ev_def_[par], S_MAIN);
  }
  for (int64_t i = 0; i < C; ++i) {
    const int64_t c = (start + i) % C;
    const int64_t c0 = cb0_[c] * m, c1 = cb1_[c] * m, W = c1 - c0;
    const int ms = S_MAIN;
    if (!dropped("b")) dev_.wait(ms, ev_b_[par][c]);
    if (i == 0 && vlocal_on()) vlocal_hash(u, V_LC, true, ms);  // At as the first chunk update reads it
    if (vparts_)  // what this chunk's update is about to read, segment by segment (one root each)
      for (int64_t j = 0; j < q; ++j)
        vhash(u, vslot(V_RB, j, c), rb_chunk(par, c) + j * m * W * (int64_t)esz(), W * (int64_t)esz(),
              W * (int64_t)esz(), m, ms);
    const int pe = prof_begin(ms);
    int64_t ra[2], rb[2], nr = 0;
    // the look-ahead columns [x0, x1) are done: one launch around them (GemmExtra::skip_c0/c1) when
    // the device can skip whole tiles there, else one launch per side.  N = 8192: the two launches
    // of a split chunk took 346-353 us against 321 us for one launch of the same tiles (two launch
    // tails), profiles/side_chain_r5.md
    int64_t sk0 = 0, sk1 = 0;
    if (has_next && x0 >= c0 && x0 < c1) {
      const int64_t al = dev_.skip_align();
      if ((x0 - c0) % al == 0 && (x1 - c0) % al == 0 && x1 <= c1 && skip_cols_) {
        ra[0] = c0; rb[0] = c1; nr = 1;
        sk0 = x0 - c0;
        sk1 = x1 - c0;
      } else {
        if (x0 > c0) { ra[nr] = c0; rb[nr] = x0; ++nr; }
        if (c1 > x1) { ra[nr] = x1; rb[nr] = c1; ++nr; }
      }
    } else {
      ra[0] = c0; rb[0] = c1; nr = 1;
    }
    // GJ_MAIN_SPLIT (A/B): the chunk's launch in two column halves -- 1: the panel's first chunk
    // only, 2: every chunk -- an extra launch boundary where a drained CU can take the pivot
    // chain's candidate inverse (profiles/rocprof_n32768_r6_final.md)
    const int pieces = (main_split_ == 2 || (main_split_ == 1 && i == 0)) ? 2 : 1;
    const int64_t s_abs0 = c0 + sk0, s_abs1 = c0 + sk1;  // skipped columns (absolute; empty if equal)
    if (rows > 0)
      for (int64_t z = 0; z < nr; ++z) {
        int64_t cut[3] = {ra[z], rb[z], rb[z]};
        int np = 1;
        if (pieces == 2 && rb[z] - ra[z] >= 256) {
          cut[1] = ra[z] + ((rb[z] - ra[z]) / 256) * 128;  // tile-aligned (128) from the range's start
          np = 2;
        }
        for (int h = 0; h < np; ++h) {
          const int64_t a = cut[h], b = cut[h + 1];
          GemmExtra ex = prows;
          const int64_t s0 = std::max(s_abs0, a), s1 = std::min(s_abs1, b);
          ex.skip_c0 = s1 > s0 ? s0 - a : 0;
          ex.skip_c1 = s1 > s0 ? s1 - a : 0;
          ex.zc0 = pc0 - a;  // the panel's own block columns enter as 0
          ex.zc1 = pc1 - a;
          // with CUs reserved for the pivot chain the trailing update may fill the rest densely:
          // N = 16384 161.6 vs 164.6 ms; without a reservation the chain starves (N = 32768 1195 vs
          // 1158 ms), profiles/gemm_stall_r4.md
          ex.dense = dense_gemm_;
          ex.c_nt = main_cnt_;
          dev_.gemm(opt_.dtype, GemmOp::Acc, ALayout::KMajor, rows, b - a, K, At, rows,
                    rb_chunk(par, c) + (a - c0) * (int64_t)esz(), W, elem(X_, a), npad, ms, ex);
        }
      }
    prof_end(PH_UPDATE, pe, ms);
    if (i + 1 == C && vlocal_on()) vlocal_hash(u, V_LE, true, ms);  // ... and after the last one
    dev_.record(ev_c_[c], ms);
  }
  dbg_sync();
}

// ---------------------------------------------------------------- solve
// A communication failure names where this rank was: step, phase and the collective it sat in
// (the message of the Comm / wait_pivot timeout), so a hang on a p-GPU node explains itself.
SolveStats Engine::solve() {
  try {
    return solve_steps();
  } catch (const Error& e) {
    if (e.status() != Status::CommError) throw;
    throw Error(Status::CommError, "rank " + std::to_string(L_.k) + "/" + std::to_string(L_.p) + ", step " +
                                       std::to_string(cur_step_) + " of " + std::to_string(L_.Nr) +
                                       ", phase " + cur_phase_ + ": " + e.what());
  }
}

SolveStats Engine::solve_steps() {
  GJ_REQUIRE(!solved_, "solve(): input panel already consumed; load the matrix again");
  cur_step_ = -1;
  cur_phase_ = "norm";
  SolveStats st;
  const int64_t m = L_.m, Nr = L_.Nr, rows = L_.rows, npad = L_.npad;
  pmarks_.clear();
  pev_next_ = 0;
  if (block_mem_fail_) {  // agreed at construction: the same answer on every rank, no collective
    st.status = Status::NoBlockMemory;
    solved_ = true;
    return st;
  }

  comm_.barrier(dev_);
  const double t_begin = now_s();
  dev_.set_gemm_tile_hint(gemm_tile_);  // (the device may be shared with another engine)

  norm_a_ = norm_inf();
  local_norm_valid_ = false;  // the sweep consumes X
  if (std::fabs(norm_a_) < opt_.eps) {  // reference main.cpp:782 second clause
    st.status = Status::Singular;
    st.singular_step = 0;
    st.seconds = now_s() - t_begin;
    solved_ = true;
    return st;
  }

  // book-keeping arrays: pos = phys_at = identity, used = 0, seq = -1 (no pivot yet: every
  // owner-predicated launch of a step enqueued ahead of its pivot -- the host-free chain -- is a
  // no-op on every rank if that step finds none, instead of treating block row 0 as the pivot)
  dev_.host_access(ihost_, sizeof(int32_t) * 2 * Nr, true);
  for (int64_t i = 0; i < Nr; ++i) {
    ihost_[i] = (int32_t)i;
    ihost_[Nr + i] = -1;
  }
  dev_.copy(pos_, ihost_, sizeof(int32_t) * Nr, S_SIDE);
  dev_.copy(phys_at_, ihost_, sizeof(int32_t) * Nr, S_SIDE);
  dev_.memset0(used_, sizeof(int32_t) * Nr, S_SIDE);
  dev_.copy(seq_, ihost_ + Nr, sizeof(int32_t) * Nr, S_SIDE);
  if (vparts_)
    dev_.memset0(vparts_, sizeof(uint64_t) * Device::kHashParts * (size_t)npanels() * (size_t)vslots(), S_SIDE);
  dev_.sync_stream(S_SIDE);

  st.pivots.assign(Nr, -1);
  for (int k = 0; k < SolveStats::kNumCommKinds; ++k) comm_bytes_[k] = 0, comm_calls_[k] = 0;
  live_ = L_.nblk;
  used_local_.assign((size_t)std::max<int64_t>(L_.nblk, 1), 0);
  for (int i = 0; i < 2; ++i) chain_sel_[i] = defer_sel_[i] = GemmExtra{};
  double host_wait = 0;
  bool ok = true;

  // prologue: column 0, pivot searches of panel 0
  if (rows > 0) dev_.extract_neg_t(opt_.dtype, At_[0], rows, X_, npad, rows, 0, m, S_MAIN);
  dev_.record(ev_L_, S_MAIN);
  begin_panel(0);
  ok = factor_panel(0, st, host_wait);

  // Per panel: the look-ahead rows and the chunk pass (SIDE / COMM), the look-ahead update (SIDE)
  // and the rest of the trailing update (MAIN), then the next panel's pivot chain.
  for (int64_t u = 0; ok && u < npanels(); ++u) {
    const bool has_next = u + 1 < npanels();
    lookahead_rows(u, /*wait_main=*/u > 0);
    chunk_pipeline(u, /*wait_main=*/u > 0);
    lookahead_update(u);
    big_update(u);
    if (has_next) {
      begin_panel(u + 1);
      ok = factor_panel(u + 1, st, host_wait);
    }
  }
  if (!ok) {
    comm_.drain_all(dev_);
    st.host_wait_ms = host_wait * 1e3;
    st.seconds = now_s() - t_begin;
    solved_ = true;
    return st;
  }

  {
    cur_phase_ = "final exchange";
    const int pe = prof_begin(S_COMM);
    finalize(st.pivots);
    prof_end(PH_FINALIZE, pe, S_COMM);
  }
  comm_.drain_all(dev_);
  const double t_end = now_s();
  for (int64_t t = 0; t < Nr; ++t)
    if (st.pivots[t] != t) st.offdiag_pivots++;
  for (int k = 0; k < SolveStats::kNumCommKinds; ++k) st.comm_bytes[k] = comm_bytes_[k], st.comm_calls[k] = comm_calls_[k];
  if (vparts_) verify_hashes(st);  // outside the timed interval; throws VerifyFailed on every rank
  st.host_wait_ms = host_wait * 1e3;
  st.seconds = t_end - t_begin;
  prof_collect(st);
  solved_ = true;
  return st;
}

// ---------------------------------------------------------------- GJ_VERIFY
int Engine::vslot(VKind k, int64_t j, int64_t c) const {
  const int64_t C = (int64_t)cb0_.size();
  const int64_t L0 = C * d_ + 3 * d_ + 1;  // first rank-local slot
  switch (k) {
    case V_RB: return (int)(c * d_ + j);
    case V_PP: return (int)(C * d_ + j);
    case V_LA: return (int)(C * d_ + d_ + j);
    case V_RECS: return (int)(C * d_ + 2 * d_ + j);
    case V_SEQ: return (int)(C * d_ + 3 * d_);
    case V_LP: return (int)(L0 + j);
    case V_LC: return (int)(L0 + vlocal_groups() + j);
    default: return (int)(L0 + 2 * vlocal_groups() + j);
  }
}

// The bytes of rank-local hand-over group g of panel v (see VKind): empty where nothing is handed
// over (no local rows, Lrow of a panel's first step, steps past the panel's end).
Engine::VRegion Engine::vlocal_region(int64_t v, int g) const {
  const int par = (int)(v & 1);
  const int64_t m = L_.m, q = panel_q(v), es = (int64_t)esz(), dm = (int64_t)d_ * m;
  VRegion r;
  const std::string P = "[" + std::to_string(par) + "]";
  if (g == 0) {
    r.name = "multiplier panel At[" + std::to_string(v % 3) + "]";
    if (L_.rows > 0) r = {At_[v % 3], L_.rows * es, L_.rows * es, q * m, r.name};
  } else if (g == 1) {
    r = {PP_[par], dm * es, q * m * es, q * m, "panel pieces PP" + P};
  } else if (g < 2 + d_) {
    const int64_t j = g - 2;
    r.name = "Lrow" + P + "[" + std::to_string(j) + "]";
    if (j >= 1 && j < q) r = {Lrow_[par][j], m * es, m * es, j * m, r.name};
  } else {
    const int64_t j = g - 2 - d_;
    r.name = "Ht" + P + "[" + std::to_string(j) + "]";
    if (j < q) r = {Ht_[par][j], m * es, m * es, m, r.name};
  }
  return r;
}

void Engine::vlocal_hash(int64_t v, VKind point, bool at_group, int s) {
  for (int g = 0; g < vlocal_groups(); ++g) {
    if ((g == 0) != at_group && point != V_LP) continue;
    const VRegion r = vlocal_region(v, g);
    if (r.base && r.rows > 0) vhash(v, vslot(point, g), r.base, r.ld, r.width, r.rows, s);
  }
}

void Engine::vhash(int64_t v, int slot, const void* base, int64_t ld_bytes, int64_t width_bytes, int64_t rows,
                   int s) {
  dev_.hash_rows(base, ld_bytes, width_bytes, rows,
                 vparts_ + ((size_t)v * vslots() + (size_t)slot) * Device::kHashParts, s);
}

// All-gather the per-slot hashes and compare every rank's with the root's: the first mismatch in
// step order (pivot records and sequence, then pieces, look-ahead rows, chunk segments in MAIN's
// order) names where a rank consumed bytes its root never sent -- a read before the data arrived, or
// a corrupted copy -- which the final residual can only report as "wrong".  Collective; every rank
// reaches the same verdict.
void Engine::verify_hashes(const SolveStats& st) {
  const int64_t P = npanels(), S = vslots(), C = (int64_t)cb0_.size(), p = L_.p;
  const size_t nparts = (size_t)P * S * Device::kHashParts;
  std::vector<uint64_t> parts(nparts);
  dev_.copy(parts.data(), vparts_, sizeof(uint64_t) * nparts, S_MAIN);
  dev_.sync_stream(S_MAIN);
  std::vector<uint64_t> mine((size_t)P * S, 0);
  for (size_t i = 0; i < mine.size(); ++i)
    for (int g = 0; g < Device::kHashParts; ++g) mine[i] += parts[i * Device::kHashParts + g];
  std::vector<uint64_t> all(mine.size() * p);
  comm_.host_allgather(dev_, mine.data(), all.data(), sizeof(uint64_t) * mine.size());
  auto h = [&](int64_t r, int64_t v, int slot) { return all[(size_t)r * P * S + (size_t)v * S + slot]; };
  auto owner = [&](int64_t t) { return (t < (int64_t)st.pivots.size() && st.pivots[t] >= 0) ? st.pivots[t] % p : 0; };
  for (int64_t v = 0; v < P; ++v) {
    const int64_t t0 = panel_t0(v), q = panel_q(v);
    const int64_t start = (v + 1 < P) ? chunk_of_[panel_t0(v + 1)] : 0;
    struct Item { int slot; int64_t step; const char* phase; std::string buffer; int64_t root; const char* stream; };
    std::vector<Item> order;
    for (int64_t j = 0; j < q; ++j)
      order.push_back({vslot(V_RECS, j), t0 + j, "pivot exchange", "gathered pivot records", -1, "SIDE"});
    order.push_back({vslot(V_SEQ, 0), t0 + q - 1, "pivot search", "pivot sequence of the panel", -1, "SIDE"});
    for (int64_t j = 0; j < q; ++j)
      order.push_back({vslot(V_PP, j), t0 + j, j + 1 < q ? "column update" : "pivot-row broadcast",
                       "panel piece PP[" + std::to_string(v & 1) + "] step " + std::to_string(j), owner(t0 + j),
                       j + 1 < q ? "SIDE" : "COMM"});
    for (int64_t j = 0; j < q; ++j)
      order.push_back({vslot(V_LA, j), t0 + j, "look-ahead update",
                       "look-ahead rows LA[" + std::to_string(v & 1) + "] step " + std::to_string(j), owner(t0 + j),
                       "SIDE"});
    // rank-local hand-overs: -2 - g = compare with this rank's own producer hash of group g
    if (vlocal_on()) {
      for (int pt = 0; pt < 2; ++pt)
        for (int g = 1; g < vlocal_groups(); ++g)
          order.push_back({vslot(pt == 0 ? V_LC : V_LE, g), t0 + q - 1,
                           pt == 0 ? "chunk pass (before its first read)" : "chunk pass (after its last read)",
                           vlocal_region(v, g).name, -2 - g, "COMM"});
      order.push_back({vslot(V_LC, 0), t0 + q - 1, "trailing update (before its first read)",
                       vlocal_region(v, 0).name, -2, "MAIN"});
    }
    for (int64_t i = 0; i < C; ++i) {
      const int64_t c = (start + i) % C;
      for (int64_t j = 0; j < q; ++j)
        order.push_back({vslot(V_RB, j, c), t0 + j, "trailing update",
                         "Rb[" + std::to_string(v & 1) + "] chunk " + std::to_string(c) + " segment " +
                             std::to_string(j),
                         owner(t0 + j), "MAIN"});
    }
    if (vlocal_on())
      order.push_back({vslot(V_LE, 0), t0 + q - 1, "trailing update (after its last read)",
                       vlocal_region(v, 0).name, -2, "MAIN"});
    for (const Item& it : order) {
      std::vector<int64_t> bad;
      if (it.root <= -2) {  // rank-local: each rank against what its own SIDE stream produced
        const int g = (int)(-2 - it.root);
        for (int64_t r = 0; r < p; ++r)
          if (h(r, v, it.slot) != h(r, v, vslot(V_LP, g))) bad.push_back(r);
        if (bad.empty()) continue;
        std::string who;
        for (int64_t r : bad) who += (who.empty() ? "" : ", ") + std::to_string(r);
        throw Error(Status::VerifyFailed,
                    "GJ_VERIFY: step " + std::to_string(it.step) + " (panel " + std::to_string(v) + "), phase " +
                        it.phase + ", rank-local buffer " + it.buffer + ": rank(s) [" + who +
                        "] saw different bytes on stream " + it.stream +
                        " than the SIDE stream left at the end of the panel (" +
                        (std::string(it.phase).find("before") != std::string::npos
                             ? "read before it was written or before the write was visible"
                             : "rewritten while still being read") +
                        "; first mismatch in step order)");
      }
      // reference value: the root's hash (broadcast buffers), else rank 0's (gathered / agreed state)
      const int64_t ref = it.root >= 0 ? it.root : 0;
      for (int64_t r = 0; r < p; ++r)
        if (h(r, v, it.slot) != h(ref, v, it.slot)) bad.push_back(r);
      if (bad.empty()) continue;
      std::string who;
      for (int64_t r : bad) who += (who.empty() ? "" : ", ") + std::to_string(r);
      throw Error(Status::VerifyFailed,
                  "GJ_VERIFY: step " + std::to_string(it.step) + " (panel " + std::to_string(v) + "), phase " +
                      it.phase + ", buffer " + it.buffer + (it.root >= 0 ? ", root rank " + std::to_string(it.root)
                                                                         : ", reference rank 0") +
                      ": rank(s) [" + who + "] consumed different bytes on stream " + it.stream +
                      " (first mismatch in step order)");
    }
  }
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
  dev_.host_access(ihost_, sizeof(int32_t) * (Nr + std::max<int64_t>(L_.nblk, 1)), true);
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
  comm_.drain(dev_, S_COMM);
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

// Bytes the fp64 check of an fp32 solve needs on this rank beyond the solve's own buffers: the
// fp64 copy of A's rows, the widened inverse and, at p > 1, the gathered fp32 inverse.
size_t Engine::residual_fp64_bytes() const {
  const size_t npad = (size_t)L_.npad, rows = (size_t)std::max<int64_t>(L_.rows, 1);
  size_t b = rows * npad * 8 + npad * npad * 8;
  if (L_.p > 1) b += npad * npad * esz() + (size_t)L_.max_nblk * L_.m * npad * esz() * (L_.p + 1);
  return b;
}

// Collective: the residual of an fp32 solve is computed in fp64 (fp64 A, widened inverse, fp64
// MFMA accumulation: the reference's check, main.cpp:490-507, is fp64) whenever that fits on every
// rank; otherwise in fp32 against the fp32 matrix (residual_precision() says which).
bool Engine::residual_wide() {
  if (opt_.dtype == DType::F64) return false;
  const bool fits = !injected_alloc_fail(L_.k, "residual64") &&
                    (!dev_.on_gpu() || residual_fp64_bytes() + (64u << 20) <= dev_.free_memory());
  return comm_.host_max(dev_, fits ? 0.0 : 1.0) == 0.0;
}

// A: this rank's rows of the matrix (ld npad), fp64 when wide, else the engine dtype.
double Engine::residual_common(const void* A, bool wide) {
  const int64_t m = L_.m, p = L_.p, npad = L_.npad;
  const size_t es = esz();
  void* full = out_;
  void* gath = nullptr;
  if (p > 1) {
    const size_t per = (size_t)L_.max_nblk * m * npad * es;
    // the whole inverse on every rank: agree that it fits everywhere before the first allocation
    const size_t need = (size_t)npad * npad * es + per * p + (L_.nblk < L_.max_nblk ? per : 0);
    const bool fits = !injected_alloc_fail(L_.k, "residual") &&
                      (!dev_.on_gpu() || need + (64u << 20) <= dev_.free_memory());
    if (comm_.host_max(dev_, fits ? 0.0 : 1.0) > 0) return residual_streamed(A, wide);
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
    comm_.drain(dev_, S_COMM);
    if (tmp) dev_.release(tmp);
    dev_.release(gath);
  }
  const DType rdt = wide ? DType::F64 : opt_.dtype;
  void* fullr = full;
  if (rdt != opt_.dtype) {  // widen the inverse (fp32 -> fp64)
    fullr = dev_.alloc((size_t)npad * npad * 8);
    dev_.widen(opt_.dtype, static_cast<double*>(fullr), npad, full, npad, npad, npad, S_MAIN);
  }
  double local = 0.0;
  if (L_.nblk > 0) {
    dev_.residual(rdt, A, fullr, L_, dscratch_, S_MAIN);
    dev_.copy(dhost_, dscratch_, sizeof(double), S_MAIN);
    dev_.sync_stream(S_MAIN);
    local = dhost_[0];
  }
  dev_.sync_stream(S_MAIN);
  if (fullr != full) dev_.release(fullr);
  if (p > 1) dev_.release(full);
  last_residual_fp64_ = (rdt == DType::F64);
  return comm_.host_max(dev_, local);
}

// p > 1 when the whole inverse does not fit on some rank: the reference's ring (matrix_mult_matrix,
// main.cpp:534-642, MPI_Sendrecv_replace of the B strips) as p broadcasts of one rank's strip at a
// time.  R = A_loc * inv accumulates strip by strip (strip q = block rows j p + q of the inverse
// meet columns (j p + q) m .. + m of A_loc), then sum_j |R - I| per row.  Needs R, one strip and
// (fp32 solves checked in fp64) its widened copy instead of two whole inverses.
double Engine::residual_streamed(const void* A, bool wide) {
  const int64_t m = L_.m, p = L_.p, npad = L_.npad, rows = std::max<int64_t>(L_.rows, 1);
  const size_t es = esz();
  const DType rdt = wide ? DType::F64 : opt_.dtype;
  const size_t res = dtype_size(rdt);
  const size_t per = (size_t)L_.max_nblk * m * npad;  // elements of the largest strip
  const size_t need = (size_t)rows * npad * res + per * es + (wide ? per * 8 : 0);
  const bool fits = !injected_alloc_fail(L_.k, "residual_stream") &&
                    (!dev_.on_gpu() || need + (64u << 20) <= dev_.free_memory());
  if (comm_.host_max(dev_, fits ? 0.0 : 1.0) > 0)
    throw Error(Status::NoMemory, "not enough device memory for the residual (" + std::to_string(need) +
                                      " bytes per rank even streamed)");
  const int s = S_COMM;  // the broadcasts' stream: every GEMM after its strip without a cross-stream hop
  void* R = dev_.alloc((size_t)rows * npad * res);
  void* S = dev_.alloc(per * es);
  void* Sw = wide ? dev_.alloc(per * 8) : nullptr;
  dev_.record(ev_main_, S_MAIN);  // A (MAIN) is complete before the first product
  dev_.wait(s, ev_main_);
  dev_.memset0(R, (size_t)rows * npad * res, s);
  for (int64_t q = 0; q < p; ++q) {
    const int64_t nbq = rows_owned(L_.Nr, p, q);
    if (nbq == 0) continue;
    void* buf = (q == L_.k) ? out_ : S;
    comm_.bcast(dev_, buf, (size_t)nbq * m * npad * es, (int)q, s);
    const void* src = buf;
    if (wide) {
      dev_.widen(opt_.dtype, static_cast<double*>(Sw), npad, buf, npad, nbq * m, npad, s);
      src = Sw;
    }
    if (L_.nblk > 0)
      for (int64_t j = 0; j < nbq; ++j)
        dev_.gemm(rdt, GemmOp::Acc, ALayout::RowMajor, L_.rows, npad, m,
                  static_cast<const char*>(A) + (size_t)(j * p + q) * m * res, npad,
                  static_cast<const char*>(src) + (size_t)j * m * npad * res, npad, R, npad, s);
  }
  double local = 0.0;
  if (L_.nblk > 0) {
    dev_.row_abs_max_minus_i(rdt, R, npad, L_, dscratch_, s);
    dev_.copy(dhost_, dscratch_, sizeof(double), s);
  }
  comm_.drain(dev_, s);
  if (L_.nblk > 0) local = dhost_[0];
  dev_.release(R);
  dev_.release(S);
  if (Sw) dev_.release(Sw);
  last_residual_fp64_ = (rdt == DType::F64);
  return comm_.host_max(dev_, local);
}

double Engine::residual_generated(GenSpec g) {
  GJ_REQUIRE(solved_, "residual: solve() first");
  if (residual_wide()) {  // fp64 A straight from the generator
    void* Aw = dev_.alloc((size_t)std::max<int64_t>(L_.rows, 1) * L_.npad * 8);
    dev_.generate(DType::F64, Aw, L_, g, S_MAIN);
    double r = 0;
    try {
      r = residual_common(Aw, true);
    } catch (...) {
      dev_.release(Aw);
      throw;
    }
    dev_.release(Aw);
    return r;
  }
  dev_.generate(opt_.dtype, X_, L_, g, S_MAIN);
  dev_.sync_stream(S_MAIN);
  local_norm_valid_ = false;
  return residual_common(X_, false);
}

// this rank's real rows from host doubles into panel P (dtype dt, ld npad): zero + identity padding,
// then through a bounded staging buffer (<= 256 MiB)
void Engine::upload_rows_into(void* P, DType dt, const double* host, int64_t ld) {
  GenSpec z;
  z.kind = GenKind::Zero;
  dev_.generate(dt, P, L_, z, S_MAIN);
  const int64_t real = real_local_rows(), n = L_.n;
  if (real > 0) {
    const int64_t rows_per = std::max<int64_t>(1, (int64_t(256) << 20) / (n * 8));
    const int64_t chunk = std::min(rows_per, real);
    double* stage = static_cast<double*>(dev_.alloc(sizeof(double) * chunk * n));
    for (int64_t r0 = 0; r0 < real; r0 += chunk) {
      const int64_t nr = std::min(chunk, real - r0);
      dev_.copy2d(stage, n * 8, host + r0 * ld, ld * 8, n * 8, nr, S_MAIN);
      dev_.upload_convert(dt, static_cast<char*>(P) + (size_t)r0 * L_.npad * dtype_size(dt), L_.npad, stage, n,
                          nr, n, S_MAIN);
      dev_.sync_stream(S_MAIN);
    }
    dev_.release(stage);
  }
  dev_.sync_stream(S_MAIN);
}

double Engine::residual_rows(const double* host, int64_t ld) {
  GJ_REQUIRE(solved_, "residual: solve() first");
  if (residual_wide()) {
    void* Aw = dev_.alloc((size_t)std::max<int64_t>(L_.rows, 1) * L_.npad * 8);
    double r = 0;
    try {
      upload_rows_into(Aw, DType::F64, host, ld);
      r = residual_common(Aw, true);
    } catch (...) {
      dev_.release(Aw);
      throw;
    }
    dev_.release(Aw);
    return r;
  }
  upload_local_rows(host, ld);
  solved_ = true;
  return residual_common(X_, false);
}

// ---------------------------------------------------------------- A x = b
namespace {
// full n-vector (double, host) -> padded device vector of the engine dtype
void* upload_vector(Device& dev, DType dt, const double* v, int64_t n, int64_t npad) {
  double* st = static_cast<double*>(dev.alloc(sizeof(double) * npad));
  dev.memset0(st, sizeof(double) * npad, S_MAIN);
  dev.copy(st, v, sizeof(double) * n, S_MAIN);
  void* d = dev.alloc(dtype_size(dt) * npad);
  dev.upload_convert(dt, d, 1, st, 1, npad, 1, S_MAIN);
  dev.sync_stream(S_MAIN);
  dev.release(st);
  return d;
}
}  // namespace

// local product y = P * v  (P: this rank's rows of a panel, v: full padded vector) -> host doubles
static std::vector<double> local_matvec(Device& dev, DType dt, const void* P, const Layout& L,
                                        const void* vd) {
  const size_t es = dtype_size(dt);
  std::vector<double> y((size_t)L.rows, 0.0);
  if (L.rows == 0) return y;
  void* yd = dev.alloc(es * L.rows);
  dev.gemm(dt, GemmOp::Store, ALayout::RowMajor, L.rows, 1, L.npad, P, L.npad, vd, 1, yd, 1, S_MAIN);
  std::vector<char> h(es * L.rows);
  dev.copy(h.data(), yd, es * L.rows, S_MAIN);
  dev.sync_stream(S_MAIN);
  dev.release(yd);
  for (int64_t i = 0; i < L.rows; ++i)
    y[i] = dt == DType::F64 ? reinterpret_cast<double*>(h.data())[i] : (double)reinterpret_cast<float*>(h.data())[i];
  return y;
}

void Engine::apply_inverse(const double* b, double* x) {
  GJ_REQUIRE(solved_, "apply_inverse: solve() first");
  const int64_t m = L_.m, n = L_.n, p = L_.p;
  void* bd = upload_vector(dev_, opt_.dtype, b, n, L_.npad);
  std::vector<double> mine = local_matvec(dev_, opt_.dtype, out_, L_, bd);
  dev_.release(bd);
  const int64_t per = L_.max_nblk * m;
  mine.resize((size_t)per, 0.0);
  std::vector<double> all((size_t)per * p);
  comm_.host_allgather(dev_, mine.data(), all.data(), sizeof(double) * per);
  for (int64_t q = 0; q < p; ++q)
    for (int64_t j = 0; j < rows_owned(L_.Nr, p, q); ++j)
      for (int64_t r = 0; r < m; ++r) {
        const int64_t gi = (j * p + q) * m + r;
        if (gi < n) x[gi] = all[(size_t)q * per + j * m + r];
      }
}

double Engine::axb_residual(const double* x, const double* b) {
  const int64_t m = L_.m, n = L_.n;
  void* xd = upload_vector(dev_, opt_.dtype, x, n, L_.npad);
  std::vector<double> y = local_matvec(dev_, opt_.dtype, X_, L_, xd);
  dev_.release(xd);
  double local = 0.0;
  for (int64_t i = 0; i < L_.rows; ++i) {
    const int64_t gi = L_.global_block(i / m) * m + i % m;
    if (gi < n) local = std::max(local, std::fabs(y[i] - b[gi]));
  }
  return comm_.host_max(dev_, local);
}

// x = inv(A) b, then iterative refinement with the residual in fp64:
//   r_k = b - A x_k  (A in fp64: regenerated, or re-uploaded from the caller's fp64 rows;
//                     fp64 MFMA GEMV, the full vector all-gathered)
//   x_{k+1} = x_k + X r_k   (X = the computed inverse, engine dtype)
// It converges when ||I - X A|| < 1; each step gains about -log10 ||I - X A|| digits.  Stops at
// the normwise backward error ||r|| / (||A|| ||x|| + ||b||) <= tol (inf-norms), after max_refine
// steps, or when the residual stops shrinking
// (refinement cannot converge: reported, not hidden).
RhsResult Engine::solve_rhs_device(const double* b, double* x, const void* dev_rows_f64, int64_t ld,
                                   int max_refine, double tol) {
  GJ_REQUIRE(dev_rows_f64 || real_local_rows() == 0, "solve_rhs_device: the matrix rows are needed");
  return solve_rhs_impl(b, x, nullptr, nullptr, dev_rows_f64, ld, max_refine, tol);
}

RhsResult Engine::solve_rhs(const double* b, double* x, const GenSpec* gen, const double* host_rows,
                            int64_t ld, int max_refine, double tol) {
  GJ_REQUIRE(gen || host_rows || real_local_rows() == 0,
             "solve_rhs: the matrix (generator or rows) is needed for the fp64 residual");
  return solve_rhs_impl(b, x, gen, host_rows, nullptr, ld, max_refine, tol);
}

RhsResult Engine::solve_rhs_impl(const double* b, double* x, const GenSpec* gen, const double* host_rows,
                                 const void* dev_rows, int64_t ld, int max_refine, double tol) {
  GJ_REQUIRE(solved_, "solve_rhs: solve() first");
  const int64_t m = L_.m, n = L_.n;
  RhsResult rr;
  void* Aw = dev_.alloc((size_t)std::max<int64_t>(L_.rows, 1) * L_.npad * 8);
  try {
    if (gen) {
      dev_.generate(DType::F64, Aw, L_, *gen, S_MAIN);
    } else if (dev_rows) {  // zero + identity padding, then the real rows device-to-device
      GenSpec z;
      z.kind = GenKind::Zero;
      dev_.generate(DType::F64, Aw, L_, z, S_MAIN);
      const int64_t real = real_local_rows();
      if (real > 0) dev_.copy2d(Aw, L_.npad * 8, dev_rows, ld * 8, n * 8, real, S_MAIN);
    } else {
      upload_rows_into(Aw, DType::F64, host_rows, ld);
    }
    dev_.sync_stream(S_MAIN);
    double bn = 0;
    for (int64_t i = 0; i < n; ++i) bn = std::max(bn, std::fabs(b[i]));
    if (bn == 0) bn = 1;
    dev_.row_abs_max(DType::F64, Aw, L_.npad, L_, dscratch_, S_MAIN);  // ||A||_inf (fp64)
    dev_.copy(dhost_, dscratch_, sizeof(double), S_MAIN);
    dev_.sync_stream(S_MAIN);
    const double an = comm_.host_max(dev_, L_.nblk > 0 ? dhost_[0] : 0.0);
    apply_inverse(b, x);
    std::vector<double> r((size_t)n), d((size_t)n);
    // the best iterate so far (a diverging refinement, e.g. an fp32 inverse with ||I - XA|| near 1,
    // must not hand back a worse x than it was given)
    std::vector<double> best_x(x, x + n);
    RhsResult best;
    double best_rn = 1e300;
    double prev = 1e300;
    for (int it = 0;; ++it) {
      // r = b - A x (this rank's rows, fp64), all-gathered to the full vector
      void* xd = upload_vector(dev_, DType::F64, x, n, L_.npad);
      std::vector<double> y = local_matvec(dev_, DType::F64, Aw, L_, xd);
      dev_.release(xd);
      const int64_t per = L_.max_nblk * m;
      std::vector<double> mine((size_t)per, 0.0), all((size_t)per * L_.p);
      for (int64_t i = 0; i < L_.rows; ++i) {
        const int64_t gi = L_.global_block(i / m) * m + i % m;
        if (gi < n) mine[(size_t)i] = b[gi] - y[(size_t)i];
      }
      comm_.host_allgather(dev_, mine.data(), all.data(), sizeof(double) * per);
      double rn = 0;
      for (int64_t q = 0; q < L_.p; ++q)
        for (int64_t j = 0; j < rows_owned(L_.Nr, L_.p, q); ++j)
          for (int64_t e = 0; e < m; ++e) {
            const int64_t gi = (j * L_.p + q) * m + e;
            if (gi < n) {
              r[(size_t)gi] = all[(size_t)q * per + j * m + e];
              rn = std::max(rn, std::fabs(r[(size_t)gi]));
            }
          }
      double xn = 0;
      for (int64_t i = 0; i < n; ++i) xn = std::max(xn, std::fabs(x[i]));
      rr.history.push_back(rn / bn);
      rr.residual = rn;
      rr.backward_error = rn / (an * xn + bn);
      if (rr.backward_error <= tol) {
        rr.converged = true;
        break;
      }
      if (rn < best_rn) {
        best_rn = rn;
        best_x.assign(x, x + n);
        best = rr;
      }
      if (it >= max_refine || (it > 0 && rn > 0.5 * prev)) {  // budget spent / not contracting
        if (rn > best_rn) {  // return the best iterate, with its own residual (history kept)
          std::copy(best_x.begin(), best_x.end(), x);
          best.history = rr.history;
          rr = best;
        }
        break;
      }
      prev = rn;
      apply_inverse(r.data(), d.data());
      for (int64_t i = 0; i < n; ++i) x[i] += d[(size_t)i];
      rr.steps = it + 1;
    }
  } catch (...) {
    dev_.release(Aw);
    throw;
  }
  dev_.release(Aw);
  return rr;
}

void SelfComm::host_allgather(Device&, const void* send, void* recv, size_t bytes) {
  if (send != recv) std::memcpy(recv, send, bytes);
}

[[noreturn]] void fail(const char* file, int line, const std::string& msg) {
  throw Error(Status::BadArgs, std::string(file) + ":" + std::to_string(line) + ": " + msg);
}

}  // namespace gj
