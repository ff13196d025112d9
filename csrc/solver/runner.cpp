// In-process multi-rank driver (see gj/runner.hpp).
#include "gj/runner.hpp"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <memory>
#include <mutex>
#include <thread>

#include "gj/async_host_device.hpp"
#include "gj/comms.hpp"
#include "gj/gen.hpp"
#include "gj/hip_device.hpp"
#include "gj/host_device.hpp"
#include "gj/io.hpp"
#include "gj/race_check.hpp"

namespace gj {

namespace {

struct Shared {
  std::mutex mu;
  RunReport rep;
  std::vector<double> b;     // right-hand side (rhs mode)
  std::vector<double> full;  // input matrix (file) shared by all rank threads
  const double* input = nullptr;
  double* inverse = nullptr;
};

void rank_main(const RunConfig& cfg, int rank, Shared& sh, std::shared_ptr<LoopbackHub> hub,
               const std::vector<std::string>& ids, bool use_rccl, std::shared_ptr<HbChecker> hb) {
  std::unique_ptr<Device> dev;
  std::unique_ptr<Comm> comm;
  const bool async = cfg.comm == "async";
  if (cfg.gpu) {
    int ndev = 0;
    (void)hipGetDeviceCount(&ndev);
    const int d = (cfg.first_device + rank) % std::max(ndev, 1);
    (void)hipSetDevice(d);
    dev.reset(new HipDevice(d));
    if (use_rccl)
      comm.reset(new RcclComm(ids, cfg.ranks, rank, d, cfg.one_comm));
    else if (cfg.ranks == 1)
      comm.reset(new SelfComm());
    else if (async)
      comm.reset(new AsyncLoopbackComm(hub, rank, cfg.jitter_us, cfg.gen.seed));
    else
      comm.reset(new LoopbackComm(hub, rank));
  } else {
    const int hw = (int)std::max(1u, std::thread::hardware_concurrency());
    const int nt = cfg.host_threads > 0 ? cfg.host_threads : std::max(1, hw / cfg.ranks);
    if (async)  // real asynchronous streams on the CPU (one worker thread per stream role)
      dev.reset(new AsyncHostDevice(nt, cfg.jitter_us, cfg.gen.seed * 131u + (uint64_t)rank,
                                    cfg.solve.comm_timeout_s));
    else
      dev.reset(new HostDevice(nt));
    if (cfg.ranks == 1)
      comm.reset(new SelfComm());
    else if (async)
      comm.reset(new AsyncLoopbackComm(hub, rank, cfg.jitter_us, cfg.gen.seed));
    else
      comm.reset(new LoopbackComm(hub, rank));
  }
  if (hb) {
    GJ_REQUIRE(!use_rccl, "--race-check needs an in-process transport (loopback / async), not RCCL");
    dev.reset(new RaceCheckDevice(std::move(dev), hb, "rank " + std::to_string(rank)));
  }

  // collective allocation check (reference main.cpp:366-381)
  std::unique_ptr<Engine> eng;
  double fail = 0.0;
  std::string err;
  try {
    eng.reset(new Engine(*dev, *comm, cfg.n, cfg.m, cfg.solve));
  } catch (const Error& e) {
    fail = 1.0;
    err = e.what();
  }
  if (comm->host_max(*dev, fail) > 0) {
    std::lock_guard<std::mutex> lk(sh.mu);
    if (sh.rep.status == Status::Ok) {
      sh.rep.status = Status::NoMemory;
      sh.rep.message = err.empty() ? "Not enough memory!" : err;
    }
    return;
  }
  const Layout& L = eng->layout();
  if (rank == 0) {
    std::lock_guard<std::mutex> lk(sh.mu);
    sh.rep.device_desc = dev->describe();
    sh.rep.comm_desc = comm->describe();
  }

  // local rows of a host matrix (block rows rank, rank+p, ...)
  std::vector<double> local;
  const double* src = sh.input ? sh.input : (sh.full.empty() ? nullptr : sh.full.data());
  auto load = [&]() {
    if (src) {
      const int64_t real = eng->real_local_rows();
      if (local.empty() && real > 0) {
        local.resize((size_t)real * cfg.n);
        for (int64_t r = 0; r < real; ++r) {
          const int64_t gr = L.global_row(r);
          std::copy(src + gr * cfg.n, src + (gr + 1) * cfg.n, local.begin() + r * cfg.n);
        }
      }
      eng->upload_local_rows(local.data(), cfg.n);
    } else {
      eng->generate(cfg.gen);
    }
  };

  const int nm = (int)std::min<int64_t>(cfg.n, cfg.print_max);
  SolveStats st;
  double best = 1e300, glob = 0;
  for (int rep = 0; rep < std::max(1, cfg.repeats); ++rep) {
    load();
    if (rep == 0 && cfg.want_corners) {
      auto c = eng->corner(nm, 0);
      if (rank == 0) {
        std::lock_guard<std::mutex> lk(sh.mu);
        sh.rep.corner_a = c;
      }
    }
    st = eng->solve();
    glob = comm->host_max(*dev, st.seconds);
    best = std::min(best, glob);
    if (st.status != Status::Ok) break;
  }
  if (st.status != Status::Ok) {
    std::lock_guard<std::mutex> lk(sh.mu);
    sh.rep.status = st.status;
    sh.rep.message = st.status == Status::NoBlockMemory ? "not enough memory for block" : "singular matrix";
    if (rank == 0) sh.rep.stats = st;
    return;
  }
  if (cfg.want_corners) {
    auto c = eng->corner(nm, 1);
    if (rank == 0) {
      std::lock_guard<std::mutex> lk(sh.mu);
      sh.rep.corner_inv = c;
    }
  }
  if (sh.inverse) {
    const int64_t real = eng->real_local_rows();
    std::vector<double> rows((size_t)std::max<int64_t>(real, 1) * cfg.n);
    eng->download_local_rows(rows.data(), cfg.n);
    for (int64_t r = 0; r < real; ++r) {
      const int64_t gr = L.global_row(r);
      std::copy(rows.begin() + r * cfg.n, rows.begin() + (r + 1) * cfg.n, sh.inverse + gr * cfg.n);
    }
  }
  bool do_res = cfg.residual == ResidualMode::Always ||
                (cfg.residual == ResidualMode::Compat &&
                 (cfg.ranks != 1 || cfg.gen.kind == GenKind::Hilbert));
  double res = 0;
  if (do_res) {
    if (src) {
      res = eng->residual_rows(local.data(), cfg.n);
    } else {
      res = eng->residual_generated(cfg.gen);
    }
  }
  if (!sh.b.empty()) {
    std::vector<double> x((size_t)cfg.n);
    comm->barrier(*dev);
    const auto t0 = std::chrono::steady_clock::now();
    const int refine = cfg.refine >= 0 ? cfg.refine : (cfg.solve.dtype == DType::F32 ? 10 : 2);
    if (src && local.empty()) load();  // the fp64 rows of A (residual_rows keeps them in `local`)
    const RhsResult rr = eng->solve_rhs(sh.b.data(), x.data(), src ? nullptr : &cfg.gen,
                                        src ? local.data() : nullptr, cfg.n, refine, cfg.refine_tol);
    const double tx = comm->host_max(
        *dev, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
    if (rank == 0) {
      std::lock_guard<std::mutex> lk(sh.mu);
      sh.rep.rhs_solved = true;
      sh.rep.rhs_residual = rr.residual;
      sh.rep.rhs_history = rr.history;
      sh.rep.rhs_steps = rr.steps;
      sh.rep.rhs_converged = rr.converged;
      sh.rep.rhs_backward_error = rr.backward_error;
      sh.rep.rhs_seconds = tx;
      sh.rep.x_head.assign(x.begin(), x.begin() + nm);
      if (cfg.keep_solution) sh.rep.x = x;
    }
  }
  if (rank == 0) {
    std::lock_guard<std::mutex> lk(sh.mu);
    sh.rep.stats = st;
    sh.rep.glob_time = glob;
    sh.rep.best_time = best;
    sh.rep.residual_computed = do_res;
    sh.rep.residual = res;
    sh.rep.residual_fp64 = eng->residual_fp64();
    sh.rep.nm = nm;
    const double n = (double)cfg.n;
    sh.rep.gflops_nominal = glob > 0 ? 2.0 * n * n * n / glob / 1e9 : 0.0;
  }
}

}  // namespace

RunReport run_local(const RunConfig& cfg) {
  Shared sh;
  if (cfg.n <= 0 || cfg.m <= 0 || cfg.ranks <= 0) {
    sh.rep.status = Status::BadArgs;
    sh.rep.message = "bad arguments";
    return sh.rep;
  }
  if (!cfg.file.empty()) {
    const Status s = read_matrix_file(cfg.file, cfg.n, sh.full, cfg.host_threads);
    if (s != Status::Ok) {
      sh.rep.status = s;
      sh.rep.message = (s == Status::CannotOpen ? "cannot open " : "cannot read ") + cfg.file;
      return sh.rep;
    }
  }
  sh.input = cfg.input;
  if (cfg.rhs_input) {
    sh.b.assign(cfg.rhs_input, cfg.rhs_input + cfg.n);
  } else if (cfg.rhs == "ones") {
    sh.b.assign((size_t)cfg.n, 1.0);
  } else if (cfg.rhs == "random") {
    sh.b.resize((size_t)cfg.n);
    for (int64_t i = 0; i < cfg.n; ++i) sh.b[i] = gen_value((int)GenKind::Random, cfg.gen.seed ^ 0x9E3779B97F4A7C15ull, cfg.n, i, 0);
  } else if (!cfg.rhs.empty()) {
    const Status s = read_values_file(cfg.rhs, (size_t)cfg.n, sh.b, cfg.host_threads);
    if (s != Status::Ok) {
      sh.rep.status = s;
      sh.rep.message = (s == Status::CannotOpen ? "cannot open " : "cannot read ") + cfg.rhs;
      return sh.rep;
    }
  }
  if (cfg.keep_inverse) {
    sh.rep.inverse.assign((size_t)cfg.n * cfg.n, 0.0);
    sh.inverse = sh.rep.inverse.data();
  }
  bool use_rccl = false;
  if (cfg.gpu) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
      sh.rep.status = Status::CommError;
      sh.rep.message = "no HIP device available (use --device cpu)";
      return sh.rep;
    }
    if (cfg.comm == "rccl")
      use_rccl = true;
    else if (cfg.comm == "auto")
      use_rccl = cfg.ranks > 1 && cfg.ranks <= ndev;
    if (use_rccl && cfg.ranks > ndev) {
      sh.rep.status = Status::BadArgs;
      sh.rep.message = "rccl needs one GPU per rank";
      return sh.rep;
    }
  }
  std::vector<std::string> ids;
  if (use_rccl) {
    ids.push_back(RcclComm::unique_id());
    ids.push_back(RcclComm::unique_id());
  }
  auto hub = std::make_shared<LoopbackHub>(cfg.ranks);
  std::shared_ptr<HbChecker> hb = cfg.race_check ? std::make_shared<HbChecker>() : nullptr;
  // A rank that throws (a transport error, a timed-out wait, a failed launch) reports it and
  // poisons the hub, so its peers leave their next rendezvous with an error instead of hanging.
  auto guarded = [&](int r) {
    try {
      rank_main(cfg, r, sh, hub, ids, use_rccl, hb);
    } catch (const Error& e) {
      hub->fail(e.what());
      std::lock_guard<std::mutex> lk(sh.mu);
      if (sh.rep.status == Status::Ok) {
        sh.rep.status = e.status();
        sh.rep.message = e.what();
      }
    } catch (const std::exception& e) {
      hub->fail(e.what());
      std::lock_guard<std::mutex> lk(sh.mu);
      if (sh.rep.status == Status::Ok) {
        sh.rep.status = Status::CommError;
        sh.rep.message = e.what();
      }
    }
  };
  if (cfg.ranks == 1) {
    guarded(0);
  } else {
    std::vector<std::thread> th;
    for (int r = 0; r < cfg.ranks; ++r) th.emplace_back([&, r] { guarded(r); });
    for (auto& t : th) t.join();
  }
  if (hb) {
    sh.rep.race_count = hb->races();
    sh.rep.races = hb->reports();
    sh.rep.race_ops = hb->ops();
  }
  return sh.rep;
}

}  // namespace gj
