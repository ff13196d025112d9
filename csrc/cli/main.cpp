// `gj` — command-line front end, compatible with the reference's `mpirun -np p ./a.out n m [file]`
// (main.cpp:65-93 + the stdout contract of solve(), main.cpp:343-519).
//
//   gj [options] n m [file]
//
// Positional arguments keep the reference semantics: n and m via atoi (non-numeric or <= 0 ->
// usage, exit 1), optional input file (text, fscanf("%lf")-compatible, or raw fp64 ".bin").
// stdout is byte-compatible with the reference:
//   A / corner / glob_time: %.2f / inverse matrix: + blank line / corner / residual: %e
// Exit codes: 0 ok, 1 usage, 2 any failure.
//
// Options (all optional; defaults reproduce the reference on one MI355X):
//   -p, --ranks P        number of ranks (GPUs with --device gpu, virtual ranks with --device cpu)
//   --gpus P             alias of --ranks for GPU runs
//   --device gpu|cpu     execution backend (default: gpu when a HIP device exists)
//   --comm auto|rccl|loopback|async   (async: stream-ordered virtual ranks; --jitter US)
//   --one-comm           rccl: one communicator for the SIDE and COMM roles (also GJ_ONE_COMM=1)
//   --dtype fp64|fp32
//   --gen absdiff|hilbert|random|randshift|identity   generator when no file is given (reference: absdiff;
//                        -DHILBERT -> --gen hilbert)
//   --seed S             seed of --gen random
//   --residual always|compat|never   compat = the reference's "p == 1!" skip (main.cpp:499-513)
//   --print-max N        corner size (reference MAX_P = 10)
//   --eps E              singularity threshold factor (reference EPS = 1e-15)
//   --chunk-cols C       broadcast pipelining granularity
//   --depth D            elimination steps fused per trailing update (1..8; default: engine.hpp)
//   --pivot block-min-inv-norm|partial   pivot rule (default: the reference's smallest ||inv||;
//                        partial = block partial pivoting, one candidate inverse per rank and step)
//   --pivot-growth G     partial pivoting: a candidate with ||inv||_inf * max|W| > G counts as
//                        singular (default by dtype: 1e8 fp64, 8.4e4 fp32; 0 = off)
//   --repeat R           time R solves, report the last (min also in --json)
//   --out FILE           write the inverse (text, or .bin)
//   --rhs ones|random|FILE  also solve A x = b (x = inv(A) b) and report ||A x - b||_inf
//   --out-x FILE         write x (text, or .bin); implies --rhs ones unless --rhs is given
//   --refine K           at most K refinement steps of x with the residual in fp64 (default: 10 for
//                        fp32 solves, 2 for fp64; Engine::solve_rhs)
//   --json               machine-readable report on stderr
//   --bcast auto|ring|direct  pivot-row broadcast algorithm at p > 2 (sets GJ_BCAST; auto = timed
//                        against each other at startup, Comm::tune_bcast)
//   --sync-debug         synchronise after every phase (race screening)
//   --verify             consumption-point hashes of every broadcast buffer, compared across ranks
//                        after the solve (also GJ_VERIFY=1; a mismatch fails with the step named)
//   --race-check         run under the happens-before schedule checker (RaceCheckDevice): every
//                        unordered conflicting access is printed to stderr and the exit code is 2
//   --check-residual TOL exit 2 (after the normal output) when the residual is not finite or
//                        exceeds TOL: a wrong inverse is a failure, not a slow success
//   --profile            per-phase device timers (in --json) + roctx ranges for rocprofv3
//   --comm-timeout S     seconds a rank waits for a pivot before declaring a peer failure
//   --wait-debugger S    sleep S seconds at start (reference -DSLEEP, main.cpp:8, :70-72)
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "gj/io.hpp"
#include "gj/runner.hpp"

using namespace gj;

static int usage(const char* prog) {
  std::printf("usage:%s n m [<file>]\n", prog);
  return 1;
}

static void json_report(const RunConfig& cfg, const RunReport& rep) {
  std::string phases;
  if (rep.stats.profiled) {
    phases = ", \"phases_ms\": {";
    for (int i = 0; i < kNumPhases; ++i) {
      char buf[96];
      std::snprintf(buf, sizeof buf, "%s\"%s\": %.3f", i ? ", " : "", phase_name(i), rep.stats.phase_ms[i]);
      phases += buf;
    }
    phases += "}";
  }
  std::string rhs;
  if (rep.rhs_solved) {
    char buf[256];
    std::snprintf(buf, sizeof buf,
                  ", \"axb_residual\": %.6e, \"axb_seconds\": %.6f, \"axb_backward_error\": %.6e, "
                  "\"refine_steps\": %d, \"refine_converged\": %s, \"axb_history\": [",
                  rep.rhs_residual, rep.rhs_seconds, rep.rhs_backward_error, rep.rhs_steps,
                  rep.rhs_converged ? "true" : "false");
    rhs = buf;
    for (size_t i = 0; i < rep.rhs_history.size(); ++i) {
      std::snprintf(buf, sizeof buf, "%s%.3e", i ? ", " : "", rep.rhs_history[i]);
      rhs += buf;
    }
    rhs += "]";
  }
  std::fprintf(stderr,
               "{\"n\": %lld, \"m\": %lld, \"ranks\": %d, \"device\": \"%s\", \"comm\": \"%s\", "
               "\"dtype\": \"%s\", \"status\": %d, \"glob_time\": %.6f, \"best_time\": %.6f, "
               "\"gflops_nominal\": %.3f, \"residual\": %.6e, \"residual_computed\": %s, "
               "\"residual_fp64\": %s, \"host_wait_ms\": %.3f, \"offdiag_pivots\": %lld, \"pivot_fallbacks\": %lld%s%s}\n",
               (long long)cfg.n, (long long)cfg.m, cfg.ranks, rep.device_desc.c_str(),
               rep.comm_desc.c_str(), dtype_name(cfg.solve.dtype), (int)rep.status, rep.glob_time,
               rep.best_time, rep.gflops_nominal, rep.residual,
               rep.residual_computed ? "true" : "false", rep.residual_fp64 ? "true" : "false",
               rep.stats.host_wait_ms,
               (long long)rep.stats.offdiag_pivots, (long long)rep.stats.pivot_fallbacks, phases.c_str(), rhs.c_str());
}

int main(int argc, char* argv[]) {
  // Before the first HIP call: one hardware queue per stream (the progress argument of the two RCCL
  // communicators, README "Progress of the two communicators"; same policy as runtime_env.py) and
  // kernel arguments in device memory.
  {
    const char* q = std::getenv("GPU_MAX_HW_QUEUES");
    if (!q || std::atoi(q) < kMinHwQueues) setenv("GPU_MAX_HW_QUEUES", std::to_string(kMinHwQueues).c_str(), 1);
    setenv("HIP_FORCE_DEV_KERNARG", "1", 0);
  }
  RunConfig cfg;
  if (const char* e = std::getenv("GJ_ONE_COMM")) cfg.one_comm = std::atoi(e) != 0;
  std::vector<const char*> pos;
  bool json = false;
  std::string device = "auto", out_file, x_file;
  int wait_dbg = 0;
  double check_tol = -1.0;  // --check-residual
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    auto val = [&](const char* name) -> const char* {
      if (i + 1 >= argc) {
        std::fprintf(stderr, "%s needs a value\n", name);
        std::exit(usage(argv[0]));
      }
      return argv[++i];
    };
    if (a.size() > 1 && a[0] == '-' && !(a[1] >= '0' && a[1] <= '9')) {
      if (a == "-p" || a == "--ranks" || a == "--gpus") cfg.ranks = std::atoi(val(a.c_str()));
      else if (a == "--device") device = val("--device");
      else if (a == "--comm") cfg.comm = val("--comm");
      else if (a == "--one-comm") cfg.one_comm = true;
      else if (a == "--jitter") cfg.jitter_us = std::atof(val("--jitter"));
      else if (a == "--dtype") {
        const std::string d = val("--dtype");
        if (d == "fp64" || d == "f64" || d == "double") cfg.solve.dtype = DType::F64;
        else if (d == "fp32" || d == "f32" || d == "float") cfg.solve.dtype = DType::F32;
        else return usage(argv[0]);
      } else if (a == "--gen") {
        const std::string g = val("--gen");
        if (g == "absdiff") cfg.gen.kind = GenKind::AbsDiff;
        else if (g == "hilbert") cfg.gen.kind = GenKind::Hilbert;
        else if (g == "random") cfg.gen.kind = GenKind::Random;
        else if (g == "identity") cfg.gen.kind = GenKind::Identity;
        else if (g == "randshift") cfg.gen.kind = GenKind::RandomShifted;
        else return usage(argv[0]);
      } else if (a == "--seed") cfg.gen.seed = std::strtoull(val("--seed"), nullptr, 10);
      else if (a == "--residual") {
        const std::string r = val("--residual");
        if (r == "always") cfg.residual = ResidualMode::Always;
        else if (r == "compat") cfg.residual = ResidualMode::Compat;
        else if (r == "never") cfg.residual = ResidualMode::Never;
        else return usage(argv[0]);
      } else if (a == "--print-max") cfg.print_max = std::atoi(val("--print-max"));
      else if (a == "--eps") cfg.solve.eps = std::atof(val("--eps"));
      else if (a == "--chunk-cols") cfg.solve.chunk_cols = std::atoll(val("--chunk-cols"));
      else if (a == "--depth") cfg.solve.depth = std::atoi(val("--depth"));
      else if (a == "--pivot") {
        const std::string pv = val("--pivot");
        if (pv == "block-min-inv-norm") cfg.solve.pivot = PivotRule::MinInvNorm;
        else if (pv == "partial") cfg.solve.pivot = PivotRule::Partial;
        else return usage(argv[0]);
      }
      else if (a == "--pivot-growth") cfg.solve.pivot_growth = std::atof(val("--pivot-growth"));
      else if (a == "--repeat") cfg.repeats = std::atoi(val("--repeat"));
      else if (a == "--out") out_file = val("--out");
      else if (a == "--rhs") cfg.rhs = val("--rhs");
      else if (a == "--out-x") x_file = val("--out-x");
      else if (a == "--refine") cfg.refine = std::atoi(val("--refine"));
      else if (a == "--json") json = true;
      else if (a == "--bcast") {
        const std::string b = val("--bcast");
        if (b != "auto" && b != "ring" && b != "direct") return usage(argv[0]);
        setenv("GJ_BCAST", b.c_str(), 1);
      }
      else if (a == "--sync-debug") cfg.solve.sync_debug = true;
      else if (a == "--verify") cfg.solve.verify = true;
      else if (a == "--race-check") cfg.race_check = true;
      else if (a == "--check-residual") check_tol = std::atof(val("--check-residual"));
      else if (a == "--profile") cfg.solve.profile = true;
      else if (a == "--comm-timeout") cfg.solve.comm_timeout_s = std::atof(val("--comm-timeout"));
      else if (a == "--wait-debugger") wait_dbg = std::atoi(val("--wait-debugger"));
      else if (a == "--host-threads") cfg.host_threads = std::atoi(val("--host-threads"));
      else if (a == "--first-device") cfg.first_device = std::atoi(val("--first-device"));
      else return usage(argv[0]);
    } else {
      pos.push_back(argv[i]);
    }
  }
  // reference: argc in {3,4}, atoi(n) != 0, atoi(m) != 0 (main.cpp:77-83); negatives rejected too
  if (pos.size() < 2 || pos.size() > 3) return usage(argv[0]);
  const long long n = std::atoll(pos[0]), m = std::atoll(pos[1]);
  if (n <= 0 || m <= 0 || cfg.ranks <= 0 || cfg.print_max < 0) return usage(argv[0]);
  cfg.n = n;
  cfg.m = m;
  if (pos.size() == 3) cfg.file = pos[2];
  if (wait_dbg > 0) sleep(wait_dbg);

  if (device == "auto") {
    int ndev = 0;
    cfg.gpu = (hipGetDeviceCount(&ndev) == hipSuccess && ndev > 0);
  } else if (device == "gpu") {
    cfg.gpu = true;
  } else if (device == "cpu") {
    cfg.gpu = false;
  } else {
    return usage(argv[0]);
  }
  cfg.keep_inverse = !out_file.empty();
  cfg.keep_solution = !x_file.empty();
  if (!x_file.empty() && cfg.rhs.empty()) cfg.rhs = "ones";

  RunReport rep;
  try {
    rep = run_local(cfg);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "gj: %s\n", e.what());
    return 2;
  }
  // error reporting mirrors main.cpp:372-449
  switch (rep.status) {
    case Status::Ok: break;
    case Status::CannotOpen: std::printf("%s\n", rep.message.c_str()); return 2;
    case Status::CannotRead: std::printf("%s\n", rep.message.c_str()); return 2;
    case Status::NoMemory: std::printf("Not enough memory!\n"); if (!rep.message.empty()) std::fprintf(stderr, "%s\n", rep.message.c_str()); return 2;
    case Status::Singular:
    case Status::NoBlockMemory:  // both are Jordan() failures: after the A corner (main.cpp:410-443)
      std::printf("A\n");
      print_corner(stdout, rep.corner_a, (int)std::min<long long>(n, cfg.print_max));
      std::printf(rep.status == Status::Singular ? "singular matrix\n" : "not enough memory for block\n");
      if (json) json_report(cfg, rep);
      return 2;
    case Status::VerifyFailed: std::fprintf(stderr, "gj: %s\n", rep.message.c_str()); return 2;
    default: std::printf("error: %s\n", rep.message.c_str()); return 2;
  }
  std::printf("A\n");
  print_corner(stdout, rep.corner_a, rep.nm);
  std::printf("glob_time: %.2f\n", rep.glob_time);
  std::printf("inverse matrix:\n\n");
  print_corner(stdout, rep.corner_inv, rep.nm);
  if (rep.residual_computed)
    std::printf("residual: %e\n", rep.residual);
  else if (cfg.residual == ResidualMode::Compat)
    std::printf("p == 1!\n");
  if (rep.rhs_solved) {  // only with --rhs: the reference has no A x = b mode
    std::printf("solution x:\n");
    for (double v : rep.x_head) std::printf("%.2f\t", v);
    std::printf("\nAx-b residual: %e\n", rep.rhs_residual);
  }
  if (!out_file.empty()) write_matrix_file(out_file, n, rep.inverse.data(), n);
  if (!x_file.empty()) write_vector_file(x_file, n, rep.x.data());
  if (json) json_report(cfg, rep);
  int rc = 0;
  if (cfg.race_check) {
    for (const auto& r : rep.races) std::fprintf(stderr, "race: %s\n", r.c_str());
    std::fprintf(stderr, "race check: %lld unordered conflicting accesses in %lld ops\n",
                 (long long)rep.race_count, (long long)rep.race_ops);
    if (rep.race_count > 0) rc = 2;
  }
  if (check_tol >= 0.0) {
    if (!rep.residual_computed) {
      std::fprintf(stderr, "residual check: no residual computed (--residual never / compat at p == 1)\n");
      rc = 2;
    } else if (!std::isfinite(rep.residual) || rep.residual > check_tol) {
      std::fprintf(stderr, "residual check failed: residual %e exceeds %e\n", rep.residual, check_tol);
      rc = 2;
    }
  }
  return rc;
}
