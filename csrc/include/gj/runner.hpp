// In-process driver: one host thread per rank (GPU or virtual host rank), the reference's solve()
// flow (main.cpp:343-519): allocate -> read/generate A -> print A -> time the inversion -> print
// inverse -> recompute A -> residual.  Shared by the `gj` CLI and the Python bindings.
#pragma once

#include <string>
#include <vector>

#include "gj/engine.hpp"

namespace gj {

enum class ResidualMode : int { Never = 0, Always = 1, Compat = 2 };

struct RunConfig {
  int64_t n = 0, m = 0;
  int ranks = 1;
  bool gpu = true;
  std::string comm = "auto";        // auto | rccl | loopback | async (stream-ordered virtual ranks)
  bool one_comm = false;            // rccl: SIDE and COMM share one communicator (RcclComm, GJ_ONE_COMM)
  double jitter_us = 0.0;           // async: random per-rank arrival delay (tests)
  int first_device = 0;
  GenSpec gen;
  std::string file;                 // input file (text or .bin); empty => generator
  const double* input = nullptr;    // or a caller-owned n x n row-major matrix
  SolveOptions solve;
  ResidualMode residual = ResidualMode::Always;
  int print_max = kDefaultPrintMax;
  bool want_corners = true;
  bool keep_inverse = false;        // gather the full inverse into RunReport::inverse
  int host_threads = 0;
  int repeats = 1;                  // timed solves (the last one is reported; min kept too)
  // A x = b after the inversion: "" (off), "ones", "random" (seeded by gen.seed), or a file of n
  // numbers (text / .bin).  x = inv(A) b, then ||A x - b||_inf.
  std::string rhs;
  const double* rhs_input = nullptr;  // or a caller-owned n-vector
  bool keep_solution = false;         // return x in RunReport::x
  // iterative refinement of x with the residual in fp64 (Engine::solve_rhs): at most `refine`
  // steps (-1 = auto: 10 for fp32 solves, 2 for fp64), stop at backward error <= refine_tol
  int refine = -1;
  double refine_tol = 1e-15;
  // Run every rank's device under the happens-before schedule checker (RaceCheckDevice, one
  // checker shared by the rank threads); reports land in RunReport::races.
  bool race_check = false;
};

struct RunReport {
  Status status = Status::Ok;
  std::string message;
  double glob_time = 0;             // max over ranks (reference glob_time, main.cpp:455-458)
  double best_time = 0;             // min over repeats of glob_time
  bool residual_computed = false;
  double residual = 0;
  int nm = 0;
  std::vector<double> corner_a, corner_inv;
  std::vector<double> inverse;      // n*n if keep_inverse
  SolveStats stats;                 // rank 0
  std::string device_desc, comm_desc;
  double gflops_nominal = 0;        // 2 n^3 / glob_time / 1e9
  bool rhs_solved = false;
  double rhs_residual = 0;          // ||A x - b||_inf (fp64)
  std::vector<double> rhs_history;  // ||A x_k - b|| / ||b|| per refinement step (k = 0: x = inv(A) b)
  int rhs_steps = 0;
  bool rhs_converged = false;
  double rhs_backward_error = 0;
  bool residual_fp64 = true;        // precision of `residual` (fp32 solves: fp64 when it fits)
  double rhs_seconds = 0;           // x = inv(A) b (GEMV + all-gather), max over ranks
  std::vector<double> x_head;       // first min(n, print_max) entries of x
  std::vector<double> x;            // n entries if keep_solution
  // race_check: unordered conflicting accesses found (total, the first distinct ones described),
  // ops checked
  int64_t race_count = 0;
  std::vector<std::string> races;
  int64_t race_ops = 0;
};

RunReport run_local(const RunConfig& cfg);

}  // namespace gj
