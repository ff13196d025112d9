// Common definitions for the MI355X-native Gauss-Jordan framework.
//
// Replaces the reference's compile-time configuration block (main.cpp:6-8: MAX_P, EPS, SLEEP)
// with typed constants plus runtime options, and adds the error/status machinery the reference
// expresses through bare integer return codes (main.cpp:87-92, :343-519).
#pragma once

#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <string>

#if defined(__HIPCC__)
#define GJ_HD __host__ __device__
#else
#define GJ_HD
#endif

namespace gj {

// Reference defaults (main.cpp:6-7).
constexpr int kDefaultPrintMax = 10;      // MAX_P: size of the printed corner
constexpr double kDefaultEps = 1e-15;     // EPS: singularity threshold (relative to ||A||_inf)

enum class DType : int { F64 = 0, F32 = 1 };

inline size_t dtype_size(DType t) { return t == DType::F64 ? 8 : 4; }
inline const char* dtype_name(DType t) { return t == DType::F64 ? "fp64" : "fp32"; }

// Status codes agreed collectively by all ranks (the reference's -1/-2 returns of Jordan,
// main.cpp:428-449, and read_matrix, main.cpp:385-397).
enum class Status : int {
  Ok = 0,
  Singular = 1,        // "singular matrix"
  NoMemory = 2,        // "Not enough memory!" (the matrix itself does not fit, main.cpp:366-381)
  CannotOpen = 3,      // "cannot open %s"
  CannotRead = 4,      // "cannot read %s"
  BadArgs = 5,
  CommError = 6,
  NoBlockMemory = 7,   // "not enough memory for block" (the elimination work space, main.cpp:428-436)
  VerifyFailed = 8,    // GJ_VERIFY: a rank consumed a broadcast buffer whose bytes differ from the root's
};

class Error : public std::runtime_error {
 public:
  Error(Status s, const std::string& msg) : std::runtime_error(msg), status_(s) {}
  Status status() const { return status_; }

 private:
  Status status_;
};

[[noreturn]] void fail(const char* file, int line, const std::string& msg);

#define GJ_REQUIRE(cond, msg)                                   \
  do {                                                          \
    if (!(cond)) ::gj::fail(__FILE__, __LINE__, (msg));         \
  } while (0)

// Stream roles.  MAIN runs the trailing (eliminate) update; SIDE runs the latency-critical
// look-ahead work (pivot search + pivot-record exchange); COMM runs pivot-row normalisation and the
// pivot-row broadcast.  Each RCCL communicator is bound to exactly one stream role.
// Hardware queues per process the engine needs (GPU_MAX_HW_QUEUES): one per stream, so that the
// SIDE and COMM communicators' RCCL kernels never wait behind each other in one in-order queue.
constexpr int kMinHwQueues = 16;

enum StreamRole : int { S_MAIN = 0, S_SIDE = 1, S_COMM = 2, kNumStreams = 3 };

}  // namespace gj
