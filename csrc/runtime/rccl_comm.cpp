// RcclComm: RCCL over xGMI (replaces the reference's MPI layer).
//
//   M9  MPI_Allreduce(PivotMin, user op)  -> ncclAllGather of 32-B records (SIDE communicator)
//   M10 MPI_Bcast(pivot row)              -> ncclBroadcast per column chunk and pivot row (COMM
//                                            communicator), pipelined behind the trailing update;
//                                            independent ones are issued as one group (bcast_many);
//                                            or, when Comm::tune_bcast measured it faster, the
//                                            direct scatter + slice exchange (runtime/comm.cpp)
//   M11 MPI_Send/Recv row swap            -> no per-step traffic; one grouped ncclSend/ncclRecv
//                                            exchange at the end (finalize)
//   M14 MPI_Sendrecv_replace ring (residual) -> ncclAllGather of the inverse strips
//   M6/M7/M13/M15 scalar allreduces       -> host_max() over a tiny device buffer
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "gj/comms.hpp"

namespace gj {

#define NCCL_OK(expr)                                                                        \
  do {                                                                                       \
    ncclResult_t r_ = (expr);                                                                \
    if (r_ != ncclSuccess)                                                                   \
      throw Error(Status::CommError, std::string("RCCL error: ") + ncclGetErrorString(r_) +  \
                                         " at " + __FILE__ + ":" + std::to_string(__LINE__)); \
  } while (0)

static_assert(sizeof(ncclUniqueId) == RcclComm::kIdBytes, "unexpected ncclUniqueId size");

std::string RcclComm::unique_id() {
  ncclUniqueId id;
  NCCL_OK(ncclGetUniqueId(&id));
  return std::string(reinterpret_cast<const char*>(&id), sizeof(id));
}

RcclComm::RcclComm(const std::vector<std::string>& ids, int nranks, int rank, int device, bool one_comm)
    : n_(nranks), r_(rank), device_(device), one_comm_(one_comm) {
  GJ_REQUIRE(ids.size() == 2, "RcclComm needs two unique ids");
  if (nranks > 1 && !one_comm_) {
    // Two concurrently active communicators need their own hardware queues (README "Progress of
    // the two communicators"): on a shared queue a SIDE kernel spinning on a peer can sit in front
    // of the COMM kernel that peer waits for -- a cross-rank deadlock that only surfaces as a comm
    // timeout.  The launchers agree on the count HIP really runs with and pass one_comm below 16
    // (parallel/dist.py agree_comm_mode, cli/main.cpp); an embedder that constructs this directly
    // with fewer queues is refused unless it opts in with GJ_ALLOW_SHARED_QUEUES=1.
    const char* q = std::getenv("GPU_MAX_HW_QUEUES");
    const char* allow = std::getenv("GJ_ALLOW_SHARED_QUEUES");
    if ((!q || std::atoi(q) < kMinHwQueues) && !(allow && std::atoi(allow) != 0))
      throw Error(Status::BadArgs,
                  std::string("two RCCL communicators need GPU_MAX_HW_QUEUES >= ") + std::to_string(kMinHwQueues) +
                      " (have " + (q ? q : "unset") + "): pass one_comm (GJ_ONE_COMM=1), raise the queue count "
                      "before the first HIP call, or set GJ_ALLOW_SHARED_QUEUES=1");
  }
  (void)hipSetDevice(device_);
  for (int c = 0; c < (one_comm_ ? 1 : 2); ++c) {
    GJ_REQUIRE(ids[c].size() == sizeof(ncclUniqueId), "bad unique id size");
    ncclUniqueId id;
    std::memcpy(&id, ids[c].data(), sizeof(id));
    ncclComm_t comm;
    NCCL_OK(ncclCommInitRank(&comm, nranks, id, rank));
    comms_[c] = comm;
  }
  dbuf_sz_ = 64 * 1024;
  if (hipMalloc(&dbuf_, dbuf_sz_) != hipSuccess) throw Error(Status::NoMemory, "RcclComm scratch");
}

RcclComm::~RcclComm() {
  (void)hipSetDevice(device_);
  for (void* c : comms_)
    if (c) ncclCommDestroy(static_cast<ncclComm_t>(c));
  if (dbuf_) (void)hipFree(dbuf_);
}

std::string RcclComm::describe() const {
  int v = 0;
  ncclGetVersion(&v);
  return "rccl(v" + std::to_string(v) + ", " + std::to_string(n_) + " ranks" +
         (one_comm_ ? ", one communicator)" : ")");
}

void* RcclComm::comm_for(int s) const {
  GJ_REQUIRE(s == S_SIDE || s == S_COMM, "RCCL collectives are only issued on SIDE/COMM streams");
  return comms_[(s == S_SIDE || one_comm_) ? 0 : 1];
}

static inline hipStream_t st(Device& dev, int s) { return static_cast<hipStream_t>(dev.native_stream(s)); }

void RcclComm::allgather(Device& dev, const void* send, void* recv, size_t bytes, int s) {
  note(s, "ncclAllGather", bytes);
  NCCL_OK(ncclAllGather(send, recv, bytes, ncclUint8, static_cast<ncclComm_t>(comm_for(s)), st(dev, s)));
}

void RcclComm::bcast(Device& dev, void* buf, size_t bytes, int root, int s) {
  if (n_ == 1) return;
  if (use_direct(bytes)) return bcast_direct(dev, {BcastOp{buf, bytes, root}}, s);
  note(s, "ncclBroadcast", bytes, root);
  NCCL_OK(ncclBroadcast(buf, buf, bytes, ncclUint8, root, static_cast<ncclComm_t>(comm_for(s)), st(dev, s)));
}

void RcclComm::bcast_many(Device& dev, const std::vector<BcastOp>& ops, int s) {
  if (n_ == 1 || ops.empty()) return;
  ncclComm_t c = static_cast<ncclComm_t>(comm_for(s));
  std::vector<BcastOp> big;
  size_t tot = 0;
  for (const auto& o : ops) tot += o.bytes;
  note(s, ops.size() == 1 ? "ncclBroadcast" : "grouped ncclBroadcast", tot, ops.front().root);
  NCCL_OK(ncclGroupStart());
  for (const auto& o : ops)
    if (use_direct(o.bytes)) big.push_back(o);
    else NCCL_OK(ncclBroadcast(o.buf, o.buf, o.bytes, ncclUint8, o.root, c, st(dev, s)));
  NCCL_OK(ncclGroupEnd());
  bcast_direct(dev, big, s);
}

void RcclComm::allreduce_max(Device& dev, double* buf, size_t count, int s) {
  note(s, "ncclAllReduce(max)", count * sizeof(double));
  NCCL_OK(ncclAllReduce(buf, buf, count, ncclFloat64, ncclMax, static_cast<ncclComm_t>(comm_for(s)), st(dev, s)));
}

void RcclComm::allreduce_sum(Device& dev, void* buf, size_t count, DType dt, int s) {
  if (n_ == 1 || count == 0) return;
  note(s, "ncclAllReduce(sum)", count * dtype_size(dt));
  NCCL_OK(ncclAllReduce(buf, buf, count, dt == DType::F64 ? ncclFloat64 : ncclFloat32, ncclSum,
                        static_cast<ncclComm_t>(comm_for(s)), st(dev, s)));
}

void RcclComm::group_p2p(Device& dev, const std::vector<P2POp>& ops, int s) {
  if (ops.empty()) return;
  ncclComm_t c = static_cast<ncclComm_t>(comm_for(s));
  size_t tot = 0;
  for (const auto& op : ops) tot += op.bytes;
  note(s, "grouped ncclSend/ncclRecv", tot);
  NCCL_OK(ncclGroupStart());
  for (const auto& op : ops) {
    if (op.send)
      NCCL_OK(ncclSend(op.ptr, op.bytes, ncclUint8, op.peer, c, st(dev, s)));
    else
      NCCL_OK(ncclRecv(op.ptr, op.bytes, ncclUint8, op.peer, c, st(dev, s)));
  }
  NCCL_OK(ncclGroupEnd());
}

void RcclComm::check_health() {
  for (void* c : comms_) {
    if (!c) continue;
    ncclResult_t st = ncclSuccess;
    NCCL_OK(ncclCommGetAsyncError(static_cast<ncclComm_t>(c), &st));
    if (st != ncclSuccess && st != ncclInProgress)
      throw Error(Status::CommError, std::string("RCCL asynchronous error: ") + ncclGetErrorString(st));
  }
}

void RcclComm::abort() {
  (void)hipSetDevice(device_);
  for (void*& c : comms_)
    if (c) {
      ncclCommAbort(static_cast<ncclComm_t>(c));
      c = nullptr;
    }
}

void RcclComm::barrier(Device& dev) {
  drain_all(dev);
  double v = 0.0;
  host_max(dev, v);
}

double RcclComm::host_max(Device& dev, double v) {
  (void)hipSetDevice(device_);
  drain(dev, S_SIDE);
  double* d = static_cast<double*>(dbuf_);
  dev.copy(d, &v, sizeof(double), S_SIDE);
  allreduce_max(dev, d, 1, S_SIDE);
  double out = 0;
  dev.copy(&out, d, sizeof(double), S_SIDE);
  drain(dev, S_SIDE);
  return out;
}

void RcclComm::host_allgather(Device& dev, const void* send, void* recv, size_t bytes) {
  (void)hipSetDevice(device_);
  const size_t need = bytes * (n_ + 1);
  void* tmp = dbuf_;
  bool owned = false;
  if (need > dbuf_sz_) {
    if (hipMalloc(&tmp, need) != hipSuccess) throw Error(Status::NoMemory, "host_allgather");
    owned = true;
  }
  char* d = static_cast<char*>(tmp);
  drain(dev, S_SIDE);
  dev.copy(d, send, bytes, S_SIDE);
  allgather(dev, d, d + bytes, bytes, S_SIDE);
  dev.copy(recv, d + bytes, bytes * n_, S_SIDE);
  drain(dev, S_SIDE);
  if (owned) (void)hipFree(tmp);
}

}  // namespace gj
