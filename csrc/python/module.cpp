// Python bindings (pybind11) of the native framework: devices, communicators, the engine and the
// in-process runner.  The module is built in-tree as mpi_jordan_crazy_acceleration_amd/_C*.so and
// shares the HIP runtime / RCCL already loaded by torch (the package imports torch first).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>

#include <thread>
#include <pybind11/stl.h>

#include <hip/hip_runtime.h>

#include <cstring>
#include <memory>
#include <tuple>

#include "gj/comms.hpp"
#include "gj/engine.hpp"
#include "gj/hip_device.hpp"
#include "gj/host_device.hpp"
#include "gj/io.hpp"
#include "gj/race_check.hpp"
#include "gj/runner.hpp"
#include "../kernels/kernels.hpp"

namespace py = pybind11;
using namespace gj;

namespace {

DType parse_dtype(const std::string& s) {
  if (s == "fp64" || s == "float64" || s == "f64" || s == "double") return DType::F64;
  if (s == "fp32" || s == "float32" || s == "f32" || s == "float") return DType::F32;
  throw std::invalid_argument("dtype must be fp64 or fp32");
}

GenKind parse_gen(const std::string& s) {
  if (s == "absdiff") return GenKind::AbsDiff;
  if (s == "hilbert") return GenKind::Hilbert;
  if (s == "identity") return GenKind::Identity;
  if (s == "random") return GenKind::Random;
  if (s == "randshift") return GenKind::RandomShifted;
  if (s == "zero") return GenKind::Zero;
  throw std::invalid_argument("unknown generator " + s);
}

// Communicator implemented in Python (torch.distributed, gloo) — host memory only.
class PyComm : public Comm {
 public:
  PyComm(py::object impl, int rank, int size) : impl_(std::move(impl)), r_(rank), n_(size) {}
  int size() const override { return n_; }
  int rank() const override { return r_; }
  std::string describe() const override { return "python(" + std::to_string(n_) + ")"; }
  void allgather(Device& dev, const void* send, void* recv, size_t bytes, int s) override {
    check(dev);
    call(s, "allgather", bytes, -1, [&] { impl_.attr("allgather")((uintptr_t)send, (uintptr_t)recv, bytes); });
  }
  void bcast(Device& dev, void* buf, size_t bytes, int root, int s) override {
    check(dev);
    call(s, "broadcast", bytes, root, [&] { impl_.attr("bcast")((uintptr_t)buf, bytes, root); });
  }
  void allreduce_max(Device& dev, double* buf, size_t count, int s) override {
    check(dev);
    call(s, "allreduce(max)", count * 8, -1, [&] { impl_.attr("allreduce_max")((uintptr_t)buf, count); });
  }
  void group_p2p(Device& dev, const std::vector<P2POp>& ops, int s) override {
    check(dev);
    size_t tot = 0;
    for (const auto& op : ops) tot += op.bytes;
    call(s, "grouped send/recv", tot, -1, [&] {
      py::list l;
      for (const auto& op : ops) l.append(py::make_tuple((uintptr_t)op.ptr, op.bytes, op.peer, op.send));
      impl_.attr("group_p2p")(l);
    });
  }
  void barrier(Device&) override {
    call(S_SIDE, "barrier", 0, -1, [&] { impl_.attr("barrier")(); });
  }
  double host_max(Device&, double v) override {
    double out = 0;
    call(S_SIDE, "host max", 8, -1, [&] { out = impl_.attr("host_max")(v).cast<double>(); });
    return out;
  }
  void host_allgather(Device&, const void* send, void* recv, size_t bytes) override {
    call(S_SIDE, "host allgather", bytes, -1,
         [&] { impl_.attr("allgather")((uintptr_t)send, (uintptr_t)recv, bytes); });
  }

 private:
  static void check(Device& dev) {
    if (dev.on_gpu()) throw std::runtime_error("PyComm works on host memory only (use RcclComm on GPUs)");
  }
  // A Python-side failure (gloo timeout, a peer that closed its connection) becomes a
  // communication error of the engine, converted while the GIL is held, naming the collective.
  template <class F>
  void call(int s, const char* kind, size_t bytes, int root, F&& f) {
    note(s, kind, bytes, root);
    py::gil_scoped_acquire g;
    try {
      f();
    } catch (py::error_already_set& e) {
      const std::string msg = e.what();
      throw Error(Status::CommError, "torch.distributed failed in the " + last_op(s) + ": " + msg);
    }
  }
  py::object impl_;
  int r_, n_;
};

PivotRule parse_pivot(const std::string& v) {
  if (v == "block-min-inv-norm" || v == "min-inv-norm") return PivotRule::MinInvNorm;
  if (v == "partial") return PivotRule::Partial;
  throw std::invalid_argument("pivot: block-min-inv-norm | partial");
}

py::dict stats_to_dict(const SolveStats& st) {
  py::dict d;
  d["status"] = (int)st.status;
  d["singular_step"] = st.singular_step;
  d["seconds"] = st.seconds;
  d["host_wait_ms"] = st.host_wait_ms;
  d["pivots"] = st.pivots;
  d["offdiag_pivots"] = st.offdiag_pivots;
  d["pivot_fallbacks"] = st.pivot_fallbacks;
  d["bcast_bytes"] = st.bcast_bytes;
  {
    static const char* kinds[SolveStats::kNumCommKinds] = {"pivot_rows", "panel_pieces", "pivot_records"};
    py::dict cb;
    for (int k = 0; k < SolveStats::kNumCommKinds; ++k) {
      py::dict e;
      e["bytes"] = st.comm_bytes[k];
      e["calls"] = st.comm_calls[k];
      cb[kinds[k]] = e;
    }
    d["comm_bytes"] = cb;
  }
  if (st.profiled) {
    py::dict ph;
    for (int i = 0; i < kNumPhases; ++i) {
      py::dict e;
      e["ms"] = st.phase_ms[i];
      e["calls"] = st.phase_calls[i];
      ph[phase_name(i)] = e;
    }
    d["phases"] = ph;
  }
  return d;
}

py::array_t<double> to_array(const std::vector<double>& v, int64_t r, int64_t c) {
  py::array_t<double> a({r, c});
  if (!v.empty()) std::memcpy(a.mutable_data(), v.data(), sizeof(double) * r * c);
  return a;
}

}  // namespace

PYBIND11_MODULE(_C, mod) {
  mod.doc() = "MI355X-native block Gauss-Jordan inversion: native engine, HIP kernels, RCCL comm";

  // gj::Error -> GJError (a RuntimeError) carrying the engine status (2 = no memory for the matrix,
  // 6 = communication failure, 7 = no memory for the work space, ...).
  static py::object gj_error = py::reinterpret_steal<py::object>(
      PyErr_NewException("mpi_jordan_crazy_acceleration_amd._C.GJError", PyExc_RuntimeError, nullptr));
  mod.attr("GJError") = gj_error;
  py::register_exception_translator([](std::exception_ptr p) {
    try {
      if (p) std::rethrow_exception(p);
    } catch (const Error& e) {
      py::object inst = gj_error(e.what());
      inst.attr("status") = (int)e.status();
      PyErr_SetObject(gj_error.ptr(), inst.ptr());
    }
  });

  mod.def("version", [] { return std::string("0.1.0"); });
  mod.def("device_count", [] {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
  });
  mod.def("rccl_unique_id", [] { return py::bytes(RcclComm::unique_id()); });
  mod.def("set_block_inverse_variant", [](const std::string& v) {
    kern::set_block_inverse_variant(kern::block_inverse_variant_id(v.c_str()));
  });
  mod.def("set_block_inverse_probe", [](uintptr_t p) { kern::set_block_inverse_probe(reinterpret_cast<int32_t*>(p)); },
          "test probe: device int32 buffer (nblk x m) receiving each candidate's pivot row per column; 0 = off");
  mod.def("set_gemm_variant", [](const std::string& v) { kern::set_gemm_variant(kern::gemm_variant_id(v.c_str())); });
  mod.def("set_glds_peel", [](bool on) { kern::set_glds_peel(on ? 1 : 0); },
          "fp64 LDS-DMA trailing-update kernel: the peeled, stage-unrolled main loop (GJ_GLDS_PEEL)");
  mod.def("set_glds_covl", [](bool on) { kern::set_glds_covl(on ? 1 : 0); },
          "fp64 LDS-DMA kernel: C loads overlapped with the first K slices (GJ_GLDS_COVL)");
  mod.def("set_glds_build", [](int b) { kern::set_glds_build(b); },
          "fp64 LDS-DMA trailing-update build for every launch: 23 | 25 | 33 | 43 | 1623, 0 = auto (GJ_GLDS_BUILD)");
  mod.def("set_glds_tile", [](int bn) { kern::set_glds_tile(bn); },
          "fp64 LDS-DMA trailing-update tile width for the 4-per-CU builds: 64 | 128 for every launch, 0 = per "
          "launch (the engine's choice; GJ_GLDS_TILE)");
  mod.def("set_lat_kernel", [](int mode) { kern::set_lat_kernel(mode); },
          "fp64 latency GEMMs on the register-fed small kernel: 1 / 0 for every launch, -1 per launch "
          "(GemmExtra::lat_reg; GJ_LAT_KERNEL)");
  mod.def("set_lat_glds", [](bool on) { kern::set_lat_glds(on ? 1 : 0); },
          "every latency GEMM of >= 1024 rows on the LDS-DMA kernel (tests; the engine sets it per launch)");

  // Kernel-level entry points (raw pointers; used by the per-kernel numerics tests and
  // mpi_jordan_crazy_acceleration_amd.ops).  Every op runs on the MAIN stream and is waited for.
  using U = uintptr_t;
  auto lay = [](int64_t n, int64_t m, int64_t p, int64_t k) { return Layout::make(n, m, p, k); };
  py::class_<Device, std::shared_ptr<Device>>(mod, "Device")
      .def_property_readonly("on_gpu", &Device::on_gpu)
      .def("describe", &Device::describe)
      .def("sync", &Device::sync_all, py::call_guard<py::gil_scoped_release>())
      .def("gemm",
           [](Device& d, const std::string& dt, const std::string& op, bool a_kmajor, int64_t M,
              int64_t N, int64_t K, U A, int64_t lda, U B, int64_t ldb, U C, int64_t ldc, int64_t zc0,
              int64_t zc1, std::vector<int64_t> zero_rows, int64_t zh, U tneg, int64_t ldtneg, bool latency,
              int64_t tneg_cols, bool dense, U c_in, int64_t ldc_in, std::vector<int64_t> row_blocks,
              int64_t row_block_m, int64_t skip_c0, int64_t skip_c1) {
             GemmExtra ex;
             ex.dense = dense;
             ex.skip_c0 = skip_c0;
             ex.skip_c1 = skip_c1;
             ex.c_in = (const void*)c_in;
             ex.ldc_in = ldc_in;
             if (row_block_m > 0) {  // GemmExtra::rsel from a list of selected row blocks
               ex.rsel_m = row_block_m;
               for (int64_t b : row_blocks) {
                 if (b < 0 || b >= 64 * GemmExtra::kRselWords) throw std::invalid_argument("row block out of range");
                 ex.rsel[b / 64] |= uint64_t(1) << (b % 64);
               }
               if (M != ex.rsel_count() * row_block_m) throw std::invalid_argument("M != selected rows");
             }
             ex.tneg = (void*)tneg;
             ex.ldtneg = ldtneg;
             ex.tneg_cols = tneg_cols;
             ex.latency = latency;
             ex.zc0 = zc0;
             ex.zc1 = zc1;
             if (zero_rows.size() > (size_t)GemmExtra::kMaxZeroRows) throw std::invalid_argument("too many zero rows");
             ex.nzr = (int)zero_rows.size();
             for (size_t i = 0; i < zero_rows.size(); ++i) ex.zr[i] = zero_rows[i];
             ex.zh = zh;
             d.gemm(parse_dtype(dt), op == "store" ? GemmOp::Store : GemmOp::Acc,
                    a_kmajor ? ALayout::KMajor : ALayout::RowMajor, M, N, K, (const void*)A, lda,
                    (const void*)B, ldb, (void*)C, ldc, S_MAIN, ex);
             d.sync_stream(S_MAIN);
           },
           py::arg("dtype"), py::arg("op"), py::arg("a_kmajor"), py::arg("M"), py::arg("N"), py::arg("K"),
           py::arg("A"), py::arg("lda"), py::arg("B"), py::arg("ldb"), py::arg("C"), py::arg("ldc"),
           py::arg("zc0") = 0, py::arg("zc1") = 0, py::arg("zero_rows") = std::vector<int64_t>(),
           py::arg("zh") = 0, py::arg("tneg") = U(0), py::arg("ldtneg") = 0, py::arg("latency") = false,
           py::arg("tneg_cols") = 0, py::arg("dense") = false, py::arg("c_in") = U(0), py::arg("ldc_in") = 0,
           py::arg("row_blocks") = std::vector<int64_t>(), py::arg("row_block_m") = 0, py::arg("skip_c0") = 0,
           py::arg("skip_c1") = 0)
      .def("gemm_batch",
           [](Device& d, const std::string& dt,
              const std::vector<std::tuple<std::string, int64_t, int64_t, int64_t, U, int64_t, U, int64_t,
                                           U, int64_t>>& ps) {
             std::vector<GemmDesc> v(ps.size());
             for (size_t i = 0; i < ps.size(); ++i) {
               const auto& t = ps[i];
               GemmDesc& g = v[i];
               g.op = std::get<0>(t) == "store" ? GemmOp::Store : GemmOp::Acc;
               g.M = std::get<1>(t); g.N = std::get<2>(t); g.K = std::get<3>(t);
               g.A = (const void*)std::get<4>(t); g.lda = std::get<5>(t);
               g.B = (const void*)std::get<6>(t); g.ldb = std::get<7>(t);
               g.C = (void*)std::get<8>(t); g.ldc = std::get<9>(t);
             }
             d.gemm_batch(parse_dtype(dt), v.data(), (int)v.size(), S_MAIN);
             d.sync_stream(S_MAIN);
           },
           py::arg("dtype"), py::arg("products"))
      .def("generate",
           [lay](Device& d, const std::string& dt, U X, int64_t n, int64_t m, int64_t p, int64_t k,
                 const std::string& kind, uint64_t seed) {
             GenSpec g;
             g.kind = parse_gen(kind);
             g.seed = seed;
             d.generate(parse_dtype(dt), (void*)X, lay(n, m, p, k), g, S_MAIN);
             d.sync_stream(S_MAIN);
           })
      .def("extract_neg_t",
           [](Device& d, const std::string& dt, U Lt, int64_t ldl, U X, int64_t ldx, int64_t rows,
              int64_t col0, int64_t m) {
             d.extract_neg_t(parse_dtype(dt), (void*)Lt, ldl, (const void*)X, ldx, rows, col0, m, S_MAIN);
             d.sync_stream(S_MAIN);
           })
      .def("block_inverse",
           [lay](Device& d, const std::string& dt, U Lt, int64_t ldl, U inv_t, U scores, U valid,
                 U used, int64_t n, int64_t m, int64_t p, int64_t k, double thresh, int64_t nlive) {
             d.block_inverse(parse_dtype(dt), (const void*)Lt, ldl, (void*)inv_t, (double*)scores,
                             (int32_t*)valid, (const int32_t*)used, lay(n, m, p, k), thresh, nlive, S_MAIN);
             d.sync_stream(S_MAIN);
           },
           py::arg("dt"), py::arg("Lt"), py::arg("ldl"), py::arg("inv_t"), py::arg("scores"), py::arg("valid"),
           py::arg("used"), py::arg("n"), py::arg("m"), py::arg("p"), py::arg("k"), py::arg("thresh"),
           py::arg("nlive") = -1)
      // pivot selection kernels (tests): local argmin of one rank's candidates -> 32-B record at rec
      .def("pivot_local",
           [lay](Device& d, U scores, U valid, U used, U pos, int64_t n, int64_t m, int64_t p, int64_t k, U rec) {
             d.pivot_local((const double*)scores, (const int32_t*)valid, (const int32_t*)used,
                           (const int32_t*)pos, lay(n, m, p, k), (PivotRec*)rec, S_MAIN);
             d.sync_stream(S_MAIN);
           })
      // one rank: argmin + book-keeping (pos / phys_at / used / seq) + result record, one launch
      .def("pivot_select_single",
           [lay](Device& d, U scores, U valid, int64_t n, int64_t m, int t, U pos, U phys_at, U used, U seq,
                 U rec, U out) {
             d.pivot_select_single((const double*)scores, (const int32_t*)valid, lay(n, m, 1, 0), (int32_t)t,
                                   (int32_t*)pos, (int32_t*)phys_at, (int32_t*)used, (int32_t*)seq,
                                   (PivotRec*)rec, (PivotResult*)out, nullptr, S_MAIN);
             d.sync_stream(S_MAIN);
           })
      // p ranks' gathered records -> winner, book-keeping, *out and the pinned host mirror (returned
      // as (step, found, phys, owner, logical, score), read after the stream completes)
      .def("pivot_global",
           [](Device& d, U recs, int p, int t, U pos, U phys_at, U used, U seq, U out) {
             auto* h = static_cast<PivotResult*>(d.alloc_pinned_coherent(sizeof(PivotResult)));
             h->step = -1;
             d.pivot_global((const PivotRec*)recs, (int32_t)p, (int32_t)t, (int32_t*)pos, (int32_t*)phys_at,
                            (int32_t*)used, (int32_t*)seq, (PivotResult*)out, h, S_MAIN);
             d.sync_stream(S_MAIN);
             py::tuple r = py::make_tuple(h->step, h->found, h->phys, h->owner, h->logical, h->score);
             d.release_pinned(h);
             return r;
           })
      // Device-side latency of the batched block inverse: `reps` back-to-back launches on one
      // stream between two timing events (no host work in between); returns microseconds per call.
      .def("time_block_inverse",
           [lay](Device& d, const std::string& dt, U Lt, int64_t ldl, U inv_t, U scores, U valid,
                 U used, int64_t n, int64_t m, int64_t p, int64_t k, double thresh, int reps, int64_t nlive) {
             py::gil_scoped_release rel;
             const Layout L = lay(n, m, p, k);
             const DType t = parse_dtype(dt);
             d.block_inverse(t, (const void*)Lt, ldl, (void*)inv_t, (double*)scores, (int32_t*)valid,
                             (const int32_t*)used, L, thresh, nlive, S_SIDE);
             const int e0 = d.create_event(true), e1 = d.create_event(true);
             d.record(e0, S_SIDE);
             for (int i = 0; i < reps; ++i)
               d.block_inverse(t, (const void*)Lt, ldl, (void*)inv_t, (double*)scores, (int32_t*)valid,
                               (const int32_t*)used, L, thresh, nlive, S_SIDE);
             d.record(e1, S_SIDE);
             d.sync_stream(S_SIDE);
             return 1e3 * d.event_ms(e0, e1) / std::max(reps, 1);
           },
           py::arg("dt"), py::arg("Lt"), py::arg("ldl"), py::arg("inv_t"), py::arg("scores"), py::arg("valid"),
           py::arg("used"), py::arg("n"), py::arg("m"), py::arg("p"), py::arg("k"), py::arg("thresh"),
           py::arg("reps"), py::arg("nlive") = -1)
      .def("permute_blocks",
           [](Device& d, const std::string& dt, U dst, int64_t ldd, U X, int64_t ldx, int64_t nblk,
              int64_t m, int64_t Nr, U dst_blk, U colsrc) {
             d.permute_blocks(parse_dtype(dt), (void*)dst, ldd, (const void*)X, ldx, nblk, m, Nr,
                              (const int32_t*)dst_blk, (const int32_t*)colsrc, S_MAIN);
             d.sync_stream(S_MAIN);
           })
      .def("row_abs_max",
           [lay](Device& d, const std::string& dt, U X, int64_t ldx, int64_t n, int64_t m, int64_t p,
                 int64_t k, U out) {
             d.row_abs_max(parse_dtype(dt), (const void*)X, ldx, lay(n, m, p, k), (double*)out, S_MAIN);
             d.sync_stream(S_MAIN);
           })
      .def("residual",
           [lay](Device& d, const std::string& dt, U A, U Full, int64_t n, int64_t m, int64_t p,
                 int64_t k, U out) {
             d.residual(parse_dtype(dt), (const void*)A, (const void*)Full, lay(n, m, p, k),
                        (double*)out, S_MAIN);
             d.sync_stream(S_MAIN);
           });
  mod.def("hip_device", [](int idx) { return std::shared_ptr<Device>(new HipDevice(idx)); });
  mod.def("host_device", [](int nthreads) { return std::shared_ptr<Device>(new HostDevice(nthreads)); },
          py::arg("nthreads") = 0);

  py::class_<Comm, std::shared_ptr<Comm>>(mod, "Comm")
      .def_property_readonly("size", &Comm::size)
      .def_property_readonly("rank", &Comm::rank)
      .def("describe", &Comm::describe)
      .def("bcast_report", &Comm::bcast_report)
      .def("tune_bcast",
           [](Comm& c, std::shared_ptr<Device> dev, size_t bytes) {
             py::gil_scoped_release r;
             c.tune_bcast(*dev, bytes);
             return c.bcast_report();
           },
           py::arg("device"), py::arg("bytes"));
  mod.def("self_comm", [] { return std::shared_ptr<Comm>(new SelfComm()); });
  mod.def("rccl_comm",
          [](std::vector<py::bytes> ids, int nranks, int rank, int device, bool one_comm) {
            std::vector<std::string> s;
            for (auto& b : ids) s.push_back(std::string(b));
            py::gil_scoped_release rel;
            return std::shared_ptr<Comm>(new RcclComm(s, nranks, rank, device, one_comm));
          },
          py::arg("ids"), py::arg("nranks"), py::arg("rank"), py::arg("device"), py::arg("one_comm") = false,
          "one_comm: the SIDE and COMM roles share one communicator (every rank must pass the same value; "
          "parallel.dist.agree_comm_mode decides it)");
  mod.def("shadow_comm", [](int p, double bw_gbs, double lat_us, int channels, int lds_kib, bool direct) {
            CostModel cm;
            cm.bw_gbs = bw_gbs;
            cm.lat_us = lat_us;
            cm.channels = channels;
            cm.lds_kib = lds_kib;
            cm.direct = direct;
            return std::shared_ptr<Comm>(new ShadowComm(p, cm));
          },
          py::arg("p"), py::arg("bw_gbs") = 0.0, py::arg("lat_us") = 0.0, py::arg("channels") = 16,
          py::arg("lds_kib") = 20, py::arg("direct") = false,
          "rank 0 of a p-rank job alone on one device (critical-path timing emulation); bw_gbs > 0 "
          "adds the communication-cost model (lat_us + bytes/bw on `channels` spin workgroups)");
  mod.def("shadow_reset", [](std::shared_ptr<Comm> c) {
    auto* sc = dynamic_cast<ShadowComm*>(c.get());
    GJ_REQUIRE(sc != nullptr, "shadow_reset: not a shadow communicator");
    sc->reset();
  });
  // One broadcast of `bytes` from `root` through a shadow communicator on the host (cost accounting
  // only: tests of the per-link model).
  mod.def("shadow_bcast_probe", [](std::shared_ptr<Comm> c, size_t bytes, int root) {
    auto* sc = dynamic_cast<ShadowComm*>(c.get());
    GJ_REQUIRE(sc != nullptr, "shadow_bcast_probe: not a shadow communicator");
    HostDevice dev(1);
    std::vector<char> buf(bytes);
    sc->bcast(dev, buf.data(), bytes, root, S_COMM);
  });
  mod.def("shadow_modelled_us", [](std::shared_ptr<Comm> c) {
    auto* sc = dynamic_cast<ShadowComm*>(c.get());
    GJ_REQUIRE(sc != nullptr, "shadow_modelled_us: not a shadow communicator");
    return sc->modelled_us();
  });
  // Two virtual ranks on the host enter collectives with different roots (rank 1 passes root_b):
  // returns the error message the loopback consistency check raised on each rank ("" = none).
  mod.def("loopback_mismatch_probe", [](int root_b) {
    auto hub = std::make_shared<LoopbackHub>(2);
    std::vector<std::string> msg(2);
    std::vector<std::thread> th;
    for (int r = 0; r < 2; ++r)
      th.emplace_back([&, r] {
        HostDevice dev(1);
        LoopbackComm c(hub, r);
        double buf[4] = {double(r), 0, 0, 0};
        try {
          c.bcast(dev, buf, sizeof(buf), r == 1 ? root_b : 0, S_COMM);
        } catch (const std::exception& e) {
          msg[r] = e.what();
        }
      });
    for (auto& t : th) t.join();
    return msg;
  });
  mod.def("py_comm", [](py::object impl, int rank, int size) {
    return std::shared_ptr<Comm>(new PyComm(std::move(impl), rank, size));
  });

  // Engine keeps its device and communicator alive.
  struct PyEngine {
    std::shared_ptr<Device> dev;
    std::shared_ptr<Comm> comm;
    std::unique_ptr<Engine> eng;
  };
  py::class_<PyEngine>(mod, "Engine")
      .def(py::init([](std::shared_ptr<Device> dev, std::shared_ptr<Comm> comm, int64_t n, int64_t m,
                       const std::string& dtype, int64_t chunk_cols, double eps, bool sync_debug,
                       int depth, bool profile, double comm_timeout_s, const std::string& pivot,
                       double pivot_growth) {
             SolveOptions o;
             o.pivot_growth = pivot_growth;
             o.dtype = parse_dtype(dtype);
             o.depth = depth;
             o.pivot = parse_pivot(pivot);
             o.profile = profile;
             o.comm_timeout_s = comm_timeout_s;
             o.chunk_cols = chunk_cols;
             o.eps = eps;
             o.sync_debug = sync_debug;
             auto* pe = new PyEngine();
             pe->dev = dev;
             pe->comm = comm;
             pe->eng.reset(new Engine(*dev, *comm, n, m, o));
             return pe;
           }),
           py::arg("device"), py::arg("comm"), py::arg("n"), py::arg("m"), py::arg("dtype") = "fp64",
           py::arg("chunk_cols") = 0, py::arg("eps") = kDefaultEps, py::arg("sync_debug") = false,
           py::arg("depth") = 0, py::arg("profile") = false, py::arg("comm_timeout_s") = 600.0,
           py::arg("pivot") = "block-min-inv-norm", py::arg("pivot_growth") = -1.0)
      .def_property_readonly("layout",
                             [](PyEngine& e) {
                               const Layout& L = e.eng->layout();
                               py::dict d;
                               d["n"] = L.n; d["m"] = L.m; d["p"] = L.p; d["k"] = L.k;
                               d["Nr"] = L.Nr; d["npad"] = L.npad; d["nblk"] = L.nblk;
                               d["rows"] = L.rows; d["real_rows"] = e.eng->real_local_rows();
                               d["depth"] = e.eng->depth();
                               d["bcast"] = e.eng->bcast_algo();
                               return d;
                             })
      .def_property_readonly("policy",
                             [](PyEngine& e) {
                               const Engine::Policy pl = e.eng->policy();
                               py::dict d;
                               d["depth"] = pl.depth;
                               d["chunk_cols"] = pl.chunk_cols;
                               d["nchunks"] = pl.nchunks;
                               d["reserve_cus"] = pl.reserve_cus;
                               d["block_inverse"] = pl.block_inverse;
                               d["comm_small_tiles"] = pl.comm_small_tiles;
                               d["dense_gemm"] = pl.dense_gemm;
                               d["look_ahead_rows"] = pl.la_side ? "SIDE" : "COMM";
                               d["pivot"] = pl.pivot;
                               if (!pl.fault_injection.empty()) d["fault_injection"] = pl.fault_injection;
                               d["env_overrides"] = pl.env_overrides;
                               d["gemm_tile"] = pl.gemm_tile;
                               d["split"] = pl.split;
                               d["lat_wide"] = pl.lat_wide;
                               d["skip_cols"] = pl.skip_cols;
                               d["lat_reg"] = pl.lat_reg;
                               d["chunk_skip"] = pl.chunk_skip;
                               d["first_depth"] = pl.first_depth;
                               d["main_cnt"] = pl.main_cnt;
                               d["bcast"] = e.eng->bcast_algo();
                               d["bcast_tuning"] = e.comm->bcast_report();
                               d["comm"] = e.comm->describe();
                               return d;
                             })
      .def("generate",
           [](PyEngine& e, const std::string& kind, uint64_t seed) {
             GenSpec g;
             g.kind = parse_gen(kind);
             g.seed = seed;
             py::gil_scoped_release rel;
             e.eng->generate(g);
           },
           py::arg("kind") = "absdiff", py::arg("seed") = 0)
      .def("upload_local_rows",
           [](PyEngine& e, py::array_t<double, py::array::c_style | py::array::forcecast> a) {
             const int64_t real = e.eng->real_local_rows(), n = e.eng->layout().n;
             if (a.ndim() != 2 || a.shape(0) != real || a.shape(1) != n)
               throw std::invalid_argument("expected (real_rows, n) float64 array");
             const double* p = a.data();
             py::gil_scoped_release rel;
             e.eng->upload_local_rows(p, n);
           })
      .def("upload_rows_device",
           [](PyEngine& e, uintptr_t ptr, int64_t ld) {
             if (ld < e.eng->layout().n) throw std::invalid_argument("ld < n");
             py::gil_scoped_release rel;
             e.eng->upload_rows_device(reinterpret_cast<const void*>(ptr), ld);
           },
           py::arg("ptr"), py::arg("ld"))
      .def("download_rows_device",
           [](PyEngine& e, uintptr_t ptr, int64_t ld) {
             if (ld < e.eng->layout().n) throw std::invalid_argument("ld < n");
             py::gil_scoped_release rel;
             e.eng->download_rows_device(reinterpret_cast<void*>(ptr), ld);
           },
           py::arg("ptr"), py::arg("ld"))
      .def("solve_rhs_device",
           [](PyEngine& e, py::array_t<double, py::array::c_style | py::array::forcecast> b, uintptr_t rows,
              int64_t ld, int max_refine, double tol) {
             const int64_t n = e.eng->layout().n;
             if (b.ndim() != 1 || b.shape(0) != n) throw std::invalid_argument("b must be an n-vector");
             if (ld < n) throw std::invalid_argument("ld < n");
             if (max_refine < 0) max_refine = e.eng->options().dtype == DType::F64 ? 2 : 10;
             py::array_t<double> x(n);
             RhsResult rr;
             {
               py::gil_scoped_release rel;
               rr = e.eng->solve_rhs_device(b.data(), x.mutable_data(), reinterpret_cast<const void*>(rows), ld,
                                            max_refine, tol);
             }
             py::dict info;
             info["residual"] = rr.residual;
             info["backward_error"] = rr.backward_error;
             info["history"] = rr.history;
             info["steps"] = rr.steps;
             info["converged"] = rr.converged;
             return py::make_tuple(x, info);
           },
           py::arg("b"), py::arg("rows_f64"), py::arg("ld"), py::arg("max_refine") = -1, py::arg("tol") = 1e-15,
           "A x = b after solve(): x = inv(A) b by the native GEMV, refined in fp64 against this rank's rows "
           "of A given as an fp64 device array (Engine::solve_rhs_device); returns (x, info)")
      .def("solve_rhs_generated",
           [](PyEngine& e, const std::string& kind, uint64_t seed,
              py::array_t<double, py::array::c_style | py::array::forcecast> b, int max_refine, double tol) {
             const int64_t n = e.eng->layout().n;
             if (b.ndim() != 1 || b.shape(0) != n) throw std::invalid_argument("b must be an n-vector");
             if (max_refine < 0) max_refine = e.eng->options().dtype == DType::F64 ? 2 : 10;
             GenSpec g;
             g.kind = parse_gen(kind);
             g.seed = seed;
             py::array_t<double> x(n);
             RhsResult rr;
             {
               py::gil_scoped_release rel;
               rr = e.eng->solve_rhs(b.data(), x.mutable_data(), &g, nullptr, 0, max_refine, tol);
             }
             py::dict info;
             info["residual"] = rr.residual;
             info["backward_error"] = rr.backward_error;
             info["history"] = rr.history;
             info["steps"] = rr.steps;
             info["converged"] = rr.converged;
             return py::make_tuple(x, info);
           },
           py::arg("kind"), py::arg("seed"), py::arg("b"), py::arg("max_refine") = -1, py::arg("tol") = 1e-15,
           "A x = b after solve() of the generated matrix (kind, seed): x = inv(A) b, refined in fp64 against A "
           "regenerated in fp64 (Engine::solve_rhs); returns (x, info) -- BASELINE config 5 as a solve")
      .def("input_panel_ptr", [](PyEngine& e) { return (uintptr_t)e.eng->input_panel(); })
      .def("result_panel_ptr", [](PyEngine& e) { return (uintptr_t)e.eng->result_panel(); })
      .def("norm_inf", [](PyEngine& e) {
        py::gil_scoped_release rel;
        return e.eng->norm_inf();
      })
      .def("input_norm_inf", [](PyEngine& e) { return e.eng->input_norm_inf(); },
           "||A||_inf of the last solve's input")
      .def("result_norm_inf",
           [](PyEngine& e) {
             py::gil_scoped_release rel;
             return e.eng->result_norm_inf();
           },
           "||inv(A)||_inf of the last solve's result (collective)")
      .def("set_profile", [](PyEngine& e, bool on) { e.eng->set_profile(on); },
           "per-phase device timers for the following solves (between solves only)")
      .def("solve", [](PyEngine& e) {
        SolveStats st;
        {
          py::gil_scoped_release rel;
          st = e.eng->solve();
        }
        return stats_to_dict(st);
      })
      .def("download_local_rows", [](PyEngine& e) {
        const int64_t real = e.eng->real_local_rows(), n = e.eng->layout().n;
        py::array_t<double> a({real, n});
        double* p = a.mutable_data();
        {
          py::gil_scoped_release rel;
          e.eng->download_local_rows(p, n);
        }
        return a;
      })
      .def("corner", [](PyEngine& e, int nm, int which) {
        std::vector<double> c;
        {
          py::gil_scoped_release rel;
          c = e.eng->corner(nm, which);
        }
        return to_array(c, nm, nm);
      })
      .def("residual_generated",
           [](PyEngine& e, const std::string& kind, uint64_t seed) {
             GenSpec g;
             g.kind = parse_gen(kind);
             g.seed = seed;
             py::gil_scoped_release rel;
             return e.eng->residual_generated(g);
           },
           py::arg("kind") = "absdiff", py::arg("seed") = 0)
      .def("load_file",
           [](PyEngine& e, const std::string& path, int nthreads) {
             py::gil_scoped_release rel;
             return (int)e.eng->load_file(path, nthreads);
           },
           py::arg("path"), py::arg("nthreads") = 0,
           "collective: this rank's rows of a matrix file; returns 0, 3 (cannot open) or 4 (cannot read)")
      .def("residual_file",
           [](PyEngine& e, const std::string& path, int nthreads) {
             Status s = Status::Ok;
             double r;
             {
               py::gil_scoped_release rel;
               r = e.eng->residual_file(path, nthreads, &s);
             }
             return py::make_tuple((int)s, r);
           },
           py::arg("path"), py::arg("nthreads") = 0)
      .def("residual_rows", [](PyEngine& e, py::array_t<double, py::array::c_style | py::array::forcecast> a) {
        const int64_t real = e.eng->real_local_rows(), n = e.eng->layout().n;
        if (a.ndim() != 2 || a.shape(0) != real || a.shape(1) != n)
          throw std::invalid_argument("expected (real_rows, n) float64 array");
        const double* p = a.data();
        py::gil_scoped_release rel;
        return e.eng->residual_rows(p, n);
      });

  // geometry of the schedule checker (tests): regions as (base, pitch, width, height) in bytes
  auto region = [](py::tuple t) {
    MemRegion r;
    r.base = reinterpret_cast<const char*>((uintptr_t)t[0].cast<int64_t>());
    r.pitch = t[1].cast<int64_t>();
    r.width = t[2].cast<int64_t>();
    r.height = t[3].cast<int64_t>();
    return r;
  };
  mod.def("_regions_overlap", [region](py::tuple a, py::tuple b) { return regions_overlap(region(a), region(b)); });
  mod.def("_region_covers", [region](py::tuple a, py::tuple b) { return region_covers(region(a), region(b)); });

  mod.def("run_local", [](py::dict d) {
    RunConfig c;
    c.n = d["n"].cast<int64_t>();
    c.m = d["m"].cast<int64_t>();
    if (d.contains("ranks")) c.ranks = d["ranks"].cast<int>();
    if (d.contains("device")) c.gpu = d["device"].cast<std::string>() == "gpu";
    if (d.contains("comm")) c.comm = d["comm"].cast<std::string>();
    if (d.contains("jitter_us")) c.jitter_us = d["jitter_us"].cast<double>();
    if (d.contains("gen")) c.gen.kind = parse_gen(d["gen"].cast<std::string>());
    if (d.contains("seed")) c.gen.seed = d["seed"].cast<uint64_t>();
    if (d.contains("file")) c.file = d["file"].cast<std::string>();
    if (d.contains("dtype")) c.solve.dtype = parse_dtype(d["dtype"].cast<std::string>());
    if (d.contains("chunk_cols")) c.solve.chunk_cols = d["chunk_cols"].cast<int64_t>();
    if (d.contains("eps")) c.solve.eps = d["eps"].cast<double>();
    if (d.contains("sync_debug")) c.solve.sync_debug = d["sync_debug"].cast<bool>();
    if (d.contains("verify")) c.solve.verify = d["verify"].cast<bool>();
    if (d.contains("one_comm")) c.one_comm = d["one_comm"].cast<bool>();
    if (d.contains("depth")) c.solve.depth = d["depth"].cast<int>();
    if (d.contains("pivot")) c.solve.pivot = parse_pivot(d["pivot"].cast<std::string>());
    if (d.contains("pivot_growth")) c.solve.pivot_growth = d["pivot_growth"].cast<double>();
    if (d.contains("profile")) c.solve.profile = d["profile"].cast<bool>();
    if (d.contains("rhs")) c.rhs = d["rhs"].cast<std::string>();
    if (d.contains("keep_solution")) c.keep_solution = d["keep_solution"].cast<bool>();
    if (d.contains("comm_timeout_s")) c.solve.comm_timeout_s = d["comm_timeout_s"].cast<double>();
    if (d.contains("residual")) {
      const std::string r = d["residual"].cast<std::string>();
      c.residual = r == "never" ? ResidualMode::Never : r == "compat" ? ResidualMode::Compat : ResidualMode::Always;
    }
    if (d.contains("print_max")) c.print_max = d["print_max"].cast<int>();
    if (d.contains("keep_inverse")) c.keep_inverse = d["keep_inverse"].cast<bool>();
    if (d.contains("host_threads")) c.host_threads = d["host_threads"].cast<int>();
    if (d.contains("repeats")) c.repeats = d["repeats"].cast<int>();
    if (d.contains("refine")) c.refine = d["refine"].cast<int>();
    if (d.contains("refine_tol")) c.refine_tol = d["refine_tol"].cast<double>();
    if (d.contains("race_check")) c.race_check = d["race_check"].cast<bool>();
    py::array_t<double, py::array::c_style | py::array::forcecast> inp;
    if (d.contains("input") && !d["input"].is_none()) {
      inp = d["input"].cast<py::array_t<double, py::array::c_style | py::array::forcecast>>();
      if (inp.ndim() != 2 || inp.shape(0) != c.n || inp.shape(1) != c.n)
        throw std::invalid_argument("input must be (n, n)");
      c.input = inp.data();
    }
    py::array_t<double, py::array::c_style | py::array::forcecast> rhs_in;
    if (d.contains("rhs_input") && !d["rhs_input"].is_none()) {
      rhs_in = d["rhs_input"].cast<py::array_t<double, py::array::c_style | py::array::forcecast>>();
      if (rhs_in.size() != c.n) throw std::invalid_argument("rhs_input must have n entries");
      c.rhs_input = rhs_in.data();
    }
    RunReport r;
    {
      py::gil_scoped_release rel;
      r = run_local(c);
    }
    py::dict o;
    o["status"] = (int)r.status;
    o["message"] = r.message;
    o["glob_time"] = r.glob_time;
    o["best_time"] = r.best_time;
    o["residual_computed"] = r.residual_computed;
    o["residual"] = r.residual;
    o["residual_fp64"] = r.residual_fp64;
    o["nm"] = r.nm;
    o["corner_a"] = to_array(r.corner_a, r.corner_a.empty() ? 0 : r.nm, r.corner_a.empty() ? 0 : r.nm);
    o["corner_inv"] = to_array(r.corner_inv, r.corner_inv.empty() ? 0 : r.nm, r.corner_inv.empty() ? 0 : r.nm);
    if (c.keep_inverse && r.status == Status::Ok) o["inverse"] = to_array(r.inverse, c.n, c.n);
    o["stats"] = stats_to_dict(r.stats);
    o["device"] = r.device_desc;
    o["comm"] = r.comm_desc;
    o["gflops_nominal"] = r.gflops_nominal;
    if (c.race_check) {
      o["race_count"] = r.race_count;
      o["races"] = r.races;
      o["race_ops"] = r.race_ops;
    }
    if (r.rhs_solved) {
      o["axb_residual"] = r.rhs_residual;
      o["axb_seconds"] = r.rhs_seconds;
      o["axb_history"] = r.rhs_history;
      o["refine_steps"] = r.rhs_steps;
      o["refine_converged"] = r.rhs_converged;
      o["axb_backward_error"] = r.rhs_backward_error;
      o["x_head"] = r.x_head;
      if (c.keep_solution) o["x"] = to_array(r.x, c.n, 1);
    }
    return o;
  });

  mod.def("read_matrix_file", [](const std::string& path, int64_t n) {
    std::vector<double> v;
    Status s;
    {
      py::gil_scoped_release rel;
      s = read_matrix_file(path, n, v);
    }
    if (s == Status::CannotOpen) throw std::runtime_error("cannot open " + path);
    if (s == Status::CannotRead) throw std::runtime_error("cannot read " + path);
    return to_array(v, n, n);
  }, py::arg("path"), py::arg("n"));
  mod.def("read_matrix_rows", [](const std::string& path, int64_t n, std::vector<int64_t> rows, int nthreads) {
    std::vector<double> v;
    Status s;
    {
      py::gil_scoped_release rel;
      s = read_matrix_rows(path, n, rows, v, nthreads);
    }
    if (s == Status::CannotOpen) throw std::runtime_error("cannot open " + path);
    if (s == Status::CannotRead) throw std::runtime_error("cannot read " + path);
    return to_array(v, (int64_t)rows.size(), n);
  }, py::arg("path"), py::arg("n"), py::arg("rows"), py::arg("nthreads") = 0,
     "the given rows of an n x n matrix file (one rank's share), same accept set as read_matrix_file");
}
