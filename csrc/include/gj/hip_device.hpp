// HipDevice — the MI355X execution backend (csrc/runtime/hip_device.cpp).
#pragma once

#include <vector>

#include "gj/device.hpp"

namespace gj {

class HipDevice : public Device {
 public:
  explicit HipDevice(int device_index);
  ~HipDevice() override;
  bool on_gpu() const override { return true; }
  std::string describe() const override;
  int device_index() const override { return dev_; }

  void* alloc(size_t bytes) override;
  void release(void* p) override;
  void* alloc_pinned(size_t bytes) override;
  void* alloc_pinned_coherent(size_t bytes) override;
  void release_pinned(void* p) override;
  size_t free_memory() const override;
  void memset0(void* p, size_t bytes, int s) override;
  void memset2d(void* p, size_t pitch, size_t width_bytes, size_t height, int s) override;
  void copy(void* dst, const void* src, size_t bytes, int s) override;
  void copy2d(void* dst, size_t dpitch, const void* src, size_t spitch, size_t width_bytes,
              size_t height, int s) override;

  int create_event(bool timing = false) override;
  void record(int ev, int s) override;
  void wait(int s, int ev) override;
  void sync_event(int ev) override;
  bool query_event(int ev) override;
 private:
  int reserved_ = 0;

 public:
  int reserve_cus(int n) override;
  int64_t skip_align() const override { return 128; }  // whole tiles of every GEMM kernel
  void generate_norm(DType dt, void* X, const Layout& L, GenSpec g, double* out, int s) override;
  void sync_stream(int s) override;
  bool stream_idle(int s) override;
  void sync_all() override;
  float event_ms(int ev_start, int ev_end) override;
  void* native_stream(int s) override;
  std::shared_ptr<void> mark(int s) override;
  void wait_mark(int s, const std::shared_ptr<void>& h) override;
  void occupy(int s, int nwg, double us, int lds_bytes = 0) override;
  void zero_channels(void* p, size_t bytes, int s, int nwg, int lds_bytes) override;

  void generate(DType dt, void* X, const Layout& L, GenSpec g, int s) override;
  void widen(DType dt, double* dst, int64_t ldd, const void* X, int64_t ldx, int64_t rows, int64_t cols,
             int s) override;
  void upload_convert(DType dt, void* X, int64_t ldx, const double* src_dev, int64_t src_ld,
                      int64_t rows, int64_t cols, int s) override;
  void extract_neg_t(DType dt, void* Lt, int64_t ldl, const void* X, int64_t ldx, int64_t rows,
                     int64_t col0, int64_t m, int s) override;
  void add_diag(DType dt, void* A, int64_t ld, int64_t nd, double alpha, int s) override;
  void block_inverse(DType dt, const void* Lt, int64_t ldl, void* inv_t, double* scores,
                     int32_t* valid, const int32_t* used, const Layout& L, double thresh, int64_t nlive,
                     int s) override;
  bool block_inverse_select(DType dt, const void* Lt, int64_t ldl, void* inv_t, double* scores,
                            int32_t* valid, const int32_t* used, const Layout& L, double thresh, int64_t nlive,
                            const PivotSelectArgs& sel, int s) override;
  void set_block_inverse_hint(int variant) override { bi_hint_ = variant; }
  void set_gemm_tile_hint(int bn) override { tile_hint_ = bn; }
  size_t block_inverse_scratch_bytes(DType dt, const Layout& L, int variant) const override;
  void prepare_block_inverse(DType dt, const Layout& L, int variant) override;
  void candidate_maxabs(DType dt, const void* Lt, int64_t ldl, double* scores, int32_t* valid,
                        const int32_t* used, const Layout& L, double thresh, int s) override;
  void gather_candidate(DType dt, void* sel, const void* Lt, int64_t ldl, const PivotRec* rec, const Layout& L,
                        int s) override;
  void commit_candidate(DType dt, void* inv_t, const void* inv1, const int32_t* valid1, const double* score1, double growth, PivotRec* rec,
                        const Layout& L, int s) override;
  void pivot_local(const double* scores, const int32_t* valid, const int32_t* used,
                   const int32_t* pos, const Layout& L, PivotRec* out, int s) override;
  void pivot_select_single(const double* scores, const int32_t* valid, const Layout& L, int32_t t,
                           int32_t* pos, int32_t* phys_at, int32_t* used, int32_t* seq, PivotRec* rec,
                           PivotResult* out, PivotResult* host_out, int s) override;
  void pivot_global(const PivotRec* recs, int32_t p, int32_t t, int32_t* pos, int32_t* phys_at,
                    int32_t* used, int32_t* seq, PivotResult* out, PivotResult* host_out,
                    int s) override;
  void owner_edits(DType dt, void* At, int64_t ldl, const int32_t* phys, int64_t p, int64_t k, int64_t j,
                   int64_t m, void* lrow, void* ht, const void* inv, const PieceMove& mv, int s) override;
  void take_rows(DType dt, void* dst, int64_t ldd, void* X, int64_t ldx, const int32_t* phys, int64_t p, int64_t k,
                 int64_t col0, int64_t w, int64_t m, int s) override;
  void sum_slices(DType dt, void* dst, const void* src, int64_t count, int64_t nslices, int s) override;
  void zero_unless_owner(DType dt, void* buf, int64_t count, const int32_t* phys, int64_t p, int64_t k,
                         int s) override;
  void h_block(DType dt, void* R, int64_t ldr, const void* Ht, int64_t m, int s) override;
  void gemm(DType dt, GemmOp op, ALayout al, int64_t M, int64_t N, int64_t K, const void* A,
            int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int s,
            const GemmExtra& ex = GemmExtra()) override;
  void gemm_batch(DType dt, const GemmDesc* d, int n, int s) override;
  void permute_blocks(DType dt, void* dst, int64_t ldd, const void* X, int64_t ldx, int64_t nblk,
                      int64_t m, int64_t Nr, const int32_t* dst_blk, const int32_t* colsrc,
                      int s) override;
  void row_abs_max_minus_i(DType dt, const void* X, int64_t ldx, const Layout& L, double* out,
                           int s) override;
  void hash_rows(const void* base, int64_t ld_bytes, int64_t width_bytes, int64_t rows, uint64_t* parts,
                 int s) override;
  void row_abs_max(DType dt, const void* X, int64_t ldx, const Layout& L, double* out,
                   int s) override;
  void residual(DType dt, const void* A, const void* Full, const Layout& L, double* out,
                int s) override;

 private:
  void* scratch(size_t bytes, int slot);
  void activate() const;

  int dev_ = 0;
  void* streams_[kNumStreams] = {};
  int bi_hint_ = -1;  // set_block_inverse_hint
  int tile_hint_ = 0;  // set_gemm_tile_hint
  std::vector<void*> events_;
  void* scratch_[2] = {nullptr, nullptr};
  size_t scratch_sz_[2] = {0, 0};
};

}  // namespace gj
