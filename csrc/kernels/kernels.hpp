// Launch wrappers of the hand-written gfx950 kernels (implemented in csrc/kernels/*.hip).
#pragma once

#include <hip/hip_runtime.h>

#include "gj/common.hpp"
#include "gj/device.hpp"
#include "gj/layout.hpp"
#include "gj/pivot.hpp"

namespace gj {
namespace kern {

// gemm.hip
void gemm(DType dt, int op /*0 acc, 1 store*/, int a_kmajor, int64_t M, int64_t N, int64_t K,
          const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc,
          hipStream_t s, const GemmExtra* ex = nullptr);
// n independent small K-major GEMMs, one launch per 4 (small tiles; Store = C never read)
void gemm_batch(DType dt, const GemmDesc* d, int n, hipStream_t s);
int residual_nparts(int64_t N);
int gemm_variant_id(const char* name);  // big | narrow | squarepf | bigpf | glds | auto; else throws
void set_gemm_variant(int v);
void set_glds_peel(int on);  // fp64 LDS-DMA trailing update: peeled stage-unrolled loop (1) or not (0)
void set_glds_covl(int on);   // fp64 LDS-DMA kernel: C loads overlapped with the first slices (GJ_GLDS_COVL)
void set_lat_glds(int on);   // every latency GEMM of >= 1024 rows on the LDS-DMA kernel (tests; GemmExtra::lat_wide per call)
void set_lat_kernel(int mode); // fp64 latency GEMMs on the register-fed kernel: 1 / 0 forced, -1 per launch (GemmExtra::lat_reg)
void set_glds_build(int b);  // 23 | 25 | 33 (stages * 10 + waves-per-SIMD bound), 0 = auto
void set_glds_tile(int bn);  // 64 | 128: the fp64 LDS-DMA kernel's tile width for every launch, 0 = per launch (GJ_GLDS_TILE)
void set_block_inverse_variant(int v);  // 0 = default families, 1 = register sweep, 5 = co-resident, 6 = generic
int block_inverse_variant();
int block_inverse_variant_id(const char* name);  // panel | sweep | co | generic; else throws
const char* block_inverse_kernel_name(DType dt, int64_t m, int variant);
void residual_partial(DType dt, int64_t M, int64_t N, int64_t K, const void* A, int64_t lda,
                      const void* B, int64_t ldb, int64_t n_real, int64_t blk_m, int64_t p,
                      int64_t k, double* partial, hipStream_t s);

// misc.hip: partial pivoting (SolveOptions::pivot = Partial)
void candidate_maxabs(DType dt, const void* Lt, int64_t ldl, double* scores, int32_t* valid,
                      const int32_t* used, const Layout& L, double thresh, hipStream_t s);
void gather_candidate(DType dt, void* sel, const void* Lt, int64_t ldl, const PivotRec* rec, const Layout& L,
                      hipStream_t s);
void commit_candidate(DType dt, void* inv_t, const void* inv1, const int32_t* valid1, const double* score1, double growth, PivotRec* rec,
                      const Layout& L, hipStream_t s);

// blockinv.hip
void block_inverse(DType dt, const void* Lt, int64_t ldl, void* inv_t, double* scores,
                   int32_t* valid, const int32_t* used, const Layout& L, double thresh, int64_t nlive,
                   hipStream_t s, void* scratch, int* iscratch, int variant = -1);
// blockinv_mfma.hip: 16 < m <= 128 (false = not handled)
bool block_inverse_mfma(DType dt, const void* Lt, int64_t ldl, void* inv_t, double* scores,
                        int32_t* valid, const int32_t* used, const Layout& L, double thresh, int64_t nlive,
                        hipStream_t s, const PivotSelectArgs* sel = nullptr);
// block_inverse with the pivot selection fused into the launch (PivotSelectArgs) where the kernel
// family the call resolves to supports it (the matrix-core register kernel); false = nothing was
// launched, the caller runs block_inverse and the selection separately
bool block_inverse_select(DType dt, const void* Lt, int64_t ldl, void* inv_t, double* scores,
                          int32_t* valid, const int32_t* used, const Layout& L, double thresh, int64_t nlive,
                          hipStream_t s, const PivotSelectArgs& sel, int variant = -1, void* scratch = nullptr);
// test probe: when set, the matrix-core block inverses write the pivot row of every column of
// every candidate to piv_out[b * m + c] (device memory; nullptr = off)
void set_block_inverse_probe(int32_t* piv_out);
int32_t* block_inverse_probe();
// blockinv_big.hip: fp64 128 < m <= 256 (false = not handled); scratch: nblk 256 x 256 images
bool block_inverse_big(DType dt, const void* Lt, int64_t ldl, void* inv_t, double* scores, int32_t* valid,
                       const int32_t* used, const Layout& L, double thresh, int64_t nlive, hipStream_t s, void* scratch);
size_t block_inverse_big_scratch_bytes(DType dt, const Layout& L);
// blockinv_huge.hip: m > 4096 (or GJ_BI_VARIANT=huge), one candidate at a time with the whole GPU
// (panel factor + MFMA GEMM updates); scratch: nblk m x m slabs (the generic path's)
void block_inverse_huge(DType dt, const void* Lt, int64_t ldl, void* inv_t, double* scores, int32_t* valid,
                        const int32_t* used, const Layout& L, double thresh, int64_t nlive, hipStream_t s,
                        void* scratch);
// the co-resident form (4 waves, fits the slot one trailing-update workgroup frees): fp64 32 < m <= 128;
// with sel, the batch's last workgroup also runs the selection (as block_inverse_mfma)
bool block_inverse_co(DType dt, const void* Lt, int64_t ldl, void* inv_t, double* scores, int32_t* valid,
                      const int32_t* used, const Layout& L, double thresh, int64_t nlive, hipStream_t s, void* scratch,
                      const PivotSelectArgs* sel = nullptr);
// scratch needed by the fp64 m > 128 paths (big kernel / generic sweep)
// (variant: the kernel family to use for this call, -1 = the process-wide setting)
size_t block_inverse_scratch_bytes(DType dt, const Layout& L, int variant = -1);
size_t block_inverse_iscratch_bytes(const Layout& L);

// misc.hip
void generate(DType dt, void* X, const Layout& L, int kind, uint64_t seed, hipStream_t s);
// generate() fused with row_abs_max() of the result (out zeroed here): one pass over the matrix
void generate_norm(DType dt, void* X, const Layout& L, int kind, uint64_t seed, double* out, hipStream_t s);
void widen(DType dt, double* dst, int64_t ldd, const void* X, int64_t ldx, int64_t rows, int64_t cols,
           hipStream_t s);
void upload_convert(DType dt, void* X, int64_t ldx, const double* src, int64_t src_ld, int64_t rows,
                    int64_t cols, hipStream_t s);
void extract_neg_t(DType dt, void* Lt, int64_t ldl, const void* X, int64_t ldx, int64_t rows,
                   int64_t col0, int64_t m, hipStream_t s);
void add_diag(DType dt, void* A, int64_t ld, int64_t nd, double alpha, hipStream_t s);
// nwg workgroups that each spin for `us` microseconds (lds_bytes > 0: 256 threads + that much LDS)
void spin(int nwg, double us, hipStream_t s, int lds_bytes = 0);
// zero `bytes` at p (16-byte vector stores, scalar tail) on nwg 256-thread workgroups holding
// lds_bytes of LDS each: the receiving RCCL channels' footprint in ShadowComm's cost model
void zero_channels(void* p, size_t bytes, int nwg, int lds_bytes, hipStream_t s);
void pivot_local(const double* scores, const int32_t* valid, const int32_t* used, const int32_t* pos,
                 const Layout& L, PivotRec* out, hipStream_t s);
void pivot_select_single(const double* scores, const int32_t* valid, const Layout& L, int32_t t,
                         int32_t* pos, int32_t* phys_at, int32_t* used, int32_t* seq, PivotRec* rec,
                         PivotResult* out, PivotResult* host_out, hipStream_t s);
int host_fence();  // GJ_HOST_FENCE (misc.hip): 1 = system-scope fences around the host pivot mirror
void pivot_global(const PivotRec* recs, int32_t p, int32_t t, int32_t* pos, int32_t* phys_at,
                  int32_t* used, int32_t* seq, PivotResult* out, PivotResult* host_out, hipStream_t s);
void owner_edits(DType dt, void* At, int64_t ldl, const int32_t* phys, int64_t p, int64_t k, int64_t j,
                 int64_t m, void* lrow, void* ht, const void* inv, const PieceMove& mv, hipStream_t s);
void take_rows(DType dt, void* dst, int64_t ldd, void* X, int64_t ldx, const int32_t* phys, int64_t p, int64_t k,
               int64_t col0, int64_t w, int64_t m, hipStream_t s);
void sum_slices(DType dt, void* dst, const void* src, int64_t count, int64_t nslices, hipStream_t s);
void zero_unless_owner(DType dt, void* buf, int64_t count, const int32_t* phys, int64_t p, int64_t k, hipStream_t s);
void h_block(DType dt, void* R, int64_t ldr, const void* Ht, int64_t m, hipStream_t s);
void permute_blocks(DType dt, void* dst, int64_t ldd, const void* X, int64_t ldx, int64_t nblk,
                    int64_t m, int64_t Nr, const int32_t* dst_blk, const int32_t* colsrc,
                    hipStream_t s);
// Device::hash_rows: nparts workgroups, parts[g] = workgroup g's partial hash
void hash_rows(const void* base, int64_t ld_bytes, int64_t width_bytes, int64_t rows, uint64_t* parts,
               int nparts, hipStream_t s);
// minus_identity: sum_j |X[r][j] - delta(global(r), j)| (the streamed residual's row sums)
void row_abs_max(DType dt, const void* X, int64_t ldx, const Layout& L, double* out, hipStream_t s,
                 bool minus_identity = false);
// reduce residual partials: out = max over real local rows of sum_parts partial[r][*]
void residual_reduce(const double* partial, int nparts, const Layout& L, double* out, hipStream_t s);

}  // namespace kern
}  // namespace gj
