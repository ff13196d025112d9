// Candidate-block inverse for m > 4096 (and GJ_BI_VARIANT=huge for any m > 256, tests): reference
// inverse_block (main.cpp:746-820) + block_norm (main.cpp:669-683) with the whole GPU per block.
//
// The per-step global sweep (block_inverse_generic: one 256-thread workgroup per block, m passes over
// all m^2 elements) was the only path above m = 4096 -- hours at m = 8192.  Here one candidate at a
// time, the working block column-major in a global slab Wc (Wc[j m + i] = W[i][j]):
//   * a panel of PB = 32 columns is factored by ONE 1024-thread workgroup (huge_panel): per step the
//     exact argmax of the reference (largest magnitude, ties to the lowest current position under
//     the reference's row swaps -- the same rule and book-keeping as block_inverse_blocked), the
//     pivot row's panel values through LDS, the rank-1 sweep update of the panel's columns only,
//     kept in the "U" form (pivot row: inv - 1, others: -w inv), as the panel-blocked kernel does;
//   * the rest of the block takes the panel as one rank-PB update X += U R (R = the PB pivot rows
//     before the panel, U = the panel), which in the column-major slab is  Wc^T[rest, :] +=
//     R[:, rest]^T U^T: two K = PB GEMMs on the engine's MFMA kernels (K-major A = R, B = U^T);
//   * the panel's columns then become U + E (E: 1 at each pivot row of its column).
// The result is permuted into inv_t exactly like block_inverse_generic (out[prow[u] m + kinv[i]] =
// W[i][u]), the score is ||W||_inf (row sums are permutation invariant).
//
// The host needs which local blocks are still candidates (a used block is skipped without its
// GEMMs): one 4-byte-per-block device-to-host copy and a stream synchronisation per batch -- only on
// this path.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <stdexcept>
#include <vector>

#include "kernels.hpp"
#include "wave_ops.hpp"

namespace gj {
namespace kern {

namespace {

constexpr int kPB = 32;       // panel width = the update GEMM's K
constexpr int kFT = 1024;     // threads of the panel workgroup
// int book-keeping per candidate: prow[m] kinv[m] usedr[m] pos[m] posrow[m] flag[4]
// flag[0]: 0 = ok, 1 = singular, 2 = block already used (not a candidate)
struct Ints {
  int* prow;
  int* kinv;
  int* usedr;
  int* pos;
  int* posrow;
  int* flag;
};
__host__ __device__ inline Ints ints_of(int* base, int m) {
  return Ints{base, base + m, base + 2 * m, base + 3 * m, base + 4 * m, base + 5 * m};
}

template <typename T>
__global__ __launch_bounds__(256) void huge_init(const T* __restrict__ Lt, int64_t ldl, T* __restrict__ Wc, int m,
                                                 int b, int used_flag, int* ibase) {
  const Ints in = ints_of(ibase, m);
  const int64_t n = (int64_t)m * m;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (int64_t)gridDim.x * blockDim.x;
  if (!used_flag)  // W[i][j] = -Lt[j ldl + b m + i]: column j of W is row j of the K-major panel
    for (int64_t e = tid; e < n; e += stride) {
      const int64_t j = e / m, i = e - j * m;
      Wc[e] = -Lt[j * ldl + (int64_t)b * m + i];
    }
  for (int64_t i = tid; i < m; i += stride) {
    in.usedr[i] = 0;
    in.pos[i] = (int)i;
    in.posrow[i] = (int)i;
  }
  if (tid == 0) in.flag[0] = used_flag ? 2 : 0;
}

// PB steps of the scalar sweep on the panel columns [c0, c0 + pb), every row; U form.
template <typename T>
__global__ __launch_bounds__(kFT) void huge_panel(T* __restrict__ Wc, int m, int c0, int pb, double thresh,
                                                  int* ibase) {
  const Ints in = ints_of(ibase, m);
  if (in.flag[0] != 0) return;  // uniform
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  __shared__ unsigned long long redk[kFT / 64];
  __shared__ int redp[kFT / 64], redr[kFT / 64];
  __shared__ T rowb[kPB];
  __shared__ int s_r;
  for (int jj = 0; jj < pb; ++jj) {
    const int64_t col = (int64_t)(c0 + jj) * m;
    // block-wide argmax of |column c0 + jj| over the unused rows: larger magnitude, then lower position
    unsigned long long bk = 0;
    int bp = 0x7fffffff, br = -1;
    for (int i = tid; i < m; i += kFT) {
      if (in.usedr[i]) continue;
      const unsigned long long key = __builtin_bit_cast(unsigned long long, (double)Wc[col + i]) & 0x7FFFFFFFFFFFFFFFull;
      const int ps = in.pos[i];
      if (br < 0 || key > bk || (key == bk && ps < bp)) {
        bk = key;
        bp = ps;
        br = i;
      }
    }
    for (int o = 32; o >= 1; o >>= 1) {
      const unsigned long long ok = __shfl_xor(bk, o, 64);
      const int op = __shfl_xor(bp, o, 64), orr = __shfl_xor(br, o, 64);
      if (orr >= 0 && (br < 0 || ok > bk || (ok == bk && op < bp))) {
        bk = ok;
        bp = op;
        br = orr;
      }
    }
    if (lane == 0) {
      redk[wave] = bk;
      redp[wave] = bp;
      redr[wave] = br;
    }
    __syncthreads();  // B1: partials published; every write of the previous step is visible
    if (tid == 0) {
      int r = -1;
      unsigned long long fk = 0;
      int fp = 0x7fffffff;
      for (int w = 0; w < kFT / 64; ++w) {
        const int wr = redr[w];
        if (wr >= 0 && (r < 0 || redk[w] > fk || (redk[w] == fk && redp[w] < fp))) {
          fk = redk[w];
          fp = redp[w];
          r = wr;
        }
      }
      if (r < 0) r = in.posrow[c0 + jj];  // no free row (cannot happen): singular below
      // the reference's swap of step c0 + jj: pivot row <-> the row at that position
      const int kp = c0 + jj, r2 = in.posrow[kp], pr = in.pos[r];
      in.pos[r2] = pr;
      in.posrow[pr] = r2;
      in.pos[r] = kp;
      in.posrow[kp] = r;
      in.prow[kp] = r;
      in.kinv[r] = kp;
      in.usedr[r] = 1;
      s_r = r;
    }
    __syncthreads();  // B2: the pivot row index
    const int r = s_r;
    if (tid < pb) rowb[tid] = Wc[(int64_t)(c0 + tid) * m + r];
    __syncthreads();  // B3: the pivot row's panel values
    const T piv = rowb[jj];
    if (!(fabs((double)piv) >= thresh)) {
      if (tid == 0) in.flag[0] = 1;
      return;  // every thread read the same pivot: a uniform exit
    }
    const T inv = fast_recip(piv);
    for (int i = tid; i < m; i += kFT) {
      const T u = (i == r) ? inv - T(1) : -Wc[col + i] * inv;
      for (int kk = 0; kk < pb; ++kk)
        if (kk != jj) {
          T* w = Wc + (int64_t)(c0 + kk) * m + i;
          *w = __builtin_fma(u, rowb[kk], *w);
        }
      Wc[col + i] = u;
    }
  }
}

// Ut[j][i] = U[i][j] (the panel, K-major B of the update), R[j][c] = W[prow[c0 + j]][c] (the pivot
// rows before the panel, K-major A)
template <typename T>
__global__ __launch_bounds__(256) void huge_stage(const T* __restrict__ Wc, int m, int c0, int pb, T* __restrict__ Ut,
                                                  T* __restrict__ R, const int* ibase) {
  const Ints in = ints_of(const_cast<int*>(ibase), m);
  if (in.flag[0] != 0) return;
  const int64_t n = (int64_t)pb * m;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = tid; e < n; e += stride) {
    const int64_t j = e / m, c = e - j * m;
    Ut[e] = Wc[(int64_t)(c0 + j) * m + c];
    R[e] = Wc[c * m + in.prow[c0 + j]];
  }
}

// the panel's columns := U + E
template <typename T>
__global__ void huge_fix(T* __restrict__ Wc, int m, int c0, int pb, const int* ibase) {
  const Ints in = ints_of(const_cast<int*>(ibase), m);
  if (in.flag[0] != 0) return;
  const int jj = threadIdx.x;
  if (jj < pb) Wc[(int64_t)(c0 + jj) * m + in.prow[c0 + jj]] += T(1);
}

template <typename T>
__global__ __launch_bounds__(256) void huge_out(const T* __restrict__ Wc, int m, T* __restrict__ out, const int* ibase) {
  const Ints in = ints_of(const_cast<int*>(ibase), m);
  if (in.flag[0] != 0) return;
  const int64_t n = (int64_t)m * m;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = tid; e < n; e += stride) {  // e = u m + i: W[i][u]
    const int64_t u = e / m, i = e - u * m;
    out[(int64_t)in.prow[u] * m + in.kinv[i]] = Wc[e];
  }
}

// row sums of W (column-major: thread i walks its row), per-workgroup maximum
template <typename T>
__global__ __launch_bounds__(256) void huge_rowsum(const T* __restrict__ Wc, int m, double* __restrict__ part,
                                                   const int* ibase) {
  const Ints in = ints_of(const_cast<int*>(ibase), m);
  __shared__ double red[4];
  const int i = blockIdx.x * 256 + threadIdx.x;
  double s = 0.0;
  if (in.flag[0] == 0 && i < m)
    for (int u = 0; u < m; ++u) s += fabs((double)Wc[(int64_t)u * m + i]);
  s = wave_max_f64(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
}

__global__ __launch_bounds__(256) void huge_probe(const int* ibase, int m, int32_t* probe) {
  const Ints in = ints_of(const_cast<int*>(ibase), m);
  if (in.flag[0] != 0) return;
  for (int c = blockIdx.x * 256 + threadIdx.x; c < m; c += gridDim.x * 256) probe[c] = in.prow[c];
}

__global__ __launch_bounds__(256) void huge_score(const double* __restrict__ part, int nparts, double* scores,
                                                  int32_t* valid, int b, const int* ibase, int m) {
  const Ints in = ints_of(const_cast<int*>(ibase), m);
  __shared__ double red[4];
  double s = 0.0;
  for (int q = threadIdx.x; q < nparts; q += 256) s = fmax(s, part[q]);
  s = wave_max_f64(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    if (in.flag[0] != 0) {
      valid[b] = 0;
      scores[b] = 0.0;
    } else {
      const double sc = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
      scores[b] = sc;
      valid[b] = isfinite(sc) ? 1 : 0;
    }
  }
}

// device scratch of this path (Ut, R, row-sum partials, int book-keeping) and the pinned used copy;
// per host thread (one thread drives one GPU in the multi-GPU runner), kept for the process
struct HugeScratch {
  void* dev = nullptr;
  size_t bytes = 0;
  int32_t* host_used = nullptr;
  size_t host_n = 0;
};
thread_local HugeScratch g_huge;

unsigned grid_of(int64_t n) { return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 4096)); }

}  // namespace

// touch_used = false (the engine's live-candidate launch, nlive >= 0): a used block's score, flag and
// inverse are left as they are, like the one-workgroup-per-live-candidate kernels; true (one launch
// per block): they are set to 0, like block_inverse_generic.
template <typename T>
static void huge_launch(const void* Lt, int64_t ldl, void* inv_t, double* scores, int32_t* valid,
                        const int32_t* used, const Layout& L, double thresh, hipStream_t s, void* scratch,
                        bool touch_used) {
  const int m = (int)L.m;
  const int64_t nblk = L.nblk;
  const int nparts = (m + 255) / 256;
  const size_t need = 2 * (size_t)kPB * m * sizeof(T) + (size_t)nparts * sizeof(double) + (6 * (size_t)m + 4) * sizeof(int) + 256;
  if (g_huge.bytes < need) {
    (void)hipStreamSynchronize(s);
    if (g_huge.dev) (void)hipFree(g_huge.dev);
    g_huge.dev = nullptr;
    if (hipMalloc(&g_huge.dev, need) != hipSuccess) throw Error(Status::NoMemory, "block inverse (m > 4096): scratch");
    g_huge.bytes = need;
  }
  if (g_huge.host_n < (size_t)std::max<int64_t>(nblk, 1)) {
    if (g_huge.host_used) (void)hipHostFree(g_huge.host_used);
    g_huge.host_used = nullptr;
    if (hipHostMalloc(reinterpret_cast<void**>(&g_huge.host_used), sizeof(int32_t) * std::max<int64_t>(nblk, 1),
                      hipHostMallocDefault) != hipSuccess)
      throw Error(Status::NoMemory, "block inverse (m > 4096): pinned flags");
    g_huge.host_n = (size_t)std::max<int64_t>(nblk, 1);
  }
  char* base = static_cast<char*>(g_huge.dev);
  T* Ut = reinterpret_cast<T*>(base);
  T* R = Ut + (size_t)kPB * m;
  double* part = reinterpret_cast<double*>(R + (size_t)kPB * m);
  int* ib = reinterpret_cast<int*>(part + nparts);
  // which local blocks are candidates: used is indexed by global block row g = b p + k
  for (int64_t b = 0; b < nblk; ++b)
    (void)hipMemcpyAsync(g_huge.host_used + b, used + b * L.p + L.k, sizeof(int32_t), hipMemcpyDeviceToHost, s);
  if (hipStreamSynchronize(s) != hipSuccess) throw Error(Status::CommError, "block inverse (m > 4096): stream");
  const T* lt = static_cast<const T*>(Lt);
  for (int64_t b = 0; b < nblk; ++b) {
    T* Wc = static_cast<T*>(scratch) + b * (int64_t)m * m;
    T* out = static_cast<T*>(inv_t) + b * (int64_t)m * m;
    const int is_used = g_huge.host_used[b] != 0;
    if (is_used && !touch_used) continue;
    hipLaunchKernelGGL((huge_init<T>), dim3(grid_of((int64_t)m * m)), dim3(256), 0, s, lt, ldl, Wc, m, (int)b, is_used,
                       ib);
    if (!is_used) {
      for (int c0 = 0; c0 < m; c0 += kPB) {
        const int pb = std::min(kPB, m - c0);
        hipLaunchKernelGGL((huge_panel<T>), dim3(1), dim3(kFT), 0, s, Wc, m, c0, pb, thresh, ib);
        hipLaunchKernelGGL((huge_stage<T>), dim3(grid_of((int64_t)pb * m)), dim3(256), 0, s, Wc, m, c0, pb, Ut, R,
                           ib);
        // Wc^T[rest, :] += R[:, rest]^T Ut  (a singular panel leaves garbage here: the score marks it)
        if (c0 > 0)
          gemm(sizeof(T) == 8 ? DType::F64 : DType::F32, 0, 1, c0, m, pb, R, m, Ut, m, Wc, m, s, nullptr);
        const int r0 = c0 + pb;
        if (r0 < m)
          gemm(sizeof(T) == 8 ? DType::F64 : DType::F32, 0, 1, m - r0, m, pb, R + r0, m, Ut, m,
               Wc + (int64_t)r0 * m, m, s, nullptr);
        hipLaunchKernelGGL((huge_fix<T>), dim3(1), dim3(64), 0, s, Wc, m, c0, pb, ib);
      }
      hipLaunchKernelGGL((huge_out<T>), dim3(grid_of((int64_t)m * m)), dim3(256), 0, s, Wc, m, out, ib);
      if (int32_t* probe = block_inverse_probe())  // the pivot row of every column (tests)
        hipLaunchKernelGGL(huge_probe, dim3(grid_of(m)), dim3(256), 0, s, ib, m, probe + b * m);
    }
    hipLaunchKernelGGL((huge_rowsum<T>), dim3((unsigned)nparts), dim3(256), 0, s, Wc, m, part, ib);
    hipLaunchKernelGGL(huge_score, dim3(1), dim3(256), 0, s, part, nparts, scores, valid, (int)b, ib, m);
  }
}

void block_inverse_huge(DType dt, const void* Lt, int64_t ldl, void* inv_t, double* scores, int32_t* valid,
                        const int32_t* used, const Layout& L, double thresh, int64_t nlive, hipStream_t s,
                        void* scratch) {
  if (L.nblk <= 0) return;
  if (dt == DType::F64)
    huge_launch<double>(Lt, ldl, inv_t, scores, valid, used, L, thresh, s, scratch, nlive < 0);
  else
    huge_launch<float>(Lt, ldl, inv_t, scores, valid, used, L, thresh, s, scratch, nlive < 0);
}

}  // namespace kern
}  // namespace gj
