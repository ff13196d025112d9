// What a small pivot-chain launch pays while a trailing-update-like kernel loads the GPU
// (profiles/side_latency_r5.md).  A high-priority stream runs back-to-back one-wave probe kernels.
// Each probe stamps wall_clock64 (100 MHz) at its start, then follows a dependent pointer chain
// of 16 loads, then stamps again.  The same probes run (a) on an idle GPU, and (b) next to a
// streaming kernel (read + write 2 GiB) on a low-priority stream, over all CUs or the engine's
// 224-CU mask.  Printed medians:
//   gap   = start of probe i+1 - end of probe i   (launch and dispatch cost on a busy chip)
//   load  = (end - start) / 16 per dependent load, for an 8 MiB chain (L2 / MALL) and a 1 GiB chain (HBM)
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 bench/side_latency_probe.hip -o build/side_latency_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <numeric>
#include <random>
#include <vector>

#define CHECK(x)                                                                 \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      std::fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));        \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

constexpr int kLoads = 16;
constexpr int kProbes = 64;

__global__ __launch_bounds__(64) void probe(const uint32_t* __restrict__ next, uint32_t start,
                                            unsigned long long* __restrict__ stamp, uint32_t* sink) {
  const unsigned long long t0 = wall_clock64();
  uint32_t i = start;
  if (next) {
#pragma unroll 1
    for (int k = 0; k < kLoads; ++k) i = __builtin_nontemporal_load(next + i);
  }
  const unsigned long long t1 = wall_clock64();
  if (threadIdx.x == 0) {
    stamp[0] = t0;
    stamp[1] = t1;
    sink[0] = i;
  }
}

// Background: each workgroup streams its slice (read, scale, write back), `reps` passes.
__global__ __launch_bounds__(256) void stream_rw(double* __restrict__ b, size_t n, int reps) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (int r = 0; r < reps; ++r)
    for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += stride) b[e] = b[e] * 0.999 + 1e-3;
}

// Occupancy hog: 96 KiB of LDS per workgroup (one per CU, like the trailing update's LDS-DMA
// tiles), an FMA loop of ~`iters` steps, then retire.
__global__ __launch_bounds__(256) void hog(double* out, int iters) {
  extern __shared__ double lds[];
  double v = threadIdx.x;
#pragma unroll 1
  for (int i = 0; i < iters; ++i) v = __builtin_fma(v, 0.999999, 1e-9);
  lds[threadIdx.x] = v;
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x & 1023] = lds[(threadIdx.x + 1) & 255];
}

// Register hog: 256 threads whose waves keep ~126 doubles live (256 VGPRs: two waves fill a SIMD) (most of a SIMD's register file,
// like the trailing update's accumulators), ~`iters` passes, then retire.
__global__ __launch_bounds__(256) void vhog(double* out, int iters) {
  double a[126];
#pragma unroll
  for (int k = 0; k < 126; ++k) a[k] = threadIdx.x + k;
#pragma unroll 1
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 126; ++k) a[k] = __builtin_fma(a[k], 0.999999, 1e-9);
  }
  double v = 0;
#pragma unroll
  for (int k = 0; k < 126; ++k) v += a[k];
  if (threadIdx.x == 0) out[blockIdx.x & 1023] = v;
}

// owner_edits-shaped probe: `gridDim.x` workgroups of 256 threads, one dependent load + store each;
// the first start and the last end over all workgroups (vector atomics on global memory).
__global__ __launch_bounds__(256) void wide_probe(const uint32_t* __restrict__ next, uint32_t* __restrict__ dst,
                                                  unsigned long long* __restrict__ stamp) {
  const unsigned long long t0 = wall_clock64();
  const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  dst[e] = next[e] + 1u;
  __syncthreads();
  const unsigned long long t1 = wall_clock64();
  if (threadIdx.x == 0) {
    atomicMin(stamp, t0);
    atomicMax(stamp + 1, t1);
  }
}

static double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v.empty() ? 0.0 : v[v.size() / 2];
}

int main() {
  const size_t small_n = (8u << 20) / 4, big_n = (size_t(1) << 30) / 4;  // chain lengths in uint32
  std::vector<uint32_t> h(big_n);
  uint32_t* chain_small = nullptr;
  uint32_t* chain_big = nullptr;
  // one random cycle over every element, each element pointing at the next
  auto build = [&](size_t n) {
    std::vector<uint32_t> perm(n);
    std::iota(perm.begin(), perm.end(), 0u);
    std::shuffle(perm.begin(), perm.end(), std::mt19937(7));
    for (size_t i = 0; i < n; ++i) h[perm[i]] = perm[(i + 1) % n];
  };
  build(small_n);
  CHECK(hipMalloc(&chain_small, small_n * 4));
  CHECK(hipMemcpy(chain_small, h.data(), small_n * 4, hipMemcpyHostToDevice));
  build(big_n);
  CHECK(hipMalloc(&chain_big, big_n * 4));
  CHECK(hipMemcpy(chain_big, h.data(), big_n * 4, hipMemcpyHostToDevice));

  const size_t bn = (size_t(2) << 30) / 8;
  double* bg = nullptr;
  CHECK(hipMalloc(&bg, bn * 8));
  CHECK(hipMemset(bg, 0, bn * 8));
  unsigned long long* stamps = nullptr;
  uint32_t* sink = nullptr;
  CHECK(hipMalloc(&stamps, kProbes * 2 * 8));
  CHECK(hipMalloc(&sink, 64));

  int lo = 0, hi = 0;
  CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  hipStream_t side, main_all, main_mask;
  CHECK(hipStreamCreateWithPriority(&side, hipStreamNonBlocking, hi));
  CHECK(hipStreamCreateWithPriority(&main_all, hipStreamNonBlocking, lo));
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int ncu = prop.multiProcessorCount;
  std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
  for (int c = 0; c < ncu; ++c) mask[c / 32] |= 1u << (c % 32);
  for (int i = 0; i < 32; ++i) mask[i / 32] &= ~(1u << (i % 32));
  CHECK(hipExtStreamCreateWithCUMask(&main_mask, (uint32_t)mask.size(), mask.data()));

  // background run length: one pass of 2 GiB read + write is ~0.6 ms; 120 passes ~ 70 ms, far longer
  // than the 64 probes
  const int reps = 120;
  struct Case {
    const char* name;
    hipStream_t bg;
  } cases[] = {{"idle", nullptr}, {"stream_rw on all CUs", main_all}, {"stream_rw on 224-CU mask", main_mask}};
  double* hog_out = nullptr;
  CHECK(hipMalloc(&hog_out, 1024 * 8));
  hipStream_t comm;
  CHECK(hipStreamCreateWithPriority(&comm, hipStreamNonBlocking, hi));
  const size_t hog_lds = 96 * 1024;
  CHECK(hipFuncSetAttribute((const void*)hog, hipFuncAttributeMaxDynamicSharedMemorySize, (int)hog_lds));
  for (const Case& c : cases) {
    for (int which = 0; which < 3; ++which) {
      const uint32_t* chain = which == 0 ? nullptr : which == 1 ? chain_small : chain_big;
      if (c.bg) hipLaunchKernelGGL(stream_rw, dim3(8192), dim3(256), 0, c.bg, bg, bn, reps);
      for (int i = 0; i < kProbes; ++i)
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, side, chain, (uint32_t)(i * 977u), stamps + 2 * i, sink);
      CHECK(hipGetLastError());
      CHECK(hipStreamSynchronize(side));
      std::vector<unsigned long long> s(kProbes * 2);
      CHECK(hipMemcpy(s.data(), stamps, s.size() * 8, hipMemcpyDeviceToHost));
      if (c.bg) CHECK(hipStreamSynchronize(c.bg));
      std::vector<double> gap, load;
      for (int i = 1; i < kProbes; ++i) {
        gap.push_back((double)(s[2 * i] - s[2 * i - 1]) * 10.0);  // ns
        load.push_back((double)(s[2 * i + 1] - s[2 * i]) * 10.0 / kLoads);
      }
      const char* what = which == 0 ? "no loads" : which == 1 ? "8 MiB chain" : "1 GiB chain";
      std::printf("%-26s %-12s gap median %7.2f us | per dependent load %7.0f ns\n", c.name, what,
                  median(gap) / 1e3, which == 0 ? 0.0 : median(load));
    }
  }
  // LDS-holding background: workgroups of ~`iters` FMA steps, one per CU at a time
  struct HogCase {
    const char* name;
    hipStream_t bg;
    int comm_wgs;  // extra hog workgroups on an unmasked high-priority stream (the COMM chunk pass)
  } hogs[] = {{"hog on 224-CU mask", main_mask, 0},
              {"hog on all CUs", main_all, 0},
              {"hog on mask + 32 COMM wgs", main_mask, 32},
              {"hog on mask + 256 COMM wgs", main_mask, 256}};
  const int iters = 20000;  // ~20 us per workgroup at ~1 FMA per 4 clk per wave
  for (const HogCase& c : hogs) {
    for (int which = 0; which < 2; ++which) {
      const uint32_t* chain = which == 0 ? nullptr : chain_small;
      hipLaunchKernelGGL(hog, dim3(224 * 20), dim3(256), hog_lds, c.bg, hog_out, iters);
      if (c.comm_wgs) hipLaunchKernelGGL(hog, dim3(c.comm_wgs * 4), dim3(256), hog_lds, comm, hog_out, iters);
      for (int i = 0; i < kProbes; ++i)
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, side, chain, (uint32_t)(i * 977u), stamps + 2 * i, sink);
      CHECK(hipGetLastError());
      CHECK(hipStreamSynchronize(side));
      std::vector<unsigned long long> s(kProbes * 2);
      CHECK(hipMemcpy(s.data(), stamps, s.size() * 8, hipMemcpyDeviceToHost));
      CHECK(hipStreamSynchronize(c.bg));
      CHECK(hipStreamSynchronize(comm));
      std::vector<double> gap, load;
      for (int i = 1; i < kProbes; ++i) {
        gap.push_back((double)(s[2 * i] - s[2 * i - 1]) * 10.0);
        load.push_back((double)(s[2 * i + 1] - s[2 * i]) * 10.0 / kLoads);
      }
      std::printf("%-26s %-12s gap median %7.2f us (p90 %7.2f) | per dependent load %7.0f ns\n", c.name,
                  which == 0 ? "no loads" : "8 MiB chain", median(gap) / 1e3,
                  [&] { auto g = gap; std::sort(g.begin(), g.end()); return g[g.size() * 9 / 10] / 1e3; }(),
                  which == 0 ? 0.0 : median(load));
    }
  }
  // register-holding background, one-wave probes and 256-workgroup probes
  uint32_t* wdst = nullptr;
  CHECK(hipMalloc(&wdst, 256 * 256 * 4));
  struct VCase {
    const char* name;
    hipStream_t bg;
    int comm_wgs;
  } vhogs[] = {{"none", nullptr, 0},
               {"vhog on 224-CU mask", main_mask, 0},
               {"vhog on all CUs", main_all, 0},
               {"vhog on mask + 256 COMM wgs", main_mask, 256}};
  for (const VCase& c : vhogs) {
    if (c.bg) hipLaunchKernelGGL(vhog, dim3(224 * 800), dim3(256), 0, c.bg, hog_out, 300);
    if (c.comm_wgs) hipLaunchKernelGGL(vhog, dim3(c.comm_wgs * 100), dim3(256), 0, comm, hog_out, 300);
    for (int i = 0; i < kProbes; ++i)
      hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, side, nullptr, 0u, stamps + 2 * i, sink);
    std::vector<unsigned long long> init(kProbes * 2);
    for (int i = 0; i < kProbes; ++i) init[2 * i] = ~0ull, init[2 * i + 1] = 0ull;
    unsigned long long* wst = nullptr;
    CHECK(hipMalloc(&wst, kProbes * 2 * 8));
    CHECK(hipMemcpy(wst, init.data(), init.size() * 8, hipMemcpyHostToDevice));
    for (int i = 0; i < kProbes; ++i)
      hipLaunchKernelGGL(wide_probe, dim3(256), dim3(256), 0, side, chain_small, wdst, wst + 2 * i);
    CHECK(hipGetLastError());
    CHECK(hipStreamSynchronize(side));
    std::vector<unsigned long long> s(kProbes * 2), w(kProbes * 2);
    CHECK(hipMemcpy(s.data(), stamps, s.size() * 8, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(w.data(), wst, w.size() * 8, hipMemcpyDeviceToHost));
    CHECK(hipDeviceSynchronize());
    CHECK(hipFree(wst));
    std::vector<double> gap, wdur, wgap;
    for (int i = 1; i < kProbes; ++i) {
      gap.push_back((double)(s[2 * i] - s[2 * i - 1]) * 10.0);
      wdur.push_back((double)(w[2 * i + 1] - w[2 * i]) * 10.0);
      wgap.push_back((double)(w[2 * i] - w[2 * i - 1]) * 10.0);
    }
    std::printf("%-28s one-wave gap %6.2f us | 256-wg probe: first start -> last end %6.2f us, gap %6.2f us\n",
                c.name, median(gap) / 1e3, median(wdur) / 1e3, median(wgap) / 1e3);
  }
  CHECK(hipDeviceSynchronize());
  return 0;
}
