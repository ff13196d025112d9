// Dependent-chain latency (shader clocks) of the cross-lane primitives used by the pivot search,
// measured with one wave:  hipcc --offload-arch=gfx950 -O3 -std=c++17 -Icsrc/include -Icsrc/kernels
//                           bench/latency_probe.hip -o build/latency_probe
#include "../csrc/kernels/blockinv.hip"

#include <cstdio>

using namespace gj::kern;

constexpr int N = 1024;

__global__ void probe(double* out, long long* cyc, double seed, int lanesel) {
  const int lane = threadIdx.x;
  double v = seed + lane;
  long long t0, t1;
  // 1. fma chain
  t0 = clock64();
  for (int i = 0; i < N; ++i) v = __builtin_fma(v, 0.999, 1e-3);
  t1 = clock64();
  cyc[0] = t1 - t0;
  // 2. wave max chain
  t0 = clock64();
  for (int i = 0; i < N; ++i) v = wave_max_f64(v) * 0.5 + lane;
  t1 = clock64();
  cyc[1] = t1 - t0;
  // 3. readfirstlane chain
  int r = lane;
  t0 = clock64();
  for (int i = 0; i < N; ++i) r = __builtin_amdgcn_readfirstlane(r + lane) & 63;
  t1 = clock64();
  cyc[2] = t1 - t0;
  // 4. readlane double chain (uniform index)
  t0 = clock64();
  for (int i = 0; i < N; ++i) v = readlane_t(v, (r + i) & 63) + lane;
  t1 = clock64();
  cyc[3] = t1 - t0;
  // 5. rcp chain
  t0 = clock64();
  for (int i = 0; i < N; ++i) v = __builtin_amdgcn_rcp(v) + 1.0;
  t1 = clock64();
  cyc[4] = t1 - t0;
  // 6. dpp only chain
  t0 = clock64();
  for (int i = 0; i < N; ++i) v = dpp64<0xB1>(v) + 1.0;
  t1 = clock64();
  cyc[5] = t1 - t0;
  // 7. permlane32 swap chain
  t0 = clock64();
  for (int i = 0; i < N; ++i) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const auto l = __builtin_amdgcn_permlane32_swap((unsigned)b, (unsigned)b, false, false);
    const auto h = __builtin_amdgcn_permlane32_swap((unsigned)(b >> 32), (unsigned)(b >> 32), false, false);
    v = join64(l[0], h[0]) + 1.0;
  }
  t1 = clock64();
  cyc[6] = t1 - t0;
  // 8. 16 independent readlanes (throughput)
  double acc = 0;
  t0 = clock64();
  for (int i = 0; i < N / 16; ++i) {
#pragma unroll
    for (int k = 0; k < 16; ++k) acc += readlane_t(v + k, (lanesel + k) & 63);
    v += acc * 1e-30;
  }
  t1 = clock64();
  cyc[7] = t1 - t0;
  // 9. v_max_f64 chain
  t0 = clock64();
  for (int i = 0; i < N; ++i) v = fmax(v, v * 0.5) - 1.0;
  t1 = clock64();
  cyc[8] = t1 - t0;
  // 10. s_memrealtime vs clock: 1000 iterations of fma chain in wall_clock64 ticks
  long long w0 = wall_clock64(), c0 = clock64();
  for (int i = 0; i < 4 * N; ++i) v = __builtin_fma(v, 0.999, 1e-3);
  long long w1 = wall_clock64(), c1 = clock64();
  cyc[9] = c1 - c0;
  cyc[10] = w1 - w0;
  out[lane] = v + r + acc;
}

int main() {
  double* out;
  long long* cyc;
  (void)hipMalloc(&out, 64 * 8);
  (void)hipMalloc(&cyc, 16 * 8);
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, out, cyc, 1.0, 3);
    (void)hipDeviceSynchronize();
    long long h[16];
    (void)hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    const char* names[] = {"fma_f64", "wave_max_f64+fma", "readfirstlane", "readlane_f64", "rcp_f64",
                           "dpp64", "permlane32_swap64", "readlane_f64 x16 indep (per op)", "max_f64"};
    for (int i = 0; i < 9; ++i) std::printf("%-34s %7.1f clk/iter\n", names[i], (double)h[i] / N);
    std::printf("clock64 %lld cycles in %lld x 10ns -> %.2f GHz\n", h[9], h[10], h[9] / (h[10] * 10.0));
  }
  return 0;
}
