// Microbenchmark: sustained f64 / f32 MFMA rate on gfx950 -- the roofline denominator the
// elimination GEMM is measured against (VERDICT r5 "the roofline denominator is not measured").
//
//   hipcc --offload-arch=gfx950 -O3 bench/mfma_peak.hip -o build/mfma_peak
//   build/mfma_peak [seconds]        # burst table, then a sustained run of `seconds` (default 20)
//
// Operands stay in registers, NACC independent accumulators per wave, every CU busy.  The
// accumulators are tied to VGPRs through inline asm ("+v"): the round-1..5 version let the compiler
// keep them in AGPRs and copy all of them AGPR -> VGPR -> AGPR around every loop iteration (64
// v_accvgpr reads + 64 writes per 8 MFMAs), which is why it reported 49 TF/s, below the production
// GEMM's 65-67 TF/s.  gfx950 MFMAs read and write the accumulator in VGPRs directly.
//
// The sustained run launches the best burst configuration back to back for `seconds` and prints
// one line per ~0.5 s window, so the rate under the same sustained load as the 25-solve bench
// (power / clock settling) is measured, not only a cold burst.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

typedef double d4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));

#define HIP_OK(x)                                                              \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)

template <int NACC>
__global__ __launch_bounds__(256) void f64_loop(double* out, int iters, double seed) {
  d4 acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = d4{0, 0, 0, 0};
  const double a = seed + threadIdx.x * 1e-3, b = seed * 0.5;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i)
      asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+v"(acc[i]) : "v"(a), "v"(b));
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NACC>
__global__ __launch_bounds__(256) void f32_loop(float* out, int iters, float seed) {
  f4 acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = f4{0, 0, 0, 0};
  const float a = seed + threadIdx.x * 1e-3f, b = seed * 0.5f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i)
      asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+v"(acc[i]) : "v"(a), "v"(b));
  }
  float s = 0;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void fma64_loop(double* out, int iters, double seed) {
  double x[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) x[i] = seed + i + threadIdx.x;
  const double y = 1.0000001, z = 1e-9;
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = fma(x[i], y, z);
  double s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename K, typename... Args>
static float timeit(K kern, int blocks, int threads, Args... args) {
  hipEvent_t e0, e1;
  HIP_OK(hipEventCreate(&e0));
  HIP_OK(hipEventCreate(&e1));
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, args...);
  HIP_OK(hipDeviceSynchronize());
  HIP_OK(hipEventRecord(e0));
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, args...);
  HIP_OK(hipEventRecord(e1));
  HIP_OK(hipEventSynchronize(e1));
  float ms;
  HIP_OK(hipEventElapsedTime(&ms, e0, e1));
  HIP_OK(hipEventDestroy(e0));
  HIP_OK(hipEventDestroy(e1));
  return ms;
}

int main(int argc, char** argv) {
  const double sustain_s = argc > 1 ? std::atof(argv[1]) : 20.0;
  hipDeviceProp_t prop;
  HIP_OK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const int threads = 256, iters = 4000;
  double* d;
  HIP_OK(hipMalloc(&d, sizeof(double) * cus * 8 * threads));
  double best = 0;
  int best_bpc = 1;
  for (int bpc : {1, 2, 4}) {  // 256-thread blocks per CU = waves per SIMD
    const int blocks = cus * bpc;
    const double waves = blocks * (threads / 64.0);
    float ms = timeit(f64_loop<4>, blocks, threads, d, iters, 1.0);
    std::printf("{\"kernel\": \"mfma_f64_16x16x4 acc4\", \"waves_per_simd\": %d, \"tflops\": %.2f}\n", bpc,
                2048.0 * 4 * iters * waves / ms / 1e9);
    ms = timeit(f64_loop<8>, blocks, threads, d, iters, 1.0);
    const double tf8 = 2048.0 * 8 * iters * waves / ms / 1e9;
    std::printf("{\"kernel\": \"mfma_f64_16x16x4 acc8\", \"waves_per_simd\": %d, \"tflops\": %.2f}\n", bpc, tf8);
    if (tf8 > best) best = tf8, best_bpc = bpc;
    ms = timeit(f64_loop<16>, blocks, threads, d, iters, 1.0);
    std::printf("{\"kernel\": \"mfma_f64_16x16x4 acc16\", \"waves_per_simd\": %d, \"tflops\": %.2f}\n", bpc,
                2048.0 * 16 * iters * waves / ms / 1e9);
    ms = timeit(f32_loop<8>, blocks, threads, (float*)d, iters, 1.0f);
    std::printf("{\"kernel\": \"mfma_f32_16x16x4 acc8\", \"waves_per_simd\": %d, \"tflops\": %.2f}\n", bpc,
                2048.0 * 8 * iters * waves / ms / 1e9);
    ms = timeit(fma64_loop, blocks, threads, d, iters * 4, 1.0);
    std::printf("{\"kernel\": \"v_fma_f64\", \"waves_per_simd\": %d, \"tflops\": %.2f}\n", bpc,
                2.0 * 8 * iters * 4.0 * blocks * threads / ms / 1e9);
  }
  std::fflush(stdout);
  // sustained: the best f64 burst configuration back to back, one line per ~0.5 s window
  const int blocks = cus * best_bpc;
  const double waves = blocks * (threads / 64.0);
  const double flop_per_launch = 2048.0 * 8 * iters * waves;
  hipEvent_t e0, e1;
  HIP_OK(hipEventCreate(&e0));
  HIP_OK(hipEventCreate(&e1));
  const auto t0 = std::chrono::steady_clock::now();
  double elapsed = 0, lo = 1e30, hi = 0, sum = 0;
  int windows = 0;
  while (elapsed < sustain_s) {
    HIP_OK(hipEventRecord(e0));
    int launches = 0;
    float ms = 0;
    do {  // ~0.5 s of launches per window
      for (int i = 0; i < 8; ++i, ++launches)
        hipLaunchKernelGGL(f64_loop<8>, dim3(blocks), dim3(threads), 0, 0, d, iters, 1.0);
      HIP_OK(hipEventRecord(e1));
      HIP_OK(hipEventSynchronize(e1));
      HIP_OK(hipEventElapsedTime(&ms, e0, e1));
    } while (ms < 500.f);
    const double tf = flop_per_launch * launches / ms / 1e9;
    elapsed = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::printf("{\"kernel\": \"sustained mfma_f64 acc8\", \"waves_per_simd\": %d, \"t_s\": %.2f, \"tflops\": %.2f}\n",
                best_bpc, elapsed, tf);
    std::fflush(stdout);
    lo = tf < lo ? tf : lo;
    hi = tf > hi ? tf : hi;
    sum += tf;
    ++windows;
  }
  std::printf("{\"kernel\": \"sustained mfma_f64 acc8 summary\", \"burst_tflops\": %.2f, \"sustained_mean\": %.2f, "
              "\"sustained_min\": %.2f, \"sustained_max\": %.2f, \"seconds\": %.1f}\n",
              best, sum / windows, lo, hi, elapsed);
  HIP_OK(hipFree(d));
  return 0;
}
