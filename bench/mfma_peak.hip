// Microbenchmark: sustained f64 / f32 MFMA rate on gfx950 (operands in registers, independent
// accumulators, every CU busy).  Establishes the ceiling the elimination GEMM is measured against.
//   hipcc --offload-arch=gfx950 -O3 bench/mfma_peak.hip -o build/mfma_peak && build/mfma_peak
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ __launch_bounds__(256) void f64_loop(double* out, int iters, double seed) {
  d4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = d4{0, 0, 0, 0};
  double a = seed + threadIdx.x * 1e-3, b = seed * 0.5;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NACC>
__global__ __launch_bounds__(256) void f32_loop(float* out, int iters, float seed) {
  f4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = f4{0, 0, 0, 0};
  float a = seed + threadIdx.x * 1e-3f, b = seed * 0.5f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
  }
  float s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void fma64_loop(double* out, int iters, double seed) {
  double x[8];
  for (int i = 0; i < 8; ++i) x[i] = seed + i + threadIdx.x;
  const double y = 1.0000001, z = 1e-9;
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = fma(x[i], y, z);
  double s = 0;
  for (int i = 0; i < 8; ++i) s += x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// mixed: waves with (wave_id % 2 == 0) issue f64 MFMA, the others f64 VALU FMA
__global__ __launch_bounds__(256) void mixed_loop(double* out, int iters, double seed) {
  const int w = threadIdx.x >> 6;
  double s = 0;
  if (w % 2 == 0) {
    d4 acc[8];
    for (int i = 0; i < 8; ++i) acc[i] = d4{0, 0, 0, 0};
    double a = seed + threadIdx.x * 1e-3, b = seed * 0.5;
    for (int it = 0; it < iters; ++it)
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
    for (int i = 0; i < 8; ++i) s += acc[i][0];
  } else {
    double x[8];
    for (int i = 0; i < 8; ++i) x[i] = seed + i + threadIdx.x;
    const double y = 1.0000001, z = 1e-9;
    // 8 MFMA (2048 flops/lane-wave each = 32 flops per lane) ~ 256 flops/lane per iter -> 128 FMAs
    for (int it = 0; it < iters * 16; ++it)
#pragma unroll
      for (int i = 0; i < 8; ++i) x[i] = fma(x[i], y, z);
    for (int i = 0; i < 8; ++i) s += x[i];
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename K, typename... Args>
static float timeit(K kern, int blocks, int threads, Args... args) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, args...);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, args...);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms;
}

int main() {
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  const int cus = prop.multiProcessorCount;
  const int threads = 256, iters = 20000;
  double* d;
  (void)hipMalloc(&d, sizeof(double) * cus * 8 * threads);
  for (int bpc : {1, 2, 4, 8}) {
    const int blocks = cus * bpc;
    const double waves = blocks * (threads / 64.0);
    float ms = timeit(f64_loop<8>, blocks, threads, d, iters, 1.0);
    printf("{\"kernel\": \"mfma_f64_16x16x4 acc8\", \"waves_per_simd\": %d, \"tflops\": %.2f}\n", bpc,
           2048.0 * 8 * iters * waves / ms / 1e9);
    ms = timeit(f64_loop<16>, blocks, threads, d, iters, 1.0);
    printf("{\"kernel\": \"mfma_f64_16x16x4 acc16\", \"waves_per_simd\": %d, \"tflops\": %.2f}\n", bpc,
           2048.0 * 16 * iters * waves / ms / 1e9);
    ms = timeit(f32_loop<8>, blocks, threads, (float*)d, iters, 1.0f);
    printf("{\"kernel\": \"mfma_f32_16x16x4 acc8\", \"waves_per_simd\": %d, \"tflops\": %.2f}\n", bpc,
           2048.0 * 8 * iters * waves / ms / 1e9);
    ms = timeit(fma64_loop, blocks, threads, d, iters * 4, 1.0);
    printf("{\"kernel\": \"v_fma_f64\", \"waves_per_simd\": %d, \"tflops\": %.2f}\n", bpc,
           2.0 * 8 * iters * 4.0 * blocks * threads / ms / 1e9);
    ms = timeit(mixed_loop, blocks, threads, d, iters, 1.0);
    // half the waves: 8 MFMA/iter (16384 flops/wave), half: 16*8 FMA per lane (8192... per wave 64*2*128)
    const double fl = waves / 2 * (2048.0 * 8 * iters) + waves / 2 * (64.0 * 2 * 8 * 16 * iters);
    printf("{\"kernel\": \"mixed mfma+valu f64\", \"waves_per_simd\": %d, \"tflops\": %.2f}\n", bpc, fl / ms / 1e9);
  }
  (void)hipFree(d);
  return 0;
}
