// Phase timestamps of the panel-blocked block inverse (workgroup 0), to locate its latency.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DGJ_BI_PROBE -Icsrc/include -Icsrc/kernels \
//         bench/blockinv_probe.hip -o build/blockinv_probe
#include "../csrc/kernels/blockinv.hip"

#include <cstdio>
#include <random>
#include <vector>

int main() {
  using namespace gj::kern;
  const int m = 128, nblk = 32;
  std::vector<double> h((size_t)m * nblk * m);
  std::mt19937_64 rng(1);
  std::uniform_real_distribution<double> U(-1, 1);
  for (auto& x : h) x = U(rng);
  double *Lt, *inv, *scores;
  int *valid, *used;
  (void)hipMalloc(&Lt, h.size() * 8);
  (void)hipMalloc(&inv, h.size() * 8);
  (void)hipMalloc(&scores, nblk * 8);
  (void)hipMalloc(&valid, nblk * 4);
  (void)hipMalloc(&used, nblk * 4);
  (void)hipMemset(used, 0, nblk * 4);
  (void)hipMemcpy(Lt, h.data(), h.size() * 8, hipMemcpyHostToDevice);
  for (int rep = 0; rep < 3; ++rep) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL((block_inverse_panel_kernel<double, 128, 512>), dim3(nblk), dim3(512), 0, 0, Lt,
                       (int64_t)nblk * m, inv, scores, valid, used, m, (int64_t)1, (int64_t)0, 1e-12);
    (void)hipEventRecord(e1, 0);
    (void)hipDeviceSynchronize();
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    unsigned long long pr[256];
    (void)hipMemcpyFromSymbol(pr, HIP_SYMBOL(g_bi_probe), sizeof(pr));
    std::printf("rep %d: kernel %.1f us; wall_clock64 is 100 MHz (10 ns ticks)\n", rep, ms * 1e3);
    const double t0 = (double)pr[0];
    for (int c = 0; c < m / 16; ++c)
      std::printf("  panel %d: start %.2f us  publish %.2f  phaseA %.2f  rbuf %.2f  phaseB %.2f\n", c,
                  (pr[1 + 4 * c] - t0) / 100.0, (pr[2 + 4 * c] - pr[1 + 4 * c]) / 100.0,
                  (pr[3 + 4 * c] - pr[2 + 4 * c]) / 100.0, (pr[4 + 4 * c] - pr[3 + 4 * c]) / 100.0,
                  ((c + 1 < m / 16 ? pr[1 + 4 * (c + 1)] : pr[100]) - pr[4 + 4 * c]) / 100.0);
    std::printf("  end %.2f us\n", (pr[100] - t0) / 100.0);
  }
  return 0;
}
