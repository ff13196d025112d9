// Shader-clock timeline of the matrix-core block inverse (workgroup 0): per pivot step, per panel.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DGJ_BI_PROBE [-DGJ_BI_PROBE_STEPS] -Icsrc/include \
//         -Icsrc/kernels bench/blockinv_mfma_probe.hip -o build/blockinv_mfma_probe
// (GJ_BI_PROBE_STEPS adds a stamp per pivot step: a memtime read + store each, so the step times it
// prints include that perturbation; compare the panel totals of the two builds)
#include "../csrc/kernels/blockinv_mfma.hip"

#include <cstdio>
#include <random>
#include <vector>

template <int MP, int LAY>
static void run(int m, int nblk) {
  using namespace gj::kern;
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
    hipLaunchKernelGGL((block_inverse_mfma_kernel<double, MP, LAY>), dim3(nblk), dim3(64 * bim_hw_waves<MP, LAY>()), 0, 0, Lt,
                       (int64_t)nblk * m, inv, scores, valid, used, m, (int64_t)1, (int64_t)0, 1e-12, nullptr,
                       gj::PivotSelectArgs{}, 0);
    (void)hipEventRecord(e1, 0);
    (void)hipDeviceSynchronize();
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    unsigned long long pr[1024];
    (void)hipMemcpyFromSymbol(pr, HIP_SYMBOL(g_bim_probe), sizeof(pr));
    if (rep < 2) continue;
    const double t0 = (double)pr[1002];
    std::printf("%s m=%d nblk=%d: kernel %.1f us (event); shader cycles from wave-0 start:\n",
                LAY == 1 ? "pivot-SIMD layout" : "9-wave layout", m, nblk, ms * 1e3);
    std::printf("  load done %.0f | pivot wave at B0(0) %.0f\n", pr[512] - t0, pr[0] - t0);
    for (int q = 0; q < m / 16; ++q) {
      const unsigned long long* P = pr + 8 + 24 * q;
      std::printf("  panel %d: pivot wave start %.0f, factor+publish %.0f, B1 wait %.0f\n", q, P[0] - t0,
                  (double)(P[17] - P[0]), (double)(P[18] - P[17]));
#ifdef GJ_BI_PROBE_STEPS
      std::printf("           steps:");
      for (int j = 0; j < 16; ++j) std::printf(" %.0f", (double)((j < 15 ? P[2 + j] : P[17]) - P[1 + j]));
      std::printf("\n");
#endif
      const unsigned long long* B = pr + 520 + 8 * q;
      std::printf("           block w0: apply %.0f, Xn %.0f, wait B1 %.0f, next tile %.0f, wait B0 %.0f\n",
                  (double)(B[1] - B[0]), (double)(B[2] - B[1]), (double)(B[3] - B[2]),
                  (double)(B[4] - B[3]), q + 1 < m / 16 ? (double)(B[8] - B[4]) : 0.0);
    }
    std::printf("  epilogue (staged output + norm) %.0f; end %.0f\n", (double)(pr[1001] - pr[1000]), pr[1001] - t0);
  }
}

int main() {
  run<128, 1>(128, 32);
  run<128, 0>(128, 32);
  run<64, 0>(64, 32);
  return 0;
}
