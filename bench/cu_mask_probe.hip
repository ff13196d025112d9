// Which CUs does a CU-masked stream actually run on?  (engine.cpp's CU reservation; HipDevice::reserve_cus)
//
//   hipcc --offload-arch=gfx950 -O2 -o build/cu_mask_probe bench/cu_mask_probe.hip && build/cu_mask_probe
//
// For a few masks (bits cleared = CUs kept off the stream) a kernel of 4096 one-wave workgroups, each
// spinning ~20 us, records the hardware id of the CU it ran on (HW_ID: CU / SH / SE, XCC_ID); the
// program prints, per XCC, how many distinct CUs the stream used.  This tells whether mask bit i is
// "CU i of XCD i / 32" (XCD-major) or "CU i / 8 of XCD i % 8" (interleaved).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <set>
#include <string>
#include <vector>

#define CHECK(x)                                                                        \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                     \
    }                                                                                   \
  } while (0)

__global__ void where_kernel(unsigned* out, long long spin_ticks) {
  const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_ID, 32 bits
  const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20);  // XCC_ID, 16 bits
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < spin_ticks) {
  }
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = hw;
    out[2 * blockIdx.x + 1] = xcc;
  }
}

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int ncu = prop.multiProcessorCount;
  const int nwg = 4096;
  unsigned* d;
  CHECK(hipMalloc(&d, sizeof(unsigned) * 2 * nwg));
  std::vector<unsigned> h(2 * nwg);
  int rate = 0;
  CHECK(hipDeviceGetAttribute(&rate, hipDeviceAttributeWallClockRate, 0));  // kHz
  const long long ticks = (long long)rate * 20 / 1000;                      // ~20 us

  struct Case {
    std::string name;
    std::vector<int> off;  // mask bits cleared
  };
  std::vector<Case> cases;
  cases.push_back({"no mask", {}});
  for (int n : {8, 16, 24, 32, 40, 48, 64}) {
    Case c{"first " + std::to_string(n) + " bits off", {}};
    for (int i = 0; i < n; ++i) c.off.push_back(i);
    cases.push_back(c);
  }
  {
    Case c{"bits 32k off (k = 0..7)", {}};
    for (int i = 0; i < 8; ++i) c.off.push_back(32 * i);
    cases.push_back(c);
  }
  std::printf("device: %s, %d CUs, wall clock %d kHz\n", prop.gcnArchName, ncu, rate);
  std::set<unsigned> ref0;
  for (const auto& cs : cases) {
    hipStream_t st;
    if (cs.off.empty()) {
      CHECK(hipStreamCreate(&st));
    } else {
      std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
      for (int c = 0; c < ncu; ++c) mask[c / 32] |= 1u << (c % 32);
      for (int c : cs.off) mask[c / 32] &= ~(1u << (c % 32));
      CHECK(hipExtStreamCreateWithCUMask(&st, (uint32_t)mask.size(), mask.data()));
    }
    CHECK(hipMemsetAsync(d, 0xff, sizeof(unsigned) * 2 * nwg, st));
    hipLaunchKernelGGL(where_kernel, dim3(nwg), dim3(64), 0, st, d, ticks);
    CHECK(hipStreamSynchronize(st));
    CHECK(hipMemcpy(h.data(), d, sizeof(unsigned) * 2 * nwg, hipMemcpyDeviceToHost));
    std::vector<std::set<unsigned>> per_xcc(16);
    std::set<unsigned> all;
    int per_se0[8] = {0};  // XCC 0: distinct CUs per (SE, SH)
    for (int i = 0; i < nwg; ++i) {
      const unsigned hw = h[2 * i], xcc = h[2 * i + 1] & 0xf;
      const unsigned cu = (hw >> 8) & 0xff;  // CU_ID [11:8], SH_ID [12], SE_ID [15:13]
      if (per_xcc[xcc].insert(cu).second && xcc == 0) per_se0[(cu >> 4) & 7]++;
      all.insert((xcc << 8) | cu);
    }
    std::printf("%-26s distinct CUs %3zu | per XCC:", cs.name.c_str(), all.size());
    for (int x = 0; x < 16; ++x)
      if (!per_xcc[x].empty()) std::printf(" %d:%zu", x, per_xcc[x].size());
    std::printf(" | XCC0 per SE/SH:");
    for (int k = 0; k < 8; ++k) std::printf(" %d", per_se0[k]);
    std::printf(" | XCC0 CUs off:");
    if (!cs.off.empty())
      for (unsigned c = 0; c < 256; ++c)
        if (!per_xcc[0].count(c) && ref0.count(c)) std::printf(" %02x", c);
    std::printf("\n");
    if (cs.off.empty()) ref0 = per_xcc[0];
    // the first WGs: which XCC does workgroup i land on?
    if (cs.off.empty()) {
      std::printf("  workgroup -> XCC for wg 0..15:");
      for (int i = 0; i < 16; ++i) std::printf(" %u", h[2 * i + 1] & 0xf);
      std::printf("\n");
    }
    CHECK(hipStreamDestroy(st));
  }
  CHECK(hipFree(d));
  return 0;
}
