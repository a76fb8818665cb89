// cumask_probe: how hipExtStreamCreateWithCUMask's bits map to MI355X's CUs,
// and whether a kernel on a plain stream gets the CUs a masked stream's
// kernel leaves free while that kernel holds every other CU (round 6,
// latency_150_under_load). A "hog" kernel (one 100 KB-LDS workgroup per CU,
// each spinning a bounded 20 ms) runs on a stream masked per variant; 5 ms
// later a "probe" kernel of 8 workgroups runs on a full-mask stream. Both
// record (XCC, SE, CU) per workgroup; the probe's host-side wait says whether
// it waited for the hog.
//   hipcc --offload-arch=gfx950 -O2 tools/cumask_probe.hip -o tools/cumask_probe
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <set>
#include <thread>
#include <vector>

#define CK(x)                                                             \
  do {                                                                    \
    hipError_t e_ = (x);                                                  \
    if (e_ != hipSuccess) {                                               \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                       \
    }                                                                     \
  } while (0)

__device__ inline uint32_t where() {
  uint32_t hw, xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  const uint32_t cu = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
  return ((xcc & 15) << 16) | (se << 8) | (sh << 4) | cu;
}

// 100 KB of LDS: one workgroup per CU; spins `ticks` of the 100 MHz wall clock
__global__ void __launch_bounds__(64) k_hog(uint32_t* out, uint64_t ticks) {
  __shared__ uint32_t pad[25 * 1024];
  const uint64_t t0 = wall_clock64();
  uint32_t acc = threadIdx.x;
  while (wall_clock64() - t0 < ticks) {
    pad[(acc * 97 + threadIdx.x) % (25 * 1024)] = acc;
    acc = acc * 1664525u + 1013904223u;
  }
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = where() | (pad[blockIdx.x % 1024] & 0u);
}

__global__ void __launch_bounds__(64) k_probe(uint32_t* out) {
  __shared__ uint32_t pad[25 * 1024];
  pad[threadIdx.x] = threadIdx.x;
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = where() | (pad[1] & 0u);
}

static void show(const char* tag, const std::vector<uint32_t>& w) {
  std::set<uint32_t> s(w.begin(), w.end());
  std::set<uint32_t> xcc;
  for (uint32_t v : s) xcc.insert(v >> 16);
  std::printf("  %s: %zu distinct CUs over %zu XCDs:", tag, s.size(), xcc.size());
  if (s.size() <= 16)
    for (uint32_t v : s) std::printf(" x%u.se%u.sh%u.cu%u", v >> 16, (v >> 8) & 7, (v >> 4) & 1, v & 15);
  std::printf("\n");
}

int main() {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const uint32_t words = (cus + 31) / 32;
  std::vector<uint32_t> all(words, 0);
  for (int c = 0; c < cus; c++) all[c / 32] |= 1u << (c % 32);
  hipStream_t plain;
  CK(hipExtStreamCreateWithCUMask(&plain, words, all.data()));
  const int n_hog = 4 * cus, n_probe = 8;
  uint32_t *d_hog, *d_probe;
  CK(hipMalloc(&d_hog, 4 * n_hog));
  CK(hipMalloc(&d_probe, 4 * n_probe));
  std::printf("%d CUs\n", cus);
  struct Variant {
    const char* name;
    std::vector<int> off;  // mask bits cleared
  };
  std::vector<Variant> vs = {{"no mask", {}},
                             {"bits 0..7 cleared", {0, 1, 2, 3, 4, 5, 6, 7}},
                             {"bits 0,32,..,224 cleared", {0, 32, 64, 96, 128, 160, 192, 224}},
                             {"bits 0..15 cleared", {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}},
                             {"only bits 0..7 set", {-1}}};
  for (auto& v : vs) {
    std::vector<uint32_t> m = all;
    if (!v.off.empty() && v.off[0] == -1) {
      m.assign(words, 0);
      m[0] = 0xFF;
    } else {
      for (int b : v.off) m[b / 32] &= ~(1u << (b % 32));
    }
    hipStream_t hs;
    CK(hipExtStreamCreateWithCUMask(&hs, words, m.data()));
    CK(hipMemset(d_hog, 0xFF, 4 * n_hog));
    CK(hipMemset(d_probe, 0xFF, 4 * n_probe));
    CK(hipDeviceSynchronize());
    // warm both kernels' code objects
    hipLaunchKernelGGL(k_probe, dim3(n_probe), dim3(64), 0, plain, d_probe);
    CK(hipStreamSynchronize(plain));
    const uint64_t ticks = 2'000'000;  // 20 ms at 100 MHz
    hipLaunchKernelGGL(k_hog, dim3(n_hog), dim3(64), 0, hs, d_hog, ticks);
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
    const auto t0 = std::chrono::steady_clock::now();
    hipLaunchKernelGGL(k_probe, dim3(n_probe), dim3(64), 0, plain, d_probe);
    CK(hipStreamSynchronize(plain));
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    const auto t1 = std::chrono::steady_clock::now();
    CK(hipStreamSynchronize(hs));
    const double hog_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count();
    std::vector<uint32_t> h(n_hog), p(n_probe);
    CK(hipMemcpy(h.data(), d_hog, 4 * n_hog, hipMemcpyDeviceToHost));
    CK(hipMemcpy(p.data(), d_probe, 4 * n_probe, hipMemcpyDeviceToHost));
    std::printf("%s: probe waited %.1f us (hog still ran %.1f ms after)\n", v.name, us, hog_ms);
    show("hog", h);
    show("probe", p);
    // CUs the hog never used (sampled over 4 rounds of the chip)
    std::set<uint32_t> used(h.begin(), h.end());
    std::printf("  probe CUs the hog never used:");
    for (uint32_t w : p)
      if (!used.count(w)) std::printf(" x%u.se%u.sh%u.cu%u", w >> 16, (w >> 8) & 7, (w >> 4) & 1, w & 15);
    std::printf("\n");
    CK(hipStreamDestroy(hs));
  }
  // (A single-bit mask leaves seven XCDs with no CU of the queue; the driver
  // then runs those XCDs' share on all their CUs, so one-bit probes say
  // nothing about the map -- and a mask that truly leaves an XCD empty could
  // strand workgroups. Not probed: the "only bits 0..7 set" variant above
  // is the map's evidence.)
  CK(hipFree(d_hog));
  CK(hipFree(d_probe));
  return 0;
}
