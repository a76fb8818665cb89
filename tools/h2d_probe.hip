// h2d_probe: how fast 640 KB of signatures (a 10,000-validator commit) can
// reach a kernel on MI355X (round 6, VERDICT r5 item 3: verify_commit_10k_keyset
// spends ~19 us in its H2D copy and ~8 us between the copy's end and the
// kernel's start). Host-side wall time of each variant, median of 200:
//   copy1      one hipMemcpyAsync + a trivial dependent kernel, sync
//   copy2/4    the same bytes split over 2 / 4 streams with their own queues
//              (copy engines in parallel), the kernel's stream waiting on
//              events
//   mapped     no copy: the kernel reads the bytes from mapped pinned memory
//              (one workgroup per 3 KB, 16-byte loads), sync
//   kernel     the trivial kernel alone, sync (launch + completion floor)
//   hipcc --offload-arch=gfx950 -O2 tools/h2d_probe.hip -o tools/h2d_probe
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
      std::exit(1);                                                                    \
    }                                                                                  \
  } while (0)

// sums its workgroup's slice (so the loads cannot be dropped) into out
__global__ void __launch_bounds__(256) k_touch(const uint4* __restrict__ src, size_t n16, uint32_t* out) {
  const size_t per = (n16 + gridDim.x - 1) / gridDim.x;
  const size_t a = blockIdx.x * per, b = std::min(n16, a + per);
  uint32_t acc = 0;
  for (size_t i = a + threadIdx.x; i < b; i += blockDim.x) {
    const uint4 v = src[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[blockIdx.x] = acc;  // practically never: keeps the loads live
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  const size_t bytes = 640 * 1024, n16 = bytes / 16;
  const int blocks = 210, iters = 200;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const uint32_t words = (cus + 31) / 32;
  std::vector<uint32_t> all(words, 0);
  for (int c = 0; c < cus; c++) all[c / 32] |= 1u << (c % 32);
  hipStream_t s[4];
  for (auto& st : s) CK(hipExtStreamCreateWithCUMask(&st, words, all.data()));
  hipEvent_t ev[4];
  for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  uint8_t* h = nullptr;
  CK(hipHostMalloc(&h, bytes, hipHostMallocPortable | hipHostMallocMapped));
  for (size_t i = 0; i < bytes; i++) h[i] = (uint8_t)(i * 131 + 7);
  uint8_t* dmapped = nullptr;
  CK(hipHostGetDevicePointer((void**)&dmapped, h, 0));
  uint8_t* d = nullptr;
  uint32_t* out = nullptr;
  CK(hipMalloc(&d, bytes));
  CK(hipMalloc(&out, 4 * blocks));
  auto run = [&](const char* name, auto&& body) {
    std::vector<double> t;
    for (int i = 0; i < iters + 20; i++) {
      const double t0 = now_us();
      body();
      CK(hipStreamSynchronize(s[0]));
      if (i >= 20) t.push_back(now_us() - t0);
    }
    std::sort(t.begin(), t.end());
    std::printf("%-8s p50 %7.1f us  p10 %7.1f  p90 %7.1f\n", name, t[t.size() / 2], t[t.size() / 10],
                t[t.size() * 9 / 10]);
  };
  run("kernel", [&] { hipLaunchKernelGGL(k_touch, dim3(blocks), dim3(256), 0, s[0], (const uint4*)d, (size_t)0, out); });
  run("copy1", [&] {
    CK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s[0]));
    hipLaunchKernelGGL(k_touch, dim3(blocks), dim3(256), 0, s[0], (const uint4*)d, n16, out);
  });
  for (int k : {2, 4}) {
    run(k == 2 ? "copy2" : "copy4", [&] {
      const size_t part = bytes / k;
      for (int j = 1; j < k; j++) {
        CK(hipMemcpyAsync(d + j * part, h + j * part, part, hipMemcpyHostToDevice, s[j]));
        CK(hipEventRecord(ev[j], s[j]));
      }
      CK(hipMemcpyAsync(d, h, part, hipMemcpyHostToDevice, s[0]));
      for (int j = 1; j < k; j++) CK(hipStreamWaitEvent(s[0], ev[j], 0));
      hipLaunchKernelGGL(k_touch, dim3(blocks), dim3(256), 0, s[0], (const uint4*)d, n16, out);
    });
  }
  run("mapped", [&] {
    hipLaunchKernelGGL(k_touch, dim3(blocks), dim3(256), 0, s[0], (const uint4*)dmapped, n16, out);
  });
  run("hbm", [&] { hipLaunchKernelGGL(k_touch, dim3(blocks), dim3(256), 0, s[0], (const uint4*)d, n16, out); });
  CK(hipFree(d));
  CK(hipFree(out));
  CK(hipHostFree(h));
  return 0;
}
