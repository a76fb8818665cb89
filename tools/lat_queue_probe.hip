// lat_queue_probe: what delays a small kernel's dispatch on a queue whose CU
// mask holds only CUs a busy masked queue leaves free (round 6: the
// 150-validator commit beside a configs[2] pipeline started 40 or ~450 us
// after its launch, bimodally). A "bulk" thread keeps two long spinning
// launches (2.5 ms, one workgroup of 64 per wave slot it can take on every
// CU but the reserved 16) in flight on a masked queue; a "copy" thread
// streams 48 MB H2D DMAs; the main thread launches a small kernel (4
// workgroups of 320) every 1 ms on the latency queue and times launch ->
// completion on the host. Variants: the latency queue reserved-CU masked or
// a plain stream; preceded by a cross-stream event wait (as LatencyStreams
// does) or not; with and without the copy thread.
//   hipcc --offload-arch=gfx950 -O2 tools/lat_queue_probe.hip -o tools/lat_queue_probe -lpthread
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
      std::exit(1);                                                                    \
    }                                                                                  \
  } while (0)

// spins `ticks` of the 100 MHz wall clock (bounded), doing VALU work
__global__ void __launch_bounds__(64) k_spin(uint32_t* out, uint64_t ticks) {
  const uint64_t t0 = wall_clock64();
  uint32_t a = threadIdx.x, b = blockIdx.x;
  while (wall_clock64() - t0 < ticks) {
#pragma unroll 16
    for (int k = 0; k < 64; k++) {
      a = a * 1664525u + b;
      b ^= a >> 7;
    }
  }
  if (a == 0x9e3779b9u && b == 1u) out[0] = a;  // practically never
}

__global__ void __launch_bounds__(320) k_small(uint32_t* out, uint64_t ticks) {
  const uint64_t t0 = wall_clock64();
  uint32_t a = threadIdx.x;
  while (wall_clock64() - t0 < ticks) a = a * 1664525u + 1013904223u;
  if (a == 0x9e3779b9u) out[1] = a;
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const uint32_t words = (cus + 31) / 32;
  std::vector<uint32_t> all(words, 0), masked, reserved(words, 0);
  for (int c = 0; c < cus; c++) all[c / 32] |= 1u << (c % 32);
  masked = all;
  for (uint32_t k = 0; k < 16; k++) {  // CUs 0, 1 of SE 0 on each XCD (runtime.cpp bulk_lane_init)
    const uint32_t b = ((k / 8) % 2) * 32 + (k % 8);
    masked[b / 32] &= ~(1u << (b % 32));
    reserved[b / 32] |= 1u << (b % 32);
  }
  hipStream_t bulk, copy, lat_masked, lat_plain, other;
  CK(hipExtStreamCreateWithCUMask(&bulk, words, masked.data()));
  CK(hipExtStreamCreateWithCUMask(&copy, words, all.data()));
  CK(hipExtStreamCreateWithCUMask(&lat_masked, words, reserved.data()));
  CK(hipStreamCreateWithFlags(&lat_plain, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&other, hipStreamNonBlocking));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  uint32_t* out = nullptr;
  CK(hipMalloc(&out, 64));
  const size_t cbytes = 48u << 20;
  uint8_t *h = nullptr, *d = nullptr;
  CK(hipHostMalloc(&h, cbytes, hipHostMallocPortable));
  CK(hipMalloc(&d, cbytes));
  std::atomic<bool> stop{false}, copies_on{false};
  const int bulk_waves = 8 * (cus - 16);
  std::thread tb([&] {
    CK(hipSetDevice(0));
    hipEvent_t e2[2];
    for (auto& e : e2) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    int k = 0;
    while (!stop.load()) {
      hipLaunchKernelGGL(k_spin, dim3(bulk_waves), dim3(64), 0, bulk, out, (uint64_t)250000);  // 2.5 ms
      CK(hipEventRecord(e2[k & 1], bulk));
      k++;
      if (k >= 2) CK(hipEventSynchronize(e2[k & 1]));  // two in flight
    }
    CK(hipStreamSynchronize(bulk));
  });
  std::thread tc([&] {
    CK(hipSetDevice(0));
    while (!stop.load()) {
      if (!copies_on.load()) {
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
        continue;
      }
      CK(hipMemcpyAsync(d, h, cbytes, hipMemcpyHostToDevice, copy));
      CK(hipStreamSynchronize(copy));
    }
  });
  std::this_thread::sleep_for(std::chrono::milliseconds(50));
  struct V {
    const char* name;
    hipStream_t s;
    bool wait, copies;
  };
  std::vector<V> vs = {{"reserved-mask queue", lat_masked, false, false},
                       {"reserved-mask queue + event wait", lat_masked, true, false},
                       {"reserved-mask queue, copies on", lat_masked, false, true},
                       {"reserved-mask queue + event wait, copies on", lat_masked, true, true},
                       {"plain stream, copies on", lat_plain, false, true}};
  for (auto& v : vs) {
    copies_on = v.copies;
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
    std::vector<double> t;
    for (int i = 0; i < 400; i++) {
      const double t0 = now_us();
      if (v.wait) {
        CK(hipEventRecord(ev, other));
        CK(hipStreamWaitEvent(v.s, ev, 0));
      }
      hipLaunchKernelGGL(k_small, dim3(4), dim3(320), 0, v.s, out, (uint64_t)1000);  // 10 us
      CK(hipStreamSynchronize(v.s));
      t.push_back(now_us() - t0);
      const double t1 = now_us();
      while (now_us() - t1 < 1000) std::this_thread::yield();
    }
    std::sort(t.begin(), t.end());
    std::printf("%-46s p50 %8.1f us  p90 %8.1f  p99 %8.1f  max %8.1f\n", v.name, t[t.size() / 2],
                t[t.size() * 9 / 10], t[t.size() * 99 / 100], t.back());
    std::fflush(stdout);
  }
  stop = true;
  tb.join();
  tc.join();
  CK(hipFree(out));
  CK(hipFree(d));
  CK(hipHostFree(h));
  return 0;
}
