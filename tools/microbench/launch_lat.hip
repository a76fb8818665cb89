// Microbenchmark: what a single small launch costs on top of its waves' own
// time -- the gap between the 150-validator row kernel's wave timeline
// (tools/row_phase.py: ~87 us from the first wave's entry to the verdict)
// and its event-timed duration (~105 us).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/microbench/launch_lat tools/microbench/launch_lat.hip
//
// Each variant launches 150 workgroups of 256 threads (the row4 shape), one
// launch at a time with a stream synchronisation after each (the VerifyCommit
// call pattern), and prints per launch: the host wall time of launch + sync,
// the event-timed duration, and -- for the spinning variants -- the spin the
// waves were asked for (s_memrealtime, 100 MHz), so the difference is the
// launch's fixed cost.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
      return 1;                                                                     \
    }                                                                               \
  } while (0)

__global__ __launch_bounds__(256, 1) void k_empty(uint32_t* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && out) out[0] = 1;
}

__global__ __launch_bounds__(256, 1) void k_lds(uint32_t* out) {
  __shared__ uint32_t buf[22952 / 4];
  buf[threadIdx.x] = threadIdx.x;
  __syncthreads();
  if (threadIdx.x == 0 && blockIdx.x == 0 && out) out[0] = buf[5];
}

// every wave spins until `ticks` of the 100 MHz constant clock have passed
// since its own entry; lane 0 of wave 0 records its entry and exit stamps
__global__ __launch_bounds__(256, 1) void k_spin(uint64_t ticks, uint64_t* stamps, uint32_t* out) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint64_t t = t0;
  while (t - t0 < ticks) t = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    stamps[2 * blockIdx.x] = t0;
    stamps[2 * blockIdx.x + 1] = t;
  }
  if (threadIdx.x == 0 && out) out[blockIdx.x] = 1;
}

// the spin with a private (scratch) array indexed by a runtime value, as the
// row kernels' 48 bytes of scratch
__global__ __launch_bounds__(256, 1) void k_spin_scratch(uint64_t ticks, uint64_t* stamps, uint32_t* out, uint32_t k) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  volatile uint32_t priv[12];
  for (int i = 0; i < 12; i++) priv[i] = i * threadIdx.x;
  uint64_t t = t0;
  while (t - t0 < ticks) t = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    stamps[2 * blockIdx.x] = t0;
    stamps[2 * blockIdx.x + 1] = t;
  }
  if (threadIdx.x == 0 && out) out[blockIdx.x] = priv[k % 12];
}

// the spin followed by a long straight-line body run once (~2k instructions
// per block below x 32 blocks: a code footprint like the row kernels')
#define BIG8(i) x = x * 0x9E3779B9u + (i); x ^= x >> 13; x = x * 0x85EBCA6Bu + (i) * 7u; x ^= x >> 16; \
  x = __builtin_amdgcn_alignbit(x, x ^ (i), (i) & 31); x += __builtin_amdgcn_readfirstlane(x) ^ (i); \
  x = x * 0xC2B2AE35u + (i); x ^= x << 5;
#define BIG64(i) BIG8(i) BIG8(i + 1) BIG8(i + 2) BIG8(i + 3) BIG8(i + 4) BIG8(i + 5) BIG8(i + 6) BIG8(i + 7)
#define BIG512(i) BIG64(i) BIG64(i + 8) BIG64(i + 16) BIG64(i + 24) BIG64(i + 32) BIG64(i + 40) BIG64(i + 48) BIG64(i + 56)
__global__ __launch_bounds__(256, 1) void k_spin_bigcode(uint64_t ticks, uint64_t* stamps, uint32_t* out) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = threadIdx.x;
  BIG512(1) BIG512(1001) BIG512(2001) BIG512(3001)
  uint64_t t = t0;
  while (t - t0 < ticks) t = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    stamps[2 * blockIdx.x] = t0;
    stamps[2 * blockIdx.x + 1] = t;
  }
  if (out) out[blockIdx.x * 256 + threadIdx.x] = x;
}

// the spin, then the row kernels' bitmap epilogue: each wave writes its
// verdict byte, a release fence and an agent-scope acq_rel ticket; the last
// wave packs the bytes into bitmap words and resets the counter.
// FENCE = 1: __threadfence() + acq_rel atomic (the round-4 code: the memory
// model's agent-scope release/acquire, an L2 writeback + invalidate per wave
// on gfx950); FENCE = 0: the bytes as agent-scope relaxed atomic stores
// (written through to the coherence point), a vmcnt wait, a relaxed ticket,
// the last wave reading them with agent-scope relaxed atomic loads.
template <int FENCE>
__global__ __launch_bounds__(256, 1) void k_spin_ticket(uint64_t ticks, uint64_t* stamps, uint32_t* slot,
                                                        uint64_t* bitmap, uint32_t n) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint64_t t = t0;
  while (t - t0 < ticks) t = __builtin_amdgcn_s_memrealtime();
  const uint32_t tl = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (threadIdx.x == 0) {
    stamps[2 * blockIdx.x] = t0;
    stamps[2 * blockIdx.x + 1] = t;
  }
  if (wave != 0) return;
  uint8_t* vb = reinterpret_cast<uint8_t*>(slot + 16);
  uint32_t ticket = 0;
  if (FENCE) {
    if (tl == 0) vb[blockIdx.x] = 1;
    __threadfence();
    if (tl == 0) ticket = __hip_atomic_fetch_add(slot, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    if (tl == 0) __hip_atomic_store(vb + blockIdx.x, (uint8_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_s_waitcnt(0);
    if (tl == 0) ticket = __hip_atomic_fetch_add(slot, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  ticket = __shfl(ticket, 0);
  if (ticket != gridDim.x - 1) return;
  if (FENCE) __threadfence();
  const uint32_t words = (n + 63) / 64;
  for (uint32_t w = tl; w < words; w += 64) {
    uint64_t m = 0;
    for (uint32_t b = 0; b < 64 && 64 * w + b < n; b++) {
      const uint8_t v = FENCE ? vb[64 * w + b] : __hip_atomic_load(vb + 64 * w + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      m |= (uint64_t)(v != 0) << b;
    }
    bitmap[w] = m;
  }
  if (tl == 0) __hip_atomic_store(slot, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// the spin, then kernels.hip row_bitmap_add's epilogue: one relaxed 64-bit
// atomic add of a 2-bit verdict field per wave; the wave that fills a word's
// last field packs it with a ballot (no fence, no serial byte loop)
__global__ __launch_bounds__(256, 1) void k_spin_fields(uint64_t ticks, uint64_t* stamps, uint32_t* slot,
                                                        uint64_t* bitmap, uint32_t n) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint64_t t = t0;
  while (t - t0 < ticks) t = __builtin_amdgcn_s_memrealtime();
  const uint32_t tl = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (threadIdx.x == 0) {
    stamps[2 * blockIdx.x] = t0;
    stamps[2 * blockIdx.x + 1] = t;
  }
  if (wave != 0) return;
  uint64_t* sw = reinterpret_cast<uint64_t*>(slot);
  const uint32_t s = blockIdx.x, j = s >> 5, f = s & 31;
  uint64_t x = 0;
  if (tl == 0) {
    const uint64_t add = 2ull << (2 * f);
    x = __hip_atomic_fetch_add(sw + j, add, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + add;
  }
  x = __shfl(x, 0);
  const uint32_t nf = n - 32 * j < 32 ? n - 32 * j : 32u;
  const uint64_t m = 0x5555555555555555ull >> (64 - 2 * nf);
  if (((x | (x >> 1)) & m) != m) return;
  const uint64_t acc = __ballot(tl < 32 && ((x >> (2 * (tl & 31) + 1)) & 1) != 0);
  if (tl == 0) {
    uint32_t* ob = reinterpret_cast<uint32_t*>(bitmap);
    ob[j] = (uint32_t)acc;
    if ((j & 1) == 0 && 32 * (j + 1) >= n) ob[j + 1] = 0u;
    __hip_atomic_store(sw + j, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// the spin, then the field epilogue, and the wave that completes the last
// word writes `seq` into a flag in mapped host memory (system-scope release):
// the host can poll that flag instead of synchronising the stream
__global__ __launch_bounds__(256, 1) void k_spin_flag(uint64_t ticks, uint64_t* stamps, uint32_t* slot,
                                                      uint32_t* hbm, uint32_t n, uint32_t* hflag, uint32_t seq) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint64_t t = t0;
  while (t - t0 < ticks) t = __builtin_amdgcn_s_memrealtime();
  const uint32_t tl = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (threadIdx.x == 0) {
    stamps[2 * blockIdx.x] = t0;
    stamps[2 * blockIdx.x + 1] = t;
  }
  if (wave != 0) return;
  uint64_t* sw = reinterpret_cast<uint64_t*>(slot);
  const uint32_t s = blockIdx.x, j = s >> 5, f = s & 31;
  uint64_t x = 0;
  if (tl == 0) {
    const uint64_t add = 2ull << (2 * f);
    x = __hip_atomic_fetch_add(sw + j, add, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + add;
  }
  x = __shfl(x, 0);
  const uint32_t nf = n - 32 * j < 32 ? n - 32 * j : 32u;
  const uint64_t m = 0x5555555555555555ull >> (64 - 2 * nf);
  if (((x | (x >> 1)) & m) != m) return;
  const uint64_t acc = __ballot(tl < 32 && ((x >> (2 * (tl & 31) + 1)) & 1) != 0);
  if (tl == 0) {
    __hip_atomic_store(hbm + j, (uint32_t)acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(sw + j, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __threadfence_system();
    const uint32_t words = (n + 31) / 32;
    const uint32_t done = __hip_atomic_fetch_add(slot + 1020, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (done == words - 1) {
      __hip_atomic_store(slot + 1020, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(hflag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

static double med(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main() {
  const int grid = 150, iters = 300;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  uint32_t* dout;
  uint64_t* dst;
  CK(hipMalloc(&dout, grid * 256 * 4));
  CK(hipMalloc(&dst, grid * 16));
  uint32_t* hout;  // pinned host memory written by the kernel (zero-copy output)
  CK(hipHostMalloc(&hout, 4096, hipHostMallocMapped));
  uint32_t* hdev;
  CK(hipHostGetDevicePointer((void**)&hdev, hout, 0));
  std::vector<uint64_t> hst(grid * 2);

  auto run = [&](const char* name, auto launch, uint64_t spin_ticks) -> int {
    std::vector<double> wall, ev, span;
    for (int i = 0; i < iters + 20; i++) {
      auto t = std::chrono::steady_clock::now();
      CK(hipEventRecord(e0, s));
      launch();
      CK(hipEventRecord(e1, s));
      CK(hipStreamSynchronize(s));
      const double w = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t).count();
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (i < 20) continue;
      wall.push_back(w);
      ev.push_back(ms * 1e3);
      if (spin_ticks) {
        CK(hipMemcpy(hst.data(), dst, grid * 16, hipMemcpyDeviceToHost));
        uint64_t lo = ~0ull, hi = 0;
        for (int b = 0; b < grid; b++) {
          lo = std::min(lo, hst[2 * b]);
          hi = std::max(hi, hst[2 * b + 1]);
        }
        span.push_back((hi - lo) * 0.01);  // first entry .. last exit, us
      }
    }
    printf("%-28s wall %7.2f us  event %7.2f us", name, med(wall), med(ev));
    if (spin_ticks) printf("  waves %7.2f us  event - waves %6.2f us", med(span), med(ev) - med(span));
    printf("\n");
    return 0;
  };
  if (run("empty", [&] { hipLaunchKernelGGL(k_empty, dim3(grid), dim3(256), 0, s, dout); }, 0)) return 1;
  if (run("lds 22.9 KiB", [&] { hipLaunchKernelGGL(k_lds, dim3(grid), dim3(256), 0, s, dout); }, 0)) return 1;
  for (uint64_t us : {10ull, 40ull, 85ull}) {
    char nm[64];
    snprintf(nm, sizeof nm, "spin %llu us", (unsigned long long)us);
    if (run(nm, [&] { hipLaunchKernelGGL(k_spin, dim3(grid), dim3(256), 0, s, us * 100, dst, dout); }, us * 100)) return 1;
    snprintf(nm, sizeof nm, "spin %llu us, host output", (unsigned long long)us);
    if (run(nm, [&] { hipLaunchKernelGGL(k_spin, dim3(grid), dim3(256), 0, s, us * 100, dst, hdev); }, us * 100)) return 1;
  }
  if (run("spin 85 us, 48 B scratch", [&] { hipLaunchKernelGGL(k_spin_scratch, dim3(grid), dim3(256), 0, s, 8500ull, dst, dout, 3u); }, 8500)) return 1;
  if (run("spin 85 us, big code", [&] { hipLaunchKernelGGL(k_spin_bigcode, dim3(grid), dim3(256), 0, s, 8500ull, dst, dout); }, 8500)) return 1;
  uint32_t* slot;
  uint64_t* bm;
  CK(hipMalloc(&slot, 4096));
  CK(hipMemset(slot, 0, 4096));
  CK(hipMalloc(&bm, 64));
  if (run("spin 85 us, fenced ticket", [&] { hipLaunchKernelGGL(k_spin_ticket<1>, dim3(grid), dim3(256), 0, s, 8500ull, dst, slot, bm, (uint32_t)grid); }, 8500)) return 1;
  if (run("spin 85 us, relaxed ticket", [&] { hipLaunchKernelGGL(k_spin_ticket<0>, dim3(grid), dim3(256), 0, s, 8500ull, dst, slot, bm, (uint32_t)grid); }, 8500)) return 1;
  if (run("spin 85 us, field atomics", [&] { hipLaunchKernelGGL(k_spin_fields, dim3(grid), dim3(256), 0, s, 8500ull, dst, slot, bm, (uint32_t)grid); }, 8500)) return 1;
  {
    // the flag variant: host polls the mapped flag, no stream synchronisation
    uint32_t* hflag;
    CK(hipHostMalloc(&hflag, 64, hipHostMallocMapped | hipHostMallocCoherent));
    uint32_t* dflag;
    CK(hipHostGetDevicePointer((void**)&dflag, hflag, 0));
    uint32_t* hbm2;
    CK(hipHostMalloc(&hbm2, 64, hipHostMallocMapped | hipHostMallocCoherent));
    uint32_t* dbm2;
    CK(hipHostGetDevicePointer((void**)&dbm2, hbm2, 0));
    *hflag = 0;
    std::vector<double> wall_sync, wall_flag;
    for (int mode = 0; mode < 2; mode++) {
      for (int i = 0; i < iters + 20; i++) {
        const uint32_t seq = (uint32_t)(mode * 100000 + i + 1);
        auto t = std::chrono::steady_clock::now();
        hipLaunchKernelGGL(k_spin_flag, dim3(grid), dim3(256), 0, s, 8500ull, dst, slot, dbm2, (uint32_t)grid, dflag, seq);
        if (mode == 0) {
          CK(hipStreamSynchronize(s));
        } else {
          volatile uint32_t* vf = hflag;
          long spins = 0;
          while (*vf != seq && ++spins < 2000000000L) {
          }
        }
        const double w = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t).count();
        if (mode == 1) CK(hipStreamSynchronize(s));  // outside the timed part (the next call would not wait)
        if (i >= 20) (mode ? wall_flag : wall_sync).push_back(w);
      }
    }
    printf("%-28s wall %7.2f us (stream sync)  %7.2f us (host polls the flag)\n", "spin 85 us, flag epilogue",
           med(wall_sync), med(wall_flag));
  }
  uint64_t hb[3];
  CK(hipMemcpy(hb, bm, sizeof hb, hipMemcpyDeviceToHost));
  printf("bitmap %016llx %016llx %016llx\n", (unsigned long long)hb[0], (unsigned long long)hb[1], (unsigned long long)hb[2]);
  return 0;
}
