// Microbenchmark: how VALU issue scales with waves per SIMD on gfx950.
// Each wave runs a field-multiply-like instruction mix (v_mad_u64_u32 +
// v_add_u32 + v_lshrrev_b64, NCH independent chains per lane); the grid is
// W x 1024 single-wave blocks for W = 0.5 .. 4 waves per SIMD. If one wave
// alone already saturates its SIMD, time grows linearly with W; if a lone
// wave only uses part of the SIMD's issue slots, W = 2 costs less than 2x.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define ITERS 4096

template <int NCH>
__global__ __launch_bounds__(64) void k_mix(uint64_t* out, uint32_t seed) {
  const uint32_t tid = blockIdx.x * 64 + threadIdx.x;
  uint64_t acc[NCH];
  uint32_t a = seed ^ tid, b = seed * 2654435761u + tid, c32[NCH];
  for (int c = 0; c < NCH; ++c) {
    acc[c] = a + c * 977u;
    c32[c] = b + c;
  }
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      // 2 mads, 1 add, 1 64-bit shift: the ratio of a carried field product
      asm volatile(
          "v_mad_u64_u32 %0, vcc, %2, %3, %0\n\t"
          "v_mad_u64_u32 %0, vcc, %3, %2, %0\n\t"
          "v_add_u32 %1, %1, %2\n\t"
          "v_lshrrev_b64 %0, 1, %0"
          : "+v"(acc[c]), "+v"(c32[c])
          : "v"(a), "v"(b)
          : "vcc");
    }
  }
  uint64_t r = 0;
  for (int c = 0; c < NCH; ++c) r ^= acc[c] ^ c32[c];
  out[tid] = r;
}

template <int NCH>
static void run(const char* name) {
  const int fracs_x2[] = {1, 2, 3, 4, 6, 8};
  uint64_t* d;
  (void)hipMalloc(&d, (size_t)4 * 1024 * 64 * sizeof(uint64_t));
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int f : fracs_x2) {
    const int grid = 512 * f;  // f/2 waves per SIMD (1024 SIMDs)
    hipLaunchKernelGGL(k_mix<NCH>, dim3(grid), dim3(64), 0, 0, d, 1u);
    (void)hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
      (void)hipEventRecord(e0);
      hipLaunchKernelGGL(k_mix<NCH>, dim3(grid), dim3(64), 0, 0, d, (uint32_t)r);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) best = ms;
    }
    const double insts = (double)ITERS * NCH * 4;  // per wave
    printf("{\"chains\": %d, \"mix\": \"%s\", \"waves_per_simd\": %.1f, \"ms\": %.4f, "
           "\"cyc_per_wave_inst_at_2p4\": %.2f}\n",
           NCH, name, f / 2.0, best, best * 1e-3 * 2.4e9 / insts);
  }
  (void)hipFree(d);
}

int main() {
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  printf("# device %s CUs %d\n", p.gcnArchName, p.multiProcessorCount);
  run<1>("2 mad + add + shr64, dependent");
  run<2>("2 mad + add + shr64");
  run<4>("2 mad + add + shr64");
  run<8>("2 mad + add + shr64");
  return 0;
}
