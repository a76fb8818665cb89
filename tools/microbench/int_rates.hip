// Microbenchmark: per-instruction VALU throughput on gfx950 for the
// instructions a GF(2^255-19) field multiply can be built from.
// Each lane runs NCH independent dependency chains of one instruction;
// result = wave-instructions/s and lane-ops/s over the whole chip.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define NCH 8
#define ITERS 16384

#define K_BEGIN(name, T) __global__ void name(T* out, uint32_t seed) { \
  uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x; \
  T acc[NCH]; uint32_t a = seed ^ tid, b = seed * 2654435761u + tid; \
  for (int c = 0; c < NCH; ++c) acc[c] = (T)(a + c * 977u);
#define K_END(T) T r = 0; for (int c = 0; c < NCH; ++c) r ^= acc[c]; out[tid] = r; }

K_BEGIN(k_mad_u64_u32, uint64_t)
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < NCH; ++c)
      asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc[c]) : "v"(a), "v"(b) : "vcc");
  }
K_END(uint64_t)

K_BEGIN(k_mul_lo_u32, uint32_t)
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < NCH; ++c)
      asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(acc[c]) : "v"(b));
  }
K_END(uint32_t)

K_BEGIN(k_mul_hi_u32, uint32_t)
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < NCH; ++c)
      asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(acc[c]) : "v"(b));
  }
K_END(uint32_t)

K_BEGIN(k_mad_u32_u24, uint32_t)
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < NCH; ++c)
      asm volatile("v_mad_u32_u24 %0, %0, %1, %0" : "+v"(acc[c]) : "v"(b));
  }
K_END(uint32_t)

K_BEGIN(k_mul_hi_u32_u24, uint32_t)
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < NCH; ++c)
      asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(acc[c]) : "v"(b));
  }
K_END(uint32_t)

K_BEGIN(k_add_u32, uint32_t)
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < NCH; ++c)
      asm volatile("v_add_u32 %0, %0, %1" : "+v"(acc[c]) : "v"(b));
  }
K_END(uint32_t)

K_BEGIN(k_add_co_u32, uint32_t)
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < NCH; ++c)
      asm volatile("v_add_co_u32 %0, vcc, %0, %1\n\tv_addc_co_u32 %0, vcc, %0, %1, vcc" : "+v"(acc[c]) : "v"(b) : "vcc");
  }
K_END(uint32_t)

K_BEGIN(k_lshl_add_u64, uint64_t)
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < NCH; ++c)
      asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(acc[c]) : "v"((uint64_t)b));
  }
K_END(uint64_t)

__global__ void k_fma_f64(double* out, uint32_t seed) {
  uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  double acc[NCH]; double a = 1.0000001 + tid * 1e-12, b = 0.9999999;
  for (int c = 0; c < NCH; ++c) acc[c] = a + c;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < NCH; ++c)
      asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(acc[c]) : "v"(a), "v"(b));
  }
  double r = 0; for (int c = 0; c < NCH; ++c) r += acc[c]; out[tid] = r;
}

__global__ void k_fma_f32(float* out, uint32_t seed) {
  uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  float acc[NCH]; float a = 1.0001f + tid * 1e-9f, b = 0.9999f;
  for (int c = 0; c < NCH; ++c) acc[c] = a + c;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < NCH; ++c)
      asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(acc[c]) : "v"(a), "v"(b));
  }
  float r = 0; for (int c = 0; c < NCH; ++c) r += acc[c]; out[tid] = r;
}

template <typename T>
static void run(const char* name, void (*k)(T*, uint32_t), int insts_per_op) {
  const int block = 256;
  int grid = 256 * 8;  // 8 blocks of 4 waves per CU = 8 waves/SIMD
  size_t n = (size_t)grid * block;
  T* d; hipMalloc(&d, n * sizeof(T));
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(k, dim3(grid), dim3(block), 0, 0, d, 1u);
  hipDeviceSynchronize();
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(k, dim3(grid), dim3(block), 0, 0, d, (uint32_t)r);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1); if (ms < best) best = ms;
  }
  double ops = (double)n * ITERS * NCH;  // lane-ops (one per asm statement)
  double lane_ops_s = ops / (best * 1e-3);
  double wave_insts_s = lane_ops_s / 64.0 * insts_per_op;
  // cycles per wave-instruction per SIMD at 2.4 GHz (1024 SIMDs)
  double cyc = (1024.0 * 2.4e9) / wave_insts_s;
  printf("{\"op\": \"%s\", \"ms\": %.3f, \"lane_ops_per_s\": %.4e, \"cyc_per_wave_inst_per_simd_at_2p4\": %.2f}\n",
         name, best, lane_ops_s, cyc);
  hipFree(d);
}

int main() {
  hipDeviceProp_t p; hipGetDeviceProperties(&p, 0);
  printf("# device %s CUs %d clock %d kHz\n", p.gcnArchName, p.multiProcessorCount, p.clockRate);
  run<uint32_t>("v_add_u32", k_add_u32, 1);
  run<uint32_t>("v_add_co+addc (pair)", k_add_co_u32, 2);
  run<uint32_t>("v_mul_lo_u32", k_mul_lo_u32, 1);
  run<uint32_t>("v_mul_hi_u32", k_mul_hi_u32, 1);
  run<uint64_t>("v_mad_u64_u32", k_mad_u64_u32, 1);
  run<uint32_t>("v_mad_u32_u24", k_mad_u32_u24, 1);
  run<uint32_t>("v_mul_hi_u32_u24", k_mul_hi_u32_u24, 1);
  run<uint64_t>("v_lshl_add_u64", k_lshl_add_u64, 1);
  run<double>("v_fma_f64", k_fma_f64, 1);
  run<float>("v_fma_f32", k_fma_f32, 1);
  return 0;
}
