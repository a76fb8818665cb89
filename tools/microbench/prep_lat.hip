// Microbenchmark: the row kernels' helper-wave scalar work with ONE wave per
// SIMD (the regime of k_verify_row4_split's wave 3): SHA-512 over R || A || a
// 116-byte vote, the mod-L reduction, the half-size pair (odd k2 and any
// parity) and u = k2 s mod L -- cycles per step from s_memtime around each.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I cometbft_amd/csrc -o tools/microbench/prep_lat tools/microbench/prep_lat.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "halfscalar.h"
#include "sc25519.h"
#include "sha512.h"

using namespace cmtv;

constexpr int kSteps = 6;

// VGPR = false: uniform inputs (the compiler runs the steps on the scalar
// unit); true: the inputs XORed with a per-lane zero it cannot see through
// (the vector unit, as in the kernels, whose helper reads LDS)
template <bool VGPR>
__global__ __launch_bounds__(64, 1) void k_prep(const uint32_t* __restrict__ in, const uint8_t* __restrict__ msg,
                                               const uint32_t* __restrict__ zero, uint64_t* cyc, uint32_t* out) {
  const uint32_t b = blockIdx.x;
  const uint32_t z = VGPR ? zero[threadIdx.x] : 0u;
  uint32_t w[16], ts[8];
#pragma unroll
  for (int i = 0; i < 16; i++) w[i] = in[b * 24 + i] ^ z;
#pragma unroll
  for (int i = 0; i < 8; i++) ts[i] = in[b * 24 + 16 + i] ^ z;
  ts[7] &= 0x0FFFFFFFu;
  uint64_t st[kSteps + 1];
  uint32_t h[16], k[8];
  st[0] = __builtin_amdgcn_s_memtime();
  sha512_prefixed<16>(h, w, msg + 116 * b + (z & 64), 116);
  st[1] = __builtin_amdgcn_s_memtime();
  sc_reduce512(k, h);
  st[2] = __builtin_amdgcn_s_memtime();
  HalfScalars hs;
  half_scalars(hs, k, false, true);
  st[3] = __builtin_amdgcn_s_memtime();
  uint32_t u[8];
  hs_bscalar(u, hs.k2, hs.k2_neg, ts);
  st[4] = __builtin_amdgcn_s_memtime();
  HalfScalars hz;
  half_scalars(hz, k, false, false);
  st[5] = __builtin_amdgcn_s_memtime();
  HalfScalars hu;
  half_scalars<true, true>(hu, k, false, true);  // the row helpers' form: uniform branches
  st[6] = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0)
    for (int i = 0; i < kSteps; i++) cyc[b * kSteps + i] = st[i + 1] - st[i];
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) x ^= u[i] ^ hs.k1[i] ^ hz.k1[i] ^ hz.k2[i] ^ hu.k1[i];
  out[b * 64 + threadIdx.x] = x ^ (uint32_t)hs.windows;
}

int main() {
  const int blocks = 1024;
  std::vector<uint32_t> h(blocks * 24);
  std::vector<uint8_t> m(blocks * 116);
  uint32_t s = 7;
  for (auto& w : h) {
    s = s * 1664525u + 1013904223u;
    w = s;
  }
  for (auto& c : m) {
    s = s * 1664525u + 1013904223u;
    c = (uint8_t)(s >> 24);
  }
  uint32_t *din, *dout, *dzero;
  uint8_t* dmsg;
  uint64_t* dcyc;
  if (hipMalloc(&din, 4 * h.size()) || hipMalloc(&dmsg, m.size()) || hipMalloc(&dout, 4 * blocks * 64) ||
      hipMalloc(&dcyc, 8 * blocks * kSteps) || hipMalloc(&dzero, 4 * 64))
    return 1;
  (void)hipMemset(dzero, 0, 4 * 64);
  (void)hipMemcpy(din, h.data(), 4 * h.size(), hipMemcpyHostToDevice);
  (void)hipMemcpy(dmsg, m.data(), m.size(), hipMemcpyHostToDevice);
  for (int vg = 0; vg < 2; vg++) {
    for (int rep = 0; rep < 2; rep++) {
      if (vg)
        hipLaunchKernelGGL(k_prep<true>, dim3(blocks), dim3(64), 0, 0, din, dmsg, dzero, dcyc, dout);
      else
        hipLaunchKernelGGL(k_prep<false>, dim3(blocks), dim3(64), 0, 0, din, dmsg, dzero, dcyc, dout);
    }
    std::vector<uint64_t> c(blocks * kSteps);
    if (hipMemcpy(c.data(), dcyc, 8 * c.size(), hipMemcpyDeviceToHost) != hipSuccess) return 1;
    double sum[kSteps] = {};
    for (int b = 0; b < blocks; b++)
      for (int i = 0; i < kSteps; i++) sum[i] += (double)c[b * kSteps + i];
    const char* nm[kSteps] = {"sha512 (64 + 116 bytes)", "sc_reduce512", "half_scalars (odd k2)", "hs_bscalar",
                              "half_scalars (any parity)", "half_scalars (odd, uniform)"};
    for (int i = 0; i < kSteps; i++)
      printf("%-6s %-28s %10.1f cycles (s_memtime, %d waves, 1 per CU)\n", vg ? "vector" : "scalar", nm[i],
             sum[i] / blocks, blocks);
  }
  return 0;
}
