// Microbenchmark: latency of the quad kernels' point operations (quad.h
// q_dbl, q_add) with ONE wave per SIMD, the regime of the 10k step (one
// issue-bound quad wave per SIMD), plus one 34-window Straus
// body (4 doublings + 2 LDS-table additions).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I cometbft_amd/csrc -o tools/microbench/pt_lat tools/microbench/pt_lat.hip
//
// Grid: 1024 one-wave workgroups with 100 KiB of LDS each, so no CU holds
// two -- one wave per CU, i.e. per SIMD; lane 0 of each wave records
// s_memtime around NOPS operations (rolled loop, hidden trip count). Prints
// the mean cycles per operation; the results are checked for agreement
// between runs (the work is deterministic).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "devtables.h"
#include "quad.h"

using namespace cmtv;

template <int OP, int FOLD>
__global__ __launch_bounds__(64, 1) void k_pt(uint32_t nops, const uint32_t* __restrict__ in, uint64_t* cyc,
                                             uint32_t* out) {
  __shared__ uint2 tab[2 * 9 * 5 * 64 + 6000];  // the quad's two tables + padding (one wave per CU)
  const uint32_t t = threadIdx.x;
  DevQuad q;
  fe v, c;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    v.v[i] = in[(blockIdx.x * 64 + t) * 20 + i] & 0x1FFFFFF;
    c.v[i] = in[(blockIdx.x * 64 + t) * 20 + 10 + i] & 0x1FFFFFF;
  }
  DevATabQ ta{tab, t}, tr{tab + 9 * 5 * 64, t};
  if (OP == 2) {
    for (int e = 0; e < 9; e++) {
      ta.store(e, c);
      tr.store(e, c);
    }
  }
  __syncthreads();
  uint32_t n = nops;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  if (OP == 0) {
#pragma unroll 1
    for (uint32_t k = 0; k < n; k++) q_dbl<FOLD>(q, v);
  } else if (OP == 1) {
#pragma unroll 1
    for (uint32_t k = 0; k < n; k++) q_add<FOLD>(q, v, c);
  } else {
    // one Straus window: 4 doublings, an A and an R addition from LDS
    uint32_t d = t * 2654435761u;
#pragma unroll 1
    for (uint32_t k = 0; k < n; k++) {
      fe cA, cR;
      const int dA = (int)((d >> 4) & 15) - 8, dR = (int)((d >> 8) & 15) - 8;
      d = d * 1664525u + 1013904223u;
      ta.load_signed(q, dA < 0 ? -dA : dA, dA < 0, cA);
      tr.load_signed(q, dR < 0 ? -dR : dR, dR < 0, cR);
#pragma unroll 1
      for (int j = 0; j < 4; j++) q_dbl<FOLD>(q, v);
      q_add<FOLD>(q, v, cA);
      q_add<FOLD>(q, v, cR);
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (t == 0) cyc[blockIdx.x] = t1 - t0;
#pragma unroll
  for (int i = 0; i < 10; i++) out[(blockIdx.x * 64 + t) * 10 + i] = v.v[i];
}

template <int OP, int FOLD>
static int run(const char* name, uint32_t nops, const uint32_t* din, uint64_t* dcyc, uint32_t* dout, int blocks,
               std::vector<uint32_t>* res) {
  hipLaunchKernelGGL((k_pt<OP, FOLD>), dim3(blocks), dim3(64), 0, 0, nops, din, dcyc, dout);
  hipLaunchKernelGGL((k_pt<OP, FOLD>), dim3(blocks), dim3(64), 0, 0, nops, din, dcyc, dout);
  std::vector<uint64_t> c(blocks);
  if (hipMemcpy(c.data(), dcyc, 8 * blocks, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  res->resize((size_t)blocks * 640);
  if (hipMemcpy(res->data(), dout, 4 * res->size(), hipMemcpyDeviceToHost) != hipSuccess) return 1;
  double s = 0;
  for (uint64_t x : c) s += (double)x;
  std::printf("%-34s fold%d %8.1f cycles/op (s_memtime, %d waves)\n", name, FOLD, s / blocks / nops,
              blocks);
  return 0;
}

template <int OP>
static int ab(const char* name, uint32_t nops, const uint32_t* din, uint64_t* dcyc, uint32_t* dout, int blocks) {
  std::vector<uint32_t> r0, r1, r2;
  int rc = run<OP, 0>(name, nops, din, dcyc, dout, blocks, &r0);
  rc |= run<OP, 1>(name, nops, din, dcyc, dout, blocks, &r1);
  rc |= run<OP, 2>(name, nops, din, dcyc, dout, blocks, &r2);
  // the forms compute the same limbs (same arithmetic, only the moves differ)
  size_t bad1 = 0, bad2 = 0;
  for (size_t i = 0; i < r0.size(); i++) {
    bad1 += r0[i] != r1[i];
    bad2 += r0[i] != r2[i];
  }
  std::printf("%-34s fold1 == mov: %zu, fold2 == mov: %zu words differ of %zu\n", name, bad1, bad2, r0.size());
  return rc | (bad1 || bad2 ? 2 : 0);
}

int main() {
  const int blocks = 1024;
  std::vector<uint32_t> h(blocks * 64 * 20);
  uint32_t x = 12345;
  for (auto& w : h) {
    x = x * 1664525u + 1013904223u;
    w = x;
  }
  uint32_t *din, *dout;
  uint64_t* dcyc;
  if (hipMalloc(&din, 4 * h.size()) != hipSuccess || hipMalloc(&dout, 4 * blocks * 64 * 10) != hipSuccess ||
      hipMalloc(&dcyc, 8 * blocks) != hipSuccess)
    return 1;
  (void)hipMemcpy(din, h.data(), 4 * h.size(), hipMemcpyHostToDevice);
  int rc = 0;
  rc |= ab<0>("q_dbl", 2048, din, dcyc, dout, blocks);
  rc |= ab<1>("q_add", 2048, din, dcyc, dout, blocks);
  rc |= ab<2>("window (4 dbl + 2 LDS add)", 512, din, dcyc, dout, blocks);
  return rc;
}
