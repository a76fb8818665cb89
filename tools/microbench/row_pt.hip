// Microbenchmark: the row verifier's operations (row.h) with ONE wave per
// SIMD, the regime of k_verify_row_split: a doubling, an addition, a Straus
// window (4 doublings + 2 LDS-table additions), the decode of A and R, and
// the two tables -- cycles per operation from s_memtime around each.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 -I cometbft_amd/csrc -o tools/microbench/row_pt tools/microbench/row_pt.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "row_dev.h"

using namespace cmtv;

__global__ __launch_bounds__(64, 1) void k_rowpt(uint32_t nops, const uint32_t* __restrict__ in, uint64_t* cyc,
                                                uint32_t* out) {
  __shared__ uint32_t tab_lds[kRowTabWords + 8000];  // one wave per CU
  const uint32_t t = threadIdx.x;
  const RowCtx<DevRow> x(DevRow::lane());
  uint32_t v = in[blockIdx.x * 128 + t] & 0xFFFFu, c = in[blockIdx.x * 128 + 64 + t] & 0xFFFFu;
  DevRowTab tab{tab_lds, t};
  for (int e = 0; e < 9; e++) {
    tab.store(0, 0, e, c);
    tab.store(0, 1, e, c);
    tab.store(1, 0, e, c);
    tab.store(1, 1, e, c);
  }
  tab_lds[kRowTabWords + t] = t;
  __syncthreads();
  const uint32_t n = nops + (tab_lds[kRowTabWords + (t & 7)] > 1000 ? 1u : 0u);
  uint64_t st[8];
  st[0] = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (uint32_t k = 0; k < n; k++) rp_dbl(x, v);
  st[1] = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (uint32_t k = 0; k < n; k++) rp_add(x, v, c);
  st[2] = __builtin_amdgcn_s_memtime();
  uint32_t d = t * 2654435761u;
#pragma unroll 1
  for (uint32_t k = 0; k < n / 4; k++) {
    const int dA = (int)((d >> 4) & 15) - 8, dR = (int)((d >> 8) & 15) - 8;
    d = d * 1664525u + 1013904223u;
    const int a = __builtin_amdgcn_readfirstlane(dA), r = __builtin_amdgcn_readfirstlane(dR);
    const uint32_t cA = tab.load(0, a < 0, a < 0 ? -a : a), cR = tab.load(1, r < 0, r < 0 ? -r : r);
#pragma unroll 1
    for (int j = 0; j < 4; j++) rp_dbl(x, v);
    rp_add(x, v, cA);
    rp_add(x, v, cR);
  }
  st[3] = __builtin_amdgcn_s_memtime();
  uint32_t xo, to;
  const bool ok = rf_decode(x, v & 0xFFFFu, (v & 1) != 0, xo, to);
  st[4] = __builtin_amdgcn_s_memtime();
  // one table: to_cached / neg per entry, 1 doubling and 6 additions
  {
    uint32_t w = rf_carry32(x, xo);
    const uint32_t d2 = x.cst(RowConst::d2);
    const uint32_t c1 = rp_to_cached(x, w, d2);
    tab.store(0, 0, 1, c1);
    tab.store(0, 1, 1, rp_cached_neg(x, c1));
    rp_dbl(x, w);
#pragma unroll 1
    for (int e = 2; e <= 8; e++) {
      if (e > 2) rp_add(x, w, c1);
      const uint32_t ce = rp_to_cached(x, w, d2);
      tab.store(0, 0, e, ce);
      tab.store(0, 1, e, rp_cached_neg(x, ce));
    }
    v ^= w;
  }
  st[5] = __builtin_amdgcn_s_memtime();
  // the split decodes (row.h rf_mul_s): one y on rows {0, 2} and one on {1, 3}
  // (S = 2), one y on every row (S = 4)
  uint32_t b0, b1, b2, b3;
  DevRow::rows(v & 0xFFFFu, b0, b1, b2, b3);
  uint32_t x2, t2, x4, t4;
  const bool ok2 = rf_decode<0, 2>(x, (t & 16) ? b1 : b0, (v & 1) != 0, x2, t2);
  st[6] = __builtin_amdgcn_s_memtime();
  const bool ok4 = rf_decode<0, 4>(x, b0, (v & 1) != 0, x4, t4);
  st[7] = __builtin_amdgcn_s_memtime();
  if (t == 0)
    for (int i = 0; i < 7; i++) cyc[blockIdx.x * 7 + i] = st[i + 1] - st[i];
  out[blockIdx.x * 64 + t] = v ^ xo ^ to ^ (ok ? 1u : 0u) ^ x2 ^ t2 ^ x4 ^ t4 ^ (ok2 ? 2u : 0u) ^ (ok4 ? 4u : 0u);
}

int main() {
  const int blocks = 1024;
  const uint32_t nops = 512;
  std::vector<uint32_t> h(blocks * 128);
  uint32_t s = 99;
  for (auto& w : h) {
    s = s * 1664525u + 1013904223u;
    w = s;
  }
  uint32_t *din, *dout;
  uint64_t* dcyc;
  if (hipMalloc(&din, 4 * h.size()) || hipMalloc(&dout, 4 * blocks * 64) || hipMalloc(&dcyc, 8 * blocks * 7)) return 1;
  (void)hipMemcpy(din, h.data(), 4 * h.size(), hipMemcpyHostToDevice);
  for (int rep = 0; rep < 2; rep++) hipLaunchKernelGGL(k_rowpt, dim3(blocks), dim3(64), 0, 0, nops, din, dcyc, dout);
  std::vector<uint64_t> c(blocks * 7);
  if (hipMemcpy(c.data(), dcyc, 8 * c.size(), hipMemcpyDeviceToHost) != hipSuccess) return 1;
  double sum[7] = {0, 0, 0, 0, 0, 0, 0};
  for (int b = 0; b < blocks; b++)
    for (int i = 0; i < 7; i++) sum[i] += (double)c[b * 7 + i];
  const char* nm[7] = {"rp_dbl", "rp_add", "window (4 dbl + 2 LDS add)", "rf_decode (A and R rows)",
                       "one table (0..8), both signs", "rf_decode S=2 (A, R: 2 rows each)",
                       "rf_decode S=4 (one point)"};
  const double per[7] = {(double)nops, (double)nops, (double)(nops / 4), 1.0, 1.0, 1.0, 1.0};
  for (int i = 0; i < 7; i++) printf("%-32s %10.1f cycles (s_memtime, %d waves, 1 per CU)\n", nm[i], sum[i] / blocks / per[i], blocks);
  return 0;
}
