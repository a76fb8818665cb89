// Microbenchmark: a GF(2^255-19) product in the "row" layout -- one field
// element per 16-lane DPP row, radix 2^16, lane k of the row holding limb k --
// against the quad layout's one-lane products (fe_lat: 528 cycles per
// squaring). Checks the DPP semantics the layout relies on (row_ror, row_shr
// with an old value, row_newbcast) and the product against a host big-int.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/microbench/row_lat tools/microbench/row_lat.hip
//
// Column k of h = f g mod p (2^256 = 38):
//   h_k = sum_r f_{(k-r) mod 16} g_r (x 38 when r > k)
// lane k gets f_{k-r} by row_ror:r and g_r by row_newbcast:r; the twist is a
// per-lane multiplier t_r = (k < r ? 38 : 1) applied to the broadcast g_r.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#define DEV __device__ __forceinline__

template <int CTRL>
DEV uint32_t dpp(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
DEV uint32_t dpp_old(uint32_t old, uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)x, CTRL, 0xF, 0xF, false);
}

// three carry rounds: limbs end < 2^16 + 2^10 (lane 0: < 2^16.6)
DEV uint32_t row_carry(uint64_t c, uint32_t m0) {
  uint64_t cc = c;
  uint32_t lo = (uint32_t)cc & 0xFFFFu;
  uint32_t ca = (uint32_t)(cc >> 16);                 // < 2^32 by the operand bounds
  ca = dpp<0x121>(ca);                                // row_ror:1 -- lane k gets lane k-1
  cc = (uint64_t)ca * m0 + lo;                        // lane 0: 38 x the top carry
  lo = (uint32_t)cc & 0xFFFFu;
  ca = (uint32_t)(cc >> 16);
  ca = dpp<0x121>(ca);
  uint32_t w = __umul24(ca, m0) + lo;                 // < 2^26
  lo = w & 0xFFFFu;
  ca = dpp<0x121>(w >> 16);
  return __umul24(ca, m0) + lo;
}

template <int R>
DEV void term(uint64_t& acc, uint32_t f, uint32_t g, uint32_t k) {
  const uint32_t fr = dpp<0x120 + R>(f);       // row_ror:R
  const uint32_t gb = dpp<0x150 + R>(g);       // row_newbcast:R
  const uint32_t t = k < R ? 38u : 1u;         // loop-invariant per lane
  acc += (uint64_t)fr * __umul24(gb, t);       // v_mul_u32_u24: full rate (v_mul_lo_u32 is not)
}

DEV uint32_t row_mul(uint32_t f, uint32_t g, uint32_t k, uint32_t m0) {
  uint64_t acc = (uint64_t)f * dpp<0x150>(g);
  term<1>(acc, f, g, k);  term<2>(acc, f, g, k);  term<3>(acc, f, g, k);
  term<4>(acc, f, g, k);  term<5>(acc, f, g, k);  term<6>(acc, f, g, k);
  term<7>(acc, f, g, k);  term<8>(acc, f, g, k);  term<9>(acc, f, g, k);
  term<10>(acc, f, g, k); term<11>(acc, f, g, k); term<12>(acc, f, g, k);
  term<13>(acc, f, g, k); term<14>(acc, f, g, k); term<15>(acc, f, g, k);
  return row_carry(acc, m0);
}

__global__ __launch_bounds__(64, 1) void k_row(uint32_t nops, int op, const uint32_t* __restrict__ in,
                                              uint64_t* cyc, uint32_t* out, uint32_t* probe) {
  __shared__ uint32_t pad[25000];  // one wave per CU
  const uint32_t t = threadIdx.x, k = t & 15;
  const uint32_t m0 = k == 0 ? 38u : 1u;
  uint32_t f = in[blockIdx.x * 128 + t] & 0xFFFFu, g = in[blockIdx.x * 128 + 64 + t] & 0xFFFFu;
  if (blockIdx.x == 0) {
    // DPP semantics probe: lane t's view of ror:3, shr:3 (old = 999), newbcast:5 of x = t
    probe[t] = dpp<0x123>(t);
    probe[64 + t] = dpp_old<0x113>(999u, t);
    probe[128 + t] = dpp<0x155>(t);
    // row exchanges (devtables.h DevRow::rows): permlane32_swap(x, x) and
    // permlane16_swap(y, y) of x = lane
    const auto h = __builtin_amdgcn_permlane32_swap(t, t, false, false);
    const auto lo = __builtin_amdgcn_permlane16_swap(h[0], h[0], false, false);
    probe[192 + t] = h[0];
    probe[256 + t] = h[1];
    probe[320 + t] = lo[0];
    probe[384 + t] = lo[1];
  }
  pad[t] = t;
  __syncthreads();
  uint32_t n = nops + (pad[t & 7] > 1000 ? 1u : 0u);
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  if (op == 0) {
#pragma unroll 1
    for (uint32_t j = 0; j < n; j++) f = row_mul(f, f, k, m0);
  } else {
#pragma unroll 1
    for (uint32_t j = 0; j < n; j++) f = row_mul(f, g, k, m0);
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (t == 0) cyc[blockIdx.x] = t1 - t0;
  out[blockIdx.x * 64 + t] = f;
}

// ---- host check --------------------------------------------------------------
typedef unsigned __int128 u128;
struct Big { uint64_t w[5]; };  // little-endian 320-bit scratch
static const uint64_t P[4] = {0xFFFFFFFFFFFFFFEDull, 0xFFFFFFFFFFFFFFFFull, 0xFFFFFFFFFFFFFFFFull,
                              0x7FFFFFFFFFFFFFFFull};
static void from_limbs(uint64_t r[4], const uint32_t* l) {  // sum l_k 2^16k mod p (l_k < 2^32)
  uint64_t acc[5] = {0, 0, 0, 0, 0};
  for (int k = 0; k < 16; k++) {
    const int bit = 16 * k, w = bit / 64, sh = bit % 64;
    u128 v = (u128)l[k] << sh;
    for (int i = w; i < 5 && v; i++) {
      u128 s = (u128)acc[i] + (uint64_t)v;
      acc[i] = (uint64_t)s;
      v = (v >> 64) + (s >> 64);
    }
  }
  // fold 2^256 = 38, twice
  for (int it = 0; it < 3; it++) {
    uint64_t hi = acc[4];
    acc[4] = 0;
    u128 c = (u128)hi * 38;
    for (int i = 0; i < 5 && c; i++) {
      u128 s = (u128)acc[i] + (uint64_t)c;
      acc[i] = (uint64_t)s;
      c = (c >> 64) + (s >> 64);
    }
  }
  for (int it = 0; it < 4; it++) {  // conditional subtract p
    bool ge = true;
    for (int i = 3; i >= 0; i--) {
      if (acc[i] != P[i]) { ge = acc[i] > P[i]; break; }
    }
    if (!ge) break;
    u128 b = 0;
    for (int i = 0; i < 4; i++) {
      u128 d = (u128)acc[i] - P[i] - (uint64_t)b;
      acc[i] = (uint64_t)d;
      b = (d >> 64) ? 1 : 0;
    }
  }
  for (int i = 0; i < 4; i++) r[i] = acc[i];
}
static void mulmod(uint64_t r[4], const uint64_t a[4], const uint64_t b[4]) {
  uint64_t t[8] = {0};
  for (int i = 0; i < 4; i++) {
    u128 c = 0;
    for (int j = 0; j < 4; j++) {
      u128 s = (u128)a[i] * b[j] + t[i + j] + (uint64_t)c;
      t[i + j] = (uint64_t)s;
      c = s >> 64;
    }
    t[i + 4] = (uint64_t)c;
  }
  // t mod p via 16-bit limbs (reuse from_limbs on 2^16 pieces of t folded)
  uint32_t l[16];
  uint64_t lo[4];
  // fold: t = lo + 2^256 hi = lo + 38 hi
  u128 c = 0;
  for (int i = 0; i < 4; i++) {
    u128 s = (u128)t[i + 4] * 38 + t[i] + (uint64_t)c;
    lo[i] = (uint64_t)s;
    c = s >> 64;
  }
  for (int k = 0; k < 16; k++) l[k] = (uint32_t)(lo[k / 4] >> (16 * (k % 4))) & 0xFFFF;
  l[0] += (uint32_t)c * 38;  // c < 64: fits
  from_limbs(r, l);
}

int main() {
  const int blocks = 1024;
  std::vector<uint32_t> h(blocks * 128);
  uint32_t x = 777;
  for (auto& w : h) {
    x = x * 1664525u + 1013904223u;
    w = x;
  }
  uint32_t *din, *dout, *dprobe;
  uint64_t* dcyc;
  if (hipMalloc(&din, 4 * h.size()) || hipMalloc(&dout, 4 * blocks * 64) || hipMalloc(&dcyc, 8 * blocks) ||
      hipMalloc(&dprobe, 4 * 448))
    return 1;
  (void)hipMemcpy(din, h.data(), 4 * h.size(), hipMemcpyHostToDevice);
  int rc = 0;
  for (int op = 0; op < 2; op++) {
    const uint32_t nops = 4096;
    for (int rep = 0; rep < 2; rep++)
      hipLaunchKernelGGL(k_row, dim3(blocks), dim3(64), 0, 0, nops, op, din, dcyc, dout, dprobe);
    std::vector<uint64_t> c(blocks);
    std::vector<uint32_t> o(blocks * 64), pr(448);
    (void)hipMemcpy(c.data(), dcyc, 8 * blocks, hipMemcpyDeviceToHost);
    (void)hipMemcpy(o.data(), dout, 4 * o.size(), hipMemcpyDeviceToHost);
    (void)hipMemcpy(pr.data(), dprobe, 4 * 448, hipMemcpyDeviceToHost);
    if (op == 0) {
      std::printf("ror:3   lanes 0..15:");
      for (int i = 0; i < 16; i++) std::printf(" %u", pr[i]);
      std::printf("\nshr:3(old 999):    ");
      for (int i = 0; i < 16; i++) std::printf(" %u", pr[64 + i]);
      std::printf("\nnewbcast:5 rows:   ");
      for (int i = 0; i < 64; i += 15) std::printf(" %u", pr[128 + i]);
      std::printf("\n");
      const char* nm[4] = {"p32.first", "p32.second", "p16(p32.first).first", "p16(p32.first).second"};
      for (int q = 0; q < 4; q++) {
        std::printf("%-24s rows (lane 16c+1):", nm[q]);
        for (int c = 0; c < 4; c++) std::printf(" %u", pr[192 + 64 * q + 16 * c + 1]);
        std::printf("\n");
      }
    }
    double s = 0;
    for (auto v : c) s += (double)v;
    // host check of 8 rows
    int bad = 0;
    for (int b = 0; b < 2; b++)
      for (int row = 0; row < 4; row++) {
        uint32_t fl[16], gl[16];
        for (int k = 0; k < 16; k++) {
          fl[k] = h[b * 128 + row * 16 + k] & 0xFFFF;
          gl[k] = h[b * 128 + 64 + row * 16 + k] & 0xFFFF;
        }
        uint64_t f[4], g[4], r[4];
        from_limbs(f, fl);
        from_limbs(g, gl);
        for (uint32_t j = 0; j < nops; j++) {
          mulmod(r, f, op == 0 ? f : g);
          for (int i = 0; i < 4; i++) f[i] = r[i];
        }
        uint64_t dv[4];
        from_limbs(dv, &o[b * 64 + row * 16]);
        for (int i = 0; i < 4; i++) bad += dv[i] != f[i];
      }
    std::printf("%s chain: %.1f cycles/op (s_memtime, %d waves, 1 per CU); host check: %s\n",
                op == 0 ? "row squaring" : "row multiply", s / blocks / nops, blocks, bad ? "MISMATCH" : "ok");
    rc |= bad;
  }
  return rc;
}
