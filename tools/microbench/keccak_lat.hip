// Microbenchmark: cycles per Keccak-f[1600] and per sr25519 merlin transcript
// (merlin.h sr_transcript over the device program, STROBE state in LDS) with
// ONE wave per SIMD -- the regime of k_verify_sr25519_quad_hs's helper wave.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I cometbft_amd/csrc -o tools/microbench/keccak_lat tools/microbench/keccak_lat.hip
//
// Variants: 0 keccak_f1600 (keccak.h: funnel-shift rotates) on a register
// state, a dependent chain; 1 the same permutation with 64-bit shift rotates
// (checked to end in the same state); 2 the whole transcript of a 116-byte
// message; 3 the transcript of an empty message; 4 the Ed25519 helper's
// SHA-512(R || A || M) of a 116-byte message (two blocks). Lane 0 of every wave records
// s_memtime around the loop; prints mean cycles per item. Then the scalar
// cache's latency (a uniform-address pointer chase), alone and with an LDS
// store per step.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "merlin.h"
#include "sha512.h"

using namespace cmtv;

struct LdsState {  // sr25519.hip LdsStrobeState
  uint32_t* lds;
  uint32_t lane;
  __device__ __forceinline__ void store(int i, uint32_t x) { lds[i * 64 + lane] = x; }
  __device__ __forceinline__ uint32_t load(int i) const { return lds[i * 64 + lane]; }
};

// keccak.h's permutation with plain 64-bit shift rotates (its form before the
// funnel-shift rotate), for comparison
__device__ __forceinline__ void keccak_shift(uint64_t a[25]) {
#pragma unroll 1
  for (int rnd = 0; rnd < 24; rnd++) {
    uint64_t c[5], b[25];
#pragma unroll
    for (int x = 0; x < 5; x++) c[x] = a[x] ^ a[x + 5] ^ a[x + 10] ^ a[x + 15] ^ a[x + 20];
#pragma unroll
    for (int x = 0; x < 5; x++) {
      const uint64_t v = c[(x + 1) % 5];
      const uint64_t d = c[(x + 4) % 5] ^ ((v << 1) | (v >> 63));
#pragma unroll
      for (int y = 0; y < 5; y++) a[x + 5 * y] ^= d;
    }
#pragma unroll
    for (int i = 0; i < 25; i++) {
      const int r = keccak_rho(i);
      b[keccak_pi(i)] = r ? (a[i] << r) | (a[i] >> (64 - r)) : a[i];
    }
#pragma unroll
    for (int y = 0; y < 5; y++)
#pragma unroll
      for (int x = 0; x < 5; x++)
        a[x + 5 * y] = b[x + 5 * y] ^ (~b[(x + 1) % 5 + 5 * y] & b[(x + 2) % 5 + 5 * y]);
    a[0] ^= keccak_rc(rnd);
  }
}

template <int V>
__global__ __launch_bounds__(256, 1) void k_chain(const uint32_t* in, const uint32_t* lens, const uint8_t* msg, uint32_t mlen,
                                                  const uint32_t* prog, int nops_prog, uint32_t* out, int n,
                                                  unsigned long long* cyc) {
  __shared__ uint32_t st_lds[4][STROBE_BLOCK_WORDS * 64];
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t a[25];
  for (int i = 0; i < 25; i++) a[i] = ((uint64_t)in[(tid * 50 + 2 * i) % 4096] << 32) | in[(tid * 50 + 2 * i + 1) % 4096];
  uint32_t acc[16] = {};
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int it = 0; it < n; it++) {
    if (V == 0) keccak_f1600(a);
    if (V == 1) keccak_shift(a);
    if (V == 4) {  // SHA-512(R || A || M), the Ed25519 helper's hash, 116-byte messages
      uint32_t pre[16], h[16];
      for (int i = 0; i < 16; i++) pre[i] = (uint32_t)a[i] ^ (uint32_t)it;
      sha512_prefixed<16>(h, pre, msg + (size_t)(tid & 1023) * 128 + 1 + (tid & 1), lens[tid & 4095]);
      for (int i = 0; i < 16; i++) acc[i] ^= h[i];
    }
    if (V == 2 || V == 3) {
      LdsState st{st_lds[threadIdx.x >> 6], threadIdx.x & 63};
      uint32_t pk[8], R[8], o[16];
      for (int i = 0; i < 8; i++) {
        pk[i] = (uint32_t)a[i] ^ (uint32_t)it;
        R[i] = (uint32_t)(a[i] >> 32);
      }
      // a per-lane length (as the kernels see it), the same value in every lane
      const uint32_t ml = V == 3 ? 0u : lens[tid & 4095];
      sr_transcript(o, st, prog, nops_prog, msg + (size_t)(tid & 1023) * 128 + 1 + (tid & 1), ml,
                    pk, R);
      for (int i = 0; i < 16; i++) acc[i] ^= o[i];
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  uint32_t h = 0;
  for (int i = 0; i < 25; i++) h ^= (uint32_t)a[i] ^ (uint32_t)(a[i] >> 32) * (i + 1);
  for (int i = 0; i < 16; i++) h ^= acc[i] * (i + 3);
  out[tid] = h;
  if ((threadIdx.x & 63) == 0) cyc[tid >> 6] = t1 - t0;
}

// scalar-cache latency: a pointer chase through a 128-entry table of next
// indices with wave-uniform addresses (s_load_dword), V=1 with an LDS store
// per step in flight (s_waitcnt lgkmcnt covers both)
template <int V>
__global__ __launch_bounds__(256, 1) void k_chase(const uint32_t* tab, uint32_t* out, int n, unsigned long long* cyc) {
  __shared__ uint32_t lds[64 * 64];
  const __attribute__((address_space(4))) uint32_t* c =
      (const __attribute__((address_space(4))) uint32_t*)(reinterpret_cast<uintptr_t>(tab));
  uint32_t idx = 0, acc = threadIdx.x;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int it = 0; it < n; it++) {
    idx = c[idx];
    if (V == 1) lds[(idx & 63) * 64 + (threadIdx.x & 63)] = acc++;
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  __syncthreads();
  out[blockIdx.x * blockDim.x + threadIdx.x] = idx + lds[threadIdx.x & 4095];
  if ((threadIdx.x & 63) == 0) cyc[(blockIdx.x * blockDim.x + threadIdx.x) >> 6] = t1 - t0;
}

typedef void (*kfn)(const uint32_t*, const uint32_t*, const uint8_t*, uint32_t, const uint32_t*, int, uint32_t*, int,
                    unsigned long long*);

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 200;
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int block = 256, grid = cus;  // 51 KiB static + 64 KiB dynamic LDS: one block per CU
  const size_t nth = (size_t)grid * block;
  std::vector<uint32_t> hin(4096);
  uint32_t x = 12345;
  for (auto& w : hin) w = (x = x * 1664525u + 1013904223u);
  std::vector<uint8_t> hm(1024 * 128 + 64);
  for (auto& b : hm) b = (uint8_t)((x = x * 1664525u + 1013904223u) >> 24);
  uint32_t prog[SR_PREFIX_WORDS];
  const int np = sr_prefix_state(prog);
  uint32_t *din, *dout;
  uint8_t* dm;
  uint32_t* dp;
  unsigned long long* dcyc;
  (void)hipMalloc(&din, hin.size() * 4);
  (void)hipMalloc(&dm, hm.size());
  (void)hipMalloc(&dp, sizeof(prog));
  (void)hipMalloc(&dout, nth * 4);
  (void)hipMalloc(&dcyc, (nth / 64) * 8);
  (void)hipMemcpy(din, hin.data(), hin.size() * 4, hipMemcpyHostToDevice);
  uint32_t* dlen;
  std::vector<uint32_t> hlen(4096, 116u);
  (void)hipMalloc(&dlen, hlen.size() * 4);
  (void)hipMemcpy(dlen, hlen.data(), hlen.size() * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(dm, hm.data(), hm.size(), hipMemcpyHostToDevice);
  (void)hipMemcpy(dp, prog, sizeof(prog), hipMemcpyHostToDevice);
  const kfn ks[] = {k_chain<0>, k_chain<1>, k_chain<2>, k_chain<3>, k_chain<4>};
  const char* names[] = {"keccak alignbit", "keccak shifts", "transcript 116B", "  ... empty msg",
                         "sha512 64+116B"};
  std::vector<uint32_t> ref(nth), got(nth);
  for (int v = 0; v < 5; v++) {
    for (int r = 0; r < 2; r++)
      hipLaunchKernelGGL(ks[v], dim3(grid), dim3(block), 64 * 1024, 0, din, dlen, dm, 116u, dp, np, dout, n, dcyc);
    (void)hipDeviceSynchronize();
    std::vector<unsigned long long> cyc(nth / 64);
    (void)hipMemcpy(cyc.data(), dcyc, cyc.size() * 8, hipMemcpyDeviceToHost);
    double mean = 0;
    for (auto c : cyc) mean += (double)c;
    mean /= cyc.size();
    (void)hipMemcpy(got.data(), dout, nth * 4, hipMemcpyDeviceToHost);
    if (v == 0) ref = got;
    printf("%-16s %9.1f cyc/item (s_memtime, one wave per SIMD)%s\n", names[v], mean / n,
           v == 1 ? (got == ref ? "  (same state as alignbit)" : "  MISMATCH") : "");
    fflush(stdout);
  }
  {
    std::vector<uint32_t> tab(128);
    for (int i = 0; i < 128; i++) tab[i] = (uint32_t)((i * 37 + 11) & 127);
    (void)hipMemcpy(din, tab.data(), 128 * 4, hipMemcpyHostToDevice);
    void (*kc[])(const uint32_t*, uint32_t*, int, unsigned long long*) = {k_chase<0>, k_chase<1>};
    const char* cn[] = {"s_load chase", "  + LDS store"};
    for (int v = 0; v < 2; v++) {
      for (int r = 0; r < 2; r++) hipLaunchKernelGGL(kc[v], dim3(grid), dim3(block), 64 * 1024, 0, din, dout, 2000, dcyc);
      (void)hipDeviceSynchronize();
      std::vector<unsigned long long> cyc(nth / 64);
      (void)hipMemcpy(cyc.data(), dcyc, cyc.size() * 8, hipMemcpyDeviceToHost);
      double mean = 0;
      for (auto x : cyc) mean += (double)x;
      printf("%-16s %9.1f cyc/step\n", cn[v], mean / cyc.size() / 2000);
    }
  }
  return 0;
}
