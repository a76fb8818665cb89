// Debug tool: runs the quad pipeline (quad.h) for one signature on the GPU and
// under the host lockstep emulation, and reports the first probe snapshot
// where they differ. Also prints DPP quad_perm semantics.
#include <hip/hip_runtime.h>

#include <barrier>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#include "../../cometbft_amd/csrc/quad.h"
#include "../../tests/host/lazy_btab.h"

using namespace cmtv;

constexpr int NSNAP = 12;

template <int VAR>
struct DevQuad {
  __device__ int lane() const { return threadIdx.x & 3; }
  template <int PAT>
  __device__ uint32_t one(uint32_t x) const {
    if (VAR == 0) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, PAT, 0xF, 0xF, true);
    if (VAR == 4) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, PAT, 0xF, 0xF, false);  // kernels.hip
    if (VAR == 1) return (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, PAT, 0xF, 0xF, false);
    if (VAR == 2) {
      const int src = (threadIdx.x & ~3) | ((PAT >> (2 * (threadIdx.x & 3))) & 3);
      return (uint32_t)__shfl((int)x, src, 64);
    }
    // VAR 3: ds_swizzle in quad-perm mode (offset bit 15 = 1: QDMode)
    return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x8000 | PAT);
  }
  template <int PAT>
  __device__ void perm(fe& o, const fe& v) const {
    for (int i = 0; i < 10; i++) o.v[i] = one<PAT>(v.v[i]);
  }
  template <int PAT>
  __device__ void add_perm(fe& o, const fe& src, const fe& b) const {
    fe t;
    perm<PAT>(t, src);
    for (int i = 0; i < 10; i++) o.v[i] = t.v[i] + b.v[i];
  }
  template <int PAT>
  __device__ void xor_perm(fe& o, const fe& src, uint32_t k) const {
    perm<PAT>(o, src);
    for (int i = 0; i < 10; i++) o.v[i] ^= k;
  }
  template <int PAT>
  __device__ void perm_lane3(fe& o, const fe& src) const {
    perm<PAT>(o, src);
    for (int i = 0; i < 10; i++) o.v[i] = (threadIdx.x & 3) == 3 ? o.v[i] : 0u;
  }
  template <int PAT>
  __device__ void permc(fe& o, const fe& v) const {
    perm<PAT>(o, v);
  }
  template <int PAT>
  __device__ uint32_t perm32(uint32_t x) const { return one<PAT>(x); }
  __device__ bool any(bool x) const { return __ballot(x) != 0; }
};
struct DevBTabQ {
  const uint32_t* rows;
  __device__ void load_coord(int e, int off, fe& r) const {
    const uint32_t* p = rows + e * BTAB_ROW_WORDS + off;
    for (int i = 0; i < 10; i++) r.v[i] = p[i];
  }
};
struct DevProbe {
  uint32_t* out;
  __device__ void snap(int id, const fe& v) const {
    if (threadIdx.x < 4)
      for (int i = 0; i < 10; i++) out[(id * 4 + threadIdx.x) * 10 + i] = v.v[i];
  }
};
// timing probe: s_memtime at every snapshot point (lane 0 writes)
struct TimeProbe {
  unsigned long long* out;
  __device__ void snap(int id, const fe& v) const {
    asm volatile("" ::"v"(v.v[0]));
    unsigned long long t = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) out[id] = t;
  }
};
struct LdsTab {  // same layout as kernels.hip's DevATabQ
  uint2* lds;
  uint32_t t;
  __device__ void store(int e, const fe& c) {
    for (int k = 0; k < 5; k++) lds[(e * 5 + k) * 64 + t] = make_uint2(c.v[2 * k], c.v[2 * k + 1]);
  }
  __device__ void load(int e, fe& c) const {
    for (int k = 0; k < 5; k++) {
      const uint2 x = lds[(e * 5 + k) * 64 + t];
      c.v[2 * k] = x.x;
      c.v[2 * k + 1] = x.y;
    }
  }
  template <class Q>
  __device__ void load_signed(const Q& q, int e, bool neg, fe& c) const {
    const uint32_t src = (t & 2) ? t : (t ^ (neg ? 1u : 0u));
    for (int k = 0; k < 5; k++) {
      const uint2 x = lds[(e * 5 + k) * 64 + src];
      c.v[2 * k] = x.x;
      c.v[2 * k + 1] = x.y;
    }
    q_negate_lane3(c, (int)(t & 3), neg);
  }
};
__global__ __launch_bounds__(64, 1) void k_time(const uint32_t* pk, const uint32_t* sig, const uint8_t* msg, uint32_t mlen,
                       const uint32_t* btab, unsigned long long* ts, int* verdict) {
  DevQuad<4> q;
  DevBTabQ bt{btab};
  if (threadIdx.x == 0) ts[15] = __builtin_amdgcn_s_memtime();
  TimeProbe pr{ts};
  __shared__ uint2 lds[2 * 9 * 5 * 64];
  LdsTab ta{lds, threadIdx.x}, tr{lds + 9 * 5 * 64, threadIdx.x};
  bool v = q_verify<MODE_GO_STDLIB>(q, pk, sig, msg, mlen, bt, ta, tr, pr);
  verdict[threadIdx.x] = v;
  if (threadIdx.x == 0) ts[14] = __builtin_amdgcn_s_memtime();
}

__global__ void k_btab(uint32_t* rows) {  // the library's k_btab_init
  const int e = blockIdx.x * 64 + threadIdx.x;
  if (e < BTAB_TOTAL_ROWS) btab_row(rows + (size_t)e * BTAB_ROW_WORDS, e);
}

template <int VAR>
__global__ void k_probe(const uint32_t* pk, const uint32_t* sig, const uint8_t* msg, uint32_t mlen,
                        const uint32_t* btab, uint32_t* snaps, int* verdict) {
  DevQuad<VAR> q;
  DevBTabQ bt{btab};
  DevProbe pr{snaps};
  QArrayTab at, at2;
  bool v = q_verify<MODE_GO_STDLIB>(q, pk, sig, msg, mlen, bt, at, at2, pr);
  verdict[threadIdx.x] = v;
}

template <int PAT>
__global__ void k_dpp(int* out) {
  out[threadIdx.x] = __builtin_amdgcn_mov_dpp((int)(threadIdx.x * 10), PAT, 0xF, 0xF, true);
}

struct Exchange {
  std::barrier<> bar{4};
  fe slot[4];
};
struct HostQuad {
  int ln;
  Exchange* ex;
  int lane() const { return ln; }
  template <int PAT>
  void perm(fe& o, const fe& v) const {
    ex->slot[ln] = v;
    ex->bar.arrive_and_wait();
    const fe r = ex->slot[(PAT >> (2 * ln)) & 3];
    ex->bar.arrive_and_wait();
    o = r;
  }
  template <int PAT>
  void add_perm(fe& o, const fe& src, const fe& b) const {
    fe t;
    perm<PAT>(t, src);
    for (int i = 0; i < 10; i++) o.v[i] = t.v[i] + b.v[i];
  }
  template <int PAT>
  void xor_perm(fe& o, const fe& src, uint32_t k) const {
    perm<PAT>(o, src);
    for (int i = 0; i < 10; i++) o.v[i] ^= k;
  }
  template <int PAT>
  void perm_lane3(fe& o, const fe& src) const {
    perm<PAT>(o, src);
    for (int i = 0; i < 10; i++) o.v[i] = lane() == 3 ? o.v[i] : 0u;
  }
  template <int PAT>
  void permc(fe& o, const fe& v) const {
    perm<PAT>(o, v);
  }
  template <int PAT>
  uint32_t perm32(uint32_t x) const {
    fe t, o;
    fe_0(t);
    t.v[0] = x;
    perm<PAT>(o, t);
    return o.v[0];
  }
  bool any(bool x) const { return x; }
};
using HostBTabQ = LazyBTab;
struct HostProbe {
  uint32_t* out;
  int ln;
  void snap(int id, const fe& v) const {
    for (int i = 0; i < 10; i++) out[(id * 4 + ln) * 10 + i] = v.v[i];
  }
};

static void hex2w(uint32_t* w, const char* hex, int nw) {
  for (int i = 0; i < 4 * nw; i++) {
    unsigned b;
    sscanf(hex + 2 * i, "%2x", &b);
    ((uint8_t*)w)[i] = (uint8_t)b;
  }
}

int main() {
  {
    int* d;
    (void)hipMalloc(&d, 256);
    int h[64];
    hipLaunchKernelGGL(k_dpp<0x55>, dim3(1), dim3(64), 0, 0, d);
    (void)hipMemcpy(h, d, 256, hipMemcpyDeviceToHost);
    printf("dpp B1:");
    for (int i = 0; i < 8; i++) printf(" %d", h[i]);
    hipLaunchKernelGGL(k_dpp<(1 | (0 << 2) | (2 << 4) | (3 << 6))>, dim3(1), dim3(64), 0, 0, d);
    (void)hipMemcpy(h, d, 256, hipMemcpyDeviceToHost);
    printf("\ndpp SWAP01:");
    for (int i = 0; i < 8; i++) printf(" %d", h[i]);
    printf("\n");
  }
  // RFC 8032 test 2
  uint32_t pk[8], sig[16];
  hex2w(pk, "3d4017c3e843895a92b70aa74d1b7ebc9c982ccf2ec4968cc0cd55f12af4660c", 8);
  hex2w(sig, "92a009a9f0d4cab8720e820b5f642540a2b27b5416503f8fb3762223ebdb69da085ac1e43e15996e458f3613d0f11d8c387b2eaeb4302aeeb00d291612bb0c00", 16);
  uint8_t msg[4] = {0x72, 0, 0, 0};
  uint32_t mlen = 1;

  std::vector<uint32_t> btab(BT16_BASE * BTAB_ROW_WORDS);  // the radix-256 blocks, for the device check
  for (int e = 0; e < BT16_BASE; e++) btab_entry(&btab[e * BTAB_ROW_WORDS], e % BTAB_ENTRIES + 1, e / BTAB_ENTRIES);
  LazyBTab hbt;

  // host emulation
  std::vector<uint32_t> hs(NSNAP * 40, 0);
  bool hres[4];
  {
    Exchange ex;
    std::vector<std::thread> th;
    for (int l = 0; l < 4; l++)
      th.emplace_back([&, l] {
        HostQuad q{l, &ex};
        const HostBTabQ& bt = hbt;
        HostProbe pr{hs.data(), l};
        QArrayTab at, at2;
        hres[l] = q_verify<MODE_GO_STDLIB>(q, pk, sig, msg, mlen, bt, at, at2, pr);
      });
    for (auto& t : th) t.join();
  }
  // device
  uint32_t *dpk, *dsig, *dbt, *dsn;
  uint8_t* dmsg;
  int* dv;
  (void)hipMalloc(&dpk, 32);
  (void)hipMalloc(&dsig, 64);
  (void)hipMalloc(&dmsg, 16);
  (void)hipMalloc(&dbt, (size_t)BTAB_TOTAL_ROWS * BTAB_ROW_WORDS * 4);
  (void)hipMalloc(&dsn, NSNAP * 40 * 4);
  (void)hipMalloc(&dv, 64 * 4);
  (void)hipMemcpy(dpk, pk, 32, hipMemcpyHostToDevice);
  (void)hipMemcpy(dsig, sig, 64, hipMemcpyHostToDevice);
  (void)hipMemcpy(dmsg, msg, 4, hipMemcpyHostToDevice);
  // device-built table must equal the host-built one
  hipLaunchKernelGGL(k_btab, dim3((BTAB_TOTAL_ROWS + 63) / 64), dim3(64), 0, 0, dbt);
  std::vector<uint32_t> dbtab(btab.size());
  (void)hipMemcpy(dbtab.data(), dbt, btab.size() * 4, hipMemcpyDeviceToHost);
  printf("btab device==host: %d\n", (int)(dbtab == btab));
  auto run = [&](auto kern, const char* name) {
    (void)hipMemset(dsn, 0, NSNAP * 40 * 4);
    hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, dpk, dsig, dmsg, mlen, dbt, dsn, dv);
    std::vector<uint32_t> ds(NSNAP * 40);
    int dres[64];
    (void)hipMemcpy(ds.data(), dsn, ds.size() * 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(dres, dv, 256, hipMemcpyDeviceToHost);
    printf("[%s] host verdict %d%d%d%d device verdict %d%d%d%d\n", name, hres[0], hres[1], hres[2], hres[3], dres[0],
           dres[1], dres[2], dres[3]);
    for (int id = 0; id < NSNAP; id++) {
      bool same = true;
      for (int j = 0; j < 40; j++) same = same && hs[id * 40 + j] == ds[id * 40 + j];
      if (!same) {
        printf("  first diff at snap %d\n", id);
        for (int l = 0; l < 4; l++) {
          printf("  lane %d host:", l);
          for (int i = 0; i < 10; i++) printf(" %07x", hs[(id * 4 + l) * 10 + i]);
          printf("\n  lane %d dev :", l);
          for (int i = 0; i < 10; i++) printf(" %07x", ds[(id * 4 + l) * 10 + i]);
          printf("\n");
        }
        break;
      }
    }
  };
  {
    unsigned long long* dts;
    (void)hipMalloc(&dts, 16 * 8);
    for (int rep = 0; rep < 3; rep++) {
      hipLaunchKernelGGL(k_time, dim3(1), dim3(64), 0, 0, dpk, dsig, dmsg, mlen, dbt, dts, dv);
      unsigned long long ts[16];
      (void)hipMemcpy(ts, dts, 16 * 8, hipMemcpyDeviceToHost);
      printf("cycles: decode %llu sha %llu halfscalar %llu tables+win0 %llu win1 %llu win2 %llu win3 %llu loop(rest) %llu final %llu total %llu\n",
             ts[0] - ts[15], ts[2] - ts[1], ts[11] - ts[2], ts[6] - ts[11], ts[7] - ts[6], ts[8] - ts[7], ts[9] - ts[8],
             ts[10] - ts[6], ts[14] - ts[10], ts[14] - ts[15]);
    }
  }
  run(k_probe<0>, "mov_dpp");
  run(k_probe<1>, "update_dpp");
  run(k_probe<2>, "shfl");
  run(k_probe<3>, "ds_swizzle");
  return 0;
}
