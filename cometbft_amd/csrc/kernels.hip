// kernels.hip -- gfx950 kernels of libcmtverify.
//
//   k_btab_init   : builds the shared fixed-base table (1..128)B (affine niels)
//   k_verify<MODE>: one signature per lane: SHA-512 + mod-L + decompression +
//                   Straus [s]B - [k]A + GO_STDLIB / ZIP215 final check, then a
//                   wavefront ballot packs 64 verdicts into one bitmap word
//   k_pubkey / k_sign : RFC 8032 key generation and signing (synthetic data)
//
// Memory layout (HBM):
//   pk   : n x 32 B   (row i = 8 words, read as 2 x dwordx4)
//   sig  : n x 64 B   (row i = 16 words, 4 x dwordx4)
//   msg  : flat bytes + (n+1) u32 offsets
//   btab : 128 rows x 32 words (ypx, ymx, 2dxy; 10 limbs each; 2 pad) = 16 KiB,
//          L1/L2-resident, rows gathered per lane as 8 x dwordx4
//   atab : per-lane (1..8)(-A) cached table, word-major / lane-minor
//          [(e*40 + w) * stride + lane] so each of the 40 word loads of a row
//          is one coalesced 256-byte wave access when lanes share the digit
//          magnitude, and at most 8 distinct 256-byte segments otherwise.
#include <hip/hip_runtime.h>

#include "kernels.h"
#include "verify_core.h"

namespace cmtv {

struct DevBTab {
  const uint32_t* __restrict__ rows;
  __device__ __forceinline__ void load(int e, ge_niels& r) const {
    const uint4* p = reinterpret_cast<const uint4*>(rows + e * BTAB_ROW_WORDS);
    uint32_t w[32];
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const uint4 v = p[q];
      w[4 * q] = v.x;
      w[4 * q + 1] = v.y;
      w[4 * q + 2] = v.z;
      w[4 * q + 3] = v.w;
    }
#pragma unroll
    for (int i = 0; i < 10; i++) {
      r.ypx.v[i] = w[i];
      r.ymx.v[i] = w[10 + i];
      r.xy2d.v[i] = w[20 + i];
    }
  }
};

struct DevATab {
  uint32_t* __restrict__ base;
  uint32_t stride;
  uint32_t lane;
  __device__ __forceinline__ void load(int e, ge_cached& r) const {
    const uint32_t* p = base + (size_t)(e * 40) * stride + lane;
#pragma unroll
    for (int i = 0; i < 10; i++) {
      r.YpX.v[i] = p[(size_t)i * stride];
      r.YmX.v[i] = p[(size_t)(10 + i) * stride];
      r.Z.v[i] = p[(size_t)(20 + i) * stride];
      r.T2d.v[i] = p[(size_t)(30 + i) * stride];
    }
  }
  __device__ __forceinline__ void store(int e, const ge_cached& r) {
    uint32_t* p = base + (size_t)(e * 40) * stride + lane;
#pragma unroll
    for (int i = 0; i < 10; i++) {
      p[(size_t)i * stride] = r.YpX.v[i];
      p[(size_t)(10 + i) * stride] = r.YmX.v[i];
      p[(size_t)(20 + i) * stride] = r.Z.v[i];
      p[(size_t)(30 + i) * stride] = r.T2d.v[i];
    }
  }
};

__device__ __forceinline__ void load_words(uint32_t* w, const uint32_t* __restrict__ src, int nquads) {
  const uint4* p = reinterpret_cast<const uint4*>(src);
#pragma unroll
  for (int q = 0; q < nquads; q++) {
    const uint4 v = p[q];
    w[4 * q] = v.x;
    w[4 * q + 1] = v.y;
    w[4 * q + 2] = v.z;
    w[4 * q + 3] = v.w;
  }
}

__global__ __launch_bounds__(64) void k_btab_init(uint32_t* __restrict__ rows) {
  const int m = blockIdx.x * 64 + threadIdx.x + 1;
  if (m > BTAB_ENTRIES) return;
  uint32_t row[BTAB_ROW_WORDS];
  btab_entry(row, m);
#pragma unroll
  for (int i = 0; i < BTAB_ROW_WORDS; i++) rows[(m - 1) * BTAB_ROW_WORDS + i] = row[i];
}

template <uint32_t MODE>
__global__ __launch_bounds__(64) void k_verify(uint32_t n, const uint32_t* __restrict__ pk,
                                               const uint32_t* __restrict__ sig, const uint8_t* __restrict__ msg,
                                               const uint32_t* __restrict__ off, const uint32_t* __restrict__ btab,
                                               uint32_t* __restrict__ atab, uint8_t* __restrict__ out_valid,
                                               uint64_t* __restrict__ out_bitmap) {
  const uint32_t gid = blockIdx.x * 64 + threadIdx.x;
  const bool active = gid < n;
  const uint32_t i = active ? gid : n - 1;
  uint32_t pkw[8], sigw[16];
  load_words(pkw, pk + 8 * (size_t)i, 2);
  load_words(sigw, sig + 16 * (size_t)i, 4);
  const uint32_t m0 = off[i], m1 = off[i + 1];
  DevATab at{atab, gridDim.x * 64u, gid};
  DevBTab bt{btab};
  bool v = verify_one<MODE>(pkw, sigw, msg + m0, m1 - m0, at, bt);
  v = v && active;
  if (active && out_valid) out_valid[gid] = v ? 1 : 0;
  const uint64_t mask = __ballot(v);
  if (threadIdx.x == 0 && out_bitmap) out_bitmap[gid >> 6] = mask;
}

__global__ __launch_bounds__(64) void k_pubkey(uint32_t n, const uint32_t* __restrict__ seeds,
                                               const uint32_t* __restrict__ btab, uint32_t* __restrict__ out_pk) {
  const uint32_t gid = blockIdx.x * 64 + threadIdx.x;
  if (gid >= n) return;
  uint32_t sw[8], pkw[8];
  load_words(sw, seeds + 8 * (size_t)gid, 2);
  DevBTab bt{btab};
  pubkey_from_seed(pkw, sw, bt);
#pragma unroll
  for (int q = 0; q < 8; q++) out_pk[8 * (size_t)gid + q] = pkw[q];
}

__global__ __launch_bounds__(64) void k_sign(uint32_t n, const uint32_t* __restrict__ seeds,
                                             const uint32_t* __restrict__ key_idx, const uint8_t* __restrict__ msg,
                                             const uint32_t* __restrict__ off, const uint32_t* __restrict__ btab,
                                             uint32_t* __restrict__ out_sig) {
  const uint32_t gid = blockIdx.x * 64 + threadIdx.x;
  if (gid >= n) return;
  const uint32_t kid = key_idx ? key_idx[gid] : gid;
  uint32_t sw[8], sg[16];
  load_words(sw, seeds + 8 * (size_t)kid, 2);
  DevBTab bt{btab};
  const uint32_t m0 = off[gid], m1 = off[gid + 1];
  sign_one(sg, sw, msg + m0, m1 - m0, bt);
#pragma unroll
  for (int q = 0; q < 16; q++) out_sig[16 * (size_t)gid + q] = sg[q];
}

static inline unsigned blocks_for(uint32_t n) { return (n + 63) / 64; }

hipError_t launch_btab_init(uint32_t* d_rows, hipStream_t s) {
  hipLaunchKernelGGL(k_btab_init, dim3(blocks_for(BTAB_ENTRIES)), dim3(64), 0, s, d_rows);
  return hipGetLastError();
}

hipError_t launch_verify(uint32_t mode, uint32_t n, const void* pk, const void* sig, const void* msg,
                         const void* off, const uint32_t* btab, uint32_t* atab, void* valid, void* bitmap,
                         hipStream_t s) {
  if (n == 0) return hipSuccess;
  const dim3 grid(blocks_for(n)), block(64);
  auto pkp = static_cast<const uint32_t*>(pk);
  auto sgp = static_cast<const uint32_t*>(sig);
  auto mp = static_cast<const uint8_t*>(msg);
  auto op = static_cast<const uint32_t*>(off);
  auto vp = static_cast<uint8_t*>(valid);
  auto bp = static_cast<uint64_t*>(bitmap);
  if (mode == MODE_ZIP215)
    hipLaunchKernelGGL(k_verify<MODE_ZIP215>, grid, block, 0, s, n, pkp, sgp, mp, op, btab, atab, vp, bp);
  else
    hipLaunchKernelGGL(k_verify<MODE_GO_STDLIB>, grid, block, 0, s, n, pkp, sgp, mp, op, btab, atab, vp, bp);
  return hipGetLastError();
}

hipError_t launch_pubkey(uint32_t n, const void* seeds, const uint32_t* btab, void* out_pk, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_pubkey, dim3(blocks_for(n)), dim3(64), 0, s, n, static_cast<const uint32_t*>(seeds), btab,
                     static_cast<uint32_t*>(out_pk));
  return hipGetLastError();
}

hipError_t launch_sign(uint32_t n, const void* seeds, const void* key_idx, const void* msg, const void* off,
                       const uint32_t* btab, void* out_sig, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_sign, dim3(blocks_for(n)), dim3(64), 0, s, n, static_cast<const uint32_t*>(seeds),
                     static_cast<const uint32_t*>(key_idx), static_cast<const uint8_t*>(msg),
                     static_cast<const uint32_t*>(off), btab, static_cast<uint32_t*>(out_sig));
  return hipGetLastError();
}

}  // namespace cmtv
