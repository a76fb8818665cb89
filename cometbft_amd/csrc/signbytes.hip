// signbytes.hip -- k_sign_bytes: CanonicalVote sign-bytes of commit
// signatures written on the device from per-commit templates (signbytes.h;
// SURVEY 8f rank 1). One thread per signature writes its message at the
// offset the host computed with the same length functions; the verify kernels
// then read the messages from HBM as usual.
#include <hip/hip_runtime.h>

#include "kernels.h"
#include "signbytes.h"

namespace cmtv {

struct DevBytes {
  uint8_t* __restrict__ p;
  __device__ __forceinline__ void put(uint32_t pos, uint8_t b) { p[pos] = b; }
  __device__ __forceinline__ void copy(uint32_t pos, const uint8_t* src, uint32_t len) {
    for (uint32_t i = 0; i < len; i++) p[pos + i] = src[i];
  }
};

// The same writer into the block's LDS image
struct LdsBytes {
  uint8_t* p;
  __device__ __forceinline__ void put(uint32_t pos, uint8_t b) { p[pos] = b; }
  __device__ __forceinline__ void copy(uint32_t pos, const uint8_t* src, uint32_t len) {
    for (uint32_t i = 0; i < len; i++) p[pos + i] = src[i];
  }
};

// LDS image of one block's messages: 256 messages of up to 188 bytes on
// average (commit votes are 116-161 bytes), + 4 bytes of alignment slack
constexpr uint32_t kSbLdsBytes = 256 * 188 + 4;

// A block of 256 signatures writes its messages -- contiguous in the output
// -- into an LDS image aligned like the output (byte p of the image is output
// byte (off[first] & ~3) + p), then copies the image out with 4-byte stores
// that a wave issues as whole cache lines. Writing each message byte by byte
// straight to HBM (one store instruction per byte per lane, 64 scattered
// lines each) cost ~280 us per 2^20 signatures. A block whose messages do not
// fit the image writes them directly.
__global__ __launch_bounds__(256) void k_sign_bytes(uint32_t n, const SbTemplate* __restrict__ tmpls,
                                                    const uint8_t* __restrict__ blob,
                                                    const uint32_t* __restrict__ tidx,
                                                    const uint8_t* __restrict__ commit_flag,
                                                    const int64_t* __restrict__ sec,
                                                    const int32_t* __restrict__ nanos,
                                                    const uint32_t* __restrict__ off, uint8_t* __restrict__ msg) {
  __shared__ uint8_t img[kSbLdsBytes];
  const uint32_t b0 = blockIdx.x * 256, i = b0 + threadIdx.x;
  const uint32_t b1 = b0 + 256 < n ? b0 + 256 : n;
  const uint32_t start = off[b0], span = off[b1] - start;
  const uint32_t base = start & ~3u, lo = start - base;
  // the 16 zero bytes after the last message (the SHA block loader's slack)
  if (i == n - 1) {
#pragma unroll
    for (int j = 0; j < 16; j++) msg[off[n] + j] = 0;
  }
  if (lo + span > kSbLdsBytes) {  // block-uniform: too long for the image
    if (i < n) {
      const SbTemplate t = tmpls[tidx[i]];
      DevBytes out{msg + off[i]};
      sb_write(out, t, blob, commit_flag[i] != 0, sec[i], nanos[i]);
    }
    return;
  }
  if (i < n) {
    const SbTemplate t = tmpls[tidx[i]];
    LdsBytes out{img + lo + (off[i] - start)};
    sb_write(out, t, blob, commit_flag[i] != 0, sec[i], nanos[i]);
  }
  __syncthreads();
  // image bytes [lo, lo + span) -> msg + base + [lo, lo + span): whole
  // dwords inside the span by every thread, the partial ones at its two ends
  // byte by byte (their other bytes belong to the neighbouring blocks)
  const uint32_t end = lo + span;
  const uint32_t d0 = (lo + 3) / 4, d1 = end / 4;
  uint32_t* out32 = reinterpret_cast<uint32_t*>(msg + base);
  const uint32_t* img32 = reinterpret_cast<const uint32_t*>(img);
  for (uint32_t d = d0 + threadIdx.x; d < d1; d += 256) out32[d] = img32[d];
  if (threadIdx.x == 0) {
    const uint32_t h_end = 4 * d0 < end ? 4 * d0 : end;
    for (uint32_t p = lo; p < h_end; p++) msg[base + p] = img[p];
    for (uint32_t p = (4 * d1 > h_end ? 4 * d1 : h_end); p < end; p++) msg[base + p] = img[p];
  }
}

// ---- direct chunks: the per-signature staging built on the device from the
// caller's arrays (DMA'd from its pinned arena), so the host packs nothing
// per signature (pipeline.cpp). Three steps on the chunk's exec stream:
//   k_bulk_gather   one workgroup per commit: signature, flag, seconds, nanos,
//                   template / key index of each planned signature into the
//                   chunk layout, and its message offset within the commit
//                   (a workgroup scan of sb_msg_len); the commit's message
//                   bytes into ctot[c]
//   k_bulk_bases    one workgroup: exclusive scan of ctot -> cbase, off[m]
//   k_bulk_rebase   off[i] += cbase[tidx[i]]
// after which k_sign_bytes and the verify kernel run as for a packed chunk.

// inclusive sum of x over the 256 threads' positions; *total = block total
__device__ __forceinline__ uint32_t block_scan256(uint32_t x, uint32_t* wsum, uint32_t* total) {
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (uint32_t j = 0; j < 4; j++) {
    const uint32_t v = wsum[j];
    pre += j < w ? v : 0;
    tot += v;
  }
  __syncthreads();  // wsum is rewritten by the next round
  *total = tot;
  return pre + x;
}

__global__ __launch_bounds__(256) void k_bulk_gather(const BulkDesc* __restrict__ desc,
                                                     const SbTemplate* __restrict__ tmpls,
                                                     const uint8_t* __restrict__ arena, uint32_t* __restrict__ kidx,
                                                     uint8_t* __restrict__ sig, uint32_t* __restrict__ off,
                                                     uint32_t* __restrict__ tidx, uint8_t* __restrict__ flag,
                                                     int64_t* __restrict__ sec, int32_t* __restrict__ nanos,
                                                     uint32_t* __restrict__ ctot) {
  __shared__ uint32_t wsum[4];
  const uint32_t c = blockIdx.x;
  const BulkDesc D = desc[c];
  uint32_t carry = 0;
  if (D.m) {
    const SbTemplate T = tmpls[c];
    for (uint32_t k0 = 0; k0 < D.m; k0 += 256) {
      const uint32_t k = k0 + threadIdx.x;
      uint32_t len = 0;
      if (k < D.m) {
        const uint32_t i = D.sp + k;
        const bool fb = arena[D.flags + k] == 2;  // BlockIDFlagCommit
        const int64_t s = *reinterpret_cast<const int64_t*>(arena + D.sec + 8ull * k);
        const int32_t ns = *reinterpret_cast<const int32_t*>(arena + D.nanos + 4ull * k);
        const uint2* src = reinterpret_cast<const uint2*>(arena + D.sig + 64ull * k);
        uint2* dst = reinterpret_cast<uint2*>(sig + 64ull * i);
#pragma unroll
        for (int j = 0; j < 8; j++) dst[j] = src[j];
        flag[i] = fb ? 1 : 0;
        sec[i] = s;
        nanos[i] = ns;
        tidx[i] = c;
        kidx[i] = k;  // a prefix plan: signature k is by validator k
        len = sb_msg_len(T, fb, s, ns);
      }
      uint32_t tot;
      const uint32_t inc = block_scan256(len, wsum, &tot);
      if (k < D.m) off[D.sp + k] = carry + inc - len;
      carry += tot;
    }
  }
  if (threadIdx.x == 0) ctot[c] = carry;
}

__global__ __launch_bounds__(256) void k_bulk_bases(uint32_t n_c, const uint32_t* __restrict__ ctot,
                                                    uint32_t* __restrict__ cbase, uint32_t* __restrict__ off,
                                                    uint32_t m) {
  __shared__ uint32_t wsum[4];
  uint32_t carry = 0;
  for (uint32_t c0 = 0; c0 < n_c; c0 += 256) {
    const uint32_t c = c0 + threadIdx.x;
    const uint32_t v = c < n_c ? ctot[c] : 0;
    uint32_t tot;
    const uint32_t inc = block_scan256(v, wsum, &tot);
    if (c < n_c) cbase[c] = carry + inc - v;
    carry += tot;
  }
  if (threadIdx.x == 0) off[m] = carry;
}

__global__ __launch_bounds__(256) void k_bulk_rebase(uint32_t m, const uint32_t* __restrict__ cbase,
                                                     const uint32_t* __restrict__ tidx, uint32_t* __restrict__ off) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i < m) off[i] += cbase[tidx[i]];
}

hipError_t launch_bulk_gather(uint32_t n_c, uint32_t m, const void* desc, const void* tmpls, const uint8_t* arena,
                              uint32_t* kidx, uint8_t* sig, uint32_t* off, uint32_t* tidx, uint8_t* flag,
                              int64_t* sec, int32_t* nanos, uint32_t* ctot, uint32_t* cbase, hipStream_t s) {
  if (n_c == 0) return hipSuccess;
  hipLaunchKernelGGL(k_bulk_gather, dim3(n_c), dim3(256), 0, s, static_cast<const BulkDesc*>(desc),
                     static_cast<const SbTemplate*>(tmpls), arena, kidx, sig, off, tidx, flag, sec, nanos, ctot);
  hipLaunchKernelGGL(k_bulk_bases, dim3(1), dim3(256), 0, s, n_c, ctot, cbase, off, m);
  if (m) hipLaunchKernelGGL(k_bulk_rebase, dim3((m + 255) / 256), dim3(256), 0, s, m, cbase, tidx, off);
  return hipGetLastError();
}

hipError_t launch_sign_bytes(uint32_t n, const void* tmpls, const uint8_t* blob, const uint32_t* tidx,
                             const uint8_t* commit_flag, const int64_t* sec, const int32_t* nanos,
                             const uint32_t* off, uint8_t* msg, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_sign_bytes, dim3((n + 255) / 256), dim3(256), 0, s, n,
                     static_cast<const SbTemplate*>(tmpls), blob, tidx, commit_flag, sec, nanos, off, msg);
  return hipGetLastError();
}

}  // namespace cmtv
