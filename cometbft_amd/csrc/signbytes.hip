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

hipError_t launch_sign_bytes(uint32_t n, const void* tmpls, const uint8_t* blob, const uint32_t* tidx,
                             const uint8_t* commit_flag, const int64_t* sec, const int32_t* nanos,
                             const uint32_t* off, uint8_t* msg, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_sign_bytes, dim3((n + 255) / 256), dim3(256), 0, s, n,
                     static_cast<const SbTemplate*>(tmpls), blob, tidx, commit_flag, sec, nanos, off, msg);
  return hipGetLastError();
}

}  // namespace cmtv
