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

__global__ __launch_bounds__(256) void k_sign_bytes(uint32_t n, const SbTemplate* __restrict__ tmpls,
                                                    const uint8_t* __restrict__ blob,
                                                    const uint32_t* __restrict__ tidx,
                                                    const uint8_t* __restrict__ commit_flag,
                                                    const int64_t* __restrict__ sec,
                                                    const int32_t* __restrict__ nanos,
                                                    const uint32_t* __restrict__ off, uint8_t* __restrict__ msg) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  // the 16 zero bytes after the last message (the SHA block loader's slack)
  if (i == n - 1) {
#pragma unroll
    for (int j = 0; j < 16; j++) msg[off[n] + j] = 0;
  }
  const SbTemplate t = tmpls[tidx[i]];
  DevBytes out{msg + off[i]};
  sb_write(out, t, blob, commit_flag[i] != 0, sec[i], nanos[i]);
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
