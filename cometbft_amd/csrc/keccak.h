// keccak.h -- Keccak-f[1600] (FIPS 202) for the merlin/STROBE transcript of
// sr25519 verification (merlin.h). One permutation per call on 25 64-bit
// lanes held in registers; on gfx950 every 64-bit XOR/AND is a pair of 32-bit
// VALU ops and every rotation a pair of v_alignbit_b32. The round loop stays
// rolled; the 25-lane theta/rho/pi/chi body is fully unrolled so every lane
// index and rotation count is a compile-time constant (no scratch).
#pragma once
#include <stdint.h>

#ifndef CMTV_HD
#define CMTV_HD __host__ __device__ __forceinline__
#endif

namespace cmtv {

CMTV_HD uint64_t keccak_rc(int r) {
  const uint64_t RC[24] = {
      0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808AULL, 0x8000000080008000ULL,
      0x000000000000808BULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
      0x000000000000008AULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000AULL,
      0x000000008000808BULL, 0x800000000000008BULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
      0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800AULL, 0x800000008000000AULL,
      0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};
  return RC[r];
}

// 64-bit rotate; n is a constant after unrolling. On the device each half is
// one funnel shift (v_alignbit_b32) instead of two 64-bit shifts and an or.
CMTV_HD uint64_t keccak_rotl(uint64_t x, int n) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  const uint32_t h = n < 32 ? hi : lo, l = n < 32 ? lo : hi;
  const int m = n & 31;
  if (m == 0) return ((uint64_t)h << 32) | l;
  return ((uint64_t)__builtin_amdgcn_alignbit(h, l, 32 - m) << 32) | __builtin_amdgcn_alignbit(l, h, 32 - m);
#else
  return n ? (x << n) | (x >> (64 - n)) : x;
#endif
}

// rho offset of lane i = x + 5y, and pi destination y + 5((2x + 3y) mod 5)
CMTV_HD int keccak_rho(int i) {
  const int R[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};
  return R[i];
}
CMTV_HD int keccak_pi(int i) {
  const int x = i % 5, y = i / 5;
  return y + 5 * ((2 * x + 3 * y) % 5);
}

CMTV_HD void keccak_f1600(uint64_t a[25]) {
#pragma unroll 1
  for (int rnd = 0; rnd < 24; rnd++) {
    uint64_t c[5], b[25];
#pragma unroll
    for (int x = 0; x < 5; x++) c[x] = a[x] ^ a[x + 5] ^ a[x + 10] ^ a[x + 15] ^ a[x + 20];
#pragma unroll
    for (int x = 0; x < 5; x++) {
      const uint64_t d = c[(x + 4) % 5] ^ keccak_rotl(c[(x + 1) % 5], 1);
#pragma unroll
      for (int y = 0; y < 5; y++) a[x + 5 * y] ^= d;
    }
#pragma unroll
    for (int i = 0; i < 25; i++) b[keccak_pi(i)] = keccak_rotl(a[i], keccak_rho(i));
#pragma unroll
    for (int y = 0; y < 5; y++)
#pragma unroll
      for (int x = 0; x < 5; x++)
        a[x + 5 * y] = b[x + 5 * y] ^ (~b[(x + 1) % 5 + 5 * y] & b[(x + 2) % 5 + 5 * y]);
    a[0] ^= keccak_rc(rnd);
  }
}

}  // namespace cmtv
