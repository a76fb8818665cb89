// sc25519.h -- scalars modulo L = 2^252 + 27742317777372353535851937790883648493.
//
//   sc_reduce512   : Scalar.SetUniformBytes (64-byte hash -> k mod L)
//   sc_is_canonical: Scalar.SetCanonicalBytes acceptance test (s < L)
//   sc_muladd      : (a*b + c) mod L (deterministic RFC 8032 signing, test data)
//   signed_digits  : t = s + 0x88..8 (radix-16) / 0x80..80 (radix-256) so that
//                    every signed digit is "window - 8" / "window - 128" and can
//                    be read left-to-right with no carry chain -- the recoding
//                    that keeps all 64 lanes of a wave on the same add schedule
//                    (a sparse wNAF would make every position an add for SOME
//                    lane and so cost the whole wave an add per bit).
//
// Reduction folds 2^252 == -delta (delta = L - 2^252 < 2^125) three times with
// a fixed schedule sized for 512-bit input, keeping every intermediate
// non-negative by adding a multiple of L first, then one conditional subtract.
#pragma once
#include <stdint.h>

#ifndef CMTV_HD
#define CMTV_HD __host__ __device__ __forceinline__
#endif

namespace cmtv {

CMTV_HD uint32_t sc_L(int i) {
  const uint32_t L[8] = {0x5cf5d3ed, 0x5812631a, 0xa2f79cd6, 0x14def9de, 0, 0, 0, 0x10000000};
  return L[i];
}
CMTV_HD uint32_t sc_delta(int i) {
  const uint32_t D[4] = {0x5cf5d3ed, 0x5812631a, 0xa2f79cd6, 0x14def9de};
  return D[i];
}

// out[NOUT] = (x mod 2^252) + L * 2^SHIFT - (x >> 252) * delta
template <int NIN, int NOUT, int SHIFT>
CMTV_HD void sc_fold(uint32_t out[NOUT], const uint32_t x[NIN]) {
  constexpr int NH = NIN - 7;  // limbs of x >> 252
  uint32_t h[NH];
#pragma unroll
  for (int j = 0; j < NH; j++) {
    uint32_t lo = x[7 + j] >> 28;
    uint32_t hi = (8 + j < NIN) ? (x[8 + j] << 4) : 0;
    h[j] = lo | hi;
  }
  // hd = h * delta
  uint32_t hd[NOUT];
#pragma unroll
  for (int i = 0; i < NOUT; i++) hd[i] = 0;
#pragma unroll
  for (int i = 0; i < NH; i++) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      if (i + j < NOUT) {
        uint64_t t = (uint64_t)h[i] * sc_delta(j) + hd[i + j] + carry;
        hd[i + j] = (uint32_t)t;
        carry = t >> 32;
      }
    }
#pragma unroll
    for (int k = i + 4; k < NOUT; k++) {
      uint64_t t = (uint64_t)hd[k] + carry;
      hd[k] = (uint32_t)t;
      carry = t >> 32;
    }
  }
  // m = L << SHIFT
  constexpr int WS = SHIFT / 32, BS = SHIFT % 32;
  int64_t acc = 0;
#pragma unroll
  for (int i = 0; i < NOUT; i++) {
    uint32_t li = (i < 7) ? x[i] : (i == 7 ? (x[7] & 0x0FFFFFFF) : 0);
    uint32_t mi = 0;
    const int k = i - WS;
    if (k >= 0 && k < 8) mi |= BS ? (sc_L(k) << BS) : sc_L(k);
    if (BS && k - 1 >= 0 && k - 1 < 8) mi |= sc_L(k - 1) >> (32 - BS);
    acc += (int64_t)li + (int64_t)mi - (int64_t)hd[i];
    out[i] = (uint32_t)acc;
    acc >>= 32;  // arithmetic: borrow propagates as -1
  }
}

// r = x mod L, x = 16 little-endian words (512 bits)
CMTV_HD void sc_reduce512(uint32_t r[8], const uint32_t x[16]) {
  uint32_t a[13], b[10], c[8];
  sc_fold<16, 13, 134>(a, x);  // < 2^252 + 2^387
  sc_fold<13, 10, 9>(b, a);    // < 2^252 + 2^262
  sc_fold<10, 8, 0>(c, b);     // < 2^252 + L < 2L
  // conditional subtract L
  uint32_t d[8];
  int64_t acc = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    acc += (int64_t)c[i] - (int64_t)sc_L(i);
    d[i] = (uint32_t)acc;
    acc >>= 32;
  }
  const bool ge = (acc == 0);  // no final borrow -> c >= L
#pragma unroll
  for (int i = 0; i < 8; i++) r[i] = ge ? d[i] : c[i];
}

// s < L ?
CMTV_HD bool sc_is_canonical(const uint32_t s[8]) {
  int64_t acc = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    acc += (int64_t)s[i] - (int64_t)sc_L(i);
    acc >>= 32;
  }
  return acc != 0;  // borrow -> s < L
}

// r = (a*b + c) mod L  (all 8-word little-endian)
CMTV_HD void sc_muladd(uint32_t r[8], const uint32_t a[8], const uint32_t b[8], const uint32_t c[8]) {
  uint32_t p[16];
#pragma unroll
  for (int i = 0; i < 16; i++) p[i] = (i < 8) ? c[i] : 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      uint64_t t = (uint64_t)a[i] * b[j] + p[i + j] + carry;
      p[i + j] = (uint32_t)t;
      carry = t >> 32;
    }
#pragma unroll
    for (int k = i + 8; k < 16; k++) {
      uint64_t t = (uint64_t)p[k] + carry;
      p[k] = (uint32_t)t;
      carry = t >> 32;
    }
  }
  sc_reduce512(r, p);
}

// t = s + (pattern repeated): radix-16 signed digits use 0x88888888,
// radix-256 use 0x80808080.
CMTV_HD void sc_bias(uint32_t t[8], const uint32_t s[8], uint32_t pattern) {
  uint64_t carry = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t v = (uint64_t)s[i] + pattern + carry;
    t[i] = (uint32_t)v;
    carry = v >> 32;
  }
}

// t <<= n (0 < n < 32), returns the bits shifted out of the top
CMTV_HD uint32_t sc_shift_out(uint32_t t[8], int n) {
  const uint32_t out = t[7] >> (32 - n);
#pragma unroll
  for (int i = 7; i > 0; i--) t[i] = (t[i] << n) | (t[i - 1] >> (32 - n));
  t[0] <<= n;
  return out;
}

}  // namespace cmtv
