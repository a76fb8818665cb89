// halfscalar.h -- half-size scalar decomposition for signature verification.
//
// Verification asks whether R' = [s]B - [k]A equals R. For any integers
// (k1, k2) with k1 == k2 * k (mod 8L),
//
//     [k2](R' - R) = [k2 s mod L]B - [k1]A - [k2]R
//
// because every point of edwards25519 has order dividing 8L (so [k2 k]A =
// [k1]A even for A with a torsion component) and B has order L. The partial
// extended Euclid on (8L, k) yields such a pair with |k1|, |k2| ~ 2^127
// (Antipa et al., "Accelerated verification of ECDSA signatures", SAC 2005;
// Pornin, "Optimized lattice basis reduction in dimension 2", 2020), which
// halves the doublings of the variable-base part: 33 four-bit windows shared
// by A, R and the two halves of the fixed-base scalar instead of 64.
//
// Exactness (the verdicts must equal Go 1.19 crypto/ed25519.Verify's,
// /root/reference/crypto/ed25519/ed25519.go:148-155):
//   * GO_STDLIB (odd_k2): k2 is chosen ODD, and 0 < |k2| < L, so
//     gcd(k2, 8L) = 1 and [k2]X = O  <=>  X = O. Cofactorless mode therefore
//     checks R' == R exactly; with R canonical this is encode(R') == R bytes.
//   * ZIP215 checks [8][k2](R' - R) = O  <=>  [8](R' - R) = O, which needs
//     only L not dividing k2 (0 < |k2| < L): any parity will do, so the
//     shorter of the two reduced basis vectors is taken -- never above 128
//     bits in 3e5 random k, against 1.2% above 130 bits for the odd choice.
//   * The window count follows the pair's size: 33 windows hold pairs up to
//     130 bits (every ZIP-215 pair; all but 1.2% of odd pairs), 34 / 35 /
//     36 / 37 windows up to 134 / 138 / 142 / 146 bits. Only if no pair fits
//     146 bits (odd: about 1e-6), or a quotient >= 2^31 appears, is the
//     decomposition marked `wide`: the caller then uses k1 = k, k2 = 1 over
//     64 windows -- the same equation, so no input changes its verdict, only
//     its cost. (The window count is uniform over a wave, so with a plain
//     fixed-or-64 rule one such signature in a 10k commit -- ~40% of
//     commits -- made its whole wave run 64 windows.)
//
// Arithmetic: the Euclid runs on 8-word values kept left-normalised (r0's top
// bit at bit 255, both remainders shifted by the same e) and t values in
// 6-word two's complement. Lehmer rounds run ~9 Euclid steps at a time on the
// 30-bit leading digits (single-word cofactors, exact quotients by f64
// division) and apply the 2x2 cofactor matrix to the full values once per
// round: ~10 multi-word updates per scalar instead of ~75. A round that
// cannot certify a quotient falls back to one exact multi-word step, whose
// quotient comes from the top 64 bits in one f64 division corrected by at
// most a few add/subtract steps.
#pragma once
#include <math.h>
#include <stdint.h>

#include "sc25519.h"

#ifndef CMTV_HD
#define CMTV_HD __host__ __device__ __forceinline__
#endif

namespace cmtv {

constexpr int HS_WINDOWS = 33;      // 4-bit windows for normal pairs (132 bits)
constexpr int HS_MAX_WINDOWS = 37;  // graded: up to 37 windows before the wide fallback
constexpr int HS_WIDE_WINDOWS = 64; // k1 = k, k2 = 1
constexpr int HS_MAX_BITS = 130;    // (2^130 + bias) < 16^33 for the signed-digit bias
// windows for a pair of `bits` bits: (2^bits + bias) < 16^W  <=>  bits <= 4W - 2
CMTV_HD int hs_windows_for(int bits) { return bits <= HS_MAX_BITS ? HS_WINDOWS : (bits + 5) / 4; }
constexpr int HS_MAX_ROUNDS = 192;  // outer rounds before giving up (Lehmer: ~10; exact steps: ~75)
constexpr int HS_MAX_INNER = 40;    // Lehmer inner steps per round (30-bit digits: ~9)

// A branch condition of the split. UNI: every lane of the wave holds the same
// scalar (the row kernels' helper waves), so the condition is taken from the
// ballot -- a scalar compare and branch instead of the exec-mask bookkeeping
// of a divergent one (~a quarter of the Lehmer loop's instructions).
template <bool UNI>
CMTV_HD bool hs_uni(bool c) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (UNI) return __builtin_amdgcn_ballot_w64(c) != 0;
#endif
  return c;
}

struct HalfScalars {
  uint32_t k1[8];  // >= 0
  uint32_t k2[8];  // |k2|, odd
  bool k2_neg;
  bool wide;
  int windows;     // 33..37 (the pair's size), HS_WIDE_WINDOWS when wide
};

CMTV_HD uint32_t hs_N(int i) {  // 8L
  const uint32_t N[8] = {0xe7ae9f68u, 0xc09318d2u, 0x17bce6b2u, 0xa6f7cef5u, 0u, 0u, 0u, 0x80000000u};
  return N[i];
}

CMTV_HD int hs_clz(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return x ? __clz((int)x) : 32;
#else
  return x ? __builtin_clz(x) : 32;
#endif
}

// bit length of an 8-word value
CMTV_HD int hs_bitlen8(const uint32_t r[8]) {
  int bl = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) bl = r[i] ? 32 * i + 32 - hs_clz(r[i]) : bl;
  return bl;
}

// |t| bit length and sign of a 6-word two's complement value
CMTV_HD int hs_bitlen6s(const uint32_t t[6], bool& neg) {
  neg = (t[5] >> 31) != 0;
  uint32_t m[6];
  uint64_t c = 1;
#pragma unroll
  for (int i = 0; i < 6; i++) {
    const uint64_t v = (uint64_t)(neg ? ~t[i] : t[i]) + (neg ? c : 0);
    m[i] = (uint32_t)v;
    c = v >> 32;
  }
  int bl = 0;
#pragma unroll
  for (int i = 0; i < 6; i++) bl = m[i] ? 32 * i + 32 - hs_clz(m[i]) : bl;
  return bl;
}

// r <<= sh (0 <= sh < 32), 8 words. Word-sized shifts only: pairing two
// array words into a 64-bit value lets the compiler merge their loads, which
// keeps the whole array in scratch memory on the device.
CMTV_HD void hs_shl8(uint32_t r[8], int sh) {
#pragma unroll
  for (int i = 7; i > 0; i--) r[i] = (r[i] << sh) | ((r[i - 1] >> (31 - sh)) >> 1);
  r[0] <<= sh;
}

// r >>= sh (0 <= sh < 32), 8 words
CMTV_HD void hs_shr8(uint32_t r[8], int sh) {
#pragma unroll
  for (int i = 0; i < 7; i++) r[i] = (r[i] >> sh) | ((r[i + 1] << (31 - sh)) << 1);
  r[7] >>= sh;
}

// one Euclid step on normalised (r0, r1): rr = r0 - q r1 with q = floor(r0 / r1),
// tt = t0 - q t1. Returns false if q does not fit the one-word estimate.
template <bool UNI = false>
CMTV_HD bool hs_step(uint32_t rr[8], uint32_t tt[6], const uint32_t r0[8], const uint32_t r1[8],
                     const uint32_t t0[6], const uint32_t t1[6]) {
  if (hs_uni<UNI>(r1[7] == 0)) return false;  // r1 < r0 / 2^31: quotient too wide for one word
  // the top 64 bits of each as an f64 (one rounding of the exact value)
  const double a = (double)r0[7] * 4294967296.0 + (double)r0[6];
  const double b = (double)r1[7] * 4294967296.0 + (double)r1[6];
  const double qd = floor(a / b);
  uint32_t q = qd >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)qd;
  // x = r0 - q r1 as 9-word two's complement; y = t0 - q t1 (6 words)
  uint32_t x[9];
  {
    uint64_t mc = 0;
    int64_t acc = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const uint64_t p = (uint64_t)q * r1[i] + mc;
      mc = p >> 32;
      acc += (int64_t)r0[i] - (int64_t)(uint32_t)p;
      x[i] = (uint32_t)acc;
      acc >>= 32;
    }
    acc -= (int64_t)mc;
    x[8] = (uint32_t)acc;
  }
  {
    uint64_t mc = 0;
    int64_t acc = 0;
#pragma unroll
    for (int i = 0; i < 6; i++) {
      const uint64_t p = (uint64_t)q * t1[i] + mc;
      mc = p >> 32;
      acc += (int64_t)t0[i] - (int64_t)(uint32_t)p;
      tt[i] = (uint32_t)acc;
      acc >>= 32;
    }
  }
  // the estimate is within a few units of q: fix it up (rarely entered)
  bool ok = true;
#pragma unroll 1
  for (int it = 0; it < 4 && hs_uni<UNI>((x[8] >> 31) != 0); it++) {  // x < 0: add r1 back
    uint64_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const uint64_t v = (uint64_t)x[i] + r1[i] + c;
      x[i] = (uint32_t)v;
      c = v >> 32;
    }
    x[8] += (uint32_t)c;
    c = 0;
#pragma unroll
    for (int i = 0; i < 6; i++) {
      const uint64_t v = (uint64_t)tt[i] + t1[i] + c;
      tt[i] = (uint32_t)v;
      c = v >> 32;
    }
  }
  ok = ok && !(x[8] >> 31);
#pragma unroll 1
  for (int it = 0; it < 4; it++) {  // x >= r1: subtract once more
    int64_t acc = 0;
    uint32_t y[8];
#pragma unroll
    for (int i = 0; i < 8; i++) {
      acc += (int64_t)x[i] - (int64_t)r1[i];
      y[i] = (uint32_t)acc;
      acc >>= 32;
    }
    acc += (int64_t)x[8];
    if (hs_uni<UNI>(acc < 0)) break;
#pragma unroll
    for (int i = 0; i < 8; i++) x[i] = y[i];
    x[8] = (uint32_t)acc;
    acc = 0;
#pragma unroll
    for (int i = 0; i < 6; i++) {
      acc += (int64_t)tt[i] - (int64_t)t1[i];
      tt[i] = (uint32_t)acc;
      acc >>= 32;
    }
  }
  ok = ok && x[8] == 0;
#pragma unroll
  for (int i = 0; i < 8; i++) rr[i] = x[i];
  return ok;
}

// floor(a / b) for 0 <= a < 2^31, 0 < b < 2^31: the correctly rounded f64
// quotient never reaches the next integer (a/b = n - m/b sits at least 2^-31
// below n relative, far more than an f64 ulp), so truncation is exact
CMTV_HD uint32_t hs_udiv31(uint32_t a, uint32_t b) { return (uint32_t)((double)a / (double)b); }

// Lehmer's inner loop (Knuth TAOCP vol. 2, 4.5.2, Algorithm L) on the 30-bit
// leading digits u = r0 >> h', v = r1 >> h' of the normalised pair (h the
// digits' bit position at true scale): returns the cofactor matrix of the
// Euclid steps whose quotients the digits determine for certain
// (floor((u+A)/(v+C)) == floor((u+B)/(v+D))), and stops before any step whose
// divisor might already be below 2^127, where the exact Euclid stops: after
// the accepted steps the true divisor lies in 2^h (v + min(C,D), v + max(C,D)).
// B == 0 on return: no step was certain.
template <bool UNI = false>
CMTV_HD void hs_lehmer(int32_t& A, int32_t& B, int32_t& C, int32_t& D, uint32_t u, uint32_t v, int h) {
  const int32_t thr = h >= 127 ? 1 : (int32_t)(1u << (127 - h));
  int32_t a = 1, b = 0, c = 0, d = 1;
  int32_t uu = (int32_t)u, vv = (int32_t)v;
#pragma unroll 1
  for (int it = 0; it < HS_MAX_INNER; it++) {
    const int32_t vc = vv + c, vd = vv + d;
    const int32_t lo = vc < vd ? vc : vd;
    if (hs_uni<UNI>(lo < thr)) break;  // divisor not certainly >= 2^127 (also keeps vc, vd > 0)
    const uint32_t q = hs_udiv31((uint32_t)(uu + a), (uint32_t)vc);
    // the other corner must give the same quotient: 0 <= (u+b) - q (v+d) < v+d
    const int64_t x = (int64_t)(uu + b) - (int64_t)q * vd;
    if (hs_uni<UNI>(x < 0 || x >= vd)) break;
    const int32_t nc = (int32_t)((int64_t)a - (int64_t)q * c);
    const int32_t nd = (int32_t)((int64_t)b - (int64_t)q * d);
    const int32_t nv = (int32_t)((int64_t)uu - (int64_t)q * vv);
    a = c;
    b = d;
    c = nc;
    d = nd;
    uu = vv;
    vv = nv;
  }
  A = a;
  B = b;
  C = c;
  D = d;
}

// out = P x + Q y modulo 2^(32 W), for cofactors P, Q of opposite signs (or
// zero) and an exact result in range: evaluated as |P| x - |Q| y or
// |Q| y - |P| x on unsigned words (x, y two's complement when W = 6)
template <int W>
CMTV_HD void hs_lin(uint32_t out[W], int32_t P, const uint32_t x[], int32_t Q, const uint32_t y[]) {
  const bool pneg = Q > 0;  // then P <= 0 and the positive term is Q y
  const uint32_t pm = P < 0 ? (uint32_t)(-(int64_t)P) : (uint32_t)P;
  const uint32_t qm = Q < 0 ? (uint32_t)(-(int64_t)Q) : (uint32_t)Q;
  const uint32_t mp = pneg ? qm : pm;  // multiplier of the positive term
  const uint32_t mq = pneg ? pm : qm;
  uint64_t cp = 0, cq = 0;
  int64_t acc = 0;
#pragma unroll
  for (int i = 0; i < W; i++) {
    const uint64_t tp = (uint64_t)mp * (pneg ? y[i] : x[i]) + cp;
    const uint64_t tq = (uint64_t)mq * (pneg ? x[i] : y[i]) + cq;
    cp = tp >> 32;
    cq = tq >> 32;
    acc += (int64_t)(uint32_t)tp - (int64_t)(uint32_t)tq;
    out[i] = (uint32_t)acc;
    acc >>= 32;
  }
}

// (k1, k2) with k1 == k2 k (mod 8L), k2 odd if odd_k2, both < 2^146, or wide.
// LEHMER = false: one exact Euclid step per round (the schedule the host test
// compares against); both give the same pair.
// force_wide: take the wide schedule regardless (CMTV_FORCE_WIDE test knob,
// so the 64-window path -- ~never reached by real k -- is exercised)
// odd_k2: the cofactorless (GO_STDLIB) requirement; ZIP215 passes false
// UNI: the wave's lanes all hold the same k (hs_uni)
template <bool LEHMER = true, bool UNI = false>
CMTV_HD void half_scalars(HalfScalars& h, const uint32_t k[8], bool force_wide = false, bool odd_k2 = true) {
  uint32_t r0[8], r1[8], t0[6], t1[6];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    r0[i] = hs_N(i);  // already normalised: bit 255 set
    r1[i] = k[i];
  }
#pragma unroll
  for (int i = 0; i < 6; i++) {
    t0[i] = 0;
    t1[i] = i == 0 ? 1u : 0u;
  }
  int e = 0;  // common left shift of r0, r1
  bool ok = true;
#pragma unroll 1
  for (int round = 0; round < HS_MAX_ROUNDS; round++) {
    const int bl1 = (r1[7] ? 256 - hs_clz(r1[7]) : hs_bitlen8(r1)) - e;
    if (hs_uni<UNI>(bl1 <= 127)) break;
    if (round == HS_MAX_ROUNDS - 1) {
      ok = false;
      break;
    }
    int32_t A = 1, B = 0, C = 0, D = 1;
    if (LEHMER) hs_lehmer<UNI>(A, B, C, D, r0[7] >> 2, r1[7] >> 2, 226 - e);
    if (hs_uni<UNI>(B == 0)) {
      // no quotient certain from the leading digits: one exact step
      uint32_t rr[8], tt[6];
      if (hs_uni<UNI>(!hs_step<UNI>(rr, tt, r0, r1, t0, t1))) {
        ok = false;
        break;
      }
#pragma unroll
      for (int i = 0; i < 8; i++) {
        r0[i] = r1[i];
        r1[i] = rr[i];
      }
#pragma unroll
      for (int i = 0; i < 6; i++) {
        t0[i] = t1[i];
        t1[i] = tt[i];
      }
    } else {
      // (r0, r1) <- (A r0 + B r1, C r0 + D r1), likewise (t0, t1)
      uint32_t s0[8], s1[8], u0[6], u1[6];
      hs_lin<8>(s0, A, r0, B, r1);
      hs_lin<8>(s1, C, r0, D, r1);
      hs_lin<6>(u0, A, t0, B, t1);
      hs_lin<6>(u1, C, t0, D, t1);
#pragma unroll
      for (int i = 0; i < 8; i++) {
        r0[i] = s0[i];
        r1[i] = s1[i];
      }
#pragma unroll
      for (int i = 0; i < 6; i++) {
        t0[i] = u0[i];
        t1[i] = u1[i];
      }
    }
    // renormalise: r0's top bit back to bit 255
#pragma unroll 1
    while (hs_uni<UNI>(r0[7] == 0)) {
#pragma unroll
      for (int i = 7; i > 0; i--) {
        r0[i] = r0[i - 1];
        r1[i] = r1[i - 1];
      }
      r0[0] = 0;
      r1[0] = 0;
      e += 32;
    }
    const int sh = hs_clz(r0[7]);
    hs_shl8(r0, sh);
    hs_shl8(r1, sh);
    e += sh;
  }

  // odd_k2: candidates with odd t: (r1, t1); else (r0, t0) [t0 odd then] or
  // one more step (r2, t2) [t2 = t0 - q t1 odd then]. Any parity: the
  // shorter of (r1, t1) and (r0, t0) (t0 = 0 only while r0 = 8L).
  bool n1, n0, n2;
  const int b1 = hs_bitlen6s(t1, n1);
  const int c1 = (hs_bitlen8(r1) - e) > b1 ? (hs_bitlen8(r1) - e) : b1;
  const bool t1_odd = t1[0] & 1;
  uint32_t r2[8], t2[6];
  bool ok2 = false;
  if (hs_uni<UNI>(ok && !t1_odd && odd_k2)) ok2 = hs_step<UNI>(r2, t2, r0, r1, t0, t1);
  const int br0 = hs_bitlen8(r0) - e, bt0 = hs_bitlen6s(t0, n0);
  const int c0 = br0 > bt0 ? br0 : bt0;
  int c2 = 1 << 20;
  if (ok2) {
    const int br2 = hs_bitlen8(r2) - e, bt2 = hs_bitlen6s(t2, n2);
    c2 = br2 > bt2 ? br2 : bt2;
  }
  // choose: 1 if t1 odd, else the smaller of 0 and 2 (any parity: of 1 and 0)
  const int pick = odd_k2 ? (t1_odd ? 1 : (c2 < c0 ? 2 : 0)) : (c1 <= c0 ? 1 : 0);
  const int cost = pick == 1 ? c1 : (pick == 2 ? c2 : c0);
  h.wide = force_wide || !ok || cost > 4 * HS_MAX_WINDOWS - 2;
  h.windows = h.wide ? HS_WIDE_WINDOWS : hs_windows_for(cost);
  uint32_t rs[8], ts[6];
#pragma unroll
  for (int i = 0; i < 8; i++) rs[i] = pick == 1 ? r1[i] : (pick == 2 ? r2[i] : r0[i]);
#pragma unroll
  for (int i = 0; i < 6; i++) ts[i] = pick == 1 ? t1[i] : (pick == 2 ? t2[i] : t0[i]);
  // denormalise r (e <= 129 whenever the pair is used)
  int ew = h.wide ? 0 : e;
#pragma unroll 1
  while (hs_uni<UNI>(ew >= 32)) {
#pragma unroll
    for (int i = 0; i < 7; i++) rs[i] = rs[i + 1];
    rs[7] = 0;
    ew -= 32;
  }
  hs_shr8(rs, ew);
  bool tneg = (ts[5] >> 31) != 0;
  uint64_t c = 1;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint32_t w = i < 6 ? ts[i] : (tneg ? 0xFFFFFFFFu : 0u);
    const uint64_t v = (uint64_t)(tneg ? ~w : w) + (tneg ? c : 0);
    h.k2[i] = (uint32_t)v;
    c = v >> 32;
  }
#pragma unroll
  for (int i = 0; i < 8; i++) {
    h.k1[i] = h.wide ? k[i] : rs[i];
    h.k2[i] = h.wide ? (i == 0 ? 1u : 0u) : h.k2[i];
  }
  h.k2_neg = !h.wide && tneg;
}

// u = k2 * s mod L (signed k2 = neg ? -mag : mag), s < L
CMTV_HD void hs_bscalar(uint32_t u[8], const uint32_t k2mag[8], bool neg, const uint32_t s[8]) {
  uint32_t z[8];
#pragma unroll
  for (int i = 0; i < 8; i++) z[i] = 0;
  sc_muladd(u, k2mag, s, z);
  // L - u (and 0 stays 0)
  uint32_t d[8];
  int64_t acc = 0;
  uint32_t nz = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    acc += (int64_t)sc_L(i) - (int64_t)u[i];
    d[i] = (uint32_t)acc;
    acc >>= 32;
    nz |= u[i];
  }
  const bool flip = neg && nz != 0;
#pragma unroll
  for (int i = 0; i < 8; i++) u[i] = flip ? d[i] : u[i];
}

// Signed radix-16 digit stream of x (|digits| <= 8) read from the top with
// sc_shift_out(t, 4) over W windows: W = HS_WIDE_WINDOWS (64, any x < 2^255)
// or HS_WINDOWS..HS_MAX_WINDOWS (x < 2^(4W-2)), left-aligned so the first
// shift_out yields the top digit.
CMTV_HD void hs_digits16(uint32_t t[8], const uint32_t x[8], int W) {
  uint32_t a[8], b[8];
  sc_bias(a, x, 0x88888888u);
  // W nibbles of 8: words 0-3 whole, word 4 holds W - 32 (1..5) of them
  const uint32_t w4 = 0x88888888u & ((1u << (4 * (W - 32))) - 1u);
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint32_t bias = i < 4 ? 0x88888888u : (i == 4 ? w4 : 0u);
    const uint64_t v = (uint64_t)x[i] + bias + c;
    b[i] = (uint32_t)v;
    c = v >> 32;
  }
  // b < 2^(4W): shift left by 4 (64 - W) = 96 + bs bits, bs = 4 (40 - W) in 12..28
  const int bs = 4 * (40 - (W > HS_MAX_WINDOWS ? HS_MAX_WINDOWS : W));
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint32_t hi = i >= 3 ? b[i - 3] : 0u;
    const uint32_t lo = i >= 4 ? b[i - 4] : 0u;
    const uint32_t sh = (hi << bs) | (lo >> (32 - bs));
    t[i] = W == HS_WIDE_WINDOWS ? a[i] : sh;
  }
}

// Signed radix-2^16 digit streams of u < L (< 2^253): t = u + 0x8000 in every
// 16-bit field (the top field stays below 2^16), tLo yields digits 7..0
// (bits 0..127) and tHi digits 15..8, each read from the top with
// sc_shift_out(t, 16); digit = out - 0x8000, in [-2^15, 2^15).
CMTV_HD void hs_digits65536(uint32_t tLo[8], uint32_t tHi[8], const uint32_t u[8]) {
  uint32_t t[8];
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint64_t v = (uint64_t)u[i] + 0x80008000u + c;
    t[i] = (uint32_t)v;
    c = v >> 32;
  }
#pragma unroll
  for (int i = 0; i < 4; i++) {
    tLo[i] = 0;
    tLo[4 + i] = t[i];
    tHi[i] = 0;
    tHi[4 + i] = t[4 + i];
  }
}

// Signed radix-256 digit streams of u < L split at 2^128, each read from the
// top with sc_shift_out(t, 8): tLo yields digits 16..0 of u mod 2^128
// (17 digits), tHi digits 15..0 of u >> 128 (< 2^125, 16 digits).
CMTV_HD void hs_digits256(uint32_t tLo[8], uint32_t tHi[8], const uint32_t u[8]) {
  uint32_t lo[5];
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 5; i++) {
    const uint64_t v = (uint64_t)(i < 4 ? u[i] : 0u) + (i < 4 ? 0x80808080u : 0x80u) + c;
    lo[i] = (uint32_t)v;
    c = v >> 32;
  }
  // lo < 2^136: shift left by 120 bits
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint32_t hi = (i >= 3 && i - 3 < 5) ? lo[i - 3] : 0u;
    const uint32_t lw = (i >= 4 && i - 4 < 5) ? lo[i - 4] : 0u;
    tLo[i] = (hi << 24) | (lw >> 8);
  }
  c = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const uint64_t v = (uint64_t)u[4 + i] + 0x80808080u + c;
    tHi[4 + i] = (uint32_t)v;
    tHi[i] = 0;
    c = v >> 32;
  }
}

}  // namespace cmtv
