// fe25519.h -- GF(2^255-19) arithmetic for gfx950 VALU.
//
// Representation: 10 unsigned 32-bit limbs in radix 2^25.5 (limb i holds bits
// [ceil(25.5 i), ceil(25.5 (i+1))) : 26,25,26,25,... bits). A limb product is a
// 32x32->64 multiply-accumulate, which hipcc lowers to v_mad_u64_u32 -- the
// measured-fastest full-width integer MAC on gfx950 (tools/microbench). No MFMA:
// field multiplication is a per-lane convolution, not a shared-operand GEMM.
//
// Lazy reduction, all limbs unsigned:
//   "carried"  : even limbs < 2^26, odd limbs < 2^25 (+tiny)      (output of mul/sq/carry)
//   fe_add     : no carry; limbs < 2^27 / 2^26 when both inputs carried
//   fe_sub     : f + 2p - g, no carry; g must be carried; limbs < 3*2^26 / 3*2^25
// Multiplier input bound: every limb < 2^27.7 (19*g_i must fit in 32 bits and
// the 267*B^2 worst-case column sum must fit in 64 bits). Square input bound:
// odd limbs < 2^26.7 (38*f_i fits 32 bits). The point formulas in ge25519.h
// keep every operand inside these bounds (checked by tests/host/ in a bounds-
// checking host build).
//
// This is the arithmetic Go 1.19's crypto/internal/edwards25519/field performs
// (reference call site /root/reference/crypto/ed25519/ed25519.go:154), laid out
// for 64-wide wavefronts instead of 64-bit scalar registers.
#pragma once
#include <stdint.h>

#ifndef CMTV_HD
#define CMTV_HD __host__ __device__ __forceinline__
#endif

// Scheduling fence between field operations. Without it the AMDGPU machine
// scheduler interleaves the 100-product DAGs of neighbouring multiplications
// for ILP and needs >512 VGPRs; fencing each multiply bounds the live set to
// one operation's working set so the verify kernel fits its occupancy target.
#if defined(__HIP_DEVICE_COMPILE__)
#define CMTV_SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define CMTV_SCHED_FENCE() ((void)0)
#endif

// (x ^ m) & k for per-lane masks m, k: one v_bitop3_b32 on gfx950 (truth
// table 0x28); from plain C the masks' selects lower to xor + v_cndmask
#if defined(__HIP_DEVICE_COMPILE__)
#define CMTV_XOR_AND(x, m, k) __builtin_amdgcn_bitop3_b32((x), (m), (k), 0x28)
#else
#define CMTV_XOR_AND(x, m, k) (((x) ^ (m)) & (k))
#endif

#ifdef CMTV_BOUNDS_CHECK
#include <cassert>
#define CMTV_ASSERT(x) assert(x)
#else
#define CMTV_ASSERT(x) ((void)0)
#endif

namespace cmtv {

struct fe {
  uint32_t v[10];
};

constexpr uint32_t M26 = (1u << 26) - 1;
constexpr uint32_t M25 = (1u << 25) - 1;
// 2p in this radix
constexpr uint32_t P2_0 = 0x7FFFFDA;  // 2*(2^26-19)
constexpr uint32_t P2_E = 0x7FFFFFE;  // 2*(2^26-1)
constexpr uint32_t P2_O = 0x3FFFFFE;  // 2*(2^25-1)
constexpr uint32_t MUL_BOUND = 226000000u;   // < 2^32/19
constexpr uint32_t SQ_ODD_BOUND = 113000000u;  // < 2^32/38

CMTV_HD void fe_0(fe& h) {
#pragma unroll
  for (int i = 0; i < 10; i++) h.v[i] = 0;
}
CMTV_HD void fe_1(fe& h) {
  fe_0(h);
  h.v[0] = 1;
}
CMTV_HD void fe_copy(fe& h, const fe& f) {
#pragma unroll
  for (int i = 0; i < 10; i++) h.v[i] = f.v[i];
}

CMTV_HD void fe_add(fe& h, const fe& f, const fe& g) {
#pragma unroll
  for (int i = 0; i < 10; i++) h.v[i] = f.v[i] + g.v[i];
}

// h = f + 2p - g  (g carried)
CMTV_HD void fe_sub(fe& h, const fe& f, const fe& g) {
  h.v[0] = f.v[0] + P2_0 - g.v[0];
#pragma unroll
  for (int i = 1; i < 10; i++) h.v[i] = f.v[i] + ((i & 1) ? P2_O : P2_E) - g.v[i];
}

// h = 2p - f  (f carried)
CMTV_HD void fe_neg(fe& h, const fe& f) {
  h.v[0] = P2_0 - f.v[0];
#pragma unroll
  for (int i = 1; i < 10; i++) h.v[i] = ((i & 1) ? P2_O : P2_E) - f.v[i];
}

// weak carry of 32-bit limbs back into the "carried" range
CMTV_HD void fe_carry(fe& h) {
  uint32_t c;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    if (i & 1) {
      c = h.v[i] >> 25;
      h.v[i] &= M25;
    } else {
      c = h.v[i] >> 26;
      h.v[i] &= M26;
    }
    h.v[i + 1] += c;
  }
  c = h.v[9] >> 25;
  h.v[9] &= M25;
  h.v[0] += 19 * c;
  c = h.v[0] >> 26;
  h.v[0] &= M26;
  h.v[1] += c;
}

CMTV_HD void fe_select(fe& h, const fe& a, const fe& b, bool take_b) {
#pragma unroll
  for (int i = 0; i < 10; i++) h.v[i] = take_b ? b.v[i] : a.v[i];
}

#define CMTV_MUL64(a, b) ((uint64_t)(a) * (uint64_t)(b))

// carry chain on ten 64-bit column sums (ref10 interleaving shortens the
// dependency chain: two independent carry streams 0->4 and 4->9)
CMTV_HD void fe_reduce64(fe& h, uint64_t h0, uint64_t h1, uint64_t h2, uint64_t h3, uint64_t h4,
                         uint64_t h5, uint64_t h6, uint64_t h7, uint64_t h8, uint64_t h9) {
  uint64_t c;
  c = h0 >> 26; h1 += c; h0 &= M26;
  c = h4 >> 26; h5 += c; h4 &= M26;
  c = h1 >> 25; h2 += c; h1 &= M25;
  c = h5 >> 25; h6 += c; h5 &= M25;
  c = h2 >> 26; h3 += c; h2 &= M26;
  c = h6 >> 26; h7 += c; h6 &= M26;
  c = h3 >> 25; h4 += c; h3 &= M25;
  c = h7 >> 25; h8 += c; h7 &= M25;
  c = h4 >> 26; h5 += c; h4 &= M26;
  c = h8 >> 26; h9 += c; h8 &= M26;
  c = h9 >> 25; h0 += c * 19; h9 &= M25;
  c = h0 >> 26; h1 += c; h0 &= M26;
  h.v[0] = (uint32_t)h0; h.v[1] = (uint32_t)h1; h.v[2] = (uint32_t)h2; h.v[3] = (uint32_t)h3;
  h.v[4] = (uint32_t)h4; h.v[5] = (uint32_t)h5; h.v[6] = (uint32_t)h6; h.v[7] = (uint32_t)h7;
  h.v[8] = (uint32_t)h8; h.v[9] = (uint32_t)h9;
}

CMTV_HD void fe_mul(fe& h, const fe& f, const fe& g) {
  CMTV_SCHED_FENCE();
#ifdef CMTV_BOUNDS_CHECK
  for (int i = 0; i < 10; i++) CMTV_ASSERT(f.v[i] < MUL_BOUND && g.v[i] < MUL_BOUND);
#endif
  const uint32_t f0 = f.v[0], f1 = f.v[1], f2 = f.v[2], f3 = f.v[3], f4 = f.v[4];
  const uint32_t f5 = f.v[5], f6 = f.v[6], f7 = f.v[7], f8 = f.v[8], f9 = f.v[9];
  const uint32_t g0 = g.v[0], g1 = g.v[1], g2 = g.v[2], g3 = g.v[3], g4 = g.v[4];
  const uint32_t g5 = g.v[5], g6 = g.v[6], g7 = g.v[7], g8 = g.v[8], g9 = g.v[9];
  const uint32_t g1_19 = 19 * g1, g2_19 = 19 * g2, g3_19 = 19 * g3, g4_19 = 19 * g4, g5_19 = 19 * g5;
  const uint32_t g6_19 = 19 * g6, g7_19 = 19 * g7, g8_19 = 19 * g8, g9_19 = 19 * g9;
  const uint32_t f1_2 = 2 * f1, f3_2 = 2 * f3, f5_2 = 2 * f5, f7_2 = 2 * f7, f9_2 = 2 * f9;

  uint64_t h0 = CMTV_MUL64(f0, g0) + CMTV_MUL64(f1_2, g9_19) + CMTV_MUL64(f2, g8_19) + CMTV_MUL64(f3_2, g7_19) +
                CMTV_MUL64(f4, g6_19) + CMTV_MUL64(f5_2, g5_19) + CMTV_MUL64(f6, g4_19) + CMTV_MUL64(f7_2, g3_19) +
                CMTV_MUL64(f8, g2_19) + CMTV_MUL64(f9_2, g1_19);
  uint64_t h1 = CMTV_MUL64(f0, g1) + CMTV_MUL64(f1, g0) + CMTV_MUL64(f2, g9_19) + CMTV_MUL64(f3, g8_19) +
                CMTV_MUL64(f4, g7_19) + CMTV_MUL64(f5, g6_19) + CMTV_MUL64(f6, g5_19) + CMTV_MUL64(f7, g4_19) +
                CMTV_MUL64(f8, g3_19) + CMTV_MUL64(f9, g2_19);
  uint64_t h2 = CMTV_MUL64(f0, g2) + CMTV_MUL64(f1_2, g1) + CMTV_MUL64(f2, g0) + CMTV_MUL64(f3_2, g9_19) +
                CMTV_MUL64(f4, g8_19) + CMTV_MUL64(f5_2, g7_19) + CMTV_MUL64(f6, g6_19) + CMTV_MUL64(f7_2, g5_19) +
                CMTV_MUL64(f8, g4_19) + CMTV_MUL64(f9_2, g3_19);
  uint64_t h3 = CMTV_MUL64(f0, g3) + CMTV_MUL64(f1, g2) + CMTV_MUL64(f2, g1) + CMTV_MUL64(f3, g0) +
                CMTV_MUL64(f4, g9_19) + CMTV_MUL64(f5, g8_19) + CMTV_MUL64(f6, g7_19) + CMTV_MUL64(f7, g6_19) +
                CMTV_MUL64(f8, g5_19) + CMTV_MUL64(f9, g4_19);
  uint64_t h4 = CMTV_MUL64(f0, g4) + CMTV_MUL64(f1_2, g3) + CMTV_MUL64(f2, g2) + CMTV_MUL64(f3_2, g1) +
                CMTV_MUL64(f4, g0) + CMTV_MUL64(f5_2, g9_19) + CMTV_MUL64(f6, g8_19) + CMTV_MUL64(f7_2, g7_19) +
                CMTV_MUL64(f8, g6_19) + CMTV_MUL64(f9_2, g5_19);
  uint64_t h5 = CMTV_MUL64(f0, g5) + CMTV_MUL64(f1, g4) + CMTV_MUL64(f2, g3) + CMTV_MUL64(f3, g2) +
                CMTV_MUL64(f4, g1) + CMTV_MUL64(f5, g0) + CMTV_MUL64(f6, g9_19) + CMTV_MUL64(f7, g8_19) +
                CMTV_MUL64(f8, g7_19) + CMTV_MUL64(f9, g6_19);
  uint64_t h6 = CMTV_MUL64(f0, g6) + CMTV_MUL64(f1_2, g5) + CMTV_MUL64(f2, g4) + CMTV_MUL64(f3_2, g3) +
                CMTV_MUL64(f4, g2) + CMTV_MUL64(f5_2, g1) + CMTV_MUL64(f6, g0) + CMTV_MUL64(f7_2, g9_19) +
                CMTV_MUL64(f8, g8_19) + CMTV_MUL64(f9_2, g7_19);
  uint64_t h7 = CMTV_MUL64(f0, g7) + CMTV_MUL64(f1, g6) + CMTV_MUL64(f2, g5) + CMTV_MUL64(f3, g4) +
                CMTV_MUL64(f4, g3) + CMTV_MUL64(f5, g2) + CMTV_MUL64(f6, g1) + CMTV_MUL64(f7, g0) +
                CMTV_MUL64(f8, g9_19) + CMTV_MUL64(f9, g8_19);
  uint64_t h8 = CMTV_MUL64(f0, g8) + CMTV_MUL64(f1_2, g7) + CMTV_MUL64(f2, g6) + CMTV_MUL64(f3_2, g5) +
                CMTV_MUL64(f4, g4) + CMTV_MUL64(f5_2, g3) + CMTV_MUL64(f6, g2) + CMTV_MUL64(f7_2, g1) +
                CMTV_MUL64(f8, g0) + CMTV_MUL64(f9_2, g9_19);
  uint64_t h9 = CMTV_MUL64(f0, g9) + CMTV_MUL64(f1, g8) + CMTV_MUL64(f2, g7) + CMTV_MUL64(f3, g6) +
                CMTV_MUL64(f4, g5) + CMTV_MUL64(f5, g4) + CMTV_MUL64(f6, g3) + CMTV_MUL64(f7, g2) +
                CMTV_MUL64(f8, g1) + CMTV_MUL64(f9, g0);
  fe_reduce64(h, h0, h1, h2, h3, h4, h5, h6, h7, h8, h9);
  CMTV_SCHED_FENCE();
}

CMTV_HD void fe_sq(fe& h, const fe& f) {
  CMTV_SCHED_FENCE();
#ifdef CMTV_BOUNDS_CHECK
  for (int i = 0; i < 10; i++) CMTV_ASSERT(f.v[i] < ((i & 1) ? SQ_ODD_BOUND : MUL_BOUND));
#endif
  const uint32_t f0 = f.v[0], f1 = f.v[1], f2 = f.v[2], f3 = f.v[3], f4 = f.v[4];
  const uint32_t f5 = f.v[5], f6 = f.v[6], f7 = f.v[7], f8 = f.v[8], f9 = f.v[9];
  const uint32_t f0_2 = 2 * f0, f1_2 = 2 * f1, f2_2 = 2 * f2, f3_2 = 2 * f3, f4_2 = 2 * f4;
  const uint32_t f5_2 = 2 * f5, f6_2 = 2 * f6, f7_2 = 2 * f7;
  const uint32_t f5_38 = 38 * f5, f6_19 = 19 * f6, f7_38 = 38 * f7, f8_19 = 19 * f8, f9_38 = 38 * f9;

  uint64_t h0 = CMTV_MUL64(f0, f0) + CMTV_MUL64(f1_2, f9_38) + CMTV_MUL64(f2_2, f8_19) + CMTV_MUL64(f3_2, f7_38) +
                CMTV_MUL64(f4_2, f6_19) + CMTV_MUL64(f5, f5_38);
  uint64_t h1 = CMTV_MUL64(f0_2, f1) + CMTV_MUL64(f2, f9_38) + CMTV_MUL64(f3_2, f8_19) + CMTV_MUL64(f4, f7_38) +
                CMTV_MUL64(f5_2, f6_19);
  uint64_t h2 = CMTV_MUL64(f0_2, f2) + CMTV_MUL64(f1_2, f1) + CMTV_MUL64(f3_2, f9_38) + CMTV_MUL64(f4_2, f8_19) +
                CMTV_MUL64(f5_2, f7_38) + CMTV_MUL64(f6, f6_19);
  uint64_t h3 = CMTV_MUL64(f0_2, f3) + CMTV_MUL64(f1_2, f2) + CMTV_MUL64(f4, f9_38) + CMTV_MUL64(f5_2, f8_19) +
                CMTV_MUL64(f6, f7_38);
  uint64_t h4 = CMTV_MUL64(f0_2, f4) + CMTV_MUL64(f1_2, f3_2) + CMTV_MUL64(f2, f2) + CMTV_MUL64(f5_2, f9_38) +
                CMTV_MUL64(f6_2, f8_19) + CMTV_MUL64(f7, f7_38);
  uint64_t h5 = CMTV_MUL64(f0_2, f5) + CMTV_MUL64(f1_2, f4) + CMTV_MUL64(f2_2, f3) + CMTV_MUL64(f6, f9_38) +
                CMTV_MUL64(f7_2, f8_19);
  uint64_t h6 = CMTV_MUL64(f0_2, f6) + CMTV_MUL64(f1_2, f5_2) + CMTV_MUL64(f2_2, f4) + CMTV_MUL64(f3_2, f3) +
                CMTV_MUL64(f7_2, f9_38) + CMTV_MUL64(f8, f8_19);
  uint64_t h7 = CMTV_MUL64(f0_2, f7) + CMTV_MUL64(f1_2, f6) + CMTV_MUL64(f2_2, f5) + CMTV_MUL64(f3_2, f4) +
                CMTV_MUL64(f8, f9_38);
  uint64_t h8 = CMTV_MUL64(f0_2, f8) + CMTV_MUL64(f1_2, f7_2) + CMTV_MUL64(f2_2, f6) + CMTV_MUL64(f3_2, f5_2) +
                CMTV_MUL64(f4, f4) + CMTV_MUL64(f9, f9_38);
  uint64_t h9 = CMTV_MUL64(f0_2, f9) + CMTV_MUL64(f1_2, f8) + CMTV_MUL64(f2_2, f7) + CMTV_MUL64(f3_2, f6) +
                CMTV_MUL64(f4_2, f5);
  fe_reduce64(h, h0, h1, h2, h3, h4, h5, h6, h7, h8, h9);
  CMTV_SCHED_FENCE();
}

// Kept as a rolled loop: the exponentiation chains call it with n up to 100,
// and an unrolled chain would stream hundreds of KB of code through the
// instruction cache once per wave. The trip count is hidden from the
// optimiser: with a constant n (every call site) LLVM rotates the loop and
// splits the 64-bit column sums, 129 VALU instructions per squaring instead of
// 107 (gfx950 listing) -- a fifth of the square-root chains' cost.
CMTV_HD void fe_sqn(fe& h, const fe& f, int n) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("" : "+s"(n));
#endif
  fe_sq(h, f);
#pragma unroll 1
  for (int i = 1; i < n; i++) fe_sq(h, h);
}

// load 255 bits (bit 255 ignored) from 8 little-endian 32-bit words; the value
// may be >= p (Go's field.Element.SetBytes accepts non-canonical input)
CMTV_HD void fe_frombytes(fe& h, const uint32_t w[8]) {
  // word-sized shifts (pos is a constant): no 64-bit pairing of array words
  auto bits = [&](int pos, uint32_t mask) -> uint32_t {
    const int wi = pos >> 5, sh = pos & 31;
    uint32_t x = w[wi] >> sh;
    if (wi < 7 && sh) x |= w[wi + 1] << (32 - sh);
    return x & mask;
  };
  h.v[0] = bits(0, M26);
  h.v[1] = bits(26, M25);
  h.v[2] = bits(51, M26);
  h.v[3] = bits(77, M25);
  h.v[4] = bits(102, M26);
  h.v[5] = bits(128, M25);
  h.v[6] = bits(153, M26);
  h.v[7] = bits(179, M25);
  h.v[8] = bits(204, M26);
  h.v[9] = bits(230, M25);
}

// canonical little-endian encoding (value mod p) as 8 32-bit words
CMTV_HD void fe_tobytes(uint32_t s[8], const fe& f) {
  fe h = f;
  fe_carry(h);
  fe_carry(h);
  // q = floor((h + 19) / 2^255) in {0, 1}
  uint32_t q = (h.v[0] + 19) >> 26;
#pragma unroll
  for (int i = 1; i < 10; i++) q = (h.v[i] + q) >> ((i & 1) ? 25 : 26);
  h.v[0] += 19 * q;
  uint32_t c;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    if (i & 1) {
      c = h.v[i] >> 25;
      h.v[i] &= M25;
    } else {
      c = h.v[i] >> 26;
      h.v[i] &= M26;
    }
    h.v[i + 1] += c;
  }
  h.v[9] &= M25;
  s[0] = h.v[0] | (h.v[1] << 26);
  s[1] = (h.v[1] >> 6) | (h.v[2] << 19);
  s[2] = (h.v[2] >> 13) | (h.v[3] << 13);
  s[3] = (h.v[3] >> 19) | (h.v[4] << 6);
  s[4] = h.v[5] | (h.v[6] << 25);
  s[5] = (h.v[6] >> 7) | (h.v[7] << 19);
  s[6] = (h.v[7] >> 13) | (h.v[8] << 12);
  s[7] = (h.v[8] >> 20) | (h.v[9] << 6);
}

CMTV_HD bool fe_iszero(const fe& f) {
  uint32_t s[8];
  fe_tobytes(s, f);
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r |= s[i];
  return r == 0;
}

CMTV_HD bool fe_isneg(const fe& f) {
  uint32_t s[8];
  fe_tobytes(s, f);
  return s[0] & 1;
}

// canonical comparison (inputs may be any 32-bit-limb representation)
CMTV_HD bool fe_equal(const fe& f, const fe& g) {
  uint32_t a[8], b[8];
  fe_tobytes(a, f);
  fe_tobytes(b, g);
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r |= a[i] ^ b[i];
  return r == 0;
}

// z^(2^250-1); also returns z^11
CMTV_HD void fe_pow2_250m1(fe& out, fe& z11, const fe& z) {
  fe t0, t1, t2, z2, z9;
  fe_sq(z2, z);
  fe_sqn(t0, z2, 2);
  fe_mul(z9, t0, z);
  fe_mul(z11, z9, z2);
  fe_sq(t0, z11);
  fe_mul(t0, t0, z9);     // 2^5 - 1
  fe_sqn(t1, t0, 5);
  fe_mul(t0, t1, t0);     // 2^10 - 1
  fe_sqn(t1, t0, 10);
  fe_mul(t1, t1, t0);     // 2^20 - 1
  fe_sqn(t2, t1, 20);
  fe_mul(t1, t2, t1);     // 2^40 - 1
  fe_sqn(t1, t1, 10);
  fe_mul(t0, t1, t0);     // 2^50 - 1
  fe_sqn(t1, t0, 50);
  fe_mul(t1, t1, t0);     // 2^100 - 1
  fe_sqn(t2, t1, 100);
  fe_mul(t1, t2, t1);     // 2^200 - 1
  fe_sqn(t1, t1, 50);
  fe_mul(out, t1, t0);    // 2^250 - 1
}

CMTV_HD void fe_invert(fe& out, const fe& z) {
  fe t, z11;
  fe_pow2_250m1(t, z11, z);
  fe_sqn(t, t, 5);
  fe_mul(out, t, z11);  // p - 2
}

CMTV_HD void fe_pow22523(fe& out, const fe& z) {
  fe t, z11;
  fe_pow2_250m1(t, z11, z);
  fe_sqn(t, t, 2);
  fe_mul(out, t, z);  // (p-5)/8
}

// curve constants
CMTV_HD void fe_const_d(fe& h) {
  const uint32_t c[10] = {0x35978a3, 0x0d37284, 0x3156ebd, 0x06a0a0e, 0x001c029,
                          0x179e898, 0x3a03cbb, 0x1ce7198, 0x2e2b6ff, 0x1480db3};
#pragma unroll
  for (int i = 0; i < 10; i++) h.v[i] = c[i];
}
CMTV_HD void fe_const_d2(fe& h) {
  const uint32_t c[10] = {0x2b2f159, 0x1a6e509, 0x22add7a, 0x0d4141d, 0x0038052,
                          0x0f3d130, 0x3407977, 0x19ce331, 0x1c56dff, 0x0901b67};
#pragma unroll
  for (int i = 0; i < 10; i++) h.v[i] = c[i];
}
CMTV_HD void fe_const_sqrtm1(fe& h) {
  const uint32_t c[10] = {0x20ea0b0, 0x186c9d2, 0x08f189d, 0x035697f, 0x0bd0c60,
                          0x1fbd7a7, 0x2804c9e, 0x1e16569, 0x004fc1d, 0x0ae0c92};
#pragma unroll
  for (int i = 0; i < 10; i++) h.v[i] = c[i];
}

}  // namespace cmtv
