// sr25519.h -- per-signature sr25519 (schnorrkel over ristretto255)
// verification, one signature per lane, for the gfx950 kernel in
// sr25519.hip and the host-compiled check in tests/host/srcheck.cpp.
//
// Restates sr25519.PubKey.VerifySignature,
// /root/reference/crypto/sr25519/pubkey.go:34-60, over go-schnorrkel v1.0.0 /
// gtank/ristretto255 v0.1.2 / gtank/merlin v0.1.1 (not in the reference tree;
// restated from their published algorithms, see oracle/sr25519_ref.py):
//
//   A = ristretto255 Decode(pk)                     (error -> false)
//   sig[63] & 0x80 set (schnorrkel marker)          (else false)
//   R = ristretto255 Decode(sig[0:32])              (error -> false)
//   s = sig[32:64] with bit 255 cleared, s < L      (else false)
//   k = merlin transcript challenge mod L           (merlin.h)
//   R' = [s]B - [k]A                                (Straus, verify_core.h)
//   R'.Equal(R):  X'y_R == Y'x_R  or  Y'y_R == X'x_R (ristretto equality)
//
// The curve is edwards25519 (ristretto255 is a quotient of it), so the field,
// point formulas and the fixed-base B tables are the Ed25519 kernel's.
#pragma once
#include "merlin.h"
#include "verify_core.h"

namespace cmtv {

// RFC 9496 SQRT_RATIO_M1(u, v): r = |sqrt(u/v)| or |sqrt(i u/v)|; returns
// was_square. u, v carried.
CMTV_HD bool fe_sqrt_ratio_m1(fe& r, const fe& u, const fe& v) {
  fe v3, v7, t, check, nu, nui, i;
  fe_sq(v3, v);
  fe_mul(v3, v3, v);  // v^3
  fe_sq(v7, v3);
  fe_mul(v7, v7, v);  // v^7
  fe_mul(t, u, v7);
  fe_pow22523(t, t);  // (u v^7)^((p-5)/8)
  fe_mul(t, t, v3);
  fe_mul(r, t, u);    // (u v^3)(u v^7)^((p-5)/8)
  fe_sq(check, r);
  fe_mul(check, check, v);
  fe_neg(nu, u);
  fe_carry(nu);
  fe_const_sqrtm1(i);
  fe_mul(nui, nu, i);
  const bool correct = fe_equal(check, u);
  const bool flipped = fe_equal(check, nu);
  const bool flipped_i = fe_equal(check, nui);
  fe_mul(t, r, i);
  fe_select(r, r, t, flipped || flipped_i);
  fe_neg(t, r);
  fe_carry(t);
  fe_select(r, r, t, fe_isneg(r));  // CT_ABS
  return correct || flipped;
}

// s (8 little-endian words) < p with bit 255 clear
CMTV_HD bool rist_canonical(const uint32_t w[8]) {
  if (w[7] >> 31) return false;
  bool all_ones = w[7] == 0x7FFFFFFFu;
#pragma unroll
  for (int i = 1; i < 7; i++) all_ones = all_ones && w[i] == 0xFFFFFFFFu;
  return !(all_ones && w[0] >= 0xFFFFFFEDu);
}

// RFC 9496 4.3.1 DECODE into extended coordinates (Z = 1). Computes on every
// input (uniform schedule); returns false for non-canonical, negative or
// invalid encodings.
CMTV_HD bool ristretto_decode(ge_p3& h, const uint32_t w[8]) {
  const bool enc_ok = rist_canonical(w) && (w[0] & 1) == 0;
  fe s, ss, u1, u2, u2sq, v, t, one, invsqrt, den_x, den_y, d;
  fe_frombytes(s, w);
  fe_1(one);
  fe_sq(ss, s);
  fe_sub(u1, one, ss);
  fe_carry(u1);                 // 1 - s^2
  fe_add(u2, one, ss);
  fe_carry(u2);                 // 1 + s^2
  fe_sq(u2sq, u2);
  fe_sq(t, u1);
  fe_const_d(d);
  fe_mul(t, t, d);              // d u1^2
  fe_neg(v, t);
  fe_carry(v);
  fe_sub(v, v, u2sq);
  fe_carry(v);                  // v = -d u1^2 - u2^2
  fe_mul(t, v, u2sq);
  const bool was_square = fe_sqrt_ratio_m1(invsqrt, one, t);
  fe_mul(den_x, invsqrt, u2);
  fe_mul(den_y, invsqrt, den_x);
  fe_mul(den_y, den_y, v);
  fe_add(t, s, s);
  fe_carry(t);
  fe_mul(h.X, t, den_x);
  fe_neg(t, h.X);
  fe_carry(t);
  fe_select(h.X, h.X, t, fe_isneg(h.X));  // x = |2 s den_x|
  fe_mul(h.Y, u1, den_y);
  fe_1(h.Z);
  fe_mul(h.T, h.X, h.Y);
  return enc_ok && was_square && !fe_isneg(h.T) && !fe_iszero(h.Y);
}

// Full single-signature verification (pubkey.go:34-60 for a 32-byte key and
// a 64-byte signature). prog/nops: the transcript's prefix sponge (merlin.h sr_prefix_state).
template <class ATab, class BTab, class State>
CMTV_HD bool sr_verify_one(const uint32_t* pk_ptr, const uint32_t* sig_ptr, const uint8_t* msg, uint32_t mlen,
                           const uint32_t* prog, int nops, State& st, ATab& atab, const BTab& btab) {
  uint32_t pk[8], rw[8], ts[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    pk[i] = pk_ptr[i];
    rw[i] = sig_ptr[i];
    ts[i] = sig_ptr[8 + i];
  }
  const bool marker = (ts[7] >> 31) != 0;
  ts[7] &= 0x7FFFFFFFu;
  const bool s_ok = marker && sc_is_canonical(ts);

  // challenge first: only pk / R words are live across the transcript
  uint32_t kb[16], k[8];
  sr_transcript(kb, st, prog, nops, msg, mlen, pk, rw);
  sc_reduce512(k, kb);

  ge_p3 A;
  const bool a_ok = ristretto_decode(A, pk);
  ge_p3 nA;
  cached_neg_point(nA, A);
  build_cached_table(atab, nA);

  ge_p3 Rp;
  straus_double_scalarmult<true>(Rp, k, ts, atab, btab);

  ge_p3 R;
  const bool r_ok = ristretto_decode(R, rw);
  fe l, r;
  fe_mul(l, Rp.X, R.Y);
  fe_mul(r, Rp.Y, R.X);
  const bool e1 = fe_equal(l, r);
  fe_mul(l, Rp.Y, R.Y);
  fe_mul(r, Rp.X, R.X);
  const bool e2 = fe_equal(l, r);
  return s_ok && a_ok && r_ok && (e1 || e2);
}

}  // namespace cmtv
