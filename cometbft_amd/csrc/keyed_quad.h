// keyed_quad.h -- registered-key verification (keyed.h) with one signature
// per quad of lanes (quad.h), for latency-bound batches: a 10k-signature
// commit against a registered validator set, or a 150-validator commit.
//
// Same verdict as verify_keyed<MODE> (and so verify_one<MODE>) on every input:
//   R' = sum_j T_B[j][s_j] + T_A[j][k_j]     32 + 32 comb additions, no doublings
//   GO_STDLIB: R canonical, decodable, and R' == R projectively
//              (X' = x_R Z', Y' = y_R Z': encode(R') == R bytes, no inversion)
//   ZIP215:    R decodable and [8](R' - R) == O
// Every lane decodes R (the same bytes); lane c then keeps coordinate c. The
// split kernel hashes and decodes on a helper wave while the quads add.
#pragma once
#include "keyed.h"
#include "quad.h"

namespace cmtv {

// 10 limbs of a comb row (affine niels: y+x[10] y-x[10] 2dxy[10] pad[2]) at
// word `off`
CMTV_HD void comb_load(const uint32_t* row, int off, fe& r) {
#pragma unroll
  for (int i = 0; i < 10; i++) r.v[i] = row[off + i];
}

// k = SHA-512(R || A || M) mod L as biased radix-256 digits (sc_bias), the
// half of a keyed verification that the helper wave computes first
CMTV_HD void q_keyed_challenge(uint32_t tk[8], const uint32_t* key_pk, const uint32_t* sig_ptr, const uint8_t* msg,
                               uint32_t mlen) {
  uint32_t w[16], h[16], k[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    w[i] = sig_ptr[i];  // R
    w[8 + i] = key_pk[i];
  }
  sha512_prefixed<16>(h, w, msg, mlen);
  sc_reduce512(k, h);
  sc_bias(tk, k, 0x80808080u);
}

// R decoded (the other helper-wave half): its extended coordinates (Z = 1)
// and whether it passes the mode's decoding rules
template <uint32_t MODE>
CMTV_HD bool q_keyed_decode_r(ge_p3& R, const uint32_t* sig_ptr) {
  uint32_t w[8];
#pragma unroll
  for (int i = 0; i < 8; i++) w[i] = sig_ptr[i];
  const bool r_ok = p3_frombytes(R, w);
  if (MODE == MODE_GO_STDLIB) return r_ok && y_is_canonical(w) && !(fe_iszero(R.X) && (w[7] >> 31));
  return r_ok;
}

// no B table (the radix-256 B comb path of q_verify_keyed_split)
struct NoBTabQ {
  CMTV_HD void load_coord(int, int, fe&) const {}
};

// The comb additions with the challenge and R supplied late: the fixed-base
// additions need only s, so they run first; get_k(tk) is called before the
// 32 key-comb additions and get_r(rc, r_ok) (this lane's coordinate of R: x,
// y, 1, t) before the final check -- a helper wave hashes and decodes
// meanwhile (kernels.hip k_verify_keyed_quad_split). [s]B: B16 = over the B
// table's radix-2^16 comb (bt.load_coord(row, off, fe&): BC16 rows, 16
// additions), else over the radix-256 comb bcomb (32).
template <uint32_t MODE, bool B16 = false, class Q, class BT = NoBTabQ, class GetK, class GetR>
CMTV_HD bool q_verify_keyed_split(const Q& q, bool key_ok, const uint32_t* sig_ptr, const uint32_t* ktab,
                                  const uint32_t* bcomb, const GetK& get_k, const GetR& get_r,
                                  const BT& bt = BT()) {
  const int lane = q.lane();
  uint32_t w[8];
#pragma unroll
  for (int i = 0; i < 8; i++) w[i] = sig_ptr[8 + i];  // S
  bool ok = key_ok && (w[7] & 0xE0000000u) == 0 && sc_is_canonical(w);
  uint32_t tk[8];

  fe v;
  q_identity(v, lane);
  if constexpr (B16) {
    uint32_t sLo[8], sHi[8];
    hs_digits65536(sLo, sHi, w);
#pragma unroll 1
    for (int j = 15; j >= 0; j--) {
      const int dB = (int)(j >= 8 ? sc_shift_out(sHi, 16) : sc_shift_out(sLo, 16)) - 0x8000;
      const int ib = dB < 0 ? -dB : dB;
      const int row = BC16_BASE + j * BT16_ENTRIES + (ib > 0 ? ib - 1 : 0);
      fe c;
      q_niels_coord(
          q, c, [&](int off, fe& r) { bt.load_coord(row, off, r); }, BTAB_COORD_WORDS, 2 * BTAB_COORD_WORDS,
          dB < 0, ib == 0);
      q_add(q, v, c);
    }
  } else {
    uint32_t ts[8];
    sc_bias(ts, w, 0x80808080u);
#pragma unroll 1
    for (int it = 0; it < COMB_WINDOWS; it++) {
      const int j = COMB_WINDOWS - 1 - it;
      const int dB = (int)sc_shift_out(ts, 8) - 128;
      const int ib = dB < 0 ? -dB : dB;
      fe c;
      const uint32_t* row = bcomb + ((size_t)j * COMB_ENTRIES + (ib > 0 ? ib - 1 : 0)) * COMB_ROW_WORDS;
      q_niels_coord(q, c, [&](int off, fe& r) { comb_load(row, off, r); }, 10, 20, dB < 0, ib == 0);
      q_add(q, v, c);
    }
  }
  get_k(tk);
  // the key comb, software-pipelined: window it + 1's row is loaded before
  // window it's addition, so its HBM latency hides behind that addition
  // (~2.5k cycles) instead of opening each window -- which matters most
  // beside a pipeline's bulk launch, when the loads queue behind its
  // traffic (round 6, CMTV_CALL_TRACE: the loaded 150-validator call's
  // launch-to-verdict p90 was 50 us over its p50)
  int dA = (int)sc_shift_out(tk, 8) - 128;
  int ia = dA < 0 ? -dA : dA;
  fe cn;
  {
    const uint32_t* row = ktab + ((size_t)(COMB_WINDOWS - 1) * COMB_ENTRIES + (ia > 0 ? ia - 1 : 0)) * COMB_ROW_WORDS;
    q_niels_load(q, cn, [&](int off, fe& r) { comb_load(row, off, r); }, 10, 20, dA < 0);
  }
#pragma unroll 1
  for (int it = 0; it < COMB_WINDOWS; it++) {
    fe c = cn;
    q_niels_fix(c, lane, dA < 0, ia == 0);
    if (it + 1 < COMB_WINDOWS) {
      const int j = COMB_WINDOWS - 2 - it;
      dA = (int)sc_shift_out(tk, 8) - 128;
      ia = dA < 0 ? -dA : dA;
      const uint32_t* row = ktab + ((size_t)j * COMB_ENTRIES + (ia > 0 ? ia - 1 : 0)) * COMB_ROW_WORDS;
      q_niels_load(q, cn, [&](int off, fe& r) { comb_load(row, off, r); }, 10, 20, dA < 0);
    }
    q_add(q, v, c);
  }
  fe rc;
  bool r_ok;
  get_r(rc, r_ok);
  ok = ok && r_ok;

  if (MODE == MODE_GO_STDLIB) {
    fe z, t;
    q.template perm<QP_B2>(z, v);  // Z'
    fe_mul(t, z, rc);              // lane 0: x_R Z', lane 1: y_R Z'
    const bool eq = fe_equal(t, v);
    const bool e0 = q.template perm32<QP_B0>(eq ? 1u : 0u) != 0;
    const bool e1 = q.template perm32<QP_B1>(eq ? 1u : 0u) != 0;
    return ok && e0 && e1;
  }
  fe c;
  q_to_cached(q, c, rc);
  q_cached_cneg(q, c, true);
  q_add(q, v, c);
  const bool so = q_small_order(q, v);  // [8](R' - R) = O; every lane takes part in its DPP moves
  return ok && so;
}

// One wave does everything (k_verify_keyed_quad; the host checks): every
// lane hashes and decodes R itself, at the same points of the chain
template <uint32_t MODE, class Q>
CMTV_HD bool q_verify_keyed(const Q& q, const uint32_t* key_pk, bool key_ok, const uint32_t* sig_ptr,
                            const uint8_t* msg, uint32_t mlen, const uint32_t* ktab, const uint32_t* bcomb) {
  const int lane = q.lane();
  return q_verify_keyed_split<MODE>(
      q, key_ok, sig_ptr, ktab, bcomb, [&](uint32_t tk[8]) { q_keyed_challenge(tk, key_pk, sig_ptr, msg, mlen); },
      [&](fe& rc, bool& r_ok) {
        ge_p3 R;
        r_ok = q_keyed_decode_r<MODE>(R, sig_ptr);
        fe one;
        fe_1(one);
        fe_pick(rc, lane, R.X, R.Y, one, R.T);
      });
}

}  // namespace cmtv
