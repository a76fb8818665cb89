// oct.h -- 8 lanes per signature ("oct"): two quads split the multi-scalar
// multiplication of the half-size-scalar verifier (quad.h q_straus_half) for
// batches small enough that the chip has idle SIMDs (VerifyCommit on a
// 150-validator set, light-client headers, small blocksync batches).
//
// The quad verifier runs ONE Straus chain per signature:
//   X = [u]B + [k1](-A) + [|k2|](k2 < 0 ? R : -R),  per window 4 doublings +
//       an A, an R and (33 of 34 windows) a B addition.
// The oct splits it into two chains of the same length, one per quad:
//   lower quad (lanes 0-3):  P_lo = [k1](-A)           + [u mod 2^128]B
//   upper quad (lanes 4-7):  P_hi = [|k2|](+/-R)       + [u >> 128][2^128]B
// with the radix-2^16 B digits of both on windows 0, 4, .., 28 (the
// (1..2^15)B and (1..2^15)[2^128]B tables, verify_core.h), so a window is 4
// doublings + 1 table addition (+ 1 B addition every 4th window): ~2/3 of
// the quad's window work per lane, and each quad builds only its own
// (0..8)P table.
// Decoding, hashing and the half-scalar split are per-lane work that both
// quads repeat (the lower quad decodes A, the upper quad R), so the total
// lane-work per signature grows; the oct wins on latency (fewer
// instructions per wave) while the chip is not full, i.e. up to 1,024 waves
// = 8,192 signatures at one wave per SIMD.
//
// Merge: the upper quad's P_hi moves to the lower quad with one DPP row
// shift per word (lane i <- lane i + 4), the lower quad adds it, and the
// final check is the quad's (quad.h q_verify). Oct policy = the quad policy
// plus   bool upper() const;  void from_upper(fe& o, const fe& v) const;
//        uint32_t from_upper32(uint32_t x) const;
#pragma once
#include "quad.h"

namespace cmtv {

// The oct verifier with the scalar work supplied by get_prep(SigPrep&), which
// is called after the decompression (every lane of the wave calls it once).
// EXT_B: [u]B comes ready-made from get_b (the lower quad's cached
// coordinate, a helper wave's q_bcomb16) and is added after the merge; the
// quads then add no fixed-base digits.
template <uint32_t MODE, bool EXT_B = false, class Q, class BTab, class ATab, class GetPrep, class GetB = NoExtB>
CMTV_HD bool o_verify_split(const Q& q, const uint32_t* pk_ptr, const uint32_t* sig_ptr, const BTab& btab, ATab& tab,
                            const GetPrep& get_prep, const GetB& get_b = GetB()) {
  const int lane = q.lane();
  const bool up = q.upper();
  uint32_t w[8];

  // ---- decode: A on the lower quad, R on the upper one
  const uint32_t* src = up ? sig_ptr : pk_ptr;
#pragma unroll
  for (int i = 0; i < 8; i++) w[i] = src[i];
  fe v;
  bool dec, canon;
  {
    ge_p3 P;
    dec = p3_frombytes(P, w);
    canon = y_is_canonical(w) && !(fe_iszero(P.X) && (w[7] >> 31));
    fe one;
    fe_1(one);
    fe_pick(v, lane, P.X, P.Y, one, P.T);
  }

  // ---- half-size scalars (halfscalar.h), u = k2 s mod L; W uniform per wave
  SigPrep hs;
  get_prep(hs);
  const bool k2_neg = hs.flags & 1u, s_ok = (hs.flags & 4u) != 0;
  const int W = q_wave_windows(q, hs.flags);
  const uint32_t* u = hs.u;

  // ---- this quad's point: -A (lower), k2 < 0 ? R : -R (upper); its table
  {
    fe t;
    fe_neg(t, v);
    fe_carry(t);
    const bool neg = up ? !k2_neg : true;
    fe_select(v, v, t, neg && (lane == 0 || lane == 3));
  }
  q_build_table(q, tab, v);

  // ---- Straus over W windows: own 4-bit digits, B digits on even windows
  uint32_t tS[8], tB[8];
  {
    uint32_t sc[8], tHi[8];
#pragma unroll
    for (int i = 0; i < 8; i++) sc[i] = up ? hs.k2[i] : hs.k1[i];
    hs_digits16(tS, sc, W);
    hs_digits65536(tB, tHi, u);
#pragma unroll
    for (int i = 0; i < 8; i++) tB[i] = up ? tHi[i] : tB[i];
  }
  const int bblock = BT16_BASE + (up ? 2 * BT16_ENTRIES : 0);
  q_identity(v, lane);
#pragma unroll 1
  for (int win = W - 1; win >= 0; win--) {
    fe cS, cB;
    {
      const int d = (int)sc_shift_out(tS, 4) - 8;
      tab.load_signed(q, d < 0 ? -d : d, d < 0, cS);
    }
    const bool has_b = !EXT_B && (win & 3) == 0 && win <= 28;
    bool b_neg = false, b_ident = false;
    if (has_b) {
      const int dB = (int)sc_shift_out(tB, 16) - 0x8000;
      const int ib = dB < 0 ? -dB : dB;
      const int row = (ib > 0 ? ib - 1 : 0) + bblock;
      q_niels_load(
          q, cB, [&](int off, fe& r) { btab.load_coord(row, off, r); }, BTAB_COORD_WORDS, 2 * BTAB_COORD_WORDS,
          dB < 0);
      b_neg = dB < 0;
      b_ident = ib == 0;
    }
    if (win != W - 1) {
#pragma unroll 1
      for (int d = 0; d < 4; d++) q_dbl(q, v);
    }
    q_add(q, v, cS);
    if (has_b) {
      q_niels_fix(cB, lane, b_neg, b_ident);
      q_add(q, v, cB);
    }
  }

  // ---- merge: X = P_lo + P_hi on the lower quad
  {
    fe ph, c;
    q.from_upper(ph, v);
    q_to_cached(q, c, ph);
    q_add(q, v, c);
    if constexpr (EXT_B) {
      get_b(c);
      q_add(q, v, c);
    }
  }
  const bool a_ok = dec;                        // lower quad: A decoded
  const bool r_ok = q.from_upper32(dec ? 1u : 0u) != 0;
  const bool r_canon = q.from_upper32(canon ? 1u : 0u) != 0;

  // ---- final check (quad.h q_verify): X = O / [8]X = O
  if (MODE == MODE_ZIP215) {
    const bool so = q_small_order(q, v);  // every lane takes part in its DPP moves
    return s_ok && a_ok && r_ok && so;
  }
  fe z;
  q.template perm<QP_B2>(z, v);
  const bool x0 = fe_iszero(v);
  const bool yz = fe_equal(v, z);
  const bool e0 = q.template perm32<QP_B0>(x0 ? 1u : 0u) != 0;
  const bool e1 = q.template perm32<QP_B1>(yz ? 1u : 0u) != 0;
  return s_ok && a_ok && r_ok && r_canon && e0 && e1;
}

// One wave does everything (k_verify_oct; the host check)
template <uint32_t MODE, class Q, class BTab, class ATab>
CMTV_HD bool o_verify(const Q& q, const uint32_t* pk_ptr, const uint32_t* sig_ptr, const uint8_t* msg,
                      uint32_t mlen, const BTab& btab, ATab& tab, bool force_wide = false) {
  return o_verify_split<MODE>(q, pk_ptr, sig_ptr, btab, tab,
                              [&](SigPrep& p) { q_prepare<MODE>(p, pk_ptr, sig_ptr, msg, mlen, force_wide); });
}

}  // namespace cmtv
