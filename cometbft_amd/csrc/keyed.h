// keyed.h -- verification against registered keys (comb tables, no doublings).
//
// A validator set signs commit after commit with the same keys (blocksync and
// light-client replay, BASELINE configs[2]: 100k commits x 150 validators).
// Decompressing A and doubling through [k]A again for every signature repeats
// per-key work, so cmtv_register_keys precomputes, once per key, the comb
//
//     T_A[j][e] = (e+1) * 256^j * (-A)      j = 0..31, e = 0..127
//
// and the context holds the same comb for the base point B. With signed
// radix-256 digits (t = k + 0x80..80, digit_j = byte_j(t) - 128 in
// [-128, 127]) the double scalar multiplication becomes
//
//     R' = [s]B - [k]A = sum_j  T_B[j][s_j] + T_A[j][k_j]
//
// 64 mixed additions and no doublings (the generic path: 256 doublings + 96
// additions + decompression of A). The final check (check_R) is unchanged,
// so verdicts are identical to verify_one's on every input: the key's
// decompression result (Go Point.SetBytes semantics, non-canonical y
// accepted) is recorded at registration, and its original 32 bytes are what
// SHA-512(R || A || M) hashes.
//
// Row layout: 32 words per entry = one 128-byte line: y+x[10] y-x[10] 2dxy[10]
// pad[2], affine (Z = 1). Row (j, e) of a comb is at (j * 128 + e) * 32.
#pragma once
#include "verify_core.h"

namespace cmtv {

constexpr int COMB_WINDOWS = 32;
constexpr int COMB_ENTRIES = 128;
constexpr int COMB_ROW_WORDS = 32;
constexpr uint32_t COMB_TABLE_WORDS = COMB_WINDOWS * COMB_ENTRIES * COMB_ROW_WORDS;  // 512 KiB

// Column d (multiple d = 1..128) of the comb of P: the 32 points d*256^j*P.
// The points are built projectively (8 doublings per window), written as
// (X, Y, Z) into their rows, then normalised with one inversion (Montgomery's
// batch trick over the 32 Z's; prefix products go through Scratch .store(j,
// fe) / .load(j, fe)) and rewritten as affine niels.
template <class Scratch>
CMTV_HD void comb_build_column(uint32_t* tab, const ge_p3& P, int d, Scratch& sc) {
  // Q = d * P (double-and-add over the 8 bits of d)
  ge_cached Pc;
  p3_to_cached(Pc, P);
  ge_p3 acc;
  p3_identity(acc);
  ge_efgh t;
  ge_p2 q;
#pragma unroll 1
  for (int bit = 7; bit >= 0; bit--) {
    p3_to_p2(q, acc);
    p2_dbl(t, q);
    efgh_to_p3(acc, t);
    ge_add_cached(t, acc, Pc);
    ge_p3 added;
    efgh_to_p3(added, t);
    const bool take = (d >> bit) & 1;
    fe_select(acc.X, acc.X, added.X, take);
    fe_select(acc.Y, acc.Y, added.Y, take);
    fe_select(acc.Z, acc.Z, added.Z, take);
    fe_select(acc.T, acc.T, added.T, take);
  }
  p3_to_p2(q, acc);
  fe prod;
#pragma unroll 1
  for (int j = 0; j < COMB_WINDOWS; j++) {
    uint32_t* row = tab + (size_t)(j * COMB_ENTRIES + (d - 1)) * COMB_ROW_WORDS;
#pragma unroll
    for (int i = 0; i < 10; i++) {
      row[i] = q.X.v[i];
      row[10 + i] = q.Y.v[i];
      row[20 + i] = q.Z.v[i];
    }
    if (j == 0)
      prod = q.Z;
    else
      fe_mul(prod, prod, q.Z);
    sc.store(j, prod);
    if (j + 1 < COMB_WINDOWS) {
#pragma unroll 1
      for (int r = 0; r < 8; r++) {
        p2_dbl(t, q);
        efgh_to_p2(q, t);
      }
    }
  }
  fe inv, d2;
  fe_invert(inv, prod);
  fe_const_d2(d2);
#pragma unroll 1
  for (int j = COMB_WINDOWS - 1; j >= 0; j--) {
    uint32_t* row = tab + (size_t)(j * COMB_ENTRIES + (d - 1)) * COMB_ROW_WORDS;
    fe X, Y, Z, zi, x, y, o;
#pragma unroll
    for (int i = 0; i < 10; i++) {
      X.v[i] = row[i];
      Y.v[i] = row[10 + i];
      Z.v[i] = row[20 + i];
    }
    if (j > 0) {
      sc.load(j - 1, zi);
      fe_mul(zi, inv, zi);  // 1 / Z_j
      fe_mul(inv, inv, Z);  // 1 / (Z_0 ... Z_{j-1})
    } else {
      zi = inv;
    }
    fe_mul(x, X, zi);
    fe_mul(y, Y, zi);
    fe_add(o, y, x);
    fe_carry(o);
#pragma unroll
    for (int i = 0; i < 10; i++) row[i] = o.v[i];
    fe_sub(o, y, x);
    fe_carry(o);
#pragma unroll
    for (int i = 0; i < 10; i++) row[10 + i] = o.v[i];
    fe_mul(o, x, y);
    fe_mul(o, o, d2);
#pragma unroll
    for (int i = 0; i < 10; i++) row[20 + i] = o.v[i];
    row[30] = 0;
    row[31] = 0;
  }
}

// One window of a comb as an ge_add_table<false> source (niels, Z2 = 1).
struct CombWindow {
  const uint32_t* rows;  // row (j, 0)
  CMTV_HD void load_fe(int e, int c, fe& r) const {
    const uint32_t* p = rows + e * COMB_ROW_WORDS + c * 10;
#pragma unroll
    for (int i = 0; i < 10; i++) r.v[i] = p[i];
  }
};

// The comb half of a registered-key verification: R' = [s]B - [k]A into acc,
// and whether the key decoded and s is canonical (the final check against
// R is the caller's: check_R, or the batched encode of
// k_verify_keyed_batch).
template <class Win>
CMTV_HD bool keyed_comb(ge_p3& acc, const uint32_t* key_pk, bool key_ok, const uint32_t* sig_ptr, const uint8_t* msg,
                        uint32_t mlen, const uint32_t* ktab, const uint32_t* bcomb) {
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 8; i++) w[i] = sig_ptr[8 + i];  // S
  const bool ok = key_ok && (w[7] & 0xE0000000u) == 0 && sc_is_canonical(w);
  uint32_t ts[8], tk[8];
  sc_bias(ts, w, 0x80808080u);

  uint32_t h[16], k[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    w[i] = sig_ptr[i];  // R
    w[8 + i] = key_pk[i];
  }
  sha512_prefixed<16>(h, w, msg, mlen);
  sc_reduce512(k, h);
  sc_bias(tk, k, 0x80808080u);

  p3_identity(acc);
  ge_efgh t;
  // digits are taken from the top byte down: window j = 31 - it
#pragma unroll 1
  for (int it = 0; it < COMB_WINDOWS; it++) {
    const int j = COMB_WINDOWS - 1 - it;
    const int dA = (int)sc_shift_out(tk, 8) - 128;
    const int ia = dA < 0 ? -dA : dA;
    Win wa{ktab + (size_t)j * COMB_ENTRIES * COMB_ROW_WORDS};
    ge_add_table<false>(t, acc, wa, ia > 0 ? ia - 1 : 0, dA < 0, ia == 0);
    efgh_to_p3(acc, t);
    const int dB = (int)sc_shift_out(ts, 8) - 128;
    const int ib = dB < 0 ? -dB : dB;
    Win wb{bcomb + (size_t)j * COMB_ENTRIES * COMB_ROW_WORDS};
    ge_add_table<false>(t, acc, wb, ib > 0 ? ib - 1 : 0, dB < 0, ib == 0);
    efgh_to_p3(acc, t);
  }
  return ok;
}

// ---------------------------------------------------------------- wide combs
//
// For bulk replay of one validator set (configs[2]) the registration can also
// build the radix-2^16 comb of each key,
//
//     W_A[j][e] = (e+1) * 2^(16j) * (-A)      j = 0..15, e = 0..32767
//
// (64 MiB per key, same 128-byte rows), which halves the additions: with the
// signed radix-2^16 digits of hs_digits65536 (t = k + 0x8000 in every 16-bit
// field, digit in [-2^15, 2^15)) and the context's B comb of the same shape
// (verify_core.h BC16 blocks of the B table),
//
//     R' = [s]B - [k]A = sum_j  T_B16[j][s_j] + W_A[j][k_j]
//
// is 32 mixed additions. The final check is the caller's, as for keyed_comb.
constexpr int WIDE_POSITIONS = 16;
constexpr int WIDE_ENTRIES = 32768;
constexpr size_t WIDE_TABLE_WORDS = (size_t)WIDE_POSITIONS * WIDE_ENTRIES * COMB_ROW_WORDS;  // 64 MiB
// entries per build thread: one run of consecutive multiples, normalised
// together with one inversion
constexpr int WIDE_RUN = 64;

// Rows e0 .. e0 + WIDE_RUN - 1 of one position of a wide comb: the points
// (e+1) * P for the position's base P = 2^(16j) (-A). Q = (e0+1) P by
// double-and-add over 15 bits, then one addition of P per row; rows are
// written projectively, normalised with one inversion (prefix products
// through Scratch .store/.load, slots 0 .. WIDE_RUN-1) and rewritten as
// affine niels -- comb_build_column's scheme along e instead of j.
template <class Scratch>
CMTV_HD void wide_build_run(uint32_t* rows, const ge_p3& P, int e0, Scratch& sc) {
  ge_cached Pc;
  p3_to_cached(Pc, P);
  ge_p3 acc;
  p3_identity(acc);
  ge_efgh t;
  ge_p2 q;
  const int m = e0 + 1;
#pragma unroll 1
  for (int bit = 14; bit >= 0; bit--) {
    p3_to_p2(q, acc);
    p2_dbl(t, q);
    efgh_to_p3(acc, t);
    ge_add_cached(t, acc, Pc);
    ge_p3 added;
    efgh_to_p3(added, t);
    const bool take = (m >> bit) & 1;
    fe_select(acc.X, acc.X, added.X, take);
    fe_select(acc.Y, acc.Y, added.Y, take);
    fe_select(acc.Z, acc.Z, added.Z, take);
    fe_select(acc.T, acc.T, added.T, take);
  }
  fe prod;
#pragma unroll 1
  for (int r = 0; r < WIDE_RUN; r++) {
    uint32_t* row = rows + (size_t)(e0 + r) * COMB_ROW_WORDS;
#pragma unroll
    for (int i = 0; i < 10; i++) {
      row[i] = acc.X.v[i];
      row[10 + i] = acc.Y.v[i];
      row[20 + i] = acc.Z.v[i];
    }
    if (r == 0)
      prod = acc.Z;
    else
      fe_mul(prod, prod, acc.Z);
    sc.store(r, prod);
    if (r + 1 < WIDE_RUN) {
      ge_add_cached(t, acc, Pc);
      efgh_to_p3(acc, t);
    }
  }
  fe inv, d2;
  fe_invert(inv, prod);
  fe_const_d2(d2);
#pragma unroll 1
  for (int r = WIDE_RUN - 1; r >= 0; r--) {
    uint32_t* row = rows + (size_t)(e0 + r) * COMB_ROW_WORDS;
    fe X, Y, Z, zi, x, y, o;
#pragma unroll
    for (int i = 0; i < 10; i++) {
      X.v[i] = row[i];
      Y.v[i] = row[10 + i];
      Z.v[i] = row[20 + i];
    }
    if (r > 0) {
      sc.load(r - 1, zi);
      fe_mul(zi, inv, zi);  // 1 / Z_r
      fe_mul(inv, inv, Z);  // 1 / (Z_0 ... Z_{r-1})
    } else {
      zi = inv;
    }
    fe_mul(x, X, zi);
    fe_mul(y, Y, zi);
    fe_add(o, y, x);
    fe_carry(o);
#pragma unroll
    for (int i = 0; i < 10; i++) row[i] = o.v[i];
    fe_sub(o, y, x);
    fe_carry(o);
#pragma unroll
    for (int i = 0; i < 10; i++) row[10 + i] = o.v[i];
    fe_mul(o, x, y);
    fe_mul(o, o, d2);
#pragma unroll
    for (int i = 0; i < 10; i++) row[20 + i] = o.v[i];
    row[30] = 0;
    row[31] = 0;
  }
}

// keyed_comb over the wide combs: wtab = the key's wide comb of -A, btab =
// the B table whose BC16 blocks hold (1..2^15) 2^(16j) B (a load_fe policy
// over absolute rows).
// The digit streams of a wide-comb verification: k = SHA-512(R || A || M)
// mod L and s, as hs_digits65536 streams (Hi: digits 15..8, Lo: 7..0); returns
// whether the key decoded and s is canonical.
CMTV_HD bool keyed_wide_digits(uint32_t kLo[8], uint32_t kHi[8], uint32_t sLo[8], uint32_t sHi[8],
                               const uint32_t* key_pk, bool key_ok, const uint32_t* sig_ptr, const uint8_t* msg,
                               uint32_t mlen) {
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 8; i++) w[i] = sig_ptr[8 + i];  // S
  const bool ok = key_ok && (w[7] & 0xE0000000u) == 0 && sc_is_canonical(w);
  hs_digits65536(sLo, sHi, w);
  uint32_t h[16], k[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    w[i] = sig_ptr[i];  // R
    w[8 + i] = key_pk[i];
  }
  sha512_prefixed<16>(h, w, msg, mlen);
  sc_reduce512(k, h);
  hs_digits65536(kLo, kHi, k);
  return ok;
}

template <class Win, class BTab>
CMTV_HD bool keyed_comb_wide(ge_p3& acc, const uint32_t* key_pk, bool key_ok, const uint32_t* sig_ptr,
                             const uint8_t* msg, uint32_t mlen, const uint32_t* wtab, const BTab& btab) {
  uint32_t kLo[8], kHi[8], sLo[8], sHi[8];
  const bool ok = keyed_wide_digits(kLo, kHi, sLo, sHi, key_pk, key_ok, sig_ptr, msg, mlen);
  p3_identity(acc);
  ge_efgh t;
#pragma unroll 1
  for (int j = WIDE_POSITIONS - 1; j >= 0; j--) {
    const bool hi = j >= 8;
    const int dA = (int)(hi ? sc_shift_out(kHi, 16) : sc_shift_out(kLo, 16)) - 0x8000;
    const int ia = dA < 0 ? -dA : dA;
    Win wa{wtab + (size_t)j * WIDE_ENTRIES * COMB_ROW_WORDS};
    ge_add_table<false>(t, acc, wa, ia > 0 ? ia - 1 : 0, dA < 0, ia == 0);
    efgh_to_p3(acc, t);
    const int dB = (int)(hi ? sc_shift_out(sHi, 16) : sc_shift_out(sLo, 16)) - 0x8000;
    const int ib = dB < 0 ? -dB : dB;
    ge_add_table<false>(t, acc, btab, BC16_BASE + j * BT16_ENTRIES + (ib > 0 ? ib - 1 : 0), dB < 0, ib == 0);
    efgh_to_p3(acc, t);
  }
  return ok;
}

// keyed_comb with [s]B over the B table's radix-2^16 comb (BC16: 16 additions)
// and [k](-A) over the key's radix-256 comb (32): 48 additions instead of 64,
// for key sets whose wide combs do not fit (64 MiB per key against 512 KiB;
// a 10k-validator set's would take 640 GiB). One B addition follows every
// other A addition (B position j >> 1 after A position j, j odd), so the two
// tables' rows alternate. The sum is R' = [s]B - [k]A as keyed_comb's.
template <class Win, class BTab>
CMTV_HD bool keyed_comb_mixed(ge_p3& acc, const uint32_t* key_pk, bool key_ok, const uint32_t* sig_ptr,
                              const uint8_t* msg, uint32_t mlen, const uint32_t* ktab, const BTab& btab) {
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 8; i++) w[i] = sig_ptr[8 + i];  // S
  const bool ok = key_ok && (w[7] & 0xE0000000u) == 0 && sc_is_canonical(w);
  uint32_t sLo[8], sHi[8], tk[8];
  hs_digits65536(sLo, sHi, w);
  uint32_t h[16], k[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    w[i] = sig_ptr[i];  // R
    w[8 + i] = key_pk[i];
  }
  sha512_prefixed<16>(h, w, msg, mlen);
  sc_reduce512(k, h);
  sc_bias(tk, k, 0x80808080u);
  p3_identity(acc);
  ge_efgh t;
#pragma unroll 1
  for (int j = COMB_WINDOWS - 1; j >= 0; j--) {
    const int dA = (int)sc_shift_out(tk, 8) - 128;
    const int ia = dA < 0 ? -dA : dA;
    Win wa{ktab + (size_t)j * COMB_ENTRIES * COMB_ROW_WORDS};
    ge_add_table<false>(t, acc, wa, ia > 0 ? ia - 1 : 0, dA < 0, ia == 0);
    efgh_to_p3(acc, t);
    if (j & 1) {
      const int jb = j >> 1;
      const int dB = (int)(jb >= 8 ? sc_shift_out(sHi, 16) : sc_shift_out(sLo, 16)) - 0x8000;
      const int ib = dB < 0 ? -dB : dB;
      ge_add_table<false>(t, acc, btab, BC16_BASE + jb * BT16_ENTRIES + (ib > 0 ? ib - 1 : 0), dB < 0, ib == 0);
      efgh_to_p3(acc, t);
    }
  }
  return ok;
}

// Verification of one signature by a registered key. key_pk: the key's 32
// original bytes; key_ok: its decompression succeeded; ktab: its comb of -A;
// bcomb: the comb of B. Same verdict as verify_one<MODE>(key_pk, ...).
template <uint32_t MODE, class Win>
CMTV_HD bool verify_keyed(const uint32_t* key_pk, bool key_ok, const uint32_t* sig_ptr, const uint8_t* msg,
                          uint32_t mlen, const uint32_t* ktab, const uint32_t* bcomb) {
  ge_p3 acc;
  const bool ok = keyed_comb<Win>(acc, key_pk, key_ok, sig_ptr, msg, mlen, ktab, bcomb);
  return check_R<MODE>(acc, sig_ptr) && ok;
}

// GO_STDLIB's final check from a precomputed 1/Z (Montgomery batch
// inversion, k_verify_keyed_batch): encode(R') == R bytes, exactly as
// check_R<MODE_GO_STDLIB> with p3_tobytes' own inversion replaced by zi.
CMTV_HD bool check_R_go_zi(const fe& X, const fe& Y, const fe& zi, const uint32_t* sig_ptr) {
  fe x, y;
  fe_mul(x, X, zi);
  fe_mul(y, Y, zi);
  uint32_t enc[8];
  fe_tobytes(enc, y);
  enc[7] |= (uint32_t)fe_isneg(x) << 31;
  uint32_t diff = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) diff |= enc[i] ^ sig_ptr[i];
  return diff == 0;
}

}  // namespace cmtv
