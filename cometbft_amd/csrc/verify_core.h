// verify_core.h -- per-signature Ed25519 verification pipeline (one signature
// per lane), shared by the gfx950 kernels in verify.hip.
//
// Restates Go 1.19 crypto/ed25519.Verify as reached from
// /root/reference/crypto/ed25519/ed25519.go:148-155 (MODE_GO_STDLIB) and the
// ZIP-215 cofactored check (MODE_ZIP215):
//
//   sig[63] & 0xE0 == 0,  s < L,  A = decode(pk) (non-canonical accepted)
//   k  = SHA-512(R || A || M) mod L
//   R' = [s]B - [k]A      (Straus, shared doublings, fixed windows)
//   GO_STDLIB: encode(R') == R bytes      ZIP215: [8](R' - decode(R)) == O
//   (efgh_small_order: no doublings)
//
// Scalar multiplication layout (SIMD-uniform schedule):
//   * [k](-A): signed radix-16 digits in [-8, 7], per-lane table of
//     (1..8)(-A) in cached form, 64 additions;
//   * [s]B:   signed radix-256 digits in [-128, 127], shared table of
//     (1..128)B in affine niels form, 32 mixed additions;
//   * 256 doublings shared by both.
// Every lane of a wave executes exactly the same instruction stream (no wNAF,
// no data-dependent branches); the digit only selects table rows.
#pragma once
#include "fe25519.h"
#include "ge25519.h"
#include "halfscalar.h"
#include "sc25519.h"
#include "sha512.h"

namespace cmtv {

enum : uint32_t { MODE_GO_STDLIB = 0, MODE_ZIP215 = 1 };

// B-table row layout: 36 words per entry, each coordinate 16-byte aligned:
// ypx[10] pad[2] ymx[10] pad[2] xy2d[10] pad[2].
constexpr int BTAB_ROW_WORDS = 36;
constexpr int BTAB_COORD_WORDS = 12;
constexpr int BTAB_ENTRIES = 128;
// A-table: 8 cached points x 40 words per lane.
constexpr int ATAB_WORDS = 8 * 40;

// canonical encoding words of the base point (y = 4/5, x even)
CMTV_HD void basepoint_words(uint32_t w[8]) {
  w[0] = 0x66666658u;
#pragma unroll
  for (int i = 1; i < 8; i++) w[i] = 0x66666666u;
}

// y (255 bits, sign stripped) < p ?  -- the canonical-encoding test for R
CMTV_HD bool y_is_canonical(const uint32_t w[8]) {
  const uint32_t top = w[7] & 0x7FFFFFFFu;
  bool all_ones = top == 0x7FFFFFFFu;
#pragma unroll
  for (int i = 1; i < 7; i++) all_ones = all_ones && w[i] == 0xFFFFFFFFu;
  return !(all_ones && w[0] >= 0xFFFFFFEDu);
}

CMTV_HD void cached_neg_point(ge_p3& r, const ge_p3& p) {
  fe_neg(r.X, p.X);
  fe_carry(r.X);
  r.Y = p.Y;
  r.Z = p.Z;
  fe_neg(r.T, p.T);
  fe_carry(r.T);
}

// [m]B for m = 1..128 in affine niels form (one entry; used by the table
// initialisation kernel and by host-side tests). The device table holds
// three blocks of 128 rows: block 0 = [m]B, block 1 = [m 2^124]B (the quad
// verifier's odd windows, halfscalar.h), block 2 = [m 2^128]B (the oct
// verifier's upper quad, oct.h).
CMTV_HD int btab_block_shift(int block) { return block == 0 ? 0 : (block == 1 ? 124 : 128); }

// Radix-2^16 fixed-base tables of the quad and oct verifiers (quad.h, oct.h),
// after the three radix-256 blocks: block b = rows (1..2^15)[2^shift]B with
// shift 0 (u's digits 0..7), 120 (quad: digits 8..15 on windows 4j+2) and
// 128 (oct upper quad: digits 8..15 on windows 4j).
constexpr int BT16_ENTRIES = 32768;
constexpr int BT16_BASE = 3 * BTAB_ENTRIES;
constexpr int BT16_ROWS = 3 * BT16_ENTRIES;
CMTV_HD int bt16_block_shift(int block) { return block == 0 ? 0 : (block == 1 ? 120 : 128); }

// 16-position radix-2^16 comb of B for the helper waves (quad.h q_bcomb16):
// block j = (1..2^15)[2^(16j)]B, j = 0..15
constexpr int BC16_BASE = BT16_BASE + BT16_ROWS;
constexpr int BC16_ROWS = 16 * BT16_ENTRIES;
constexpr int BTAB_TOTAL_ROWS = BC16_BASE + BC16_ROWS;  // 622,976 rows, 89.7 MB

// [m][2^shift]B, m < 2^bits, in affine niels form
CMTV_HD void btab_entry_shift(uint32_t row[BTAB_ROW_WORDS], int m, int shift, int bits);
CMTV_HD void btab_entry(uint32_t row[BTAB_ROW_WORDS], int m, int block = 0) {
  btab_entry_shift(row, m, btab_block_shift(block), 8);
}
CMTV_HD void btab_entry_shift(uint32_t row[BTAB_ROW_WORDS], int m, int shift, int bits) {
  uint32_t bw[8];
  basepoint_words(bw);
  ge_p3 B, acc;
  p3_frombytes(B, bw);
  if (shift) {
    ge_efgh t;
    ge_p2 q;
    p3_to_p2(q, B);
#pragma unroll 1
    for (int i = 0; i < shift; i++) {
      p2_dbl(t, q);
      efgh_to_p2(q, t);
    }
    efgh_to_p3(B, t);
  }
  ge_cached Bc;
  p3_to_cached(Bc, B);
  p3_identity(acc);
  ge_efgh t;
  ge_p2 q;
  for (int bit = bits - 1; bit >= 0; bit--) {
    p3_to_p2(q, acc);
    p2_dbl(t, q);
    efgh_to_p3(acc, t);
    ge_add_cached(t, acc, Bc);
    ge_p3 added;
    efgh_to_p3(added, t);
    const bool take = (m >> bit) & 1;
    fe_select(acc.X, acc.X, added.X, take);
    fe_select(acc.Y, acc.Y, added.Y, take);
    fe_select(acc.Z, acc.Z, added.Z, take);
    fe_select(acc.T, acc.T, added.T, take);
  }
  fe zi, x, y, ypx, ymx, xy, d2;
  fe_invert(zi, acc.Z);
  fe_mul(x, acc.X, zi);
  fe_mul(y, acc.Y, zi);
  fe_add(ypx, y, x);
  fe_carry(ypx);
  fe_sub(ymx, y, x);
  fe_carry(ymx);
  fe_mul(xy, x, y);
  fe_const_d2(d2);
  fe_mul(xy, xy, d2);
  for (int i = 0; i < BTAB_ROW_WORDS; i++) row[i] = 0;
  for (int i = 0; i < 10; i++) {
    row[i] = ypx.v[i];
    row[BTAB_COORD_WORDS + i] = ymx.v[i];
    row[2 * BTAB_COORD_WORDS + i] = xy.v[i];
  }
}

// row e of the device B table, whatever its block (k_btab_init, host checks)
CMTV_HD void btab_row(uint32_t row[BTAB_ROW_WORDS], int e) {
  if (e < BT16_BASE) {
    btab_entry(row, e % BTAB_ENTRIES + 1, e / BTAB_ENTRIES);
  } else if (e < BC16_BASE) {
    const int f = e - BT16_BASE;
    btab_entry_shift(row, f % BT16_ENTRIES + 1, bt16_block_shift(f / BT16_ENTRIES), 16);
  } else {
    const int f = e - BC16_BASE;
    btab_entry_shift(row, f % BT16_ENTRIES + 1, 16 * (f / BT16_ENTRIES), 16);
  }
}

// acc = [s]B + [k]P  where the ATab holds (1..8)P in cached form.
// ATab: .load_fe(int e, int c, fe&) for e in 0..7 (multiple e+1), c = cached coordinate.
// BTab: .load_fe(int e, int c, fe&) for e in 0..127 (multiple e+1), c = niels coordinate.
// Loops are kept rolled (#pragma unroll 1): the body is ~20 inlined field
// multiplications, and the whole loop must stay resident in the instruction
// cache that the CU's waves share.
template <bool WITH_P, class ATab, class BTab>
CMTV_HD void straus_double_scalarmult(ge_p3& out, const uint32_t k[8], const uint32_t s[8], const ATab& atab,
                                      const BTab& btab) {
  uint32_t tk[8], ts[8];
  sc_bias(tk, k, 0x88888888u);
  sc_bias(ts, s, 0x80808080u);
  ge_p2 cur;
  p2_identity(cur);
  ge_p3 P;
  ge_efgh t;
#pragma unroll 1
  for (int w = 0; w < 64; w++) {
#pragma unroll 1
    for (int d = 0; d < 3; d++) {
      p2_dbl(t, cur);
      efgh_to_p2(cur, t);
    }
    p2_dbl(t, cur);
    if (WITH_P) {
      const int dA = (int)sc_shift_out(tk, 4) - 8;
      const int ia = dA < 0 ? -dA : dA;
      efgh_to_p3(P, t);
      ge_add_table<true>(t, P, atab, ia > 0 ? ia - 1 : 0, dA < 0, ia == 0);
    }
    if (w & 1) {
      const int dB = (int)sc_shift_out(ts, 8) - 128;
      const int ib = dB < 0 ? -dB : dB;
      efgh_to_p3(P, t);
      ge_add_table<false>(t, P, btab, ib > 0 ? ib - 1 : 0, dB < 0, ib == 0);
    }
    efgh_to_p2(cur, t);
  }
  efgh_to_p3(out, t);
}

// Builds (1..8)P in cached form through the ATab (.store / .load_fe); P's own
// cached form is re-read from entry 0 rather than kept in registers.
template <class ATab>
CMTV_HD void build_cached_table(ATab& atab, const ge_p3& P) {
  ge_cached c;
  p3_to_cached(c, P);
  atab.store(0, c);
  ge_efgh t;
  ge_p2 q;
  ge_p3 cur;
  p3_to_p2(q, P);
  p2_dbl(t, q);
  efgh_to_p3(cur, t);
  p3_to_cached(c, cur);
  atab.store(1, c);
#pragma unroll 1
  for (int e = 2; e < 8; e++) {
    ge_add_table<true>(t, cur, atab, 0, false, false);
    efgh_to_p3(cur, t);
    p3_to_cached(c, cur);
    atab.store(e, c);
  }
}

// [8]P = O for P = (ef : gh : fg : eh) in completed form: the torsion is
// cyclic of order 8, so [8]P = O <=> [2]P is in E[4] (the points with
// xy = 0) <=> T([2]P) = 2XY (X^2 + Y^2) = 0 <=> T = 0 or X^2 + Y^2 = 0
// (quad.h q_small_order); T = eh is zero iff e or h is.
CMTV_HD bool efgh_small_order(const ge_efgh& t) {
  fe x, y;
  fe_mul(x, t.e, t.f);
  fe_mul(y, t.g, t.h);
  fe_sq(x, x);
  fe_sq(y, y);
  fe_add(x, x, y);
  return fe_iszero(t.e) || fe_iszero(t.h) || fe_iszero(x);
}

// Final equation against the signature's R bytes (sig_ptr[0..7]):
//   GO_STDLIB: encode(R') == R bytes (Go bytes.Equal after Point.Bytes)
//   ZIP215:    [8](R' - decode(R)) == O, R decoded with the same rules as A
template <uint32_t MODE>
CMTV_HD bool check_R(const ge_p3& Rp, const uint32_t* sig_ptr) {
  uint32_t w[8];
#pragma unroll
  for (int i = 0; i < 8; i++) w[i] = sig_ptr[i];  // R
  if (MODE == MODE_GO_STDLIB) {
    uint32_t enc[8];
    p3_tobytes(enc, Rp.X, Rp.Y, Rp.Z);
    uint32_t diff = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) diff |= enc[i] ^ w[i];
    return diff == 0;
  } else {
    ge_p3 R;
    const bool r_ok = p3_frombytes(R, w);
    ge_cached Rc;
    p3_to_cached(Rc, R);
    ge_efgh t;
    cached_cneg(Rc, true);
    ge_add_cached(t, Rp, Rc);
    return r_ok && efgh_small_order(t);
  }
}

// ---------------------------------------------------------------- ZIP-215 by coset
//
// ZIP-215's final check, [8](R' - R) = O with R decoded, without decoding R
// (no square-root chain): the check holds iff R's decoding lies in the coset
// R' + E[8]. With T8 a point of order 8, E[8] = E[4] u (T8 + E[4]), and
// adding a point of E[4] only permutes and scales coordinates (a = -1):
//   + (0, -1): (x, y) -> (-x, -y);  + (i, 0): (x, y) -> (iy, ix);
//   + (-i, 0): (x, y) -> (-iy, -ix)                     (i = sqrt(-1))
// So for Q in {R', R' + T8} (projective X:Y:Z) and y_R = R's y (mod p, the
// non-canonical encodings accepted as in decoding), the coset holds a point
// with y = y_R iff one of Y, -Y, iX, -iX equals y_R Z; its x is then X, -X,
// iY, -iY over Z. A point with y = y_R on the curve means R decodes (x^2 is
// the same square), to the root whose low bit is R's sign bit (x = 0 for
// either sign), so R's decoding is that coset point iff x = 0 or x has the
// sign bit. Two matches are the two roots +-x (both in the coset): pass.
// Equivalence with the decode-and-multiply check: the 1,406-vector corpus
// and torsion-shifted / sign-flipped / non-canonical R fuzzing against the
// oracle (tests/test_host_math.py, hostcheck "zipc" mode).
//
// zip_coset returns 0 (fail), 2 (pass) or 1 (pass iff xn / z is 0 or has R's
// sign bit: z is inverted by the caller, in a batch over signatures).
struct T8Niels {  // (y+x, y-x, 2dxy) of the order-8 point used
  CMTV_HD void load_fe(int, int c, fe& r) const {
    const uint32_t k[3][10] = {
        {0x1afe924, 0x064e10d, 0x3de65cf, 0x1ec4f88, 0x1ae0131, 0x1316ae5, 0x3e92f99, 0x02ef5ff, 0x327e371, 0x0676598},
        {0x324467d, 0x1c1bdaa, 0x3502e26, 0x0eb112a, 0x2cd374e, 0x174d56e, 0x04ffd60, 0x1a4bbb3, 0x3271c47, 0x168b7cb},
        {0x3139da9, 0x108e3c9, 0x24d90e1, 0x12c8a83, 0x2f70530, 0x1e35349, 0x1fd626f, 0x1edcea2, 0x3ef68a4, 0x11762b1}};
#pragma unroll
    for (int i = 0; i < 10; i++) r.v[i] = c == 0 ? k[0][i] : (c == 1 ? k[1][i] : k[2][i]);
  }
};

CMTV_HD uint32_t zip_coset(fe& xn, fe& z, const ge_p3& Rp, const uint32_t rw[8]) {
  fe yr, sqm1;
  fe_frombytes(yr, rw);  // bit 255 (the sign) ignored, y >= p accepted
  fe_const_sqrtm1(sqm1);
  uint32_t matches = 0;
  bool have = false;
  // one base point Q = (X:Y:Z): its four E[4] translates against y_R
  auto base = [&](const fe& X, const fe& Y, const fe& Z) {
    fe a, t, iX, iY, cand;
    fe_mul(a, yr, Z);
    fe_mul(iX, sqm1, X);
    fe_mul(iY, sqm1, Y);
    fe_sub(t, Y, a);
    const bool c0 = fe_iszero(t);
    fe_add(t, Y, a);
    const bool c1 = fe_iszero(t);
    fe_sub(t, iX, a);
    const bool c2 = fe_iszero(t);
    fe_add(t, iX, a);
    const bool c3 = fe_iszero(t);
    matches += (uint32_t)c0 + (uint32_t)c1 + (uint32_t)c2 + (uint32_t)c3;
    // the first match's x numerator: X, -X, iY, -iY
    fe nX, niY;
    fe_neg(nX, X);
    fe_neg(niY, iY);
    fe_select(cand, niY, iY, c2);
    fe_select(cand, cand, nX, c1);
    fe_select(cand, cand, X, c0);
    const bool take = !have && (c0 || c1 || c2 || c3);
    fe_select(xn, xn, cand, take);
    fe_select(z, z, Z, take);
    have = have || take;
  };
  fe_1(z);
  fe_1(xn);
  base(Rp.X, Rp.Y, Rp.Z);
  {
    ge_efgh t;
    ge_add_table<false>(t, Rp, T8Niels{}, 0, false, false);  // R' + T8
    fe X1, Y1, Z1;
    fe_mul(X1, t.e, t.f);
    fe_mul(Y1, t.g, t.h);
    fe_mul(Z1, t.f, t.g);
    base(X1, Y1, Z1);
  }
  if (matches == 0) {
    fe_1(z);
    return 0u;
  }
  if (matches >= 2) {
    fe_1(z);
    return 2u;
  }
  return 1u;
}

// state 1: x = xn zi (zi = 1 / z) is 0 or has R's sign bit (rw7 = R's top word)
CMTV_HD bool zip_coset_finish(uint32_t state, const fe& xn, const fe& zi, uint32_t rw7) {
  fe x;
  fe_mul(x, xn, zi);
  uint32_t s[8];
  fe_tobytes(s, x);
  uint32_t nz = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) nz |= s[i];
  return state == 2u || (state == 1u && (nz == 0 || (s[0] & 1u) == (rw7 >> 31)));
}

// check_R<MODE_ZIP215> by coset, one inversion (the batched kernels share it
// over several signatures instead)
CMTV_HD bool check_R_zip_coset(const ge_p3& Rp, const uint32_t* sig_ptr) {
  uint32_t w[8];
#pragma unroll
  for (int i = 0; i < 8; i++) w[i] = sig_ptr[i];  // R
  fe xn, z, zi;
  const uint32_t st = zip_coset(xn, z, Rp, w);
  fe_invert(zi, z);
  return zip_coset_finish(st, xn, zi, w[7]);
}

// Full single-signature verification. pk / sig are read through pointers
// (little-endian 32-bit words) at the points they are needed, so neither is
// held in registers across the scalar multiplication.
template <uint32_t MODE, class ATab, class BTab>
CMTV_HD bool verify_one(const uint32_t* pk_ptr, const uint32_t* sig_ptr, const uint8_t* msg, uint32_t mlen,
                        ATab& atab, const BTab& btab) {
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 8; i++) w[i] = sig_ptr[8 + i];  // S
  bool ok = (w[7] & 0xE0000000u) == 0 && sc_is_canonical(w);  // sig[63] & 224, S < L
  uint32_t ts[8];
#pragma unroll
  for (int i = 0; i < 8; i++) ts[i] = w[i];

  ge_p3 A;
#pragma unroll
  for (int i = 0; i < 8; i++) w[i] = pk_ptr[i];
  ok = p3_frombytes(A, w) && ok;
  ge_p3 nA;
  cached_neg_point(nA, A);
  build_cached_table(atab, nA);

  uint32_t h[16], k[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    w[i] = sig_ptr[i];  // R
    w[8 + i] = pk_ptr[i];
  }
  sha512_prefixed<16>(h, w, msg, mlen);
  sc_reduce512(k, h);

  ge_p3 Rp;
  straus_double_scalarmult<true>(Rp, k, ts, atab, btab);
  return check_R<MODE>(Rp, sig_ptr) && ok;
}

// Wave-uniform predicate for loop bounds (the device policy ballots; one
// lane per "wave" on the host)
struct HostWave {
  CMTV_HD bool any(bool x) const { return x; }
};

// Half-size-scalar form of verify_one (halfscalar.h): with (k1, k2) the
// half-size pair of k and u = k2 s mod L,
//   X = [u]B + [k1](-A) + [|k2|](k2 < 0 ? R : -R) = [k2](R' - R)
// over 34 shared 4-bit windows (64 when the pair is wide): per window four
// doublings, one (1..8)(-A) and one (1..8)(-/+R) addition, and one fixed-base
// addition (u mod 2^128 against (1..128)B on even windows, u >> 128 against
// (1..128)[2^124]B on odd ones). k2 is odd, so X = O <=> R' = R and
// [8]X = O <=> [8](R' - R) = O: the verdicts are verify_one's.
//   GO_STDLIB: R canonical (and decodable) and X = O  -- encode(R') == R bytes
//   ZIP215:    R decodable and [8]X = O
// atabA / atabR: two (1..8)P cached tables; btab rows 0..255 (both tables).
template <uint32_t MODE, class ATab, class BTab, class Wave = HostWave>
CMTV_HD bool verify_one_half(const uint32_t* pk_ptr, const uint32_t* sig_ptr, const uint8_t* msg, uint32_t mlen,
                             ATab& atabA, ATab& atabR, const BTab& btab, const Wave& wave = Wave()) {
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 8; i++) w[i] = sig_ptr[8 + i];  // S
  bool ok = (w[7] & 0xE0000000u) == 0 && sc_is_canonical(w);  // sig[63] & 224, S < L
  uint32_t ts[8];
#pragma unroll
  for (int i = 0; i < 8; i++) ts[i] = w[i];

  // k = SHA-512(R || A || M) mod L, then the half-size pair and u
  uint32_t k[8];
  {
    uint32_t h[16];
#pragma unroll
    for (int i = 0; i < 8; i++) {
      w[i] = sig_ptr[i];  // R
      w[8 + i] = pk_ptr[i];
    }
    sha512_prefixed<16>(h, w, msg, mlen);
    sc_reduce512(k, h);
  }
  HalfScalars hs;
  half_scalars(hs, k, false, MODE != MODE_ZIP215);
  uint32_t u[8];
  hs_bscalar(u, hs.k2, hs.k2_neg, ts);
  // window count: the largest over the wave (33..37), 64 if any is wide
  const bool wide = wave.any(hs.wide);
  int W = HS_WINDOWS;
#pragma unroll 1
  for (int w = HS_WINDOWS; w < HS_MAX_WINDOWS; w++) W += wave.any(hs.windows > w) ? 1 : 0;
  W = wide ? HS_WIDE_WINDOWS : W;

  // tables: (1..8)(-A), (1..8)(k2 < 0 ? R : -R)
  {
    ge_p3 P, nP;
#pragma unroll
    for (int i = 0; i < 8; i++) w[i] = pk_ptr[i];
    ok = p3_frombytes(P, w) && ok;
    cached_neg_point(nP, P);
    build_cached_table(atabA, nP);
#pragma unroll
    for (int i = 0; i < 8; i++) w[i] = sig_ptr[i];
    const bool r_ok = p3_frombytes(P, w);
    if (MODE == MODE_GO_STDLIB) ok = ok && r_ok && y_is_canonical(w) && !(fe_iszero(P.X) && (w[7] >> 31));
    else ok = ok && r_ok;
    cached_neg_point(nP, P);
#pragma unroll
    for (int i = 0; i < 10; i++) {
      nP.X.v[i] = hs.k2_neg ? P.X.v[i] : nP.X.v[i];
      nP.T.v[i] = hs.k2_neg ? P.T.v[i] : nP.T.v[i];
    }
    build_cached_table(atabR, nP);
  }

  uint32_t tA[8], tR[8], tLo[8], tHi[8];
  hs_digits16(tA, hs.k1, W);
  hs_digits16(tR, hs.k2, W);
  hs_digits256(tLo, tHi, u);
  ge_p2 cur;
  p2_identity(cur);
  ge_p3 P;
  ge_efgh t;
#pragma unroll 1
  for (int win = W - 1; win >= 0; win--) {
#pragma unroll 1
    for (int d = 0; d < 3; d++) {
      p2_dbl(t, cur);
      efgh_to_p2(cur, t);
    }
    p2_dbl(t, cur);
    {
      const int dA = (int)sc_shift_out(tA, 4) - 8;
      const int ia = dA < 0 ? -dA : dA;
      efgh_to_p3(P, t);
      ge_add_table<true>(t, P, atabA, ia > 0 ? ia - 1 : 0, dA < 0, ia == 0);
    }
    {
      const int dR = (int)sc_shift_out(tR, 4) - 8;
      const int ir = dR < 0 ? -dR : dR;
      efgh_to_p3(P, t);
      ge_add_table<true>(t, P, atabR, ir > 0 ? ir - 1 : 0, dR < 0, ir == 0);
    }
    if (win <= 32 && ((win & 1) == 0 || win <= 31)) {
      const bool odd = win & 1;
      int dB;
      if (odd)
        dB = (int)sc_shift_out(tHi, 8) - 128;
      else
        dB = (int)sc_shift_out(tLo, 8) - 128;
      const int ib = dB < 0 ? -dB : dB;
      efgh_to_p3(P, t);
      ge_add_table<false>(t, P, btab, (ib > 0 ? ib - 1 : 0) + (odd ? BTAB_ENTRIES : 0), dB < 0, ib == 0);
    }
    efgh_to_p2(cur, t);
  }
  if (MODE == MODE_ZIP215) return ok && efgh_small_order(t);  // t: the last window's sum
  return ok && fe_iszero(cur.X) && fe_equal(cur.Y, cur.Z);
}

// RFC 8032 key expansion: h = SHA-512(seed); a = clamp(h[0:32]) mod L, prefix = h[32:64]
CMTV_HD void expand_seed(uint32_t a_modl[8], uint32_t prefix[8], const uint32_t seed[8]) {
  uint32_t h[16];
  sha512_prefixed<8>(h, seed, nullptr, 0);
  uint32_t a[16];
#pragma unroll
  for (int i = 0; i < 16; i++) a[i] = (i < 8) ? h[i] : 0;
  a[0] &= 0xFFFFFFF8u;
  a[7] &= 0x7FFFFFFFu;
  a[7] |= 0x40000000u;
  sc_reduce512(a_modl, a);
#pragma unroll
  for (int i = 0; i < 8; i++) prefix[i] = h[8 + i];
}

struct NullATab {
  CMTV_HD void load_fe(int, int, fe&) const {}
  CMTV_HD void store(int, const ge_cached&) {}
};

template <class BTab>
CMTV_HD void scalarmult_base(ge_p3& out, const uint32_t s[8], const BTab& btab) {
  const uint32_t zero[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  NullATab na;
  straus_double_scalarmult<false>(out, zero, s, na, btab);
}

template <class BTab>
CMTV_HD void pubkey_from_seed(uint32_t pk[8], const uint32_t seed[8], const BTab& btab) {
  uint32_t a[8], prefix[8];
  expand_seed(a, prefix, seed);
  ge_p3 A;
  scalarmult_base(A, a, btab);
  p3_tobytes(pk, A.X, A.Y, A.Z);
}

template <class BTab>
CMTV_HD void sign_one(uint32_t sig[16], const uint32_t seed[8], const uint8_t* msg, uint32_t mlen,
                      const BTab& btab) {
  uint32_t a[8], prefix[8], pk[8], rh[16], r[8], kh[16], k[8], pre[16];
  expand_seed(a, prefix, seed);
  ge_p3 P;
  scalarmult_base(P, a, btab);
  p3_tobytes(pk, P.X, P.Y, P.Z);
  sha512_prefixed<8>(rh, prefix, msg, mlen);
  sc_reduce512(r, rh);
  scalarmult_base(P, r, btab);
  uint32_t Rw[8];
  p3_tobytes(Rw, P.X, P.Y, P.Z);
#pragma unroll
  for (int i = 0; i < 8; i++) {
    pre[i] = Rw[i];
    pre[8 + i] = pk[i];
  }
  sha512_prefixed<16>(kh, pre, msg, mlen);
  sc_reduce512(k, kh);
  uint32_t s[8];
  sc_muladd(s, k, a, r);
#pragma unroll
  for (int i = 0; i < 8; i++) {
    sig[i] = Rw[i];
    sig[8 + i] = s[i];
  }
}

}  // namespace cmtv
