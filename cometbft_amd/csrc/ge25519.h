// ge25519.h -- edwards25519 group arithmetic (a = -1 twisted Edwards, extended
// coordinates, HWCD 2008 unified formulas -- complete on this curve, so small-
// order and mixed-order inputs need no special cases).
//
// Representations (all field elements "carried" unless noted):
//   ge_p2     (X:Y:Z)                 x = X/Z, y = Y/Z      (doubling input)
//   ge_p3     (X:Y:Z:T)               + T = XY/Z            (addition input)
//   ge_efgh   (e, f, g, h)            X = ef, Y = gh, Z = fg, T = eh
//                                     (output of dbl/add before the last mults)
//   ge_cached (Y+X, Y-X, Z, 2dT)      second addend, precomputed (Y+X, Y-X uncarried)
//   ge_niels  (y+x, y-x, 2dxy)        affine second addend (fixed-base tables)
//
// Every intermediate respects the fe25519.h operand bounds; the two fe_carry()
// calls per doubling / addition are where an unsigned lazy representation has
// to pay for not using signed limbs.
//
// Restates the group law Go 1.19 crypto/internal/edwards25519 uses underneath
// VarTimeDoubleScalarBaseMult (reference call site
// /root/reference/crypto/ed25519/ed25519.go:154).
#pragma once
#include "fe25519.h"

namespace cmtv {

struct ge_p2 {
  fe X, Y, Z;
};
struct ge_p3 {
  fe X, Y, Z, T;
};
struct ge_efgh {
  fe e, f, g, h;
};
struct ge_cached {
  fe YpX, YmX, Z, T2d;
};
struct ge_niels {
  fe ypx, ymx, xy2d;
};

CMTV_HD void efgh_to_p2(ge_p2& r, const ge_efgh& p) {
  fe_mul(r.X, p.e, p.f);
  fe_mul(r.Y, p.g, p.h);
  fe_mul(r.Z, p.f, p.g);
}

CMTV_HD void efgh_to_p3(ge_p3& r, const ge_efgh& p) {
  fe_mul(r.X, p.e, p.f);
  fe_mul(r.Y, p.g, p.h);
  fe_mul(r.Z, p.f, p.g);
  fe_mul(r.T, p.e, p.h);
}

CMTV_HD void p3_to_p2(ge_p2& r, const ge_p3& p) {
  r.X = p.X;
  r.Y = p.Y;
  r.Z = p.Z;
}

CMTV_HD void p3_identity(ge_p3& p) {
  fe_0(p.X);
  fe_1(p.Y);
  fe_1(p.Z);
  fe_0(p.T);
}

CMTV_HD void p2_identity(ge_p2& p) {
  fe_0(p.X);
  fe_1(p.Y);
  fe_1(p.Z);
}

// dbl-2008-hwcd with a = -1, all four outputs negated (a projective no-op) so
// every operand is a non-negative lazy sum:
//   A = X^2, B = Y^2, K = (X+Y)^2, S = A+B, M = A-B, E' = S-K, F' = 2Z^2 + M
//   X3 = E'F', Y3 = MS, Z3 = F'M, T3 = E'S
CMTV_HD void p2_dbl(ge_efgh& r, const ge_p2& p) {
  fe A, B, K, C;
  fe_sq(A, p.X);
  fe_sq(B, p.Y);
  fe_sq(C, p.Z);
  fe_add(K, p.X, p.Y);
  fe_sq(K, K);
  fe_add(r.h, A, B);   // S
  fe_carry(r.h);
  fe_sub(r.g, A, B);   // M
  fe_sub(r.e, r.h, K); // E'
  fe_add(C, C, C);     // 2Z^2
  fe_add(r.f, C, r.g); // F'
  fe_carry(r.f);
}

// p + q  (q cached). neg = true computes p - q.
CMTV_HD void ge_add_cached(ge_efgh& r, const ge_p3& p, const ge_cached& q, bool neg) {
  fe ymx, ypx, a, b, c, d2;
  fe_sub(ymx, p.Y, p.X);
  fe_add(ypx, p.Y, p.X);
  fe qa, qb;
  fe_select(qa, q.YmX, q.YpX, neg);
  fe_select(qb, q.YpX, q.YmX, neg);
  fe_mul(a, ymx, qa);
  fe_mul(b, ypx, qb);
  fe_mul(c, p.T, q.T2d);
  fe_mul(d2, p.Z, q.Z);
  fe_add(d2, d2, d2);
  fe_carry(d2);
  fe_sub(r.e, b, a);  // E = B - A
  fe_add(r.h, b, a);  // H = B + A
  fe F, G;
  fe_sub(F, d2, c);   // D - C
  fe_add(G, d2, c);   // D + C
  fe_select(r.f, F, G, neg);
  fe_select(r.g, G, F, neg);
}

// p + q (q affine niels). neg = true computes p - q.
CMTV_HD void ge_add_niels(ge_efgh& r, const ge_p3& p, const ge_niels& q, bool neg) {
  fe ymx, ypx, a, b, c, d2;
  fe_sub(ymx, p.Y, p.X);
  fe_add(ypx, p.Y, p.X);
  fe qa, qb;
  fe_select(qa, q.ymx, q.ypx, neg);
  fe_select(qb, q.ypx, q.ymx, neg);
  fe_mul(a, ymx, qa);
  fe_mul(b, ypx, qb);
  fe_mul(c, p.T, q.xy2d);
  fe_add(d2, p.Z, p.Z);
  fe_carry(d2);
  fe_sub(r.e, b, a);
  fe_add(r.h, b, a);
  fe F, G;
  fe_sub(F, d2, c);
  fe_add(G, d2, c);
  fe_select(r.f, F, G, neg);
  fe_select(r.g, G, F, neg);
}

CMTV_HD void p3_to_cached(ge_cached& r, const ge_p3& p) {
  fe d2;
  fe_const_d2(d2);
  fe_add(r.YpX, p.Y, p.X);
  fe_sub(r.YmX, p.Y, p.X);
  r.Z = p.Z;
  fe_mul(r.T2d, p.T, d2);
}

CMTV_HD void cached_identity(ge_cached& r) {
  fe_1(r.YpX);
  fe_1(r.YmX);
  fe_1(r.Z);
  fe_0(r.T2d);
}

CMTV_HD void niels_identity(ge_niels& r) {
  fe_1(r.ypx);
  fe_1(r.ymx);
  fe_0(r.xy2d);
}

// Go 1.19 Point.SetBytes: y = low 255 bits (non-canonical y accepted, taken
// mod p), x = sqrt((y^2-1)/(dy^2+1)) via SqrtRatio, non-negative root, negated
// when the sign bit is set (x = 0 with the sign bit set is accepted).
// Returns false when no square root exists.
CMTV_HD bool p3_frombytes(ge_p3& h, const uint32_t w[8]) {
  fe y, y2, u, v, v3, v7, t, r, check, one, d;
  fe_frombytes(y, w);
  fe_1(one);
  fe_const_d(d);
  fe_sq(y2, y);
  fe_sub(u, y2, one);     // u = y^2 - 1
  fe_mul(v, y2, d);
  fe_add(v, v, one);      // v = d y^2 + 1
  fe_sq(v3, v);
  fe_mul(v3, v3, v);      // v^3
  fe_sq(v7, v3);
  fe_mul(v7, v7, v);      // v^7
  fe_mul(t, u, v7);
  fe_pow22523(t, t);      // (u v^7)^((p-5)/8)
  fe_mul(r, u, v3);
  fe_mul(r, r, t);        // r = u v^3 (u v^7)^((p-5)/8)
  fe_sq(check, r);
  fe_mul(check, check, v);  // v r^2
  fe uc = u;
  fe_carry(uc);
  fe uneg;
  fe_neg(uneg, uc);
  const bool correct = fe_equal(check, uc);
  const bool flipped = fe_equal(check, uneg);
  fe sqm1, r2;
  fe_const_sqrtm1(sqm1);
  fe_mul(r2, r, sqm1);
  fe_select(r, r, r2, flipped);
  // Absolute(): the non-negative (even) root
  fe rn;
  fe_neg(rn, r);
  fe_carry(rn);
  fe_select(r, r, rn, fe_isneg(r));
  // sign bit selects the negative root
  fe_neg(rn, r);
  fe_carry(rn);
  fe_select(r, r, rn, (w[7] >> 31) != 0);
  h.X = r;
  h.Y = y;
  fe_1(h.Z);
  fe_mul(h.T, r, y);
  return correct || flipped;
}

// canonical encoding as 8 little-endian words (Go Point.Bytes)
CMTV_HD void p3_tobytes(uint32_t s[8], const fe& X, const fe& Y, const fe& Z) {
  fe zi, x, y;
  fe_invert(zi, Z);
  fe_mul(x, X, zi);
  fe_mul(y, Y, zi);
  fe_tobytes(s, y);
  s[7] |= (uint32_t)fe_isneg(x) << 31;
}

}  // namespace cmtv
