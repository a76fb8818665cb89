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

// p + q  (q cached). Operands are consumed in an order that lets the T and Z
// inputs die early (register pressure is the occupancy limiter).
CMTV_HD void ge_add_cached(ge_efgh& r, const ge_p3& p, const ge_cached& q) {
  fe t0, t1;
  fe_mul(r.g, p.T, q.T2d);  // C
  fe_mul(r.f, p.Z, q.Z);    // Z1 Z2
  fe_add(r.f, r.f, r.f);
  fe_carry(r.f);            // D = 2 Z1 Z2
  fe_sub(t0, p.Y, p.X);
  fe_mul(t0, t0, q.YmX);    // A
  fe_add(t1, p.Y, p.X);
  fe_mul(t1, t1, q.YpX);    // B
  fe_sub(r.e, t1, t0);      // E = B - A
  fe_add(r.h, t1, t0);      // H = B + A
  fe_add(t0, r.f, r.g);     // G = D + C
  fe_sub(r.f, r.f, r.g);    // F = D - C
  r.g = t0;
}

// p + q (q affine niels, Z2 = 1)
CMTV_HD void ge_add_niels(ge_efgh& r, const ge_p3& p, const ge_niels& q) {
  fe t0, t1;
  fe_mul(r.g, p.T, q.xy2d);  // C
  fe_add(r.f, p.Z, p.Z);
  fe_carry(r.f);             // D = 2 Z1
  fe_sub(t0, p.Y, p.X);
  fe_mul(t0, t0, q.ymx);     // A
  fe_add(t1, p.Y, p.X);
  fe_mul(t1, t1, q.ypx);     // B
  fe_sub(r.e, t1, t0);
  fe_add(r.h, t1, t0);
  fe_add(t0, r.f, r.g);
  fe_sub(r.f, r.f, r.g);
  r.g = t0;
}

// p + q with q = (neg ? -1 : 1) * table[e] (or the identity when ident),
// streamed from a table one coordinate at a time so only one 10-word
// coordinate of the addend is ever live. Tab::load_fe(e, c, fe&) with c in
// {0: Y+X, 1: Y-X, 2: Z, 3: 2dT} (cached, NZ = true) or {0: y+x, 1: y-x,
// 2: 2dxy} (niels, NZ = false, Z2 = 1). Negation swaps the (Y+X, Y-X) reads
// and negates 2dT; both are per-lane selects, not branches.
template <bool NZ, class Tab>
CMTV_HD void ge_add_table(ge_efgh& r, const ge_p3& p, const Tab& tab, int e, bool neg, bool ident) {
  fe q, t0, t1;
  const int cT = NZ ? 3 : 2;
  tab.load_fe(e, cT, q);
  {
    fe qn;
    fe_neg(qn, q);
    fe_select(q, q, qn, neg);
#pragma unroll
    for (int i = 0; i < 10; i++) q.v[i] = ident ? 0u : q.v[i];
  }
  fe_mul(r.g, p.T, q);  // C
  if (NZ) {
    tab.load_fe(e, 2, q);
#pragma unroll
    for (int i = 0; i < 10; i++) q.v[i] = ident ? (i == 0 ? 1u : 0u) : q.v[i];
    fe_mul(r.f, p.Z, q);
    fe_add(r.f, r.f, r.f);
  } else {
    fe_add(r.f, p.Z, p.Z);
  }
  fe_carry(r.f);  // D
  tab.load_fe(e, neg ? 0 : 1, q);
#pragma unroll
  for (int i = 0; i < 10; i++) q.v[i] = ident ? (i == 0 ? 1u : 0u) : q.v[i];
  fe_sub(t0, p.Y, p.X);
  fe_mul(t0, t0, q);  // A
  tab.load_fe(e, neg ? 1 : 0, q);
#pragma unroll
  for (int i = 0; i < 10; i++) q.v[i] = ident ? (i == 0 ? 1u : 0u) : q.v[i];
  fe_add(t1, p.Y, p.X);
  fe_mul(t1, t1, q);  // B
  fe_sub(r.e, t1, t0);
  fe_add(r.h, t1, t0);
  fe_add(t0, r.f, r.g);
  fe_sub(r.f, r.f, r.g);
  r.g = t0;
}

// -q for cached / niels forms: swap (Y+X, Y-X), negate the 2dT term.
// `neg` is a per-lane flag (digit sign), so this is a select, not a branch.
CMTV_HD void cached_cneg(ge_cached& q, bool neg) {
  fe a = q.YpX, t;
  fe_select(q.YpX, q.YpX, q.YmX, neg);
  fe_select(q.YmX, q.YmX, a, neg);
  fe_neg(t, q.T2d);
  fe_select(q.T2d, q.T2d, t, neg);
}

CMTV_HD void niels_cneg(ge_niels& q, bool neg) {
  fe a = q.ypx, t;
  fe_select(q.ypx, q.ypx, q.ymx, neg);
  fe_select(q.ymx, q.ymx, a, neg);
  fe_neg(t, q.xy2d);
  fe_select(q.xy2d, q.xy2d, t, neg);
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
  fe y, u, v, r0, t, one;
  fe_frombytes(y, w);
  fe_1(one);
  fe_sq(t, y);
  fe_sub(u, t, one);  // u = y^2 - 1
  fe_const_d(v);
  fe_mul(v, t, v);
  fe_add(v, v, one);  // v = d y^2 + 1
  fe_sq(t, v);        // v^2
  fe_mul(r0, t, v);   // v^3
  fe_sq(t, t);        // v^4
  fe_mul(r0, u, r0);  // u v^3
  fe_mul(t, r0, t);   // u v^7
  fe_pow22523(t, t);  // (u v^7)^((p-5)/8)
  fe_mul(r0, r0, t);  // r = u v^3 (u v^7)^((p-5)/8)
  fe_sq(t, r0);
  fe_mul(t, t, v);    // check = v r^2
  fe_carry(u);
  const bool correct = fe_equal(t, u);
  fe_neg(v, u);
  const bool flipped = fe_equal(t, v);
  fe_const_sqrtm1(t);
  fe_mul(t, r0, t);
  fe_select(r0, r0, t, flipped);
  // Absolute(): the non-negative (even) root
  fe_neg(t, r0);
  fe_carry(t);
  fe_select(r0, r0, t, fe_isneg(r0));
  // the sign bit selects the negative root (x = 0 stays 0)
  fe_neg(t, r0);
  fe_carry(t);
  fe_select(r0, r0, t, (w[7] >> 31) != 0);
  h.X = r0;
  h.Y = y;
  fe_1(h.Z);
  fe_mul(h.T, r0, y);
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
