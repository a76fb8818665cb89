// row.h -- one signature per wavefront ("row" layout) for latency-bound
// batches: a field element of GF(2^255-19) lives in one 16-lane DPP row, in
// radix 2^16 (lane k of the row holds limb k), and the four rows of a wave
// hold the four extended coordinates (X, Y, Z, T) of a point.
//
// Why: at 150 signatures the chip has ~7 SIMDs per signature and the oct and
// quad kernels are bound by one lane's chain of field products (DESIGN.md
// 4.3: ~4.4 cycles per VALU instruction, one wave per SIMD). Here one product
// is 16 column terms per lane -- a DPP row_ror:r of f (lane k gets f_{k-r}), a
// DPP row_newbcast:r of g (every lane gets g_r), a 24-bit twist (x 38 where
// the column wraps past 2^256) and a v_mad_u64_u32 -- plus three carry rounds
// whose carries move by row_ror:1: 76 VALU instructions for all four
// coordinates' products, against 107 (squaring) / 130 (product) per lane in
// the quad layout; every add, subtract and select is one instruction per
// lane instead of ten; and the cross-coordinate moves of the point formulas
// are v_permlane16/32_swap row exchanges.
//
// Column k of h = f g mod p (2^256 = 38 mod p):
//   h_k = sum_r f_{(k-r) mod 16} g_r  (x 38 when r > k)
// Bounds (asserted by tests/host/rowcheck.cpp): multiplication inputs below
// 2^19.37 per limb (the first carry of a column then fits 32 bits); products
// leave limbs below 2^16 + 2^7 ("carried"); subtraction adds 4p (limbs of
// 4p are >= 0x1FFFC, above any carried limb).
//
// Everything is written against a row policy R:
//   R::U / R::U64 / R::B     this lane's u32 / u64 / bool (the host test
//                            policy: 64-lane arrays, tests/host/rowcheck.cpp)
//   R::lane()                0..63
//   R::ror<r>(x)             lane k of a row gets lane (k - r) mod 16 of it
//   R::bcast<r>(x)           every lane of a row gets lane r of it
//   R::rows(x, b0..b3)       b_c = row c of x broadcast to all four rows
//   R::ballot(b)             64-bit mask of b over the wave
// with free functions mad64(a, b, c) = a b + c (u64), lo32, shr64(x, s) (low
// word of x >> s), mul24, sel(c, a, b). Control flow is wave-uniform.
#pragma once
#include "keyed.h"
#include "quad.h"

namespace cmtv {

// the lane-vector primitives on one lane's scalars (the device policy; the
// host test policy overloads them for 64-lane arrays)
CMTV_HD uint64_t widen(uint32_t a) { return a; }
CMTV_HD uint64_t mad64(uint32_t a, uint32_t b, uint64_t c) { return (uint64_t)a * b + c; }
CMTV_HD uint32_t lo32(uint64_t a) { return (uint32_t)a; }
CMTV_HD uint32_t shr64(uint64_t a, int s) { return (uint32_t)(a >> s); }
// the high word of a product's column sum (the host policy asserts the sum
// is below 2^48, so the word is below 2^16)
CMTV_HD uint32_t hi32(uint64_t a) { return (uint32_t)(a >> 32); }
// a b for a, b < 2^24: v_mul_u32_u24 (full rate; v_mul_lo_u32 is quarter rate)
CMTV_HD uint32_t mul24(uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __umul24(a, b);
#else
  return a * b;
#endif
}
template <class T>
CMTV_HD T sel(bool c, const T& a, const T& b) {
  return c ? a : b;
}

// 16-bit limbs of the curve constants
struct RowConst {
  static constexpr uint16_t d[16] = {0x78a3, 0x1359, 0x4dca, 0x75eb, 0xd8ab, 0x4141, 0x0a4d, 0x0070,
                                     0xe898, 0x7779, 0x4079, 0x8cc7, 0xfe73, 0x2b6f, 0x6cee, 0x5203};
  static constexpr uint16_t d2[16] = {0xf159, 0x26b2, 0x9b94, 0xebd6, 0xb156, 0x8283, 0x149a, 0x00e0,
                                      0xd130, 0xeef3, 0x80f2, 0x198e, 0xfce7, 0x56df, 0xd9dc, 0x2406};
  static constexpr uint16_t sqrtm1[16] = {0xa0b0, 0x4a0e, 0x1b27, 0xc4ee, 0xe478, 0xad2f, 0x1806, 0x2f43,
                                          0xd7a7, 0x3dfb, 0x0099, 0x2b4d, 0xdf0b, 0x4fc1, 0x2480, 0x2b83};
};

// Per-lane constants of a wave, computed once (loop-invariant vectors).
template <class R>
struct RowCtx {
  using U = typename R::U;
  using B = typename R::B;
  U k;        // limb index (lane & 15)
  U c;        // row index (lane >> 4)
  U bias;     // limb k of 4p
  U m38;      // 38 on limb 0 (the carry out of limb 15 wraps as x 38), else 1
  U m38x2;    // 38 on limbs 0 and 1 (the second carry out of limbs 14, 15 wraps), else 1
  U one;      // the constant 1 (limb 0)
  U tw[16];   // column twist of term r: 38 where limb k < r (the column wraps past 2^256), else 1
  U tw4[4];   // split products (rf_mul_s): the twists of terms 4c + j (four rows share a product)
  U tw8[8];   // ... of terms 8 (c >> 1) + j (rows c and c ^ 2 share one)
  B r0, r1, r2, r3;
  CMTV_HD explicit RowCtx(const U& lane) {
    k = lane & 15u;
#pragma unroll
    for (int r = 0; r < 16; r++) tw[r] = sel(k < (uint32_t)r, U(38u), U(1u));
    c = lane >> 4;
#pragma unroll
    for (int j = 0; j < 4; j++) tw4[j] = sel(k < (c << 2) + (uint32_t)j, U(38u), U(1u));
#pragma unroll
    for (int j = 0; j < 8; j++) tw8[j] = sel(k < ((c >> 1) << 3) + (uint32_t)j, U(38u), U(1u));
    bias = sel(k == 0u, U(4u * 0xFFEDu), sel(k == 15u, U(4u * 0x7FFFu), U(4u * 0xFFFFu)));
    m38 = sel(k == 0u, U(38u), U(1u));
    m38x2 = sel(k < 2u, U(38u), U(1u));
    one = sel(k == 0u, U(1u), U(0u));
    r0 = c == 0u;
    r1 = c == 1u;
    r2 = c == 2u;
    r3 = c == 3u;
  }
  CMTV_HD U cst(const uint16_t* tab) const { return R::load_const(tab, k); }
};

// ---- the product -------------------------------------------------------------

// The column sums (< 2^48) to limbs below 2^16 + 2^7: each sum is cut into
// three 16-bit pieces at once, piece j moving j limbs up (row_ror:j, x 38
// where it wraps past limb 15), so limb k collects c0_k + c1_{k-1} + c2_{k-2}
// (< 2^22.3), then one ordinary round. 10 VALU instructions, 4 dependent
// steps to the first sum instead of three chained rounds.
template <class R>
CMTV_HD typename R::U rf_carry64(const RowCtx<R>& x, const typename R::U64& c) {
  using U = typename R::U;
  const U l = lo32(c);
  const U c1 = R::template ror<1>(l >> 16);
  const U c2 = R::template ror<2>(hi32(c));
  U w = mul24(c1, x.m38) + (l & 0xFFFFu);
  w = mul24(c2, x.m38x2) + w;
  const U ca = R::template ror<1>(w >> 16);
  return mul24(ca, x.m38) + (w & 0xFFFFu);
}

// the same on 32-bit limbs below 2^26 (sums of a few carried values)
template <class R>
CMTV_HD typename R::U rf_carry32(const RowCtx<R>& x, const typename R::U& w0) {
  using U = typename R::U;
  U lo = w0 & 0xFFFFu;
  U ca = R::template ror<1>(w0 >> 16);
  U w = mul24(ca, x.m38) + lo;
  lo = w & 0xFFFFu;
  ca = R::template ror<1>(w >> 16);
  return mul24(ca, x.m38) + lo;
}

template <class R, int r>
CMTV_HD void rf_terms(const RowCtx<R>& x, typename R::U64& acc, const typename R::U& f, const typename R::U& g) {
  if constexpr (r < 16) {
    using U = typename R::U;
    const U fr = R::template ror<r>(f);
    const U gb = R::template bcast<r>(g);
    acc = mad64(fr, mul24(gb, x.tw[r]), acc);
    rf_terms<R, r + 1>(x, acc, f, g);
  }
}

// h = f g (each row its own product). A policy with kFusedProduct supplies
// the 15 twisted broadcasts itself (DevRow: v_mul_u32_u24_dpp row_newbcast,
// the broadcast and the twist in one instruction).
template <class R>
CMTV_HD typename R::U rf_mul(const RowCtx<R>& x, const typename R::U& f, const typename R::U& g) {
  if constexpr (R::kFusedProduct) {
    return rf_carry64(x, R::product(x.tw, f, g));
  } else {
    typename R::U64 acc = mad64(f, R::template bcast<0>(g), widen(typename R::U(0u)));
    rf_terms<R, 1>(x, acc, f, g);
    return rf_carry64(x, acc);
  }
}

template <class R>
CMTV_HD typename R::U rf_sq(const RowCtx<R>& x, const typename R::U& f) {
  return rf_mul(x, f, f);
}

template <class R>
CMTV_HD typename R::U rf_sqn(const RowCtx<R>& x, typename R::U f, int n) {
#pragma unroll 1
  for (int i = 0; i < n; i++) f = rf_sq(x, f);
  return f;
}

template <int S, class R, int j>
CMTV_HD void rf_split_rest(const typename R::U* tws, typename R::U64& acc, const typename R::U& F,
                           const typename R::U& G) {
  if constexpr (j < 16 / S) {
    acc = mad64(R::template ror<j>(F), mul24(R::template bcast<j>(G), tws[j]), acc);
    rf_split_rest<S, R, j + 1>(tws, acc, F, G);
  }
}

// ---- split products ----------------------------------------------------------
//
// A chain of products whose operands are the same on S rows (the decode's
// square-root chain: one point on all four rows, or A and R on rows {0, 2}
// and {1, 3}) shares each product among those rows: row c takes the 16/S
// terms r = (16/S) q + j, q its place in the group (c for S = 4, c >> 1 for
// S = 2), on operands rotated by (16/S) q beforehand -- F = f row_ror:(16/S)q,
// G = g rotated the other way, so that row_ror:j of F is f_{k-r} and
// row_newbcast:j of G is g_r -- and the partial column sums are added across
// the group (v_permlane32_swap / v_permlane16_swap). Per product: 4 (S = 2:
// 8) terms instead of 16, for 6 (2) rotations and 2 (1) cross-row 64-bit
// sums. The chain is latency-bound, not issue-bound: measured (row_pt), the
// decode takes 72k cycles with S = 2, 79k with S = 4 (its rotations and sums
// are deeper dependent chains), 83k unsplit -- so every decode uses S = 2,
// which needs only rows c and c ^ 2 to agree.
template <int S, class R>
CMTV_HD typename R::U64 rf_split_terms(const typename R::U* tws, const typename R::U& F, const typename R::U& G) {
  if constexpr (R::kFusedProduct) {
    return R::template product_split<S>(tws, F, G);
  } else {
    typename R::U64 acc = mad64(F, mul24(R::template bcast<0>(G), tws[0]), widen(typename R::U(0u)));
    rf_split_rest<S, R, 1>(tws, acc, F, G);
    return acc;
  }
}

template <int S, class R>
CMTV_HD typename R::U rf_mul_s(const RowCtx<R>& x, const typename R::U& f, const typename R::U& g) {
  if constexpr (S == 1) {
    return rf_mul(x, f, g);
  } else {
    using U = typename R::U;
    static_assert(S == 2 || S == 4, "rows per product: 1, 2 or 4");
    const U F = S == 4 ? R::template ror_rows<4, 8, 12>(f) : R::template ror_rows<0, 8, 8>(f);
    const U G = S == 4 ? R::template ror_rows<12, 8, 4>(g) : R::template ror_rows<0, 8, 8>(g);
    return rf_carry64(x, R::template sum_rows<S>(rf_split_terms<S, R>(S == 4 ? x.tw4 : x.tw8, F, G)));
  }
}

template <int S, class R>
CMTV_HD typename R::U rf_sq_s(const RowCtx<R>& x, const typename R::U& f) {
  return rf_mul_s<S>(x, f, f);
}

template <int S, class R>
CMTV_HD typename R::U rf_sqn_s(const RowCtx<R>& x, typename R::U f, int n) {
#pragma unroll 1
  for (int i = 0; i < n; i++) f = rf_sq_s<S>(x, f);
  return f;
}

// a - b + 4p (b carried); -a
template <class R>
CMTV_HD typename R::U rf_sub(const RowCtx<R>& x, const typename R::U& a, const typename R::U& b) {
  return a + (x.bias - b);
}
template <class R>
CMTV_HD typename R::U rf_neg(const RowCtx<R>& x, const typename R::U& a) {
  return x.bias - a;
}

// ---- canonical tests -----------------------------------------------------------

// Whether the row's value is 0 mod p, and the parity of its canonical
// representative (Go's IsNegative). Every lane of the row gathers the 16
// limbs (row_newbcast) and normalises them serially; the result is uniform
// within a row. Limbs may be any value below 2^26.
template <class R>
struct RowCanon {
  typename R::B zero, odd;
};

template <class R, int r>
CMTV_HD void rf_gather(typename R::U* l, const typename R::U& f) {
  if constexpr (r < 16) {
    l[r] = R::template bcast<r>(f);
    rf_gather<R, r + 1>(l, f);
  }
}

template <class R>
CMTV_HD void rf_ripple(typename R::U* l, typename R::U& c) {
#pragma unroll
  for (int i = 0; i < 16; i++) {
    const typename R::U t = l[i] + c;
    l[i] = t & 0xFFFFu;
    c = t >> 16;
  }
}

template <class R>
CMTV_HD RowCanon<R> rf_canon(const typename R::U& f) {
  using U = typename R::U;
  U l[16];
  rf_gather<R, 0>(l, f);
  U c(0u);
  rf_ripple<R>(l, c);  // limbs < 2^16, carry out < 2^11
#pragma unroll 1
  for (int pass = 0; pass < 2; pass++) {
    l[0] = l[0] + c * 38u;
    c = U(0u);
    rf_ripple<R>(l, c);
  }
  // value V < 2^256; fold bit 255: V' = V mod 2^255 + 19 (V >> 255) < 2^255 + 19
  const U h = l[15] >> 15;
  l[15] = l[15] & 0x7FFFu;
  c = h * 19u;
  rf_ripple<R>(l, c);  // no carry out: V' < 2^255 + 19
  // V' >= p  <=>  V' + 19 >= 2^255
  U w[16];
#pragma unroll
  for (int i = 0; i < 16; i++) w[i] = l[i];
  c = U(19u);
  rf_ripple<R>(w, c);
  const typename R::B ge = (w[15] >> 15) != 0u;
  U acc(0u);
#pragma unroll
  for (int i = 0; i < 16; i++) acc = acc | sel(ge, i == 15 ? (w[i] & 0x7FFFu) : w[i], l[i]);
  RowCanon<R> out;
  out.zero = acc == 0u;
  out.odd = (sel(ge, w[0], l[0]) & 1u) != 0u;
  return out;
}

// ---- points: four rows = (X, Y, Z, T) ---------------------------------------------

// Doubling (quad.h q_dbl with rows for lanes): round 1 squares {X, Y, Z, X+Y},
// round 2 multiplies each row's U = {F', S, M, E'} by the row {E', M, F', S}.
template <class R>
CMTV_HD void rp_dbl(const RowCtx<R>& x, typename R::U& v) {
  using U = typename R::U;
  const U m3 = sel(x.r3, U(~0u), U(0u));
  const U sh = sel(x.r0, U(1u), U(0u));
  const U n2 = sel(x.r1 || x.r3, U(0u), U(~0u));
  const U n3 = m3;
  const U mo = sel(x.r0 || x.r3, U(~0u), U(0u));
  const U corr = sel(x.r1, U(0u), U(1u));
  U b0, b1, b2, b3;
  R::rows(v, b0, b1, b2, b3);
  U m = sel(x.r3, b0, v) + (b1 & m3);  // X, Y, Z, X + Y
  m = rf_sq(x, m);                     // A, B, C', K
  R::rows(m, b0, b1, b2, b3);
  const U a = sel(x.r0, b2, b0);       // C', A, A, A
  // F' = 2C' + A - B, S = A + B, M = A - B, E' = A + B - K (+ 4p)
  m = (a << sh) + (b1 ^ n2) + ((m ^ n3) & mo) + corr + x.bias;
  R::rows(m, b0, b1, b2, b3);
  const U pr = sel(x.r0, b3, sel(x.r1, b2, sel(x.r2, b0, b1)));  // E', M, F', S
  v = rf_mul(x, m, pr);
}

// v += Q, c = this row's coordinate of Q in cached form (Y-X, Y+X, 2Z, 2dT)
// (quad.h q_add with rows for lanes)
template <class R>
CMTV_HD void rp_add(const RowCtx<R>& x, typename R::U& v, const typename R::U& c) {
  using U = typename R::U;
  const U m0 = sel(x.r0, U(~0u), U(0u));
  const U m01 = sel(x.r0 || x.r1, U(~0u), U(0u));
  const U m23 = sel(x.r2 || x.r3, U(~0u), U(0u));
  U b0, b1, b2, b3;
  R::rows(v, b0, b1, b2, b3);
  const U y = sel(x.r0, b1, sel(x.r1, b0, v));  // Y, X, Z, T
  U p = v + ((y ^ m0) & m01) + sel(x.r0, x.bias + 1u, U(0u));  // X - Y, Y + X, Z, T
  const U t = rf_mul(x, p, c);                                  // -A, B, D, C
  R::rows(t, b0, b1, b2, b3);
  const typename R::B e03 = x.r0 || x.r3;
  const U xx = sel(e03, b1, b2);  // B, D, D, B
  const U yy = sel(e03, b0, b3);  // -A, C, C, -A
  p = xx + (yy ^ m23) + sel(x.r2 || x.r3, x.bias + 1u, U(0u));  // E, G, F, H
  R::rows(p, b0, b1, b2, b3);
  const U pr = sel(x.r0, b2, sel(x.r1, b3, sel(x.r2, b1, b0)));  // F, H, G, E
  v = rf_mul(x, p, pr);
}

// this row's cached coordinate (Y-X, Y+X, 2Z, 2dT) of the extended point v
template <class R>
CMTV_HD typename R::U rp_to_cached(const RowCtx<R>& x, const typename R::U& v, const typename R::U& d2) {
  using U = typename R::U;
  U b0, b1, b2, b3;
  R::rows(v, b0, b1, b2, b3);
  const U dt = rf_mul(x, v, d2);  // row 3: 2dT
  return sel(x.r0, rf_sub(x, b1, b0), sel(x.r1, b1 + b0, sel(x.r2, v + v, dt)));
}

// the negated cached point: (Y+X, Y-X, 2Z, -2dT)
template <class R>
CMTV_HD typename R::U rp_cached_neg(const RowCtx<R>& x, const typename R::U& c) {
  using U = typename R::U;
  U b0, b1, b2, b3;
  R::rows(c, b0, b1, b2, b3);
  return sel(x.r0, b1, sel(x.r1, b0, sel(x.r3, rf_sub(x, U(0u), rf_carry32(x, c)), c)));
}

// the identity (0, 1, 1, 0) and its cached form (1, 1, 2, 0)
template <class R>
CMTV_HD typename R::U rp_identity(const RowCtx<R>& x) {
  using U = typename R::U;
  return sel((x.r1 || x.r2) && (x.k == 0u), U(1u), U(0u));
}
template <class R>
CMTV_HD typename R::U rp_cached_identity(const RowCtx<R>& x) {
  using U = typename R::U;
  return sel(x.k == 0u, sel(x.r2, U(2u), sel(x.r3, U(0u), U(1u))), U(0u));
}

// ---- decompression --------------------------------------------------------------

// Go 1.19 Point.SetBytes (ge25519.h p3_frombytes) on every row at once: y =
// the row's limbs (bit 255 already cleared, non-canonical y taken mod p), sign
// = its sign bit. Returns the decode flag; xo, to = x and x y (carried).
struct RowNoHook {
  CMTV_HD void operator()() const {}
};
// mid(): called once inside the square-root chain, MID_AT squarings into
// its run of 100 after 2^100 - 1 (~112 + MID_AT of the decode's ~265
// products): the keyed row kernel's R wave meets the workgroup barrier there
// S: rows sharing each product (rf_mul_s): 4 when y is the same on every
// row, 2 when rows c and c ^ 2 hold the same y (A on rows 0, 2, R on 1, 3)
template <int MID_AT = 0, int S = 1, class R, class Mid = RowNoHook>
CMTV_HD typename R::B rf_decode(const RowCtx<R>& x, const typename R::U& y, const typename R::B& sign,
                                typename R::U& xo, typename R::U& to, const Mid& mid = Mid()) {
  using U = typename R::U;
  const U y2 = rf_sq_s<S>(x, y);
  const U u = rf_carry32(x, rf_sub(x, y2, x.one));                     // y^2 - 1
  const U v = rf_carry32(x, rf_mul_s<S>(x, y2, x.cst(RowConst::d)) + x.one);  // d y^2 + 1
  U t = rf_sq_s<S>(x, v);                  // v^2
  U r0 = rf_mul_s<S>(x, t, v);             // v^3
  t = rf_sq_s<S>(x, t);                    // v^4
  r0 = rf_mul_s<S>(x, u, r0);              // u v^3
  t = rf_mul_s<S>(x, r0, t);               // u v^7
  // (u v^7)^((p-5)/8) (fe25519.h fe_pow22523)
  {
    const U z = t;
    U t0, t1, t2, z2, z9, z11;
    z2 = rf_sq_s<S>(x, z);
    t0 = rf_sqn_s<S>(x, z2, 2);
    z9 = rf_mul_s<S>(x, t0, z);
    z11 = rf_mul_s<S>(x, z9, z2);
    t0 = rf_mul_s<S>(x, rf_sq_s<S>(x, z11), z9);  // 2^5 - 1
    t1 = rf_sqn_s<S>(x, t0, 5);
    t0 = rf_mul_s<S>(x, t1, t0);             // 2^10 - 1
    t1 = rf_sqn_s<S>(x, t0, 10);
    t1 = rf_mul_s<S>(x, t1, t0);             // 2^20 - 1
    t2 = rf_sqn_s<S>(x, t1, 20);
    t1 = rf_mul_s<S>(x, t2, t1);             // 2^40 - 1
    t1 = rf_sqn_s<S>(x, t1, 10);
    t0 = rf_mul_s<S>(x, t1, t0);             // 2^50 - 1
    t1 = rf_sqn_s<S>(x, t0, 50);
    t1 = rf_mul_s<S>(x, t1, t0);             // 2^100 - 1
    t2 = rf_sqn_s<S>(x, t1, MID_AT);
    mid();
    t2 = rf_sqn_s<S>(x, t2, 100 - MID_AT);
    t1 = rf_mul_s<S>(x, t2, t1);             // 2^200 - 1
    t1 = rf_sqn_s<S>(x, t1, 50);
    t1 = rf_mul_s<S>(x, t1, t0);             // 2^250 - 1
    t1 = rf_sqn_s<S>(x, t1, 2);
    t = rf_mul_s<S>(x, t1, z);               // (p-5)/8
  }
  r0 = rf_mul_s<S>(x, r0, t);          // r = u v^3 (u v^7)^((p-5)/8)
  t = rf_mul_s<S>(x, rf_sq_s<S>(x, r0), v);  // v r^2
  const RowCanon<R> correct = rf_canon<R>(rf_sub(x, t, u));
  const RowCanon<R> flipped = rf_canon<R>(t + u);
  r0 = sel(flipped.zero, rf_mul_s<S>(x, r0, x.cst(RowConst::sqrtm1)), r0);
  // Absolute(): the even root; then the sign bit picks the negative one
  const RowCanon<R> rc = rf_canon<R>(r0);
  const typename R::B neg = rc.odd != sign;
  r0 = sel(neg, rf_carry32(x, rf_neg(x, r0)), r0);
  xo = r0;
  to = rf_mul_s<S>(x, r0, y);
  return correct.zero || flipped.zero;
}

// ---- verification ------------------------------------------------------------------

// Table policy: (0..8)P and (0..8)(-P) in cached form, one u32 per lane per
// entry (LDS on the device):
//   void store(int tbl, int neg, int e, const U& c);  U load(int tbl, int neg, int e) const;

// (0..8)P and (0..8)(-P) in cached form into table tb, P extended (clobbers
// nothing: v is copied)
template <class R, class Tab>
CMTV_HD void r_build_table(const RowCtx<R>& x, Tab& tab, int tb, const typename R::U& p) {
  using U = typename R::U;
  const U d2 = x.cst(RowConst::d2);
  U v = rf_carry32(x, p);
  const U ci = rp_cached_identity(x);
  tab.store(tb, 0, 0, ci);
  tab.store(tb, 1, 0, ci);
  const U c1 = rp_to_cached(x, v, d2);
  tab.store(tb, 0, 1, c1);
  tab.store(tb, 1, 1, rp_cached_neg(x, c1));
  rp_dbl(x, v);
  U c = rp_to_cached(x, v, d2);
  tab.store(tb, 0, 2, c);
  tab.store(tb, 1, 2, rp_cached_neg(x, c));
#pragma unroll 1
  for (int e = 3; e <= 8; e++) {
    rp_add(x, v, c1);
    c = rp_to_cached(x, v, d2);
    tab.store(tb, 0, e, c);
    tab.store(tb, 1, e, rp_cached_neg(x, c));
  }
}

// the window count of a prepared pair (quad.h q_wave_windows for one signature)
CMTV_HD int r_windows(uint32_t flags) {
  const int W = (int)((flags >> 8) & 0xFFu);
  return (flags & 2u) ? HS_WIDE_WINDOWS : (W < HS_WINDOWS ? HS_WINDOWS : (W > HS_MAX_WINDOWS ? HS_MAX_WINDOWS : W));
}

// The final check on X (this row's coordinate): X = O (GO_STDLIB, with R
// canonical: encode(R') == R bytes) / [8]X = O (ZIP215: T = 0 or
// X^2 + Y^2 = 0, quad.h q_small_order). ok: the s, A and R checks.
template <uint32_t MODE, class R>
CMTV_HD bool r_final(const RowCtx<R>& x, const typename R::U& v, bool ok, bool r_canon) {
  using U = typename R::U;
  if (MODE == MODE_ZIP215) {
    const U s = rf_sq(x, v);
    U s0, s1, s2, s3;
    R::rows(s, s0, s1, s2, s3);
    const uint64_t zt = R::ballot(rf_canon<R>(sel(x.r3, v, s0 + s1)).zero);
    const bool so = ((zt >> 48) & 1u) != 0 || (zt & 1u) != 0;
    return ok && so;
  }
  U v0, v1, v2, v3;
  R::rows(v, v0, v1, v2, v3);
  const uint64_t z = R::ballot(rf_canon<R>(sel(x.r0, v, rf_sub(x, v1, v2))).zero);
  const bool e0 = (z & 1u) != 0, e1 = ((z >> 16) & 1u) != 0;
  return ok && r_canon && e0 && e1;
}

// The sum over the lowest `lo` windows (all of them when lo >= W) of the
// one-wave form: decode A (rows 0, 2) and R (rows 1, 3) at once, their tables,
// then the Straus windows with one A and one R addition each. Out: the
// scalars (p) and the checks of A and R.
template <class R, class Tab, class GetPrep>
CMTV_HD typename R::U r_sum_ar(const RowCtx<R>& x, const typename R::U& limb, const uint32_t pkw[8],
                               const uint32_t sigw[8], Tab& tab, const GetPrep& get_prep, int lo, SigPrep& p,
                               bool& a_ok, bool& r_ok, bool& r_canon) {
  using U = typename R::U;
  using B = typename R::B;
  // ---- phase 1: decode A (rows 0, 2) and R (rows 1, 3) at once
  const B is_r = (x.c & 1u) != 0u;
  const bool a_sign = (pkw[7] >> 31) != 0, r_sign = (sigw[7] >> 31) != 0;
  const U y = sel(x.k == 15u, limb & 0x7FFFu, limb);
  U xo, to;
  const B dec = rf_decode<0, 2>(x, y, sel(is_r, B(r_sign), B(a_sign)), xo, to);
  const uint64_t decm = R::ballot(dec);
  a_ok = (decm & 1u) != 0;
  r_ok = ((decm >> 16) & 1u) != 0;  // lane 0 of rows 0 and 1
  const uint64_t x0m = R::ballot(rf_canon<R>(xo).zero);
  r_canon = y_is_canonical(sigw) && !(((x0m >> 16) & 1u) != 0 && r_sign);
  // -A = (-x, y, 1, -x y) and -R, extended, one coordinate per row
  U X0, X1, X2, X3, Y0, Y1, Y2, Y3, T0, T1, T2, T3;
  R::rows(xo, X0, X1, X2, X3);
  R::rows(y, Y0, Y1, Y2, Y3);
  R::rows(to, T0, T1, T2, T3);
  const U na = sel(x.r0, rf_neg(x, X0), sel(x.r1, Y0, sel(x.r2, x.one, rf_neg(x, T0))));
  const U nr = sel(x.r0, rf_neg(x, X1), sel(x.r1, Y1, sel(x.r2, x.one, rf_neg(x, T1))));
  // ---- phase 2 (before the scalars): (0..8)(-A) and (0..8)(-R), both signs
  r_build_table(x, tab, 0, na);
  r_build_table(x, tab, 1, nr);
  // ---- phase 3: Straus over the low windows of k1 (A) and k2 (R)
  get_prep(p);
  const bool r_flip = (p.flags & 1u) != 0;  // k2 < 0: R's digits flip (its table is of -R)
  const int W = r_windows(p.flags);
  const int L = lo < W ? lo : W;
  uint32_t tA[8], tR[8];
  hs_digits16(tA, p.k1, W);
  hs_digits16(tR, p.k2, W);
#pragma unroll 1
  for (int w = W; w > L; w--) {
    sc_shift_out(tA, 4);
    sc_shift_out(tR, 4);
  }
  U v = rp_identity(x);
#pragma unroll 1
  for (int win = L - 1; win >= 0; win--) {
    const int dA = (int)sc_shift_out(tA, 4) - 8;
    const int dR = (int)sc_shift_out(tR, 4) - 8;
    const U cA = tab.load(0, dA < 0 ? 1 : 0, dA < 0 ? -dA : dA);
    const U cR = tab.load(1, (dR < 0) != r_flip ? 1 : 0, dR < 0 ? -dR : dR);
    if (win != L - 1) {
#pragma unroll 1
      for (int d = 0; d < 4; d++) rp_dbl(x, v);
    }
    rp_add(x, v, cA);
    rp_add(x, v, cR);
  }
  return v;
}

// X = [u]B + [k1](-A) + [|k2|](k2 < 0 ? R : -R) = [k2](R' - R) (quad.h
// q_straus_prep_b<EXT_B, PREBUILT>) and the final check of the mode, one
// signature per wave. limb: this lane's 16-bit limb of A / R (row c & 1:
// 0 = A, 1 = R), pkw / sigw: the 8 words of A / R (uniform). get_prep(SigPrep&)
// supplies the helper's scalars, get_b() this row's cached coordinate of [u]B.
template <uint32_t MODE, class R, class Tab, class GetPrep, class GetB>
CMTV_HD bool r_verify_split(const R&, const typename R::U& limb, const uint32_t pkw[8], const uint32_t sigw[8],
                            Tab& tab, const GetPrep& get_prep, const GetB& get_b) {
  const RowCtx<R> x(R::lane());
  SigPrep p;
  bool a_ok, r_ok, r_canon;
  typename R::U v = r_sum_ar(x, limb, pkw, sigw, tab, get_prep, 1 << 20, p, a_ok, r_ok, r_canon);
  rp_add(x, v, get_b());
  return r_final<MODE>(x, v, (p.flags & 4u) != 0 && a_ok && r_ok, r_canon);
}


// The two-wave form (k_verify_row2_split, one signature per CU): wave PART
// = 0 takes A, PART = 1 takes R. Each decodes its point on every row, builds
// (0..8)(-P) (both signs), and after get_prep runs W windows of 4 doublings
// and ONE addition -- [k1](-A), or [|k2|](k2 < 0 ? R : -R) -- instead of the
// one-wave form's two additions per window. Returns this row's coordinate
// of the part's sum; dec / x0 are P's decode flag and whether its x is 0.
struct RowNoStamp {
  CMTV_HD void operator()(int) const {}
};
// windows the four-wave form leaves to its lo wave (72 bits: W >= 33, so the
// high parts take 15..19 windows, 46 on the wide schedule), and the high
// waves' doublings before the scalars' barrier: decode ~75k cycles + 48 x
// ~800 ~ the helper's hash and half-size pair (~114k, tools/row_phase.py);
// after it the lo wave's 18 windows and a high wave's 24 doublings + table +
// 15 windows both take ~87k
constexpr int kRowLoWindows = 18;
constexpr int kRowHiPreDoublings = 48;
// HI > 0 (the four-wave form): the part takes only the windows above the
// lowest HI, against [2^(4 HI)](-P) -- 4 HI doublings of -P before its table,
// while the helper hashes -- and the lo wave (r_sum_ar) takes the rest.
template <int PART, int HI = 0, class R, class Tab, class GetPrep, class Stamp = RowNoStamp>
CMTV_HD typename R::U r_part(const RowCtx<R>& x, const typename R::U& limb, bool sign, Tab& tab,
                             const GetPrep& get_prep, SigPrep& p, bool& dec, bool& x0,
                             const Stamp& stamp = Stamp()) {
  using U = typename R::U;
  const U y = sel(x.k == 15u, limb & 0x7FFFu, limb);
  U xo, to;
  dec = (R::ballot(rf_decode<0, 2>(x, y, typename R::B(sign), xo, to)) & 1u) != 0;
  x0 = (R::ballot(rf_canon<R>(xo).zero) & 1u) != 0;
  stamp(6);  // decoded
  U X0, X1, X2, X3, Y0, Y1, Y2, Y3, T0, T1, T2, T3;
  R::rows(xo, X0, X1, X2, X3);
  R::rows(y, Y0, Y1, Y2, Y3);
  R::rows(to, T0, T1, T2, T3);
  U np = sel(x.r0, rf_neg(x, X0), sel(x.r1, Y0, sel(x.r2, x.one, rf_neg(x, T0))));
  if constexpr (HI > 0) {
    // the workgroup barrier that hands over the scalars (get_prep) sits after
    // kRowHiPreDoublings of the 4 HI doublings: the high waves reach it about
    // when the helper does, and the lo wave is not held up by the rest
    np = rf_carry32(x, np);
#pragma unroll 1
    for (int j = 0; j < kRowHiPreDoublings; j++) rp_dbl(x, np);
    get_prep(p);
#pragma unroll 1
    for (int j = kRowHiPreDoublings; j < 4 * HI; j++) rp_dbl(x, np);
    r_build_table(x, tab, 0, np);
  } else {
    r_build_table(x, tab, 0, np);
    get_prep(p);
  }
  const bool flip = PART == 1 && (p.flags & 1u) != 0;
  const int W = r_windows(p.flags);
  uint32_t t[8];
  hs_digits16(t, PART == 0 ? p.k1 : p.k2, W);
  U v = rp_identity(x);
#pragma unroll 1
  for (int win = W - 1; win >= HI; win--) {
    const int d = (int)sc_shift_out(t, 4) - 8;
    const U c = tab.load(0, (d < 0) != flip ? 1 : 0, d < 0 ? -d : d);
    if (win != W - 1) {
#pragma unroll 1
      for (int j = 0; j < 4; j++) rp_dbl(x, v);
    }
    rp_add(x, v, c);
  }
  return v;
}

// The two-wave form's last step on the A wave: X = (A's sum) + (R's sum,
// cached: cR) + [u]B (cached: cB), then the mode's final check
template <uint32_t MODE, class R>
CMTV_HD bool r_join(const RowCtx<R>& x, typename R::U vA, const typename R::U& cR, const typename R::U& cB, bool ok,
                    bool r_canon) {
  rp_add(x, vA, cR);
  rp_add(x, vA, cB);
  return r_final<MODE>(x, vA, ok, r_canon);
}

// The four-wave form's last step on the lo wave: X = lo + A's high part +
// R's high part + [u]B (the last three cached), then the final check
template <uint32_t MODE, class R>
CMTV_HD bool r_join4(const RowCtx<R>& x, typename R::U v, const typename R::U& cA, const typename R::U& cR,
                     const typename R::U& cB, bool ok, bool r_canon) {
  rp_add(x, v, cA);
  return r_join<MODE>(x, v, cR, cB, ok, r_canon);
}

// ---- registered keys (keyed.h combs) in the row layout ----------------------------

// This row's cached coordinate of (neg ? -P : P) for P an affine niels row of
// 10-limb values (y+x at word 0, y-x at word ymx_off, 2dxy at xy_off): row 0
// y-x, 1 y+x, 2 the constant 2 (Z = 1), 3 2dxy; negated, rows 0 and 1 swap and
// row 3 is negated; the cached identity (1, 1, 2, 0) when ident. The policy's
// niels_limb(row, off) gives this lane's 16-bit limb of the 10-limb value at
// word off (its canonical encoding).
template <class R>
CMTV_HD typename R::U r_niels(const RowCtx<R>& x, const uint32_t* row, int ymx_off, int xy_off, bool neg,
                              bool ident) {
  using U = typename R::U;
  const U off = sel(x.r3, U((uint32_t)xy_off), sel(x.r0 != typename R::B(neg), U((uint32_t)ymx_off), U(0u)));
  const U l = R::niels_limb(row, off);
  const U c = sel(x.r2, sel(x.k == 0u, U(2u), U(0u)), sel(x.r3 && typename R::B(neg), rf_neg(x, l), l));
  return ident ? rp_cached_identity(x) : c;
}

// [s]B over the 16-position radix-2^16 comb of B (verify_core.h BC16 rows of
// the B table, 36 words: y+x at 0, y-x at 12, 2dxy at 24; q_bcomb16's digits)
template <class R, class BRow>
CMTV_HD typename R::U r_bcomb16(const RowCtx<R>& x, const uint32_t s[8], const BRow& brow) {
  uint32_t lo[8], hi[8];
  hs_digits65536(lo, hi, s);
  typename R::U v = rp_identity(x);
#pragma unroll 1
  for (int j = 15; j >= 0; j--) {
    const int d = (int)(j >= 8 ? sc_shift_out(hi, 16) : sc_shift_out(lo, 16)) - 0x8000;
    const int ib = d < 0 ? -d : d;
    rp_add(x, v, r_niels(x, brow(BC16_BASE + j * BT16_ENTRIES + (ib > 0 ? ib - 1 : 0)), BTAB_COORD_WORDS,
                         2 * BTAB_COORD_WORDS, d < 0, ib == 0));
  }
  return v;
}

// [k](-A) over a registered key's radix-256 comb (keyed.h T_A), tk = k's
// biased digits (sc_bias 0x80), top byte first as keyed_comb takes them;
// krow(j, e) = the comb row of position j, entry e (a key's table in HBM, or
// the rows a kernel prefetched into LDS), converted to
// the row layout of a wave. Positions first .. last (downwards) are added to
// v (the keyed row kernel splits the 32 between two waves).
template <class R, class KRow>
CMTV_HD void r_kcomb(const RowCtx<R>& x, typename R::U& v, uint32_t tk[8], const KRow& krow, int first = COMB_WINDOWS - 1,
                     int last = 0) {
#pragma unroll 1
  for (int j = COMB_WINDOWS - 1; j > first; j--) sc_shift_out(tk, 8);
#pragma unroll 1
  for (int j = first; j >= last; j--) {
    const int d = (int)sc_shift_out(tk, 8) - 128;
    const int ia = d < 0 ? -d : d;
    rp_add(x, v, r_niels(x, krow(j, ia > 0 ? ia - 1 : 0), 10, 20, d < 0, ia == 0));
  }
}

// R decoded on every row (limb: R's 16-bit limb k on every row), as -R in
// extended coordinates; r_ok with the mode's decoding rules (GO_STDLIB: R
// canonical, and x = 0 only without the sign bit)
template <uint32_t MODE, int MID_AT = 0, class R, class Mid = RowNoHook>
CMTV_HD typename R::U r_decode_neg_r(const RowCtx<R>& x, const typename R::U& limb, const uint32_t sigw[8], bool& r_ok,
                                     const Mid& mid = Mid()) {
  using U = typename R::U;
  const bool sign = (sigw[7] >> 31) != 0;
  const U y = sel(x.k == 15u, limb & 0x7FFFu, limb);
  U xo, to;
  r_ok = (R::ballot(rf_decode<MID_AT, 2>(x, y, typename R::B(sign), xo, to, mid)) & 1u) != 0;
  const bool x0 = (R::ballot(rf_canon<R>(xo).zero) & 1u) != 0;
  if (MODE == MODE_GO_STDLIB) r_ok = r_ok && y_is_canonical(sigw) && !(x0 && sign);
  U X0, X1, X2, X3, Y0, Y1, Y2, Y3, T0, T1, T2, T3;
  R::rows(xo, X0, X1, X2, X3);
  R::rows(y, Y0, Y1, Y2, Y3);
  R::rows(to, T0, T1, T2, T3);
  return rf_carry32(x, sel(x.r0, rf_neg(x, X0), sel(x.r1, Y0, sel(x.r2, x.one, rf_neg(x, T0)))));
}

// The keyed join: X = -R + [k](-A) + [s]B (the last two cached) = R' - R,
// then the mode's final check (GO_STDLIB: X = O; ZIP215: [8]X = O)
template <uint32_t MODE, class R>
CMTV_HD bool r_keyed_join(const RowCtx<R>& x, typename R::U nr, const typename R::U& cA, const typename R::U& cB,
                          bool ok) {
  rp_add(x, nr, cA);
  rp_add(x, nr, cB);
  return r_final<MODE>(x, nr, ok, true);
}

// [u]B's cached coordinates (Y-X, Y+X, 2Z, 2dT) as four canonical 32-byte
// encodings (8 words each): a row lane reads its 16-bit limb (the helper
// wave's output in k_verify_row_split)
CMTV_HD void bpoint_store_bytes(uint32_t* d, const ge_p3& P) {
  fe c[4], d2;
  fe_sub(c[0], P.Y, P.X);
  fe_add(c[1], P.Y, P.X);
  fe_add(c[2], P.Z, P.Z);
  fe_const_d2(d2);
  fe_mul(c[3], P.T, d2);
#pragma unroll
  for (int k = 0; k < 4; k++) fe_tobytes(d + 8 * k, c[k]);
}

}  // namespace cmtv
