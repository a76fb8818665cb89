// quad.h -- 4 lanes per signature ("quad"): coordinate-parallel edwards25519
// arithmetic for latency-bound batches (a 10k-signature commit fills only
// ~157 of the chip's 1,024 SIMDs at one signature per lane).
//
// Lane c of a quad holds coordinate c of every point:
//   extended point  (X, Y, Z, T)            lane 0: X, 1: Y, 2: Z, 3: T
//   cached addend   (Y-X, Y+X, Z, 2dT)      ordered so lane c's product in
//                                           round 1 of an addition is local
// A doubling or an addition is two rounds of ONE field multiplication per
// lane (HWCD 4-way formulas) instead of 7-8 sequential multiplications, with
// operands exchanged inside the quad by DPP quad_perm moves (a VALU operand
// modifier on gfx950, no LDS round trip).
//
// Everything is written against a Quad policy:
//   int lane() const;                               this lane's coordinate index
//   template <int PAT> void perm(fe& o, const fe& v) const;
//                          lane c receives v from lane (PAT >> 2c) & 3
//   template <int PAT> uint32_t perm32(uint32_t x) const;
//   bool any(bool x) const;   x on any lane of the wave (uniform loop bounds)
// The device policy lowers perm to v_mov_b32_dpp quad_perm; the host test
// policy (tests/host/quadcheck.cpp) runs 4 threads in lockstep, so the same
// source is checked against the oracle on the CPU.
//
// Control flow is uniform across a quad (digits, verdicts and mode are per
// signature); only data differs per lane, via pick() selects.
#pragma once
#include "halfscalar.h"
#include "verify_core.h"

namespace cmtv {

// quad_perm codes
constexpr int QP_B0 = 0x00, QP_B1 = 0x55, QP_B2 = 0xAA, QP_B3 = 0xFF;  // broadcast lane k
constexpr int QP_SWAP01 = (1 << 0) | (0 << 2) | (2 << 4) | (3 << 6);    // [1,0,2,3]

// quad_perm code: lane c reads lane s_c
constexpr int qp(int s0, int s1, int s2, int s3) { return s0 | (s1 << 2) | (s2 << 4) | (s3 << 6); }

// limb i of 2p (the bias of fe_sub / fe_neg)
CMTV_HD uint32_t fe_p2(int i) { return i == 0 ? P2_0 : ((i & 1) ? P2_O : P2_E); }

// h = {a, b, c, d}[lane]
CMTV_HD void fe_pick(fe& h, int lane, const fe& a, const fe& b, const fe& c, const fe& d) {
  const bool l1 = lane & 1, l2 = lane & 2;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    const uint32_t lo = l1 ? b.v[i] : a.v[i];
    const uint32_t hi = l1 ? d.v[i] : c.v[i];
    h.v[i] = l2 ? hi : lo;
  }
}

// the identity point's coordinate for this lane: (0, 1, 1, 0)
CMTV_HD void q_identity(fe& v, int lane) {
  fe_0(v);
  v.v[0] = (lane == 1 || lane == 2) ? 1u : 0u;
}

// Cached form of an addend, one coordinate per lane: (Y-X, Y+X, 2Z, 2dT).
// Lane 2 carries 2Z so that round 1 of an addition yields D = 2 Z1 Z2
// directly. The identity's cached coordinate: (1, 1, 2, 0).
CMTV_HD void q_cached_identity(fe& v, int lane) {
  fe_0(v);
  v.v[0] = lane == 2 ? 2u : (lane != 3 ? 1u : 0u);
}

// Doubling (dbl-2008-hwcd, a = -1, outputs negated as in ge25519.h p2_dbl):
//   round 1: lane c squares {X, Y, Z, X+Y}[c]      -> A, B, C', K
//   round 2: lane c multiplies {E'F', MS, F'M, E'S}[c],
//            S = A + B, M = A - B, E' = S - K, F' = 2C' + M
// Routing: lane c forms U_c = {F', S, M, E'}[c] (one carry for all four).
// The round-2 products form the cycle F'-E'-S-M-F', so each lane multiplies
// its own U by one neighbour's: a single quad_perm move {E', M, F', S}. The
// U_c take two moves of the round-1 results (lane 0 reads C', the rest A;
// every lane B). Input T (lane 3) is ignored; output is a full extended point.
// FOLD: how a quad move that feeds exactly one 32-bit add / xor / select
// reaches it. 0: a v_mov_b32_dpp, then the instruction; 2: the policy's fused
// forms (add_perm, xor_perm, perm_lane3 -- DevQuad: v_add_u32_dpp,
// v_xor_b32_dpp, v_cndmask_b32_dpp), 30 fewer VALU instructions per doubling
// and 10 per addition; 1: permc (update_dpp, left to DPP-combine; folds only
// some). A/B: tools/microbench/pt_lat.hip.
#ifndef CMTV_DPP_FOLD
#define CMTV_DPP_FOLD 0
#endif
constexpr int kDppFold = CMTV_DPP_FOLD;

template <int FOLD = kDppFold, class Q>
CMTV_HD void q_dbl(const Q& q, fe& v) {
  const int lane = q.lane();
  // per-lane masks (loop-invariant): the four U_c share one straight-line
  // form, U = (p1 << sh) + (p2 ^ n2) + ((own ^ n3) & mo) + corr + 2p,
  // instead of computing all four candidates and selecting
  const uint32_t m3 = lane == 3 ? ~0u : 0u;
  const uint32_t sh = lane == 0 ? 1u : 0u;                  // 2C' on lane 0
  const uint32_t s2 = lane == 2 ? 1u : 0u;                  // ... doubled at its source, lane 2 (FOLD)
  const uint32_t n2 = (lane & 1) ? 0u : ~0u;                // -B on lanes 0, 2
  const uint32_t n3 = lane == 3 ? ~0u : 0u;                 // -K on lane 3
  const uint32_t mo = (lane == 0 || lane == 3) ? ~0u : 0u;  // own A (0), K (3)
  const uint32_t corr = lane == 1 ? 0u : 1u;                // ~x = -x - 1
  fe a, b, m;
  if constexpr (FOLD == 2) {
    q.template perm_lane3<QP_B1>(b, v);                 // lane 3: Y, else 0
    q.template add_perm<qp(0, 1, 2, 0)>(m, v, b);        // X + Y on lane 3
  } else if constexpr (FOLD == 1) {
    q.template permc<QP_B1>(b, v);
#pragma unroll
    for (int i = 0; i < 10; i++) b.v[i] &= m3;  // v_and_b32_dpp
    q.template permc<qp(0, 1, 2, 0)>(a, v);
#pragma unroll
    for (int i = 0; i < 10; i++) m.v[i] = a.v[i] + b.v[i];  // v_add_u32_dpp: X + Y on lane 3
  } else {
    q.template perm<qp(0, 1, 2, 0)>(a, v);
    q.template perm<QP_B1>(b, v);
#pragma unroll
    for (int i = 0; i < 10; i++) m.v[i] = a.v[i] + (b.v[i] & m3);  // X + Y on lane 3
  }
  fe_sq(m, m);                                                     // A, B, C', K
  if constexpr (FOLD == 2) {
    fe src;
#pragma unroll
    for (int i = 0; i < 10; i++) src.v[i] = m.v[i] << s2;  // lane 2: 2C' (lane 0 reads it)
    q.template xor_perm<QP_B1>(b, m, n2);                // B ^ n2
#pragma unroll
    for (int i = 0; i < 10; i++) b.v[i] += CMTV_XOR_AND(m.v[i], n3, mo) + (corr + fe_p2(i));
    q.template add_perm<qp(2, 0, 0, 0)>(m, src, b);      // F', S, M, E' (+2p)
  } else if constexpr (FOLD == 1) {
    // lane 0 reads 2C' from lane 2, the others A from lane 0: lane 2's C'
    // is doubled before the move (its own U does not use it)
    fe src;
#pragma unroll
    for (int i = 0; i < 10; i++) src.v[i] = m.v[i] << s2;
    q.template permc<QP_B1>(b, m);  // B
#pragma unroll
    for (int i = 0; i < 10; i++) {
      const uint32_t t = b.v[i] ^ n2;  // v_xor_b32_dpp
      b.v[i] = t + (CMTV_XOR_AND(m.v[i], n3, mo) + (corr + fe_p2(i)));
    }
    q.template permc<qp(2, 0, 0, 0)>(a, src);  // 2C', A, A, A
#pragma unroll
    for (int i = 0; i < 10; i++) m.v[i] = a.v[i] + b.v[i];  // v_add_u32_dpp
  } else {
    q.template perm<qp(2, 0, 0, 0)>(a, m);  // C', A, A, A
    q.template perm<QP_B1>(b, m);           // B
#pragma unroll
    for (int i = 0; i < 10; i++) {
      // lane 0: F' = M + 2C', 1: S = A + B, 2: M = A - B, 3: E' = S - K (+2p)
      const uint32_t u = (b.v[i] ^ n2) + CMTV_XOR_AND(m.v[i], n3, mo) + corr + fe_p2(i);
      m.v[i] = (a.v[i] << sh) + u;
    }
  }
  fe_carry(m);
  q.template perm<qp(3, 2, 0, 1)>(a, m);  // E', M, F', S
  fe_mul(v, m, a);                        // F'E', SM, MF', E'S
}

// Addition v += Q where c is this lane's coordinate of Q in cached form
// (Y2-X2, Y2+X2, 2Z2, 2dT2):
//   round 1: lane c computes {(X1-Y1)(Y2-X2), (Y1+X1)(Y2+X2), Z1 2Z2, T1 2dT2}[c]
//            = {-A, B, D, C}  (lane 0 negates its own factor: X1 - Y1 needs
//            one swap move of (X, Y) where Y1 - X1 needed two broadcasts)
//   round 2: with E = B-A, F = D-C, G = D+C, H = B+A, lane c forms
//            U_c = {E, G, F, H}[c] from two quad_perm moves (no carry: every
//            U stays inside the multiplier bounds); the products form the
//            cycle E-F-G-H-E, so lane c multiplies its own U by one move
//            {F, H, G, E}: {EF, GH, FG, HE}[c] = (X3, Y3, Z3, T3).
template <int FOLD = kDppFold, class Q>
CMTV_HD void q_add(const Q& q, fe& v, const fe& c) {
  const int lane = q.lane();
  // per-lane masks (loop-invariant); ~x + 1 = -x supplies the negations
  const uint32_t m0 = lane == 0 ? ~0u : 0u;
  const uint32_t m01 = lane < 2 ? ~0u : 0u;
  const uint32_t m23 = lane >= 2 ? ~0u : 0u;
  fe x, y, p;
  q.template perm<QP_SWAP01>(y, v);  // Y, X, Z, T
#pragma unroll
  for (int i = 0; i < 10; i++) {
    // lane 0: X - Y + 2p, 1: Y + X, 2: Z, 3: T
    const uint32_t k = lane == 0 ? fe_p2(i) + 1 : 0u;
    p.v[i] = v.v[i] + CMTV_XOR_AND(y.v[i], m0, m01) + k;
  }
  fe t;
  fe_mul(t, p, c);  // -A, B, D, C
  if constexpr (FOLD == 2) {
    q.template xor_perm<qp(0, 3, 3, 0)>(y, t, m23);  // -A, C, C, -A (negated on lanes 2, 3)
#pragma unroll
    for (int i = 0; i < 10; i++) y.v[i] += lane >= 2 ? fe_p2(i) + 1 : 0u;
    q.template add_perm<qp(1, 2, 2, 1)>(p, t, y);     // E, G, F, H
  } else if constexpr (FOLD == 1) {
    q.template permc<qp(0, 3, 3, 0)>(y, t);  // -A, C, C, -A
#pragma unroll
    for (int i = 0; i < 10; i++) {
      const uint32_t k = lane >= 2 ? fe_p2(i) + 1 : 0u;
      y.v[i] = (y.v[i] ^ m23) + k;  // v_xor_b32_dpp
    }
    q.template permc<qp(1, 2, 2, 1)>(x, t);  // B, D, D, B
#pragma unroll
    for (int i = 0; i < 10; i++) p.v[i] = x.v[i] + y.v[i];  // v_add_u32_dpp
  } else {
    q.template perm<qp(1, 2, 2, 1)>(x, t);  // B, D, D, B
    q.template perm<qp(0, 3, 3, 0)>(y, t);  // -A, C, C, -A
#pragma unroll
    for (int i = 0; i < 10; i++) {
      // E = B - A, G = D + C; F = D - C, H = B + A (lanes 2, 3: + 2p)
      const uint32_t k = lane >= 2 ? fe_p2(i) + 1 : 0u;
      p.v[i] = x.v[i] + (y.v[i] ^ m23) + k;
    }
  }
  q.template perm<qp(2, 3, 1, 0)>(x, p);  // F, H, G, E
  fe_mul(v, p, x);
}

// this lane's cached-form coordinate of the extended point v
template <class Q>
CMTV_HD void q_to_cached(const Q& q, fe& c, const fe& v) {
  const int lane = q.lane();
  fe x, y, d2;
  q.template perm<QP_B0>(x, v);
  q.template perm<QP_B1>(y, v);
  fe_const_d2(d2);
  fe_mul(d2, v, d2);
#pragma unroll
  for (int i = 0; i < 10; i++) {
    const uint32_t w = lane == 0 ? fe_p2(i) - x.v[i] : x.v[i];
    const uint32_t hi = (lane & 1) ? d2.v[i] : 2 * v.v[i];
    c.v[i] = (lane & 2) ? hi : y.v[i] + w;  // Y-X, Y+X, 2Z, 2dT
  }
}

// conditional negation of a cached addend: swap (Y-X, Y+X), negate 2dT
template <class Q>
CMTV_HD void q_cached_cneg(const Q& q, fe& c, bool neg) {
  fe s, n;
  q.template perm<QP_SWAP01>(s, c);
  fe_neg(n, c);
  fe_select(s, s, n, q.lane() == 3);
  fe_select(c, c, s, neg);
}

// lane 3's half of a cached negation (lanes 0/1 swap by where they load)
CMTV_HD void q_negate_lane3(fe& c, int lane, bool neg) {
  const bool f = neg && lane == 3;
#pragma unroll
  for (int i = 0; i < 10; i++) c.v[i] = f ? fe_p2(i) - c.v[i] : c.v[i];
}

// ZIP-215's [8]P = O for the quad's extended point v (lane c: coordinate c).
// The torsion of edwards25519 is cyclic of order 8, so [8]P = O <=> [2]P is in
// E[4] = {(0, 1), (0, -1), (+/-sqrt(-1), 0)}, the points with xy = 0, i.e.
// T([2]P) = 0; and the doubling gives T([2]P) = 2XY (X^2 + Y^2) (ref10's
// p2_dbl: (A - XX - YY)(XX + YY)). So [8]P = O <=> T = 0 or X^2 + Y^2 = 0:
// one squaring round instead of three doublings.
template <class Q>
CMTV_HD bool q_small_order(const Q& q, const fe& v) {
  fe s, x2, y2;
  fe_sq(s, v);  // lane 0: X^2, lane 1: Y^2
  q.template perm<QP_B0>(x2, s);
  q.template perm<QP_B1>(y2, s);
  fe_add(s, x2, y2);
  const bool t0 = q.template perm32<QP_B3>(fe_iszero(v) ? 1u : 0u) != 0;  // T, from lane 3
  return t0 || fe_iszero(s);
}

// This lane's cached coordinate of (neg ? -P : P) for P an affine niels row
// (y+x at word 0, y-x at word ymx_off, 2dxy at word xy_off), or of the
// identity when ident. ld(off, c) loads the 10 limbs at word `off`.
template <class Q, class Ld>
CMTV_HD void q_niels_load(const Q& q, fe& c, const Ld& ld, int ymx_off, int xy_off, bool neg) {
  const int lane = q.lane();
  const int off = lane == 3 ? xy_off : (((lane == 0) != neg) ? ymx_off : 0);
  ld(off, c);
}
CMTV_HD void q_niels_fix(fe& c, int lane, bool neg, bool ident) {
  const bool cst = ident || lane == 2;  // lane 2: 2Z = 2 (affine); identity (1, 1, 2, 0)
  const uint32_t c0 = lane == 2 ? 2u : (lane == 3 ? 0u : 1u);
#pragma unroll
  for (int i = 0; i < 10; i++) c.v[i] = cst ? (i == 0 ? c0 : 0u) : c.v[i];
  q_negate_lane3(c, lane, neg && !ident);
}
template <class Q, class Ld>
CMTV_HD void q_niels_coord(const Q& q, fe& c, const Ld& ld, int ymx_off, int xy_off, bool neg, bool ident) {
  q_niels_load(q, c, ld, ymx_off, xy_off, neg);
  q_niels_fix(c, q.lane(), neg, ident);
}

}  // namespace cmtv

namespace cmtv {


// One signature per quad. Every lane returns the same verdict.
//   phase 1: lanes {0,2} decode A, lanes {1,3} decode R (same code, different
//            data, so the two square-root chains run simultaneously); every
//            lane hashes k = SHA-512(R || A || M) mod L
//   phase 2: half-size scalars k1 == k2 k (mod 8L), u = k2 s mod L
//   phase 3: (0..8)(-A) and (0..8)(-/+R) in cached form, one coordinate per
//            lane, in the ATab policy's storage (LDS on the device)
//   phase 4: Straus over 34 (wide: 64) 4-bit windows: per window 4 shared
//            doublings, one A and one R addition (signed radix-16 digits) and
//            one fixed-base addition (signed radix-256 digits of u's low half
//            against (1..128)B on even windows, of its high half against
//            (1..128)[2^124]B on odd ones)
//   final  : X = [k2](R' - R) is O (GO_STDLIB, with R canonical: encode(R')
//            == R bytes; no inversion) or [8]X = O (ZIP215, q_small_order)
// (0..8)P in cached form (entry 0 = the identity), one coordinate per lane;
// v holds this lane's coordinate of P and is clobbered.
template <class Q, class ATab>
CMTV_HD void q_build_table(const Q& q, ATab& tab, fe& v) {
  const int lane = q.lane();
  fe c1, c;
  q_cached_identity(c, lane);
  tab.store(0, c);
  q_to_cached(q, c1, v);
  tab.store(1, c1);
  q_dbl(q, v);
  q_to_cached(q, c, v);
  tab.store(2, c);
#pragma unroll 1
  for (int e = 3; e <= 8; e++) {
    q_add(q, v, c1);
    q_to_cached(q, c, v);
    tab.store(e, c);
  }
}

struct NullProbe {
  CMTV_HD void snap(int, const fe&) const {}
};

// Table policy for the per-signature (0..8)(-A) cached table (entry 0 = the
// identity), one coordinate per lane:
//   void store(int e, const fe& c);  void load(int e, fe& c) const;
// The device policy keeps it in LDS (a per-lane slot, so no barrier is needed
// and a lookup is 5 ds_read_b64 instead of an 8-way register select).
//   template <class Q> void load_signed(const Q& q, int e, bool neg, fe& c) const;
// gives (neg ? -P_e : P_e): the LDS policy negates by reading the partner
// lane's slot on lanes 0/1 and negating lane 3 (q_negate_lane3).
struct QArrayTab {  // plain-array table policy (host checks, debug kernels)
  fe t[9];
  CMTV_HD void store(int e, const fe& c) { t[e] = c; }
  CMTV_HD void load(int e, fe& c) const { c = t[e]; }
  // this lane's coordinate of (neg ? -P_e : P_e)
  template <class Q>
  CMTV_HD void load_signed(const Q& q, int e, bool neg, fe& c) const {
    c = t[e];
    q_cached_cneg(q, c, neg);
  }
};

// Per-signature scalar work that does not depend on the decoded points: the
// half-size pair of the challenge k and the fixed-base scalar u = k2 s mod L
// (plus, from q_prepare, the s check). The split kernels (kernels.hip
// k_verify_quad_split / k_verify_oct_split) compute it on a helper wave while
// the main waves decompress A and R.
struct SigPrep {
  uint32_t k1[8], k2[8], u[8];
  uint32_t flags;  // bit 0: k2 < 0, bit 1: wide, bit 2: s canonical, bits 8..15: window count
};
constexpr int SIG_PREP_WORDS = 25;

// UNI: every lane of the wave holds the same signature (halfscalar.h hs_uni)
template <bool UNI = false>
CMTV_HD void q_prepare_scalars(SigPrep& p, const uint32_t k[8], const uint32_t ts[8], bool force_wide,
                               bool odd_k2 = true) {
  HalfScalars hs;
  half_scalars<true, UNI>(hs, k, force_wide, odd_k2);
  hs_bscalar(p.u, hs.k2, hs.k2_neg, ts);
#pragma unroll
  for (int i = 0; i < 8; i++) {
    p.k1[i] = hs.k1[i];
    p.k2[i] = hs.k2[i];
  }
  p.flags = (hs.k2_neg ? 1u : 0u) | (hs.wide ? 2u : 0u) | ((uint32_t)hs.windows << 8);
}

// s check, k = SHA-512(R || A || M) mod L, then q_prepare_scalars (k2 odd
// for the cofactorless check, MODE_GO_STDLIB; any parity for MODE_ZIP215)
struct NoPrepMark {
  CMTV_HD void operator()() const {}
};

template <uint32_t MODE, bool UNI = false, class Mark = NoPrepMark>
CMTV_HD void q_prepare(SigPrep& p, const uint32_t* pk_ptr, const uint32_t* sig_ptr, const uint8_t* msg,
                       uint32_t mlen, bool force_wide, const Mark& after_hash = Mark()) {
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 8; i++) w[i] = sig_ptr[8 + i];
  const bool s_ok = (w[7] & 0xE0000000u) == 0 && sc_is_canonical(w);
  uint32_t ts[8];
#pragma unroll
  for (int i = 0; i < 8; i++) ts[i] = w[i];
  uint32_t k[8];
  {
    uint32_t h[16];
#pragma unroll
    for (int i = 0; i < 8; i++) {
      w[i] = sig_ptr[i];
      w[8 + i] = pk_ptr[i];
    }
    sha512_prefixed<16>(h, w, msg, mlen);
    after_hash();
    sc_reduce512(k, h);
  }
  q_prepare_scalars<UNI>(p, k, ts, force_wide, MODE != MODE_ZIP215);
  p.flags |= s_ok ? 4u : 0u;
}

CMTV_HD void sig_prep_store(uint32_t* d, const SigPrep& p) {
#pragma unroll
  for (int j = 0; j < 8; j++) {
    d[j] = p.k1[j];
    d[8 + j] = p.k2[j];
    d[16 + j] = p.u[j];
  }
  d[24] = p.flags;
}
CMTV_HD void sig_prep_load(SigPrep& p, const uint32_t* d) {
#pragma unroll
  for (int j = 0; j < 8; j++) {
    p.k1[j] = d[j];
    p.k2[j] = d[8 + j];
    p.u[j] = d[16 + j];
  }
  p.flags = d[24];
}

// [u]B by the 16-position radix-2^16 comb (verify_core.h BC16 blocks): 16
// mixed additions and no doublings, one lane per signature -- the helper
// waves' share of the fixed-base work. BTab: the one-lane policy (load_fe).
template <class BTab>
CMTV_HD void q_bcomb16(ge_p3& P, const uint32_t u[8], const BTab& btab) {
  uint32_t lo[8], hi[8];
  hs_digits65536(lo, hi, u);
  p3_identity(P);
  ge_efgh t;
#pragma unroll 1
  for (int j = 15; j >= 0; j--) {
    const int d = (int)(j >= 8 ? sc_shift_out(hi, 16) : sc_shift_out(lo, 16)) - 0x8000;
    const int ib = d < 0 ? -d : d;
    ge_add_table<false>(t, P, btab, BC16_BASE + j * BT16_ENTRIES + (ib > 0 ? ib - 1 : 0), d < 0, ib == 0);
    efgh_to_p3(P, t);
  }
}

// q_bcomb16 one comb position at a time (the helper-summed quad kernel
// spreads the 16 additions over the windows' slack): init, then step() while
// j >= 0
struct BComb16 {
  ge_p3 P;
  uint32_t lo[8], hi[8];
  int j;
  CMTV_HD void init(const uint32_t u[8]) {
    hs_digits65536(lo, hi, u);
    p3_identity(P);
    j = 15;
  }
  template <class BTab>
  CMTV_HD void step(const BTab& btab) {
    const int d = (int)(j >= 8 ? sc_shift_out(hi, 16) : sc_shift_out(lo, 16)) - 0x8000;
    const int ib = d < 0 ? -d : d;
    ge_efgh t;
    ge_add_table<false>(t, P, btab, BC16_BASE + j * BT16_ENTRIES + (ib > 0 ? ib - 1 : 0), d < 0, ib == 0);
    efgh_to_p3(P, t);
    j--;
  }
};

// the quad's cached coordinates of P, (Y-X, Y+X, 2Z, 2dT), as 40 words
CMTV_HD void bpoint_store(uint32_t* d, const ge_p3& P) {
  fe c[4], d2;
  fe_sub(c[0], P.Y, P.X);
  fe_add(c[1], P.Y, P.X);
  fe_add(c[2], P.Z, P.Z);
  fe_const_d2(d2);
  fe_mul(c[3], P.T, d2);
#pragma unroll
  for (int k = 0; k < 3; k++) fe_carry(c[k]);
#pragma unroll
  for (int k = 0; k < 4; k++)
#pragma unroll
    for (int i = 0; i < 10; i++) d[10 * k + i] = c[k].v[i];
}

// get_b policy of a verifier that adds its own fixed-base digits
struct NoExtB {
  CMTV_HD void operator()(fe&) const {}
};

// the wave-uniform window count: the largest over the wave (33..37), 64 if
// any signature is wide
template <class Q>
CMTV_HD int q_wave_windows(const Q& q, uint32_t flags) {
  const bool wide = q.any((flags & 2u) != 0);
  int W = HS_WINDOWS;
#pragma unroll 1
  for (int x = HS_WINDOWS; x < HS_MAX_WINDOWS; x++) W += q.any((int)(flags >> 8) > x) ? 1 : 0;
  return wide ? HS_WIDE_WINDOWS : W;
}

// Phase 3 ahead of the scalars: (0..8)(-A) and (0..8)(-R) need only the
// decoded points, so a split verifier whose helper is the longer side of
// barrier 1 (sr25519: the merlin transcript) builds them before waiting; a negative k2 then flips R's digits at lookup
// (q_straus_prep_b<EXT_B, true>) instead of negating R. v, rc are clobbered.
template <class Q, class ATab>
CMTV_HD void q_tables_early(const Q& q, fe& v, fe& rc, ATab& tabA, ATab& tabR) {
  const int lane = q.lane();
  fe t;
  fe_neg(t, rc);
  fe_carry(t);
  fe_select(rc, rc, t, lane == 0 || lane == 3);
  q_build_table(q, tabA, v);
  q_build_table(q, tabR, rc);
}

// Phases 3-4 from a prepared pair (see q_straus_half below). EXT_B: the
// fixed-base part [u]B comes ready-made from get_b (this lane's cached
// coordinate, a helper wave's q_bcomb16) and is added once after the windows.
// PREBUILT: the tables came from q_tables_early (R's table is of -R).
template <bool EXT_B, bool PREBUILT = false, class Q, class BTab, class ATab, class Probe, class GetB>
CMTV_HD void q_straus_prep_b(const Q& q, fe& v, fe& rc, const SigPrep& hs, const BTab& btab, ATab& tabA, ATab& tabR,
                             const Probe& probe, const GetB& get_b) {
  const int lane = q.lane();
  const bool k2_neg = (hs.flags & 1u) != 0;
  const bool r_flip = PREBUILT && k2_neg;
  const uint32_t* u = hs.u;
  const int W = q_wave_windows(q, hs.flags);
  {
    fe kk;
#pragma unroll
    for (int i = 0; i < 8; i++) kk.v[i] = hs.k1[i];
    kk.v[8] = hs.k2[0];
    kk.v[9] = hs.flags & 3u;
    probe.snap(11, kk);
  }

  // ---- phase 3: (0..8)(-A) and (0..8)(-/+R), this lane's cached coordinate
  if constexpr (!PREBUILT) {
    fe t;
    fe_neg(t, rc);
    fe_carry(t);
    fe_select(rc, rc, t, !k2_neg && (lane == 0 || lane == 3));
    q_build_table(q, tabA, v);
    q_build_table(q, tabR, rc);
  }

  // ---- phase 4: Straus over W shared 4-bit windows; the fixed-base scalar
  //      u in signed radix-2^16 digits: digit j on window 4j against
  //      (1..2^15)B, digit 8+j on window 4j+2 against (1..2^15)[2^120]B
  uint32_t tA[8], tR[8], tLo[8], tHi[8];
  hs_digits16(tA, hs.k1, W);
  hs_digits16(tR, hs.k2, W);
  hs_digits65536(tLo, tHi, u);
  q_identity(v, lane);
#pragma unroll 1
  for (int win = W - 1; win >= 0; win--) {
    // this window's addends are fetched first (LDS for A and R, the global
    // B row) so their latency hides under the four doublings
    fe cA, cR, cB;
    {
      const int dA = (int)sc_shift_out(tA, 4) - 8;
      tabA.load_signed(q, dA < 0 ? -dA : dA, dA < 0, cA);
      const int dR = (int)sc_shift_out(tR, 4) - 8;
      tabR.load_signed(q, dR < 0 ? -dR : dR, (dR < 0) != r_flip, cR);
    }
    const bool has_b = !EXT_B && (win & 1) == 0 && win <= 30;
    bool b_neg = false, b_ident = false;
    if (has_b) {
      const bool hi = (win & 2) != 0;
      int dB;
      if (hi)
        dB = (int)sc_shift_out(tHi, 16) - 0x8000;
      else
        dB = (int)sc_shift_out(tLo, 16) - 0x8000;
      const int ib = dB < 0 ? -dB : dB;
      const int row = BT16_BASE + (ib > 0 ? ib - 1 : 0) + (hi ? BT16_ENTRIES : 0);
      // raw row only: the select / negation waits until after the doublings
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
    q_add(q, v, cA);
    q_add(q, v, cR);
    if (has_b) {
      q_niels_fix(cB, lane, b_neg, b_ident);
      q_add(q, v, cB);
    }
    if (win >= W - 4) probe.snap(6 + (W - 1 - win), v);
  }
  if constexpr (EXT_B) {
    fe c;
    get_b(c);
    q_add(q, v, c);
  }
  probe.snap(10, v);
}

template <class Q, class BTab, class ATab, class Probe>
CMTV_HD void q_straus_prep(const Q& q, fe& v, fe& rc, const SigPrep& hs, const BTab& btab, ATab& tabA, ATab& tabR,
                           const Probe& probe) {
  q_straus_prep_b<false>(q, v, rc, hs, btab, tabA, tabR, probe, NoExtB());
}

// Phases 2-4 of a quad verification, shared by the Ed25519 (q_verify) and
// sr25519 (q_verify_sr, sr25519_quad.h) kernels. In: v = this lane's
// coordinate of -A, rc = of R (both extended, Z = 1), k the challenge, ts the
// fixed-base scalar s. Out: v = this lane's coordinate of
//   X = [u]B + [k1](-A) + [|k2|](k2 < 0 ? R : -R) = [k2](R' - R),   R' = [s]B - [k]A
// with (k1, k2) the half-size pair of k (halfscalar.h) and u = k2 s mod L.
// rc is clobbered.
template <class Q, class BTab, class ATab, class Probe>
CMTV_HD void q_straus_half(const Q& q, fe& v, fe& rc, const uint32_t k[8], const uint32_t ts[8], const BTab& btab,
                           ATab& tabA, ATab& tabR, const Probe& probe, bool force_wide = false) {
  SigPrep p;
  q_prepare_scalars(p, k, ts, force_wide);
  q_straus_prep(q, v, rc, p, btab, tabA, tabR, probe);
}

// The quad verifier with the scalar work supplied by get_prep(SigPrep&)
// (q_prepare, or a helper wave's result), called after the decompression by
// every lane of the wave.
template <uint32_t MODE, bool EXT_B = false, class Q, class BTab, class ATab, class GetPrep, class GetB = NoExtB,
          class Probe = NullProbe>
CMTV_HD bool q_verify_split(const Q& q, const uint32_t* pk_ptr, const uint32_t* sig_ptr, const BTab& btab, ATab& tabA,
                            ATab& tabR, const GetPrep& get_prep, const GetB& get_b = GetB(),
                            const Probe& probe = Probe()) {
  const int lane = q.lane();
  uint32_t w[8];

  // ---- phase 1: decode A (even lanes) and R (odd lanes)
  const uint32_t* src = (lane & 1) ? sig_ptr : pk_ptr;
#pragma unroll
  for (int i = 0; i < 8; i++) w[i] = src[i];
  fe v, rc;
  bool a_ok, r_ok, r_canon;
  {
    ge_p3 P;
    const bool dec = p3_frombytes(P, w);
    const bool canon = y_is_canonical(w) && !(fe_iszero(P.X) && (w[7] >> 31));
    fe x, y, t, one;
    fe_1(one);
    q.template perm<QP_B0>(x, P.X);
    q.template perm<QP_B0>(y, P.Y);
    q.template perm<QP_B0>(t, P.T);
    fe_pick(v, lane, x, y, one, t);  // A
    q.template perm<QP_B1>(x, P.X);
    q.template perm<QP_B1>(y, P.Y);
    q.template perm<QP_B1>(t, P.T);
    fe_pick(rc, lane, x, y, one, t);  // R
    a_ok = q.template perm32<QP_B0>(dec ? 1u : 0u) != 0;
    r_ok = q.template perm32<QP_B1>(dec ? 1u : 0u) != 0;
    r_canon = q.template perm32<QP_B1>(canon ? 1u : 0u) != 0;
    // -A: negate X (lane 0) and T (lane 3)
    fe_neg(t, v);
    fe_carry(t);
    fe_select(v, v, t, lane == 0 || lane == 3);
  }
  probe.snap(0, v);
  probe.snap(1, rc);
  // the tables stay after get_prep here: barrier 1 is balanced (the quads'
  // decode and the helper's hash + pair both take ~150k cycles), and building
  // them first measured 1.7% slower in ZIP-215 mode (sr25519 gains: 7%)
  SigPrep p;
  get_prep(p);
  const bool s_ok = (p.flags & 4u) != 0;
  {
    fe kk;
#pragma unroll
    for (int i = 0; i < 8; i++) kk.v[i] = p.u[i];
    kk.v[8] = s_ok | (a_ok << 1) | (r_ok << 2) | (r_canon << 3);
    kk.v[9] = 0;
    probe.snap(2, kk);
  }

  // ---- phases 2-4: v <- this lane's coordinate of X = [k2](R' - R)
  q_straus_prep_b<EXT_B>(q, v, rc, p, btab, tabA, tabR, probe, get_b);

  // ---- final check: X = O (GO_STDLIB: R' == R with R canonical, i.e.
  //      encode(R') == R bytes) / [8]X = O (ZIP215)
  if (MODE == MODE_ZIP215) {
    const bool so = q_small_order(q, v);  // every lane takes part in its DPP moves
    return s_ok && a_ok && r_ok && so;
  }
  fe z;
  q.template perm<QP_B2>(z, v);
  const bool x0 = fe_iszero(v);    // meaningful on lane 0
  const bool yz = fe_equal(v, z);  // meaningful on lane 1
  const bool e0 = q.template perm32<QP_B0>(x0 ? 1u : 0u) != 0;
  const bool e1 = q.template perm32<QP_B1>(yz ? 1u : 0u) != 0;
  return s_ok && a_ok && r_ok && r_canon && e0 && e1;
}

// ---- helper-summed windows (kernels.hip k_verify_quad_hs) -----------------
//
// In the helper-wave quad kernel a third of every window went to the quads'
// two table additions (A's and R's), while the helper wave sat idle after
// [u]B. Here the helper sums a window's two table entries in its own lane
// layout, S_w = [dA](-A) + [dR](-/+R), and hands S_w to the quads through LDS
// at a per-window barrier: a window is 4 doublings and ONE addition. Both
// tables are built before barrier 1 as extended points -- of -A and of -R (a
// negative k2 flips R's digits) -- so the quads spend no cached conversions on
// them; the helper converts R's entry itself. Only the top window is summed
// by the quads (its A entry is loaded as the starting point).

// (0..8)P as extended points (entry 0 the identity), one coordinate per lane;
// v holds this lane's coordinate of P and is clobbered
template <class Q, class ATab>
CMTV_HD void q_build_table_p3(const Q& q, ATab& tab, fe& v) {
  const int lane = q.lane();
  fe c1, z;
  q_identity(z, lane);
  tab.store(0, z);
  tab.store(1, v);
  q_to_cached(q, c1, v);
  q_dbl(q, v);
  tab.store(2, v);
#pragma unroll 1
  for (int e = 3; e <= 8; e++) {
    q_add(q, v, c1);
    tab.store(e, v);
  }
}

// The helper's addend of one window for its signature (one per lane), from
// the quads' tables read through rd(P, e, c, fe&) -- P = 0: the extended
// entries of -A, 1: of -R; c = the coordinate, i.e. the quad lane that stored
// it -- as the quads' cached coordinates (Y-X, Y+X, 2Z, 2dT) in out[0..3]:
// S = [dA](-A) + [dR](r_flip ? R : -R). HWCD addition with both operands
// extended: A = (Y1-X1)(Y2-X2), B = (Y1+X1)(Y2+X2), C = T1 2dT2 (2d T2 one
// constant product), D = 2 Z1 Z2; then the cached form of the sum: 10
// multiplications. Negating an operand swaps its (Y-X, Y+X) and negates T;
// the two T signs meet in C, so one sign decides whether C is added to or
// subtracted from D (no negation is computed).
template <class Rd>
CMTV_HD void h_window_addend(fe out[4], const Rd& rd, int dA, int dR, bool r_flip) {
  const int eA = dA < 0 ? -dA : dA, eR = dR < 0 ? -dR : dR;
  const bool nA = dA < 0, nR = (dR < 0) != r_flip;
  fe x, y, s, d, m, s2, d2;
  rd(0, eA, 0, x);
  rd(0, eA, 1, y);
  fe_sub(d, y, x);  // Y1 - X1
  fe_add(s, y, x);  // Y1 + X1
  rd(1, eR, 0, x);
  rd(1, eR, 1, y);
  fe_sub(d2, y, x);  // Y2 - X2
  fe_add(s2, y, x);  // Y2 + X2
  fe_select(x, d, s, nA);
  fe_select(m, d2, s2, nR);
  fe_mul(x, x, m);  // A = (Y1 - X1)(Y2 - X2)
  fe_select(y, s, d, nA);
  fe_select(m, s2, d2, nR);
  fe_mul(y, y, m);  // B = (Y1 + X1)(Y2 + X2)
  fe e, h, f, g;
  fe_sub(e, y, x);  // E = B - A
  fe_add(h, y, x);  // H = B + A
  rd(1, eR, 3, m);
  fe_const_d2(d2);
  fe_mul(m, m, d2);  // 2d T2
  rd(0, eA, 3, x);
  fe_mul(x, x, m);  // +/- C = T1 2dT2
  rd(0, eA, 2, y);
  rd(1, eR, 2, m);
  fe_add(m, m, m);
  fe_mul(y, y, m);  // D = Z1 2Z2
  fe_add(s, y, x);  // D + C
  fe_sub(d, y, x);  // D - C
  const bool cneg = nA != nR;
  fe_select(f, d, s, cneg);  // F = D - C
  fe_select(g, s, d, cneg);  // G = D + C
  fe X3, Y3, Z3, T3;
  fe_mul(X3, e, f);
  fe_mul(Y3, g, h);
  fe_mul(Z3, f, g);
  fe_mul(T3, e, h);
  fe_sub(out[0], Y3, X3);
  fe_add(out[1], Y3, X3);
  fe_add(out[2], Z3, Z3);
  fe_const_d2(m);
  fe_mul(out[3], T3, m);
}

// The quad side of the helper-summed verifiers after the decode (v: this
// lane's coordinate of -A, rc: of -R, both extended, Z = 1): both tables,
// then get_prep (the scalars; flags bits 16..23 carry the window count W the
// whole workgroup runs, else this quad's own), the top window from the
// tables, then W - 1 windows of 4 doublings and get_s(win, c) (this lane's
// cached coordinate of the helper's S_win), and get_b(c): the helper's part
// of [u]B, comb positions 15..j0 (BComb16). The quads add positions j0-1..0
// themselves, digit j of u's radix-2^16 digits on the window the remaining
// doublings scale to 2^16j -- j < 8 against (1..2^15)B on window 4j, j >= 8
// against (1..2^15)[2^120]B on window 4(j-8)+2 -- its row fetched before the
// window's doublings. Out: v = this lane's coordinate of X = [k2](R' - R), p.
template <class Q, class BTab, class ATab, class GetPrep, class GetS, class GetB>
CMTV_HD void q_hs_straus(const Q& q, fe& v, fe& rc, const BTab& btab, ATab& tabA, ATab& tabR, int j0, SigPrep& p,
                         const GetPrep& get_prep, const GetS& get_s, const GetB& get_b) {
  const int lane = q.lane();
  q_build_table_p3(q, tabA, v);
  q_build_table_p3(q, tabR, rc);
  get_prep(p);
  const bool r_flip = (p.flags & 1u) != 0;
  const int W = (p.flags >> 16) & 0xFFu ? (int)((p.flags >> 16) & 0xFFu) : q_wave_windows(q, p.flags);
  uint32_t tA[8], tR[8];
  hs_digits16(tA, p.k1, W);
  hs_digits16(tR, p.k2, W);
  uint32_t tLo[8], tHi[8];
  hs_digits65536(tLo, tHi, p.u);
#pragma unroll 1
  for (int j = 15; j >= j0; j--) sc_shift_out(j >= 8 ? tHi : tLo, 16);  // the helper's positions
  fe c;
  {
    // the top window: v = [dA](-A) straight from A's table, + [dR](-/+R)
    const int dA = (int)sc_shift_out(tA, 4) - 8;
    const int dR = (int)sc_shift_out(tR, 4) - 8;
    tabA.load(dA < 0 ? -dA : dA, v);
    fe t, r;
    fe_neg(t, v);
    fe_carry(t);
    fe_select(v, v, t, dA < 0 && (lane == 0 || lane == 3));
    tabR.load(dR < 0 ? -dR : dR, r);
    fe_neg(t, r);
    fe_carry(t);
    fe_select(r, r, t, ((dR < 0) != r_flip) && (lane == 0 || lane == 3));
    q_to_cached(q, c, r);
    q_add(q, v, c);
  }
#pragma unroll 1
  for (int win = W - 2; win >= 0; win--) {
    const bool hi = (win & 2) != 0;
    const bool has_b = (win & 1) == 0 && win <= 30 && (hi ? 8 : 0) + (win >> 2) < j0;
    bool b_neg = false, b_ident = false;
    fe cB;
    if (has_b) {
      const int dB = (int)sc_shift_out(hi ? tHi : tLo, 16) - 0x8000;
      const int ib = dB < 0 ? -dB : dB;
      const int row = BT16_BASE + (ib > 0 ? ib - 1 : 0) + (hi ? BT16_ENTRIES : 0);
      q_niels_load(
          q, cB, [&](int off, fe& r) { btab.load_coord(row, off, r); }, BTAB_COORD_WORDS, 2 * BTAB_COORD_WORDS,
          dB < 0);
      b_neg = dB < 0;
      b_ident = ib == 0;
    }
#pragma unroll 1
    for (int d = 0; d < 4; d++) q_dbl(q, v);
    get_s(win, c);
    q_add(q, v, c);
    if (has_b) {
      q_niels_fix(cB, lane, b_neg, b_ident);
      q_add(q, v, cB);
    }
  }
  get_b(c);
  q_add(q, v, c);
}

// The Ed25519 helper-summed verifier (k_verify_quad_hs): decode as
// q_verify_split, q_hs_straus, the mode's final check
template <uint32_t MODE, class Q, class BTab, class ATab, class GetPrep, class GetS, class GetB>
CMTV_HD bool q_verify_hs(const Q& q, const uint32_t* pk_ptr, const uint32_t* sig_ptr, const BTab& btab, ATab& tabA,
                         ATab& tabR, int j0, const GetPrep& get_prep, const GetS& get_s, const GetB& get_b) {
  const int lane = q.lane();
  uint32_t w[8];
  const uint32_t* src = (lane & 1) ? sig_ptr : pk_ptr;
#pragma unroll
  for (int i = 0; i < 8; i++) w[i] = src[i];
  fe v, rc;
  bool a_ok, r_ok, r_canon;
  {
    ge_p3 P;
    const bool dec = p3_frombytes(P, w);
    const bool canon = y_is_canonical(w) && !(fe_iszero(P.X) && (w[7] >> 31));
    fe x, y, t, one;
    fe_1(one);
    q.template perm<QP_B0>(x, P.X);
    q.template perm<QP_B0>(y, P.Y);
    q.template perm<QP_B0>(t, P.T);
    fe_pick(v, lane, x, y, one, t);  // A
    q.template perm<QP_B1>(x, P.X);
    q.template perm<QP_B1>(y, P.Y);
    q.template perm<QP_B1>(t, P.T);
    fe_pick(rc, lane, x, y, one, t);  // R
    a_ok = q.template perm32<QP_B0>(dec ? 1u : 0u) != 0;
    r_ok = q.template perm32<QP_B1>(dec ? 1u : 0u) != 0;
    r_canon = q.template perm32<QP_B1>(canon ? 1u : 0u) != 0;
    // -A and -R: negate X (lane 0) and T (lane 3)
    const bool xt = lane == 0 || lane == 3;
    fe_neg(t, v);
    fe_carry(t);
    fe_select(v, v, t, xt);
    fe_neg(t, rc);
    fe_carry(t);
    fe_select(rc, rc, t, xt);
  }
  SigPrep p;
  q_hs_straus(q, v, rc, btab, tabA, tabR, j0, p, get_prep, get_s, get_b);
  const bool s_ok = (p.flags & 4u) != 0;
  if (MODE == MODE_ZIP215) {
    const bool so = q_small_order(q, v);
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

// One wave does everything (k_verify_quad; the host checks)
template <uint32_t MODE, class Q, class BTab, class ATab, class Probe = NullProbe>
CMTV_HD bool q_verify(const Q& q, const uint32_t* pk_ptr, const uint32_t* sig_ptr, const uint8_t* msg,
                      uint32_t mlen, const BTab& btab, ATab& tabA, ATab& tabR, const Probe& probe = Probe(),
                      bool force_wide = false) {
  return q_verify_split<MODE>(
      q, pk_ptr, sig_ptr, btab, tabA, tabR,
      [&](SigPrep& p) { q_prepare<MODE>(p, pk_ptr, sig_ptr, msg, mlen, force_wide); }, NoExtB(), probe);
}

}  // namespace cmtv
