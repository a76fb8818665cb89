// sr25519_quad.h -- sr25519 verification with one signature per quad of lanes
// (the Ed25519 quad kernel's structure, quad.h), for latency-bound batches.
//
// Same verdict as sr_verify_one (sr25519.h; crypto/sr25519/pubkey.go:34-60).
// The ristretto equality R'.Equal(R) holds iff R' - R lies in the 4-torsion
// E[4] = {(0, +-1), (+-i, 0)}, i.e. iff that difference has X = 0 or Y = 0
// (checked against the big-int oracle for points with arbitrary torsion
// components). With the half-size pair of k (halfscalar.h) the kernel forms
// X = [k2](R' - R); k2 is odd, so gcd(k2, 8L) = 1 and X lies in E[4] iff
// R' - R does: accept iff X.X = 0 or X.Y = 0.
//
// Per quad: every lane runs the merlin transcript (the same bytes; the State
// policy gives each lane its own slot), lanes {0,2} decode A and {1,3}
// decode R, then the quad Straus (q_straus_prep). The split kernel moves the
// transcript and the half-size split to a helper wave (sr_prepare).
#pragma once
#include "quad.h"
#include "sr25519.h"

namespace cmtv {

// The scalar half of an sr25519 quad verification (no decoded points
// needed): schnorrkel marker and canonical s, the merlin challenge k mod L,
// the half-size pair and u = k2 s mod L. k_verify_sr25519_quad_hs runs it on
// its helper wave.
struct NoMark {
  CMTV_HD void operator()() const {}
};

template <class State, class Mark = NoMark>
CMTV_HD void sr_prepare(SigPrep& p, const uint32_t* pk_ptr, const uint32_t* sig_ptr, const uint8_t* msg,
                        uint32_t mlen, const uint32_t* prog, int nops, State& st, bool force_wide,
                        const Mark& after_transcript = Mark()) {
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
  uint32_t k[8];
  {
    uint32_t kb[16];
    sr_transcript(kb, st, prog, nops, msg, mlen, pk, rw);
    after_transcript();
    sc_reduce512(k, kb);
  }
  q_prepare_scalars(p, k, ts, force_wide);
  p.flags |= s_ok ? 4u : 0u;
}

// The point half, with the scalars from get_prep(SigPrep&) (called after the
// decompression by every lane of the wave).
template <bool EXT_B = false, class Q, class BTab, class ATab, class GetPrep, class GetB = NoExtB,
          class Probe = NullProbe>
CMTV_HD bool q_verify_sr_split(const Q& q, const uint32_t* pk_ptr, const uint32_t* sig_ptr, const BTab& btab,
                               ATab& tabA, ATab& tabR, const GetPrep& get_prep, const GetB& get_b = GetB(),
                               const Probe& probe = Probe()) {
  const int lane = q.lane();
  // ---- decode A (even lanes) and R (odd lanes), broadcast coordinates
  fe v, rc;
  bool a_ok, r_ok;
  {
    uint32_t w[8];
#pragma unroll
    for (int i = 0; i < 8; i++) w[i] = (lane & 1) ? sig_ptr[i] : pk_ptr[i];
    ge_p3 P;
    const bool dec = ristretto_decode(P, w);
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
    // -A: negate X (lane 0) and T (lane 3)
    fe_neg(t, v);
    fe_carry(t);
    fe_select(v, v, t, lane == 0 || lane == 3);
  }
  probe.snap(0, v);
  probe.snap(1, rc);
  // split kernel (EXT_B): the tables are built while the helper runs the
  // transcript; the one-wave kernel's STROBE states live in the table LDS
  // until its own transcript is done, so it builds them after get_prep
  if constexpr (EXT_B) q_tables_early(q, v, rc, tabA, tabR);
  SigPrep p;
  get_prep(p);
  const bool s_ok = (p.flags & 4u) != 0;

  q_straus_prep_b<EXT_B, EXT_B>(q, v, rc, p, btab, tabA, tabR, probe, get_b);

  // ---- X in E[4]: X.X = 0 (lane 0) or X.Y = 0 (lane 1)
  const bool z = fe_iszero(v);
  const bool e0 = q.template perm32<QP_B0>(z ? 1u : 0u) != 0;
  const bool e1 = q.template perm32<QP_B1>(z ? 1u : 0u) != 0;
  return s_ok && a_ok && r_ok && (e0 || e1);
}

// The helper-summed form (k_verify_sr25519_quad_hs): the ristretto decode as
// q_verify_sr_split, the windows of quad.h q_hs_straus (the helper wave adds
// every window's two table entries), the E[4] check
template <class Q, class BTab, class ATab, class GetPrep, class GetS, class GetB>
CMTV_HD bool q_verify_sr_hs(const Q& q, const uint32_t* pk_ptr, const uint32_t* sig_ptr, const BTab& btab,
                            ATab& tabA, ATab& tabR, int j0, const GetPrep& get_prep, const GetS& get_s,
                            const GetB& get_b) {
  const int lane = q.lane();
  fe v, rc;
  bool a_ok, r_ok;
  {
    uint32_t w[8];
#pragma unroll
    for (int i = 0; i < 8; i++) w[i] = (lane & 1) ? sig_ptr[i] : pk_ptr[i];
    ge_p3 P;
    const bool dec = ristretto_decode(P, w);
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
  // ---- X in E[4]: X.X = 0 (lane 0) or X.Y = 0 (lane 1)
  const bool z = fe_iszero(v);
  const bool e0 = q.template perm32<QP_B0>(z ? 1u : 0u) != 0;
  const bool e1 = q.template perm32<QP_B1>(z ? 1u : 0u) != 0;
  return s_ok && a_ok && r_ok && (e0 || e1);
}

// One wave does everything (k_verify_sr25519_quad; the host checks)
template <class Q, class BTab, class ATab, class State, class Probe = NullProbe>
CMTV_HD bool q_verify_sr(const Q& q, const uint32_t* pk_ptr, const uint32_t* sig_ptr, const uint8_t* msg,
                         uint32_t mlen, const uint32_t* prog, int nops, State& st, const BTab& btab, ATab& tabA,
                         ATab& tabR, const Probe& probe = Probe(), bool force_wide = false) {
  return q_verify_sr_split(
      q, pk_ptr, sig_ptr, btab, tabA, tabR,
      [&](SigPrep& p) { sr_prepare(p, pk_ptr, sig_ptr, msg, mlen, prog, nops, st, force_wide); }, NoExtB(),
      probe);
}

}  // namespace cmtv
