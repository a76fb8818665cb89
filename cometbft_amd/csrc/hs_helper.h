// hs_helper.h -- the helper wave of the helper-summed quad kernels
// (kernels.hip k_verify_quad_hs, sr25519.hip k_verify_sr25519_quad_hs): the
// workgroup's window count before barrier 1, and after it the per-window sums
// S_w = [dA](-A) + [dR](-/+R) of its 48 signatures (quad.h h_window_addend,
// one per lane) handed to the quads through a 2-slot LDS ring at one barrier
// per window, then the helper's part of [u]B. The quad side is quad.h
// q_hs_straus. Device code only.
#pragma once
#include "devtables.h"
#include "quad.h"

namespace cmtv {

// [u]B's comb positions the helper adds while the quads build their tables
// (the quads add the rest inside their windows); CMTV_HS_PRE overrides it.
// Each one the helper takes saves the quads ~1 us of window time and costs
// barrier 1 ~3 us once the helper arrives last. Ed25519: 6 with the message
// in HBM (the helper reaches barrier 1 with the quads, profiles/
// r05_ed_phase_hbm.json); 3 when the helper builds the sign-bytes itself
// from zero-copy staged templates (the node's commit path: its first loads
// cross PCIe; profiles/r05_hs_pre_ab.txt). sr25519: none -- its merlin
// transcript already brings the helper to barrier 1 with the quads (1 and 2
// measured 1-3% slower, profiles/r05_sr_hs_pre_ab.txt)
constexpr int kHsCombPre = 6, kHsCombPreFused = 3, kHsCombPreSr = 0;
// one ring slot: 3 quad waves x 5 uint2 x 64 lanes
constexpr uint32_t kHsSlotU2 = 3 * 5 * 64;
// a quad wave's two tables in LDS: 2 points x 9 entries x 5 uint2 x 64 lanes
constexpr uint32_t kHsTabU2 = 2 * 9 * 5 * 64;

// the number of [u]B's comb positions the helper takes (launcher's hs_tune
// bits 0..7: CMTV_HS_PRE + 1; 0 = the kernel's default)
__device__ __forceinline__ int hs_comb_pre(uint32_t hs_tune, int dflt) {
  const int c = (hs_tune & 0xFFu) ? (int)(hs_tune & 0xFFu) - 1 : dflt;
  return c > 16 ? 16 : c;
}

// The workgroup's window count: quad.h q_wave_windows over the helper's 48
// signatures (lane t < 48 holds signature t's flags)
__device__ __forceinline__ int hs_workgroup_windows(uint32_t flags, uint32_t t) {
  const bool wide = __ballot(t < 48 && (flags & 2u) != 0) != 0;
  int W = HS_WINDOWS;
#pragma unroll 1
  for (int x = HS_WINDOWS; x < HS_MAX_WINDOWS; x++) W += __ballot(t < 48 && (int)((flags >> 8) & 0xFFu) > x) ? 1 : 0;
  return wide ? HS_WIDE_WINDOWS : W;
}

// After barrier 1: windows W-2 .. 0 (the top one is the quads'), each sum
// written to ring slot (win & 1) before that window's barrier (a slot is
// rewritten only after the quads read it, one barrier later), then [u]B's
// partial sum bc.P in slot 1 before the last barrier. tabs = the workgroup's
// three quad waves' tables, ring = 2 slots; lane t < 48 owns signature t
// (quad wave t >> 4, quad t & 15). Meets W barriers. hwait: cycles spent at
// the window barriers when clock() counts them (the probe build).
template <class Clock>
__device__ __forceinline__ void hs_helper_windows(const SigPrep& p, int W, const BComb16& bc, const uint2* tabs,
                                                  uint2* ring, uint32_t t, const Clock& clock, uint64_t& hwait) {
  const uint32_t slot = t < 48 ? t : 47;
  const bool r_flip = (p.flags & 1u) != 0;
  uint32_t tA[8], tR[8];
  hs_digits16(tA, p.k1, W);
  hs_digits16(tR, p.k2, W);
  sc_shift_out(tA, 4);  // the top window is the quads' own
  sc_shift_out(tR, 4);
  const uint2* tw = tabs + (slot >> 4) * kHsTabU2;
  const uint32_t qb = 4 * (slot & 15);
  auto rd = [&](int P, int e, int c, fe& r) {
    const uint2* src = tw + (P * 9 + e) * 5 * 64 + qb + c;
#pragma unroll
    for (int k = 0; k < 5; k++) {
      const uint2 x = src[k * 64];
      r.v[2 * k] = x.x;
      r.v[2 * k + 1] = x.y;
    }
  };
  auto put = [&](uint2* dst, const fe* out) {
    if (t < 48) {
#pragma unroll
      for (int c = 0; c < 4; c++)
#pragma unroll
        for (int k = 0; k < 5; k++)
          dst[(slot >> 4) * 320 + k * 64 + qb + c] = make_uint2(out[c].v[2 * k], out[c].v[2 * k + 1]);
    }
  };
#pragma unroll 1
  for (int win = W - 2; win >= 0; win--) {
    const int dA = (int)sc_shift_out(tA, 4) - 8;
    const int dR = (int)sc_shift_out(tR, 4) - 8;
    fe out[4];
    h_window_addend(out, rd, dA, dR, r_flip);
    put(ring + (win & 1) * kHsSlotU2, out);
    const uint64_t c0 = clock();
    __syncthreads();  // window win
    hwait += clock() - c0;
  }
  fe out[4], d2;
  fe_sub(out[0], bc.P.Y, bc.P.X);
  fe_add(out[1], bc.P.Y, bc.P.X);
  fe_add(out[2], bc.P.Z, bc.P.Z);
  fe_const_d2(d2);
  fe_mul(out[3], bc.P.T, d2);
  put(ring + kHsSlotU2, out);  // slot 1: last read for window 1, before barrier 0
}

// the quads' read of their coordinate of a ring slot (or of [u]B)
__device__ __forceinline__ void hs_slot_load(const uint2* sl, uint32_t wave, uint32_t t, fe& c) {
#pragma unroll
  for (int k = 0; k < 5; k++) {
    const uint2 x = sl[wave * 320 + k * 64 + t];
    c.v[2 * k] = x.x;
    c.v[2 * k + 1] = x.y;
  }
}

}  // namespace cmtv
