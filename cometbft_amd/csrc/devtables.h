// devtables.h -- device-side table policies shared by the gfx950 kernels
// (kernels.hip, sr25519.hip): the fixed-base B table and the per-lane
// (1..8)(-A) table of the one-signature-per-lane Straus (verify_core.h), and
// the quad kernels' B-table, DPP quad and LDS table policies (quad.h).
#pragma once
#include <hip/hip_runtime.h>

#include "keyed.h"
#include "oct.h"
#include "quad.h"
#include "row_dev.h"
#include "verify_core.h"

namespace cmtv {

__device__ __forceinline__ void load_words(uint32_t* w, const uint32_t* __restrict__ src, int nquads) {
  const uint4* p = reinterpret_cast<const uint4*>(src);
#pragma unroll
  for (int q = 0; q < nquads; q++) {
    const uint4 v = p[q];
    w[4 * q] = v.x;
    w[4 * q + 1] = v.y;
    w[4 * q + 2] = v.z;
    w[4 * q + 3] = v.w;
  }
}

// Prefix products of comb_build_column, word-major / lane-minor per launch.
struct DevCombScratch {
  uint32_t* __restrict__ base;
  uint32_t stride;
  uint32_t lane;
  __device__ __forceinline__ void store(int j, const fe& v) {
#pragma unroll
    for (int i = 0; i < 10; i++) base[(size_t)(j * 10 + i) * stride + lane] = v.v[i];
  }
  __device__ __forceinline__ void load(int j, fe& v) const {
#pragma unroll
    for (int i = 0; i < 10; i++) v.v[i] = base[(size_t)(j * 10 + i) * stride + lane];
  }
};

// One comb window as a table source: 32-word rows, coordinates at 8-byte
// aligned offsets 0 / 40 / 80 bytes -> 5 x dwordx2 per coordinate.
struct DevCombWindow {
  const uint32_t* __restrict__ rows;
  __device__ __forceinline__ void load_fe(int e, int c, fe& r) const {
    const uint2* p = reinterpret_cast<const uint2*>(rows + e * COMB_ROW_WORDS + c * 10);
#pragma unroll
    for (int i = 0; i < 5; i++) {
      const uint2 v = p[i];
      r.v[2 * i] = v.x;
      r.v[2 * i + 1] = v.y;
    }
  }
};

// wave-uniform predicate (verify_one_half's loop bound)
struct DevWave {
  __device__ __forceinline__ bool any(bool x) const { return __ballot(x) != 0; }
};

struct DevBTab {
  const uint32_t* __restrict__ rows;
  // one niels coordinate (10 words at a 16-byte aligned offset): 2 x dwordx4 + dwordx2
  __device__ __forceinline__ void load_fe(int e, int c, fe& r) const {
    const uint32_t* p = rows + e * BTAB_ROW_WORDS + c * BTAB_COORD_WORDS;
    const uint4 a = *reinterpret_cast<const uint4*>(p);
    const uint4 b = *reinterpret_cast<const uint4*>(p + 4);
    const uint2 d = *reinterpret_cast<const uint2*>(p + 8);
    r.v[0] = a.x; r.v[1] = a.y; r.v[2] = a.z; r.v[3] = a.w;
    r.v[4] = b.x; r.v[5] = b.y; r.v[6] = b.z; r.v[7] = b.w;
    r.v[8] = d.x; r.v[9] = d.y;
  }
};

// Per-lane (1..8)(-A) table, word-major / lane-minor: word w of entry e for
// lane l lives at base[(e * 40 + w) * stride + l], so a wave's load of one
// word is a 256-byte coalesced access whenever its lanes share the entry.
struct DevATab {
  uint32_t* __restrict__ base;
  uint32_t stride;
  uint32_t lane;
  __device__ __forceinline__ void load_fe(int e, int c, fe& r) const {
    const uint32_t* p = base + (uint32_t)((e * 4 + c) * 10) * stride + lane;
#pragma unroll
    for (int i = 0; i < 10; i++) r.v[i] = p[i * stride];
  }
  __device__ __forceinline__ void store(int e, const ge_cached& r) {
    uint32_t* p = base + (uint32_t)(e * 40) * stride + lane;
#pragma unroll
    for (int i = 0; i < 10; i++) {
      p[i * stride] = r.YpX.v[i];
      p[(10 + i) * stride] = r.YmX.v[i];
      p[(20 + i) * stride] = r.Z.v[i];
      p[(30 + i) * stride] = r.T2d.v[i];
    }
  }
};


// B-table access for the quad kernel: each lane reads its own coordinate
// (word offset `off` inside the row) of entry e.
struct DevBTabQ {
  const uint32_t* __restrict__ rows;
  __device__ __forceinline__ void load_coord(int e, int off, fe& r) const {
    const uint32_t* p = rows + e * BTAB_ROW_WORDS + off;
    const uint4 a = *reinterpret_cast<const uint4*>(p);
    const uint4 b = *reinterpret_cast<const uint4*>(p + 4);
    const uint2 d = *reinterpret_cast<const uint2*>(p + 8);
    r.v[0] = a.x; r.v[1] = a.y; r.v[2] = a.z; r.v[3] = a.w;
    r.v[4] = b.x; r.v[5] = b.y; r.v[6] = b.z; r.v[7] = b.w;
    r.v[8] = d.x; r.v[9] = d.y;
  }
};

// Quad policy (quad.h): 4 consecutive lanes = one signature; operand exchange
// inside the quad is a DPP quad_perm move. mov_dpp with bound_ctrl off: one
// v_mov_b32_dpp per word (update_dpp(old = src) costs an extra v_mov for the
// tied old operand), and DPP-combine leaves it alone -- the bound_ctrl:1 form
// miscompiles on ROCm 7.2 / gfx950 once DPP-combine folds it into its
// consumers (lanes 0-1 of a quad read wrong values; tools/dbg/quad_debug.hip).
struct DevQuad {
  __device__ __forceinline__ int lane() const { return threadIdx.x & 3; }
  template <int PAT>
  __device__ __forceinline__ uint32_t dpp(uint32_t x) const {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, PAT, 0xF, 0xF, false);
  }
  template <int PAT>
  __device__ __forceinline__ void perm(fe& o, const fe& v) const {
#pragma unroll
    for (int i = 0; i < 10; i++) o.v[i] = dpp<PAT>(v.v[i]);
  }
  template <int PAT>
  __device__ __forceinline__ uint32_t perm32(uint32_t x) const {
    return dpp<PAT>(x);
  }
  // Fused quad moves (quad.h, FOLD = 2): a DPP quad_perm read as the first
  // operand of the 32-bit VOP2 that consumes it, written out as one asm
  // block per field element -- ROCm 7.2's DPP-combine folds only some of
  // them, and its bound_ctrl:1 folds miscompiled. Each block
  // starts with s_nop 1: the two wait states a DPP read needs after the VALU
  // that wrote its source (the compiler inserts none in front of inline asm);
  // inside a block no DPP source is written.
  //   add_perm:  o = perm(src) + b        v_add_u32_dpp
  //   xor_perm:  o = perm(src) ^ k        v_xor_b32_dpp
  //   perm_lane3: o = lane 3 ? perm(src) : 0   v_cndmask_b32_dpp (vcc = lanes 0-2)
#define CMTV_DPP10_CND(PATS)                                                                                 \
  "s_nop 1\n"                                                                                               \
  "v_cndmask_b32_dpp %0, %10, %20, vcc " PATS "\n v_cndmask_b32_dpp %1, %11, %20, vcc " PATS                \
  "\n v_cndmask_b32_dpp %2, %12, %20, vcc " PATS "\n v_cndmask_b32_dpp %3, %13, %20, vcc " PATS             \
  "\n v_cndmask_b32_dpp %4, %14, %20, vcc " PATS "\n v_cndmask_b32_dpp %5, %15, %20, vcc " PATS             \
  "\n v_cndmask_b32_dpp %6, %16, %20, vcc " PATS "\n v_cndmask_b32_dpp %7, %17, %20, vcc " PATS             \
  "\n v_cndmask_b32_dpp %8, %18, %20, vcc " PATS "\n v_cndmask_b32_dpp %9, %19, %20, vcc " PATS "\n"
#define CMTV_QP_STR(a, b, c, d) "quad_perm:[" #a "," #b "," #c "," #d "] row_mask:0xf bank_mask:0xf"
#define CMTV_DPP10(OP, PATS)                                                                                 \
  "s_nop 1\n"                                                                                               \
  OP " %0, %10, %20 " PATS "\n" OP " %1, %11, %21 " PATS "\n" OP " %2, %12, %22 " PATS "\n" OP            \
     " %3, %13, %23 " PATS "\n" OP " %4, %14, %24 " PATS "\n" OP " %5, %15, %25 " PATS "\n" OP             \
     " %6, %16, %26 " PATS "\n" OP " %7, %17, %27 " PATS "\n" OP " %8, %18, %28 " PATS "\n" OP            \
     " %9, %19, %29 " PATS "\n"
#define CMTV_DPP10_K(OP, PATS)                                                                               \
  "s_nop 1\n"                                                                                               \
  OP " %0, %10, %20 " PATS "\n" OP " %1, %11, %20 " PATS "\n" OP " %2, %12, %20 " PATS "\n" OP            \
     " %3, %13, %20 " PATS "\n" OP " %4, %14, %20 " PATS "\n" OP " %5, %15, %20 " PATS "\n" OP             \
     " %6, %16, %20 " PATS "\n" OP " %7, %17, %20 " PATS "\n" OP " %8, %18, %20 " PATS "\n" OP            \
     " %9, %19, %20 " PATS "\n"
#define CMTV_FE_OUT(o)                                                                                       \
  "=&v"(o.v[0]), "=&v"(o.v[1]), "=&v"(o.v[2]), "=&v"(o.v[3]), "=&v"(o.v[4]), "=&v"(o.v[5]), "=&v"(o.v[6]),   \
      "=&v"(o.v[7]), "=&v"(o.v[8]), "=&v"(o.v[9])
#define CMTV_FE_IN(x)                                                                                        \
  "v"(x.v[0]), "v"(x.v[1]), "v"(x.v[2]), "v"(x.v[3]), "v"(x.v[4]), "v"(x.v[5]), "v"(x.v[6]), "v"(x.v[7]),     \
      "v"(x.v[8]), "v"(x.v[9])
#define CMTV_QP_CASES(BODY)                                                                                  \
  if constexpr (PAT == 0x55) { BODY(CMTV_QP_STR(1, 1, 1, 1)); }                                               \
  else if constexpr (PAT == (0 | (1 << 2) | (2 << 4) | (0 << 6))) { BODY(CMTV_QP_STR(0, 1, 2, 0)); }           \
  else if constexpr (PAT == 2) { BODY(CMTV_QP_STR(2, 0, 0, 0)); }                                             \
  else if constexpr (PAT == (0 | (3 << 2) | (3 << 4) | (0 << 6))) { BODY(CMTV_QP_STR(0, 3, 3, 0)); }           \
  else if constexpr (PAT == (1 | (2 << 2) | (2 << 4) | (1 << 6))) { BODY(CMTV_QP_STR(1, 2, 2, 1)); }           \
  else { static_assert(PAT < 0, "quad_perm pattern without an asm string"); }
  template <int PAT>
  __device__ __forceinline__ void add_perm(fe& o, const fe& src, const fe& b) const {
#define CMTV_BODY(PATS) asm volatile(CMTV_DPP10("v_add_u32_dpp", PATS) : CMTV_FE_OUT(o) : CMTV_FE_IN(src), CMTV_FE_IN(b))
    CMTV_QP_CASES(CMTV_BODY)
#undef CMTV_BODY
  }
  template <int PAT>
  __device__ __forceinline__ void xor_perm(fe& o, const fe& src, uint32_t k) const {
#define CMTV_BODY(PATS) asm volatile(CMTV_DPP10_K("v_xor_b32_dpp", PATS) : CMTV_FE_OUT(o) : CMTV_FE_IN(src), "v"(k))
    CMTV_QP_CASES(CMTV_BODY)
#undef CMTV_BODY
  }
  template <int PAT>
  __device__ __forceinline__ void perm_lane3(fe& o, const fe& src) const {
    // vcc = lanes other than 3 of each quad; v_cndmask_b32 o = vcc ? 0 : perm(src)
    const uint64_t keep = 0x7777777777777777ull;
    const uint32_t zero = 0;
#define CMTV_BODY(PATS)                                                                                      \
  asm volatile("s_mov_b64 vcc, %21\n" CMTV_DPP10_CND(PATS)                                                  \
               : CMTV_FE_OUT(o)                                                                              \
               : CMTV_FE_IN(src), "v"(zero), "s"(keep)                                                      \
               : "vcc")
    CMTV_QP_CASES(CMTV_BODY)
#undef CMTV_BODY
  }
  // A move meant to fold into its one consumer: update_dpp(old = 0), which
  // DPP-combine turns into that VOP2's own DPP operand (v_add_u32_dpp,
  // v_and_b32_dpp, v_xor_b32_dpp ...; quad_perm reads no invalid lane, so
  // the zero old value never shows). Use only where the result has a single
  // VOP2 use: otherwise it stays a move.
  template <int PAT>
  __device__ __forceinline__ void permc(fe& o, const fe& v) const {
#pragma unroll
    for (int i = 0; i < 10; i++) o.v[i] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v.v[i], PAT, 0xF, 0xF, false);
  }
  __device__ __forceinline__ bool any(bool x) const { return __ballot(x) != 0; }
};

// Oct policy (oct.h): two quads per signature; the upper quad's words reach
// the lower one by a DPP row shift (lane i <- lane i + 4, inside a 16-lane row).
struct DevOct : DevQuad {
  __device__ __forceinline__ bool upper() const { return (threadIdx.x & 4) != 0; }
  __device__ __forceinline__ uint32_t from_upper32(uint32_t x) const {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x104 /* row_shl:4 */, 0xF, 0xF, false);
  }
  __device__ __forceinline__ void from_upper(fe& o, const fe& v) const {
#pragma unroll
    for (int i = 0; i < 10; i++) o.v[i] = from_upper32(v.v[i]);
  }
};

// Quad (0..8)(-A) table in LDS: entry e, limb pair k of lane t at
// slot (e * 5 + k) * 64 + t -- a wave's ds_read_b64 covers 512 contiguous
// bytes whatever entries its 16 signatures pick, so lookups are conflict-free.
struct DevATabQ {
  uint2* lds;
  uint32_t t;
  __device__ __forceinline__ void store(int e, const fe& c) {
#pragma unroll
    for (int k = 0; k < 5; k++) lds[(e * 5 + k) * 64 + t] = make_uint2(c.v[2 * k], c.v[2 * k + 1]);
  }
  __device__ __forceinline__ void load(int e, fe& c) const {
#pragma unroll
    for (int k = 0; k < 5; k++) {
      const uint2 x = lds[(e * 5 + k) * 64 + t];
      c.v[2 * k] = x.x;
      c.v[2 * k + 1] = x.y;
    }
  }
  // (neg ? -P_e : P_e): lanes 0/1 read each other's slot (Y-X <-> Y+X),
  // lane 3 negates 2dT
  template <class Q>
  __device__ __forceinline__ void load_signed(const Q& q, int e, bool neg, fe& c) const {
    const uint32_t src = (t & 2) ? t : (t ^ (neg ? 1u : 0u));
#pragma unroll
    for (int k = 0; k < 5; k++) {
      const uint2 x = lds[(e * 5 + k) * 64 + src];
      c.v[2 * k] = x.x;
      c.v[2 * k + 1] = x.y;
    }
    q_negate_lane3(c, (int)(t & 3), neg);
  }
};



}  // namespace cmtv
