// devtables.h -- device-side table policies shared by the gfx950 kernels
// (kernels.hip, sr25519.hip): the fixed-base B table and the per-lane
// (1..8)(-A) table of the one-signature-per-lane Straus (verify_core.h), and
// the quad kernels' B-table, DPP quad and LDS table policies (quad.h).
#pragma once
#include <hip/hip_runtime.h>

#include "oct.h"
#include "quad.h"
#include "verify_core.h"

namespace cmtv {

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
