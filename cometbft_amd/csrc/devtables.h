// devtables.h -- device-side table policies shared by the gfx950 kernels
// (kernels.hip, sr25519.hip): the fixed-base B table and the per-lane
// (1..8)(-A) table of the one-signature-per-lane Straus (verify_core.h).
#pragma once
#include <hip/hip_runtime.h>

#include "verify_core.h"

namespace cmtv {

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

}  // namespace cmtv
