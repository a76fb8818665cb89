// row_dev.h -- the device row policy and LDS table policy of the
// one-signature-per-wave verifier (row.h; k_verify_row_split in kernels.hip,
// tools/microbench/row_lat.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "row.h"

namespace cmtv {

// Row policy (row.h): one signature per wave, a field element per 16-lane
// row. Row moves are DPP (row_ror:r 0x120+r, row_newbcast:r 0x150+r, with
// bound_ctrl off as in DevQuad); the four row broadcasts of a value are one
// v_permlane32_swap and two v_permlane16_swap:
//   permlane32_swap(x, x) = {[x0 x1 x0 x1], [x2 x3 x2 x3]}  (rows)
//   permlane16_swap(y, y) = {[y0 y0 y2 y2], [y1 y1 y3 y3]}
#ifndef CMTV_ROW_FUSED
#define CMTV_ROW_FUSED 1
#endif

// five column terms r .. r+4 of a product: row_ror:r of f, and g_r's
// broadcast times the twist in one v_mul_u32_u24_dpp row_newbcast:r (src0 is
// the DPP operand). The s_nop covers a VALU write of f or g just before (the
// compiler inserts no wait states in front of inline asm).
#define CMTV_ROW_TERM(r, F, G, T)                                                \
  "v_mov_b32_dpp " F ", %[f] row_ror:" #r " row_mask:0xf bank_mask:0xf\n\t"    \
  "v_mul_u32_u24_dpp " G ", %[g], " T " row_newbcast:" #r " row_mask:0xf bank_mask:0xf\n\t"
#define CMTV_ROW_TERMS5(r0, r1, r2, r3, r4)                                                          \
  asm("s_nop 1\n\t" CMTV_ROW_TERM(r0, "%[a0]", "%[b0]", "%[t0]") CMTV_ROW_TERM(r1, "%[a1]", "%[b1]", "%[t1]") \
          CMTV_ROW_TERM(r2, "%[a2]", "%[b2]", "%[t2]") CMTV_ROW_TERM(r3, "%[a3]", "%[b3]", "%[t3]")             \
              CMTV_ROW_TERM(r4, "%[a4]", "%[b4]", "%[t4]")                                                     \
      : [a0] "=&v"(fr[r0]), [b0] "=&v"(gt[r0]), [a1] "=&v"(fr[r1]), [b1] "=&v"(gt[r1]), [a2] "=&v"(fr[r2]),  \
        [b2] "=&v"(gt[r2]), [a3] "=&v"(fr[r3]), [b3] "=&v"(gt[r3]), [a4] "=&v"(fr[r4]), [b4] "=&v"(gt[r4])    \
      : [f] "v"(f), [g] "v"(g), [t0] "v"(tw[r0]), [t1] "v"(tw[r1]), [t2] "v"(tw[r2]), [t3] "v"(tw[r3]),      \
        [t4] "v"(tw[r4]))

#ifndef CMTV_ROW_ASM_BLOCKS
#define CMTV_ROW_ASM_BLOCKS 1
#endif
// all fifteen terms in one asm block: one s_nop instead of three
#define CMTV_ROW_TERMS15()                                                                                     \
  asm("s_nop 1\n\t" CMTV_ROW_TERM(1, "%[a1]", "%[b1]", "%[t1]") CMTV_ROW_TERM(2, "%[a2]", "%[b2]", "%[t2]")      \
          CMTV_ROW_TERM(3, "%[a3]", "%[b3]", "%[t3]") CMTV_ROW_TERM(4, "%[a4]", "%[b4]", "%[t4]")                  \
              CMTV_ROW_TERM(5, "%[a5]", "%[b5]", "%[t5]") CMTV_ROW_TERM(6, "%[a6]", "%[b6]", "%[t6]")              \
                  CMTV_ROW_TERM(7, "%[a7]", "%[b7]", "%[t7]") CMTV_ROW_TERM(8, "%[a8]", "%[b8]", "%[t8]")          \
                      CMTV_ROW_TERM(9, "%[a9]", "%[b9]", "%[t9]") CMTV_ROW_TERM(10, "%[a10]", "%[b10]", "%[t10]")  \
                          CMTV_ROW_TERM(11, "%[a11]", "%[b11]", "%[t11]")                                          \
                              CMTV_ROW_TERM(12, "%[a12]", "%[b12]", "%[t12]")                                      \
                                  CMTV_ROW_TERM(13, "%[a13]", "%[b13]", "%[t13]")                                  \
                                      CMTV_ROW_TERM(14, "%[a14]", "%[b14]", "%[t14]")                              \
                                          CMTV_ROW_TERM(15, "%[a15]", "%[b15]", "%[t15]")                          \
      : [a1] "=&v"(fr[1]), [b1] "=&v"(gt[1]), [a2] "=&v"(fr[2]), [b2] "=&v"(gt[2]), [a3] "=&v"(fr[3]),             \
        [b3] "=&v"(gt[3]), [a4] "=&v"(fr[4]), [b4] "=&v"(gt[4]), [a5] "=&v"(fr[5]), [b5] "=&v"(gt[5]),             \
        [a6] "=&v"(fr[6]), [b6] "=&v"(gt[6]), [a7] "=&v"(fr[7]), [b7] "=&v"(gt[7]), [a8] "=&v"(fr[8]),             \
        [b8] "=&v"(gt[8]), [a9] "=&v"(fr[9]), [b9] "=&v"(gt[9]), [a10] "=&v"(fr[10]), [b10] "=&v"(gt[10]),         \
        [a11] "=&v"(fr[11]), [b11] "=&v"(gt[11]), [a12] "=&v"(fr[12]), [b12] "=&v"(gt[12]), [a13] "=&v"(fr[13]),   \
        [b13] "=&v"(gt[13]), [a14] "=&v"(fr[14]), [b14] "=&v"(gt[14]), [a15] "=&v"(fr[15]), [b15] "=&v"(gt[15])    \
      : [f] "v"(f), [g] "v"(g), [t1] "v"(tw[1]), [t2] "v"(tw[2]), [t3] "v"(tw[3]), [t4] "v"(tw[4]),             \
        [t5] "v"(tw[5]), [t6] "v"(tw[6]), [t7] "v"(tw[7]), [t8] "v"(tw[8]), [t9] "v"(tw[9]), [t10] "v"(tw[10]),  \
        [t11] "v"(tw[11]), [t12] "v"(tw[12]), [t13] "v"(tw[13]), [t14] "v"(tw[14]), [t15] "v"(tw[15]))

// the split products' terms (row.h rf_mul_s): term 0 is F times g_0's
// twisted broadcast (row_newbcast:0), terms 1.. as CMTV_ROW_TERM
#define CMTV_ROW_BTERM0 "v_mul_u32_u24_dpp %[b0], %[g], %[t0] row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"

struct DevRow {
  using U = uint32_t;
  using U64 = uint64_t;
  using B = bool;
  static constexpr bool kFusedProduct = CMTV_ROW_FUSED != 0;
  // the column sums of f g: 15 rotations and 15 fused twisted broadcasts in
  // three asm blocks, 16 v_mad_u64_u32
  __device__ __forceinline__ static uint64_t product(const uint32_t* tw, uint32_t f, uint32_t g) {
    uint32_t fr[16], gt[16];
#if CMTV_ROW_ASM_BLOCKS == 1
    CMTV_ROW_TERMS15();
#else
    CMTV_ROW_TERMS5(1, 2, 3, 4, 5);
    CMTV_ROW_TERMS5(6, 7, 8, 9, 10);
    CMTV_ROW_TERMS5(11, 12, 13, 14, 15);
#endif
    uint64_t acc = (uint64_t)f * (uint32_t)__builtin_amdgcn_mov_dpp((int)g, 0x150, 0xF, 0xF, false);
#pragma unroll
    for (int r = 1; r < 16; r++) acc += (uint64_t)fr[r] * gt[r];
    return acc;
  }
  // the 16 / S column terms of a split product (row.h rf_split_terms) on the
  // rotated operands F, G, with the twists tw[0 .. 16/S)
  template <int S>
  __device__ __forceinline__ static uint64_t product_split(const uint32_t* tw, uint32_t f, uint32_t g) {
    uint32_t fr[8], gt[8];
    if constexpr (S == 4) {
      asm("s_nop 1\n\t" CMTV_ROW_BTERM0 CMTV_ROW_TERM(1, "%[a1]", "%[b1]", "%[t1]")
              CMTV_ROW_TERM(2, "%[a2]", "%[b2]", "%[t2]") CMTV_ROW_TERM(3, "%[a3]", "%[b3]", "%[t3]")
          : [b0] "=&v"(gt[0]), [a1] "=&v"(fr[1]), [b1] "=&v"(gt[1]), [a2] "=&v"(fr[2]), [b2] "=&v"(gt[2]),
            [a3] "=&v"(fr[3]), [b3] "=&v"(gt[3])
          : [f] "v"(f), [g] "v"(g), [t0] "v"(tw[0]), [t1] "v"(tw[1]), [t2] "v"(tw[2]), [t3] "v"(tw[3]));
    } else {
      static_assert(S == 2, "split products share 2 or 4 rows");
      asm("s_nop 1\n\t" CMTV_ROW_BTERM0 CMTV_ROW_TERM(1, "%[a1]", "%[b1]", "%[t1]")
              CMTV_ROW_TERM(2, "%[a2]", "%[b2]", "%[t2]") CMTV_ROW_TERM(3, "%[a3]", "%[b3]", "%[t3]")
                  CMTV_ROW_TERM(4, "%[a4]", "%[b4]", "%[t4]") CMTV_ROW_TERM(5, "%[a5]", "%[b5]", "%[t5]")
                      CMTV_ROW_TERM(6, "%[a6]", "%[b6]", "%[t6]") CMTV_ROW_TERM(7, "%[a7]", "%[b7]", "%[t7]")
          : [b0] "=&v"(gt[0]), [a1] "=&v"(fr[1]), [b1] "=&v"(gt[1]), [a2] "=&v"(fr[2]), [b2] "=&v"(gt[2]),
            [a3] "=&v"(fr[3]), [b3] "=&v"(gt[3]), [a4] "=&v"(fr[4]), [b4] "=&v"(gt[4]), [a5] "=&v"(fr[5]),
            [b5] "=&v"(gt[5]), [a6] "=&v"(fr[6]), [b6] "=&v"(gt[6]), [a7] "=&v"(fr[7]), [b7] "=&v"(gt[7])
          : [f] "v"(f), [g] "v"(g), [t0] "v"(tw[0]), [t1] "v"(tw[1]), [t2] "v"(tw[2]), [t3] "v"(tw[3]),
            [t4] "v"(tw[4]), [t5] "v"(tw[5]), [t6] "v"(tw[6]), [t7] "v"(tw[7]));
    }
    uint64_t acc = (uint64_t)f * gt[0];
#pragma unroll
    for (int r = 1; r < 16 / S; r++) acc += (uint64_t)fr[r] * gt[r];
    return acc;
  }
  // rows 1..3 rotated by A1..A3 (row_ror; 0: as is), row 0 as is: DPP moves
  // with a row mask onto a copy
  template <int A1, int A2, int A3>
  __device__ __forceinline__ static U ror_rows(U x) {
    U r = x;
    if constexpr (A1 != 0) r = (uint32_t)__builtin_amdgcn_update_dpp((int)r, (int)x, 0x120 + A1, 0x2, 0xF, false);
    if constexpr (A2 != 0 && A2 == A3) {
      r = (uint32_t)__builtin_amdgcn_update_dpp((int)r, (int)x, 0x120 + A2, 0xC, 0xF, false);
    } else {
      if constexpr (A2 != 0) r = (uint32_t)__builtin_amdgcn_update_dpp((int)r, (int)x, 0x120 + A2, 0x4, 0xF, false);
      if constexpr (A3 != 0) r = (uint32_t)__builtin_amdgcn_update_dpp((int)r, (int)x, 0x120 + A3, 0x8, 0xF, false);
    }
    return r;
  }
  // S = 2: rows c and c ^ 2 summed (v_permlane32_swap: {[x0 x1 x0 x1], [x2 x3 x2 x3]});
  // S = 4: then rows c and c ^ 1 (v_permlane16_swap): the four-row sum everywhere
  template <int S>
  __device__ __forceinline__ static uint64_t sum_rows(uint64_t x) {
    uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
    {
      const auto l = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
      const auto h = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
      x = (((uint64_t)h[0] << 32) | l[0]) + (((uint64_t)h[1] << 32) | l[1]);
    }
    if constexpr (S == 4) {
      lo = (uint32_t)x;
      hi = (uint32_t)(x >> 32);
      const auto l = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
      const auto h = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
      x = (((uint64_t)h[0] << 32) | l[0]) + (((uint64_t)h[1] << 32) | l[1]);
    }
    return x;
  }
  __device__ __forceinline__ static U lane() { return threadIdx.x & 63; }
  template <int R>
  __device__ __forceinline__ static U ror(U x) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x120 + R, 0xF, 0xF, false);
  }
  template <int R>
  __device__ __forceinline__ static U bcast(U x) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x150 + R, 0xF, 0xF, false);
  }
  __device__ __forceinline__ static void rows(U x, U& b0, U& b1, U& b2, U& b3) {
    const auto h = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    const auto lo = __builtin_amdgcn_permlane16_swap(h[0], h[0], false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap(h[1], h[1], false, false);
    b0 = lo[0];
    b1 = lo[1];
    b2 = hi[0];
    b3 = hi[1];
  }
  __device__ __forceinline__ static uint64_t ballot(bool b) { return __ballot(b); }
  __device__ __forceinline__ static U load_const(const uint16_t* tab, U k) { return tab[k]; }
  // this lane's 16-bit limb of the 10-limb (radix 2^25.5) value at word off
  // of row: its canonical encoding (fe_tobytes), word k / 2
  __device__ __forceinline__ static U niels_limb(const uint32_t* row, U off) {
    const uint32_t* p = row + off;
    fe f;
#pragma unroll
    for (int i = 0; i < 10; i++) f.v[i] = p[i];
    uint32_t b[8];
    fe_tobytes(b, f);
    const uint32_t k = threadIdx.x & 15u;
    uint32_t w = b[0];
#pragma unroll
    for (int i = 1; i < 8; i++) w = (k >> 1) == (uint32_t)i ? b[i] : w;
    return (w >> (16 * (k & 1))) & 0xFFFFu;
  }
};

// the row verifier's (0..8)(-A), (0..8)(-R) cached tables, both signs: one
// LDS word per lane per entry (a lookup is one ds_read_b32)
struct DevRowTab {
  uint32_t* t;
  uint32_t lane;
  __device__ __forceinline__ void store(int tb, int neg, int e, uint32_t c) { t[((tb * 2 + neg) * 9 + e) * 64 + lane] = c; }
  __device__ __forceinline__ uint32_t load(int tb, int neg, int e) const { return t[((tb * 2 + neg) * 9 + e) * 64 + lane]; }
};
constexpr int kRowTabWords = 2 * 2 * 9 * 64;

}  // namespace cmtv
