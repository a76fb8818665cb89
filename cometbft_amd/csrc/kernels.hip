// kernels.hip -- gfx950 kernels of libcmtverify.
//
//   k_btab_init   : builds the shared fixed-base table (1..128)B (affine niels)
//   k_verify<MODE>: one signature per lane: SHA-512 + mod-L + decompression +
//                   Straus [s]B - [k]A + GO_STDLIB / ZIP215 final check, then a
//                   wavefront ballot packs 64 verdicts into one bitmap word
//   k_verify_quad_hs / k_verify_oct_split / k_verify_row_split /
//   k_verify_row4_split<MODE>: the same with 4 / 8 / 64 / 256 lanes per
//                   signature and a helper wave (smaller batches; kernels.h forms)
//   k_comb_build  : registered-key combs (keyed.h), one workgroup per key
//   k_verify_keyed_row_split / k_verify_keyed_quad_split<MODE>: one signature
//                   per workgroup / per quad of lanes against a registered key
//                   (the lane kernels: keyed_lane.hip)
//   k_pubkey / k_sign : RFC 8032 key generation and signing (synthetic data)
//
// Memory layout (HBM):
//   pk   : n x 32 B   (row i = 8 words, read as 2 x dwordx4)
//   sig  : n x 64 B   (row i = 16 words, 4 x dwordx4)
//   msg  : flat bytes + (n+1) u32 offsets
//   btab : 2 x 128 rows x 36 words (ypx, ymx, 2dxy; 10 limbs + 2 pad each) = 36 KiB:
//          (1..128)B, then (1..128)[2^124]B (quad kernel's high-half table),
//          L1/L2-resident; one coordinate gathered per lane as 2 x dwordx4 + dwordx2
//   atab : per-lane (1..8)(-A) cached table, word-major / lane-minor
//          [(e*40 + w) * stride + lane] so each of the 40 word loads of a row
//          is one coalesced 256-byte wave access when lanes share the digit
//          magnitude, and at most 8 distinct 256-byte segments otherwise.
#include <hip/hip_runtime.h>

#include "devtables.h"
#include "hs_helper.h"
#include "kernels.h"
#include "keyed.h"
#include "keyed_quad.h"
#include "quad.h"
#include "signbytes.h"
#include "verify_core.h"

// The small-batch (latency) forms raise their waves' issue priority: beside a
// pipeline's bulk launch (k_verify_keyed_batch, k_sign_bytes at priority 0)
// a 150-validator commit's workgroup lands on a SIMD that already holds bulk
// waves, and the SIMD's oldest-first arbitration starves the younger wave
// (round 6, tools/lat_trace_report.py: its kernel ran 2-2.7 ms instead of
// 0.05 ms while the bulk launch still had milliseconds to go). Within one
// kernel every wave has the same priority, so alone it changes nothing.
#define CMTV_URGENT() __builtin_amdgcn_s_setprio(2)

// Minimum waves per SIMD the verify kernel is compiled for (the second
// __launch_bounds__ argument): caps VGPRs at 512 / waves.
#ifndef CMTV_QUAD_WAVES_PER_EU
#define CMTV_QUAD_WAVES_PER_EU 1
#endif

#ifndef CMTV_VERIFY_WAVES_PER_EU
#define CMTV_VERIFY_WAVES_PER_EU 2
#endif

namespace cmtv {



// rows 0..127: (1..128)B; 128..255: (1..128)[2^124]B; 256..383: (1..128)[2^128]B;
// then the radix-2^16 blocks (1..2^15)B, (1..2^15)[2^120]B, (1..2^15)[2^128]B
// and the 16-position comb (1..2^15)[2^16j]B (verify_core.h btab_row)
__global__ __launch_bounds__(64) void k_btab_init(uint32_t* __restrict__ rows) {
  const int e = blockIdx.x * 64 + threadIdx.x;
  if (e >= BTAB_TOTAL_ROWS) return;
  uint32_t row[BTAB_ROW_WORDS];
  btab_row(row, e);
#pragma unroll
  for (int i = 0; i < BTAB_ROW_WORDS; i++) rows[e * BTAB_ROW_WORDS + i] = row[i];
}

template <uint32_t MODE>
__global__ __launch_bounds__(64, CMTV_VERIFY_WAVES_PER_EU) void k_verify(uint32_t n, const uint32_t* __restrict__ pk,
                                               const uint32_t* __restrict__ sig, const uint8_t* __restrict__ msg,
                                               const uint32_t* __restrict__ off, const uint32_t* __restrict__ btab,
                                               uint32_t* __restrict__ atab, uint8_t* __restrict__ out_valid,
                                               uint64_t* __restrict__ out_bitmap) {
  const uint32_t gid = blockIdx.x * 64 + threadIdx.x;
  const bool active = gid < n;
  const uint32_t i = active ? gid : n - 1;
  const uint32_t m0 = off[i], m1 = off[i + 1];
  DevATab at{atab, gridDim.x * 64u, gid};
  DevBTab bt{btab};
  // verify_one, not verify_one_half: with one signature per lane the kernel is
  // bound by the latency of its per-lane table loads (tables of 2 x 64 x 1280 B
  // per wave miss L2), and the half-size-scalar form keeps the number of
  // dependent lookups (68 vs 64) while removing the doublings that hid them:
  // measured 60.0 vs 61.7 M verifs/s at 1M signatures.
  bool v = verify_one<MODE>(pk + 8 * (size_t)i, sig + 16 * (size_t)i, msg + m0, m1 - m0, at, bt);
  v = v && active;
  if (active && out_valid) out_valid[gid] = v ? 1 : 0;
  const uint64_t mask = __ballot(v);
  if (threadIdx.x == 0 && out_bitmap) out_bitmap[gid >> 6] = mask;
}

struct LdsBytes {
  uint8_t* p;
  __device__ __forceinline__ void put(uint32_t pos, uint8_t b) { p[pos] = b; }
  // a template byte run from HBM: aligned dword loads issued 8 at a time
  // (one memory round trip per 32 bytes instead of one per byte), bytes
  // placed into the LDS slot
  __device__ __forceinline__ void copy(uint32_t pos, const uint8_t* src, uint32_t len) {
    const uintptr_t a = (uintptr_t)src;
    const int sh = (int)(a & 3);
    const uint32_t* w = (const uint32_t*)(a - sh);
    const uint32_t nw = ((uint32_t)sh + len + 3) >> 2;  // words holding bytes of the run
#pragma unroll 1
    for (uint32_t j = 0; j < nw; j += 8) {
      uint32_t v[8];
#pragma unroll
      for (int k = 0; k < 8; k++) v[k] = j + k < nw ? w[j + k] : 0u;
#pragma unroll
      for (int k = 0; k < 8; k++) {
#pragma unroll
        for (int b = 0; b < 4; b++) {
          const int q = 4 * (int)(j + k) + b - sh;
          if (q >= 0 && q < (int)len) p[pos + q] = (uint8_t)(v[k] >> (8 * b));
        }
      }
    }
  }
};

// Message of signature i for a helper lane: the CanonicalVote written into
// this lane's LDS slot from the commit template (sb.tmpls set; the host
// checked every message fits kSbFuseMaxMsg bytes), else msg[off[i]..off[i+1]).
// A lane hashes only bytes it wrote itself (sha512_prefixed loads only words
// holding message bytes), so no barrier is needed.
__device__ __forceinline__ void helper_message(const SbFuse& sb, uint32_t i, const uint8_t* msg, const uint32_t* off,
                                               uint32_t* slot, const uint8_t*& mp, uint32_t& ml) {
  if (sb.tmpls) {
    LdsBytes out{reinterpret_cast<uint8_t*>(slot)};
    // tidx null: one template for the whole batch (a single commit)
    const SbTemplate tp = static_cast<const SbTemplate*>(sb.tmpls)[sb.tidx ? sb.tidx[i] : 0u];
    ml = sb_write(out, tp, sb.blob, sb.flag[i] != 0, sb.sec[i], sb.nanos[i]);
    mp = reinterpret_cast<const uint8_t*>(slot);
  } else {
    const uint32_t m0 = off[i];
    mp = msg + m0;
    ml = off[i + 1] - m0;
  }
}

// Phase probe of the helper-wave kernels (tools/phase_probe.py): built
// only into a separate library with -DCMTV_PHASE_PROBE; lane 0 of every wave
// of the first 4,096 workgroups records the shader clock at fixed points
// (0 entry, 1/2 before/after barrier 1, 3/4 before/after barrier 2, 5 exit).
#ifdef CMTV_PHASE_PROBE
constexpr int kPhaseSlots = 8;
__device__ uint64_t g_phase[4096 * 4 * kPhaseSlots];
#define CMTV_STAMP(k)                                                                              \
  do {                                                                                             \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 4096)                                              \
      g_phase[((size_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * kPhaseSlots + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
// the 100 MHz constant clock, beside the shader clock (row4: slot 7 at entry,
// slot 6 at the lo wave's verdict): the launch's wall time and clock rate
#define CMTV_STAMP_RT(k)                                                                           \
  do {                                                                                             \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 4096)                                              \
      g_phase[((size_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * kPhaseSlots + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
// a value of the wave's own (cycles summed over a loop's barriers) into slot k
#define CMTV_STAMP_VAL(k, val)                                                                     \
  do {                                                                                             \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 4096)                                              \
      g_phase[((size_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * kPhaseSlots + (k)] = (val);          \
  } while (0)
#define CMTV_CLOCK() __builtin_amdgcn_s_memtime()
// five-wave workgroups (k_verify_keyed_quad_split): the same buffer indexed
// by (block * 5 + wave)
#define CMTV_STAMP5(k)                                                                             \
  do {                                                                                             \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 3200)                                              \
      g_phase[((size_t)blockIdx.x * 5 + (threadIdx.x >> 6)) * kPhaseSlots + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
// slot 6 of a five-wave workgroup's wave: its HW_ID (bits 5:4 the SIMD, 11:8 the CU)
#define CMTV_HWID5()                                                                               \
  do {                                                                                             \
    uint32_t hwid_;                                                                                \
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid_));                             \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 3200)                                              \
      g_phase[((size_t)blockIdx.x * 5 + (threadIdx.x >> 6)) * kPhaseSlots + 6] = hwid_;             \
  } while (0)
#else
#define CMTV_STAMP5(k) ((void)0)
#define CMTV_HWID5() ((void)0)
#define CMTV_STAMP(k) ((void)0)
#define CMTV_STAMP_RT(k) ((void)0)
#define CMTV_STAMP_VAL(k, val) ((void)0)
#define CMTV_CLOCK() 0ull
#endif

// The helper-summed quad verifier (quad.h q_verify_hs, hs_helper.h): a 4-wave
// workgroup takes 48 signatures; waves 0-2 are quad waves (16 signatures
// each) and wave 3 hashes and splits the scalars of all 48 (one lane each,
// q_prepare, the templated sign-bytes included) while they decompress A and R
// and build both tables (extended points); the scalars reach them at barrier
// 1. LDS (3 x 45 KiB tables + scalars + the window ring) allows one workgroup
// per CU, i.e. 4 waves on its 4 SIMDs: 256 workgroups = 12,288 signatures per
// round. After barrier 1 the helper wave sums every window's two table entries for its 48
// signatures (h_window_addend, one per lane) and hands the sums over through a
// 2-slot LDS ring, one barrier per window: the quads' windows lose one of
// their two additions. [u]B: while the quads build their tables the helper
// adds the top kHsCombPre positions of u's 16-position comb and hands that
// part over at a last barrier; the quads add the other digits inside their
// windows (q_hs_straus). Nothing of [u]B runs inside the helper's window
// loop: the per-window barriers go at the slower side's pace, so helper work
// there stalls all three quads (measured: comb additions cut into
// one-multiplication phases, two per window, cost the quads 1.6k cycles a
// window; tools/gpu_hs.sh). The slot ring overlays the fused sign-bytes
// buffer (dead once the hashes are done). hs_tune (the launcher's kflags bits
// 16..31, CMTV_HS_PRE) overrides kHsCombPre (0..16) for tuning.
template <uint32_t MODE>
__global__ __launch_bounds__(256, CMTV_QUAD_WAVES_PER_EU) void k_verify_quad_hs(
    uint32_t n, const uint32_t* __restrict__ pk, const uint32_t* __restrict__ sig, const uint8_t* __restrict__ msg,
    const uint32_t* __restrict__ off, const uint32_t* __restrict__ btab, uint8_t* __restrict__ out_valid,
    uint64_t* __restrict__ out_bitmap, uint32_t force_wide, SbFuse sb, uint32_t hs_tune, RowSlot tags) {
  CMTV_URGENT();
  const uint32_t wave = threadIdx.x >> 6, t = threadIdx.x & 63;
  const uint32_t base = blockIdx.x * 48;
  const int comb_pre = hs_comb_pre(hs_tune, sb.tmpls ? kHsCombPreFused : kHsCombPre);
  __shared__ uint32_t prep[48][SIG_PREP_WORDS + 1];
  __shared__ uint2 tab_lds[3][kHsTabU2];
  __shared__ uint2 xbuf[2 * kHsSlotU2];  // sign-bytes (48 x kSbFuseMaxMsg B), then the 2-slot ring
  static_assert(sizeof(xbuf) >= 48 * kSbFuseMaxMsg, "ring must cover the sign-bytes buffer");
  CMTV_STAMP(0);
  if (wave == 3) {
    const uint32_t slot = t < 48 ? t : 47;
    const uint32_t s = base + slot;
    const uint32_t i = s < n ? s : n - 1;
    const uint8_t* mp;
    uint32_t ml;
    CMTV_STAMP(5);  // the helper's slots 5 / 4: before / after locating its message
    helper_message(sb, i, msg, off, reinterpret_cast<uint32_t*>(xbuf) + slot * (kSbFuseMaxMsg / 4), mp, ml);
#ifdef CMTV_PHASE_PROBE
    __builtin_amdgcn_s_waitcnt(0);  // the offsets arrived
#endif
    CMTV_STAMP(4);
    SigPrep p;
    q_prepare<MODE>(p, pk + 8 * (size_t)i, sig + 16 * (size_t)i, mp, ml, force_wide != 0,
                    [] { CMTV_STAMP(7); });
    const int W = hs_workgroup_windows(p.flags, t);
    p.flags |= (uint32_t)W << 16;
    if (t < 48) sig_prep_store(prep[t], p);
    BComb16 bc;
    bc.init(p.u);
    const DevBTab bt{btab};
#pragma unroll 1
    for (int k = 0; k < comb_pre; k++) bc.step(bt);
    CMTV_STAMP(1);
    __syncthreads();  // 1: the scalars; the tables are built
    CMTV_STAMP(2);
    uint64_t hwait = 0;  // probe build: cycles the helper waits at the window barriers
    hs_helper_windows(p, W, bc, &tab_lds[0][0], xbuf, t, [] { return (uint64_t)CMTV_CLOCK(); }, hwait);
    CMTV_STAMP_VAL(6, hwait);
    CMTV_STAMP(3);
    __syncthreads();  // B: [u]B
    return;
  }
  const uint32_t ls = wave * 16 + (t >> 2);
  const uint32_t s = base + ls;
  const bool active = s < n;
  const uint32_t i = active ? s : n - 1;
  DevQuad q;
  DevATabQ ta{tab_lds[wave], t}, tr{tab_lds[wave] + 9 * 5 * 64, t};
  uint64_t qwait = 0;  // probe build: cycles this quad wave waits at the window barriers
  (void)qwait;
  DevBTabQ bt{btab};
  bool v = q_verify_hs<MODE>(
      q, pk + 8 * (size_t)i, sig + 16 * (size_t)i, bt, ta, tr, 16 - comb_pre,
      [&](SigPrep& p) {
        CMTV_STAMP(1);
        __syncthreads();
        CMTV_STAMP(2);
        sig_prep_load(p, prep[ls]);
      },
      [&](int win, fe& c) {
        const uint64_t c0 = CMTV_CLOCK();
        __syncthreads();
        qwait += CMTV_CLOCK() - c0;
        hs_slot_load(xbuf + (win & 1) * kHsSlotU2, wave, t, c);
      },
      [&](fe& c) {
        CMTV_STAMP(3);
        __syncthreads();
        CMTV_STAMP(4);
        hs_slot_load(xbuf + kHsSlotU2, wave, t, c);
      });
  CMTV_STAMP(5);
  CMTV_STAMP_VAL(6, qwait);
  v = v && active;
  if (active && (t & 3) == 0 && out_valid) out_valid[s] = v ? 1 : 0;
  uint64_t x = __ballot(v && (t & 3) == 0) & 0x1111111111111111ull;
  x = (x | (x >> 3)) & 0x0303030303030303ull;
  x = (x | (x >> 6)) & 0x000F000F000F000Full;
  x = (x | (x >> 12)) & 0x000000FF000000FFull;
  x = (x | (x >> 24)) & 0xFFFFull;
  const uint32_t slice = blockIdx.x * 3 + wave;
  if (t == 0 && slice < 4 * ((n + 63) / 64)) {
    if (tags.tagged)  // a polled host call (kernels.h RowSlot): the slice with the call's tag
      __hip_atomic_store(tags.tagged + slice, ((uint64_t)tags.seq << 32) | x, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
    else if (out_bitmap)
      reinterpret_cast<uint16_t*>(out_bitmap)[slice] = (uint16_t)x;
  }
}

// The oct verifier over two waves per 8 signatures: wave 1 hashes and splits
// the scalars (q_prepare) while wave 0 decompresses A and R; the scalars
// reach wave 0 through LDS at one barrier, and wave 1 exits. For batches up
// to 4,096 signatures (1,024 waves), where SIMDs are idle anyway, this takes
// the hash and the half-scalar Euclid (~11% of a wave) off the chain.
template <uint32_t MODE>
__global__ __launch_bounds__(128, CMTV_QUAD_WAVES_PER_EU) void k_verify_oct_split(
    uint32_t n, const uint32_t* __restrict__ pk, const uint32_t* __restrict__ sig, const uint8_t* __restrict__ msg,
    const uint32_t* __restrict__ off, const uint32_t* __restrict__ btab, uint8_t* __restrict__ out_valid,
    uint64_t* __restrict__ out_bitmap, uint32_t force_wide, SbFuse sb) {
  CMTV_URGENT();
  const uint32_t t = threadIdx.x & 63;
  const uint32_t gid = blockIdx.x * 64 + t;
  const uint32_t s = gid >> 3;
  const bool active = s < n;
  const uint32_t i = active ? s : n - 1;
  __shared__ uint32_t prep[8][SIG_PREP_WORDS + 1];
  __shared__ uint32_t bpt[8][40];
  __shared__ uint2 tab_lds[9 * 5 * 64];
  __shared__ uint32_t sbm[8][kSbFuseMaxMsg / 4];  // fused sign-bytes
  if (threadIdx.x >= 64) {
    // the oct's 8 helper lanes write the same bytes to the same slot, and
    // each hashes what it wrote
    const uint8_t* mp;
    uint32_t ml;
    helper_message(sb, i, msg, off, sbm[t >> 3], mp, ml);
    SigPrep p;
    q_prepare<MODE>(p, pk + 8 * (size_t)i, sig + 16 * (size_t)i, mp, ml, force_wide != 0);
    if ((t & 7) == 0) sig_prep_store(prep[t >> 3], p);
    __syncthreads();  // 1: the scalars
    ge_p3 B;
    q_bcomb16(B, p.u, DevBTab{btab});
    if ((t & 7) == 0) bpoint_store(bpt[t >> 3], B);
    __syncthreads();  // 2: [u]B
    return;
  }
  DevOct q;
  DevBTabQ bt{btab};
  DevATabQ ta{tab_lds, t};
  const uint32_t* bq = &bpt[t >> 3][10 * (t & 3)];
  bool v = o_verify_split<MODE, true>(
      q, pk + 8 * (size_t)i, sig + 16 * (size_t)i, bt, ta,
      [&](SigPrep& p) {
        __syncthreads();
        sig_prep_load(p, prep[t >> 3]);
      },
      [&](fe& c) {
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 10; j++) c.v[j] = bq[j];
      });
  v = v && active;
  if (active && (t & 7) == 0 && out_valid) out_valid[s] = v ? 1 : 0;
  uint64_t x = __ballot(v && (t & 7) == 0) & 0x0101010101010101ull;
  x = (x | (x >> 7)) & 0x0003000300030003ull;
  x = (x | (x >> 14)) & 0x0000000F0000000Full;
  x = (x | (x >> 28)) & 0xFFull;
  if (t == 0 && out_bitmap) reinterpret_cast<uint8_t*>(out_bitmap)[gid >> 6] = (uint8_t)x;
}

// [u]B for a helper wave whose 64 lanes all hold the same signature (the
// row forms with one signature per workgroup): the 16 comb rows (digit j of
// u is 16-bit chunk j of u + 0x8000...8000, verify_core.h BC16 blocks) are
// fetched at once -- lane L loads a quarter of row L / 4 into LDS -- and
// q_bcomb16 then reads them from LDS (one round trip to the 75 MB table
// instead of sixteen dependent ones).
struct LdsCombB {
  const uint32_t* rows;  // [16][BTAB_ROW_WORDS]
  __device__ __forceinline__ void load_fe(int e, int c, fe& r) const {
    const uint32_t* q = rows + ((e - BC16_BASE) >> 15) * BTAB_ROW_WORDS + c * BTAB_COORD_WORDS;
#pragma unroll
    for (int i = 0; i < 10; i++) r.v[i] = q[i];
  }
};
static_assert(BT16_ENTRIES == 1 << 15, "LdsCombB maps a comb row to its position by >> 15");

__device__ __forceinline__ void helper_bcomb_prefetched(ge_p3& B, const uint32_t u[8], const uint32_t* btab,
                                                        uint32_t* lds_rows, uint32_t* lds_pts, uint32_t t) {
  uint32_t tb[8];
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint64_t v = (uint64_t)u[i] + 0x80008000u + c;
    tb[i] = (uint32_t)v;
    c = v >> 32;
  }
  auto digit = [&](uint32_t j) -> int {
    uint32_t w = tb[0];
#pragma unroll
    for (int i = 1; i < 8; i++) w = (j >> 1) == (uint32_t)i ? tb[i] : w;
    return (int)((w >> (16 * (j & 1))) & 0xFFFFu) - 0x8000;
  };
  {
    const uint32_t j = t >> 2, part = t & 3;
    const int d = digit(j);
    const int ib = d < 0 ? -d : d;
    const uint32_t* src =
        btab + (size_t)(BC16_BASE + j * BT16_ENTRIES + (ib > 0 ? ib - 1 : 0)) * BTAB_ROW_WORDS + 9 * part;
    uint32_t v[9];
#pragma unroll
    for (int i = 0; i < 9; i++) v[i] = src[i];
#pragma unroll
    for (int i = 0; i < 9; i++) lds_rows[j * BTAB_ROW_WORDS + 9 * part + i] = v[i];
  }
  auto wave_sync = [] {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  wave_sync();
  // a tree instead of q_bcomb16's chain of 16: lane j (< 8) adds comb rows
  // 2j and 2j+1, then three levels of full additions through LDS (lanes
  // 0..3, 0..1, 0) -- 2 mixed + 3 full additions on the path instead of 16
  // mixed ones. The sum is the same point as q_bcomb16's in another
  // projective representation; the row kernels use it only as a point.
  const uint32_t l = t & 7;
  ge_p3 P;
  p3_identity(P);
  ge_efgh e;
#pragma unroll
  for (int h = 0; h < 2; h++) {
    const uint32_t j = 2 * l + h;
    const int d = digit(j);
    const int ib = d < 0 ? -d : d;
    ge_add_table<false>(e, P, LdsCombB{lds_rows}, BC16_BASE + (int)j * BT16_ENTRIES, d < 0, ib == 0);
    efgh_to_p3(P, e);
  }
#pragma unroll 1
  for (uint32_t width = 4; width >= 1; width >>= 1) {
    if (t < 2 * width) {
#pragma unroll
      for (int i = 0; i < 10; i++) {
        lds_pts[t * 40 + i] = P.X.v[i];
        lds_pts[t * 40 + 10 + i] = P.Y.v[i];
        lds_pts[t * 40 + 20 + i] = P.Z.v[i];
        lds_pts[t * 40 + 30 + i] = P.T.v[i];
      }
    }
    wave_sync();
    const uint32_t a = (2 * t) & 7, b = a + 1;  // lanes < width combine slots 2t, 2t+1
    ge_p3 Q, S;
#pragma unroll
    for (int i = 0; i < 10; i++) {
      Q.X.v[i] = lds_pts[a * 40 + i];
      Q.Y.v[i] = lds_pts[a * 40 + 10 + i];
      Q.Z.v[i] = lds_pts[a * 40 + 20 + i];
      Q.T.v[i] = lds_pts[a * 40 + 30 + i];
      S.X.v[i] = lds_pts[b * 40 + i];
      S.Y.v[i] = lds_pts[b * 40 + 10 + i];
      S.Z.v[i] = lds_pts[b * 40 + 20 + i];
      S.T.v[i] = lds_pts[b * 40 + 30 + i];
    }
    wave_sync();
    ge_cached sc;
    p3_to_cached(sc, S);
    ge_add_cached(e, Q, sc);
    efgh_to_p3(P, e);
  }
  B = P;
}

// The row kernels' bitmap epilogue, on one slot of the per-device ring
// (kernels.h kRowSlots). Slot word j (64 bits) collects the verdicts of
// signatures 32j .. 32j+31 as 2-bit fields (01 rejected, 10 accepted), each
// added by its signature's wave with ONE agent-scope relaxed atomic; the wave
// whose add fills the word's last field packs the word into 32-bit half j of
// out_bitmap (and the unused upper half of the last 64-bit word) and zeroes
// the slot word for the slot's next launch. Every access to a slot word is an
// atomic on that word, so nothing else needs ordering and no fence is issued:
// the round-4 form (verdict bytes, a release fence and an acq_rel ticket per
// wave, the last wave packing) made every wave write back and invalidate its
// XCD's L2 (buffer_wbl2 sc1 / buffer_inv sc1), ~10 us of a 150-signature
// launch (tools/microbench/launch_lat.hip).
__device__ __forceinline__ void row_bitmap_add(const RowSlot& slot, uint32_t s, uint32_t n, bool v,
                                               uint64_t* __restrict__ out_bitmap, uint32_t t) {
  uint64_t* sw = reinterpret_cast<uint64_t*>(slot.words);
  const uint32_t j = s >> 5, f = s & 31;
  uint64_t x = 0;
  if (t == 0) {
    const uint64_t add = (uint64_t)(v ? 2u : 1u) << (2 * f);
    x = __hip_atomic_fetch_add(sw + j, add, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + add;
  }
  x = __shfl(x, 0);
  const uint32_t nf = n - 32 * j < 32 ? n - 32 * j : 32u;  // fields of word j
  const uint64_t m = 0x5555555555555555ull >> (64 - 2 * nf);
  if (((x | (x >> 1)) & m) != m) return;  // a field of word j is still empty
  const uint64_t acc = __ballot(t < 32 && ((x >> (2 * (t & 31) + 1)) & 1) != 0);
  if (t == 0) {
    __hip_atomic_store(sw + j, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (slot.tagged) {  // kernels.h RowSlot
      __hip_atomic_store(slot.tagged + j, ((uint64_t)slot.seq << 32) | (uint32_t)acc, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
    uint32_t* ob = reinterpret_cast<uint32_t*>(out_bitmap);
    ob[j] = (uint32_t)acc;
    if ((j & 1) == 0 && 32 * (j + 1) >= n) ob[j + 1] = 0u;
  }
}

// One signature per wave (row.h): for the smallest batches (a 150-validator
// commit), where SIMDs are idle and each signature's chain of field products
// is the kernel time. A 4-wave workgroup takes 3 signatures: waves 0-2
// decode A and R (rows 0/2 and 1/3) and build their tables while wave 3's
// lanes 0-2 hash and split the scalars (q_prepare, the templated sign-bytes
// included); the scalars reach them at barrier 1 and [u]B (q_bcomb16, as
// four canonical encodings) at barrier 2, after which wave 3 exits. LDS:
// 3 x 9 KiB tables, one workgroup per CU, i.e. one wave per SIMD.
// Verdicts: lane 0 of each wave writes its byte to out_valid and adds its
// field to the launch's ring slot (row_bitmap_add).
template <uint32_t MODE>
__global__ __launch_bounds__(256, 1) void k_verify_row_split(
    uint32_t n, const uint32_t* __restrict__ pk, const uint32_t* __restrict__ sig, const uint8_t* __restrict__ msg,
    const uint32_t* __restrict__ off, const uint32_t* __restrict__ btab, uint8_t* __restrict__ out_valid,
    uint64_t* __restrict__ out_bitmap, uint32_t force_wide, SbFuse sb, RowSlot slot) {
  CMTV_URGENT();
  const uint32_t wave = threadIdx.x >> 6, t = threadIdx.x & 63;
  const uint32_t base = blockIdx.x * 3;
  __shared__ uint32_t prep[3][SIG_PREP_WORDS + 1];
  __shared__ uint32_t bpt[3][32];
  __shared__ uint32_t tab_lds[3][kRowTabWords];
  __shared__ uint32_t sbm[3][kSbFuseMaxMsg / 4];
  CMTV_STAMP(0);
  if (wave == 3) {
    const uint32_t ls = t < 3 ? t : 2;
    const uint32_t s = base + ls;
    const uint32_t i = s < n ? s : n - 1;
    const uint8_t* mp;
    uint32_t ml;
    helper_message(sb, i, msg, off, sbm[ls], mp, ml);
    SigPrep p;
    q_prepare<MODE>(p, pk + 8 * (size_t)i, sig + 16 * (size_t)i, mp, ml, force_wide != 0);
    if (t < 3) sig_prep_store(prep[t], p);
    CMTV_STAMP(1);
    __syncthreads();  // 1: the scalars
    CMTV_STAMP(2);
    ge_p3 B;
    q_bcomb16(B, p.u, DevBTab{btab});
    if (t < 3) bpoint_store_bytes(bpt[t], B);
    CMTV_STAMP(3);
    __syncthreads();  // 2: [u]B
    CMTV_STAMP(4);
    return;
  }
  const uint32_t s = base + wave;
  const bool active = s < n;
  const uint32_t i = active ? s : n - 1;
  const uint32_t* pkp = pk + 8 * (size_t)i;
  const uint32_t* sgp = sig + 16 * (size_t)i;
  uint32_t pkw[8], sigw[8];
  load_words(pkw, pkp, 2);
  load_words(sigw, sgp, 2);
  const uint32_t limb = reinterpret_cast<const uint16_t*>(((t >> 4) & 1) ? sgp : pkp)[t & 15];
  DevRowTab tab{tab_lds[wave], t};
  const uint32_t* bq = bpt[wave];
  bool v = r_verify_split<MODE>(
      DevRow(), limb, pkw, sigw, tab,
      [&](SigPrep& p) {
        CMTV_STAMP(1);
        __syncthreads();
        CMTV_STAMP(2);
        sig_prep_load(p, prep[wave]);
      },
      [&]() -> uint32_t {
        CMTV_STAMP(3);
        __syncthreads();
        CMTV_STAMP(4);
        return (bq[8 * (t >> 4) + ((t & 15) >> 1)] >> (16 * (t & 1))) & 0xFFFFu;
      });
  CMTV_STAMP(5);
  v = v && active;
  if (t == 0 && active && out_valid) out_valid[s] = v ? 1 : 0;
  if (out_bitmap && active) row_bitmap_add(slot, s, n, v, out_bitmap, t);
}

// The row verifier over four waves per signature (row.h r_sum_ar / r_part<·,
// kRowLoWindows> / r_join4), one signature per workgroup and CU, for batches
// of at most 256: wave 0 (lo) decodes A and R and runs the lowest 21
// windows of both; waves 1 and 2 (A-hi, R-hi) each decode their point, scale
// it by 2^84 while the helper (wave 3) hashes, and run the windows above;
// the helper computes [u]B. Waves 1-2 hand their sums (cached) over at
// barrier 2; wave 0 adds them and [u]B and checks. The critical path is a
// high wave's decode + 4W doublings + its additions, instead of the two-wave
// form's decode + 4W doublings + W additions + the second table.
template <uint32_t MODE>
__global__ __launch_bounds__(256, 1) void k_verify_row4_split(
    uint32_t n, const uint32_t* __restrict__ pk, const uint32_t* __restrict__ sig, const uint8_t* __restrict__ msg,
    const uint32_t* __restrict__ off, const uint32_t* __restrict__ btab, uint8_t* __restrict__ out_valid,
    uint64_t* __restrict__ out_bitmap, uint32_t force_wide, SbFuse sb, RowSlot slot) {
  CMTV_URGENT();
  const uint32_t wave = threadIdx.x >> 6, t = threadIdx.x & 63;
  const uint32_t s = blockIdx.x;
  const uint32_t i = s < n ? s : n - 1;
  __shared__ uint32_t prep[SIG_PREP_WORDS + 1];
  __shared__ uint32_t bpt[32];
  __shared__ uint32_t brows[16 * BTAB_ROW_WORDS];  // the helper's [u]B comb rows
  __shared__ uint32_t bpts[8 * 40];                // ... and its partial sums
  __shared__ uint32_t tab_lo[kRowTabWords];
  __shared__ uint32_t tab_hi[2][kRowTabWords / 2];
  __shared__ uint32_t sbm[kSbFuseMaxMsg / 4];
  __shared__ uint32_t xh[2][64];  // the high parts' sums (cached)
  const uint32_t* pkp = pk + 8 * (size_t)i;
  const uint32_t* sgp = sig + 16 * (size_t)i;
  CMTV_STAMP(0);
  CMTV_STAMP_RT(7);
  if (wave == 3) {
    const uint8_t* mp;
    uint32_t ml;
    helper_message(sb, i, msg, off, sbm, mp, ml);
    SigPrep p;
    q_prepare<MODE, true>(p, pkp, sgp, mp, ml, force_wide != 0);  // one signature on every lane
    if (t == 0) sig_prep_store(prep, p);
    CMTV_STAMP(1);
    __syncthreads();  // 1: the scalars
    CMTV_STAMP(2);
    ge_p3 B;
    helper_bcomb_prefetched(B, p.u, btab, brows, bpts, t);
    if (t == 0) bpoint_store_bytes(bpt, B);
    CMTV_STAMP(3);
    __syncthreads();  // 2: [u]B and the high parts
    CMTV_STAMP(4);
    return;
  }
  const RowCtx<DevRow> x(DevRow::lane());
  SigPrep p;
  auto stamp = [&](int k) { CMTV_STAMP(k); (void)k; };
  auto get_prep = [&](SigPrep& q) {
    CMTV_STAMP(1);
    __syncthreads();
    CMTV_STAMP(2);
    sig_prep_load(q, prep);
  };
  if (wave != 0) {
    const uint32_t* src = wave == 2 ? sgp : pkp;
    const uint32_t limb = reinterpret_cast<const uint16_t*>(src)[t & 15];
    const bool sign = (src[7] >> 31) != 0;
    DevRowTab tab{tab_hi[wave - 1], t};
    bool dec, x0;
    const uint32_t v = wave == 1 ? r_part<0, kRowLoWindows>(x, limb, sign, tab, get_prep, p, dec, x0, stamp)
                                 : r_part<1, kRowLoWindows>(x, limb, sign, tab, get_prep, p, dec, x0, stamp);
    xh[wave - 1][t] = rp_to_cached(x, v, x.cst(RowConst::d2));
    CMTV_STAMP(3);
    __syncthreads();  // 2
    CMTV_STAMP(4);
    return;
  }
  uint32_t pkw[8], sigw[8];
  load_words(pkw, pkp, 2);
  load_words(sigw, sgp, 2);
  const uint32_t limb = reinterpret_cast<const uint16_t*>(((t >> 4) & 1) ? sgp : pkp)[t & 15];
  DevRowTab tab{tab_lo, t};
  bool a_ok, r_ok, r_canon;
  const uint32_t v = r_sum_ar(x, limb, pkw, sigw, tab, get_prep, kRowLoWindows, p, a_ok, r_ok, r_canon);
  CMTV_STAMP(3);
  __syncthreads();  // 2
  CMTV_STAMP(4);
  const uint32_t cb = (bpt[8 * (t >> 4) + ((t & 15) >> 1)] >> (16 * (t & 1))) & 0xFFFFu;
  bool v_ok = r_join4<MODE>(x, v, xh[0][t], xh[1][t], cb, (p.flags & 4u) != 0 && a_ok && r_ok, r_canon);
  CMTV_STAMP(5);
  CMTV_STAMP_RT(6);
  const bool active = s < n;
  v_ok = v_ok && active;
  if (t == 0 && active && out_valid) out_valid[s] = v_ok ? 1 : 0;
  if (out_bitmap && active) row_bitmap_add(slot, s, n, v_ok, out_bitmap, t);
}

// the keyed row kernel's R wave meets barrier 1 86 squarings into the decode's
// run of 100 (~198 of its ~265 products, ~54k cycles with the split
// products: when the hash helper publishes k)
constexpr int kKeyedRowMidAt = 86;

// Registered keys, one signature per workgroup in the row layout (row.h
// r_decode_neg_r / r_kcomb / r_bcomb16 / r_keyed_join), for batches of at
// most 256 (the 150-validator VerifyCommit with the keyset cache): wave 3
// hashes k; wave 2 adds [s]B over the B table's 16-position radix-2^16 comb
// (s needs no hash), then positions 31..16 of [k](-A) over the key's
// radix-256 comb; wave 1 takes k at barrier 1 and adds positions 15..0;
// wave 0 decodes R, meeting barrier 1 inside its square-root chain (about
// when the hash is done, so it does not wait), and after barrier 2 adds both
// sums to -R and checks. Comb rows are
// converted to the row layout as they are read (DevRow::niels_limb).
// Bitmap as k_verify_row_split.
template <uint32_t MODE>
__global__ __launch_bounds__(256, 1) void k_verify_keyed_row_split(
    uint32_t n, uint32_t n_keys, const uint32_t* __restrict__ key_idx, const uint32_t* __restrict__ sig,
    const uint8_t* __restrict__ msg, const uint32_t* __restrict__ off, const uint32_t* __restrict__ keys_pk,
    const uint8_t* __restrict__ keys_ok, const uint32_t* __restrict__ ktabs, const uint32_t* __restrict__ btab,
    uint8_t* __restrict__ out_valid, uint64_t* __restrict__ out_bitmap, RowSlot slot, SbFuse sb) {
  CMTV_URGENT();
  const uint32_t wave = threadIdx.x >> 6, t = threadIdx.x & 63;
  const uint32_t s = blockIdx.x;
  const uint32_t i = s < n ? s : n - 1;
  __shared__ uint32_t tks[8];
  __shared__ uint32_t sbm[kSbFuseMaxMsg / 4];  // fused sign-bytes (every helper lane writes the same bytes)
  __shared__ uint32_t xa[64], xb[64];
  __shared__ uint32_t arows[COMB_WINDOWS * COMB_ROW_WORDS];  // the 32 key-comb rows of k's digits
  __shared__ uint32_t brows[16 * BTAB_ROW_WORDS];            // the 16 B-comb rows of s's digits
  uint32_t kid = key_idx ? key_idx[i] : i;  // null: signature i is by key i (one commit)
  const bool kin = kid < n_keys;
  kid = kin ? kid : 0;
  const uint32_t* sgp = sig + 16 * (size_t)i;
  CMTV_STAMP(0);
  if (wave == 3) {
    const uint8_t* mp;
    uint32_t ml;
    helper_message(sb, i, msg, off, sbm, mp, ml);
    uint32_t tk[8];
    q_keyed_challenge(tk, keys_pk + 8 * (size_t)kid, sgp, mp, ml);
    if (t == 0)
#pragma unroll
      for (int j = 0; j < 8; j++) tks[j] = tk[j];
    CMTV_STAMP(1);
    __syncthreads();  // 1: k
    CMTV_STAMP(2);
    __syncthreads();  // 2
    return;
  }
  const RowCtx<DevRow> x(DevRow::lane());
  const uint32_t d2 = x.cst(RowConst::d2);
  // k's key-comb rows of positions hi .. hi - 15 into LDS at once (lane L
  // fetches a quarter of row L / 4), then added onto v
  auto kcomb_half = [&](uint32_t& v, int hi) {
    uint32_t tk[8];
#pragma unroll
    for (int j = 0; j < 8; j++) tk[j] = tks[j];
    {
      const uint32_t j = (uint32_t)(hi - 15) + (t >> 2), part = t & 3;
      uint32_t w = tk[0];
#pragma unroll
      for (int q = 1; q < 8; q++) w = (j >> 2) == (uint32_t)q ? tk[q] : w;
      const int d = (int)((w >> (8 * (j & 3))) & 0xFFu) - 128;
      const int ia = d < 0 ? -d : d;
      const uint4* src = reinterpret_cast<const uint4*>(
          ktabs + (size_t)kid * COMB_TABLE_WORDS + ((size_t)j * COMB_ENTRIES + (ia > 0 ? ia - 1 : 0)) * COMB_ROW_WORDS +
          8 * part);
      const uint4 r0 = src[0], r1 = src[1];
      uint4* dst = reinterpret_cast<uint4*>(arows + j * COMB_ROW_WORDS + 8 * part);
      dst[0] = r0;
      dst[1] = r1;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    r_kcomb(x, v, tk, [&](int j, int) { return arows + j * COMB_ROW_WORDS; }, hi, hi - 15);
  };
  if (wave == 2) {
    uint32_t sw[8];
    load_words(sw, sgp + 8, 2);
    {
      // the 16 rows at once (one memory round trip instead of 16 dependent
      // ones): lane L fetches a quarter of row L / 4
      uint32_t tb[8];
      uint64_t c = 0;
#pragma unroll
      for (int j = 0; j < 8; j++) {
        const uint64_t w = (uint64_t)sw[j] + 0x80008000u + c;
        tb[j] = (uint32_t)w;
        c = w >> 32;
      }
      const uint32_t j = t >> 2, part = t & 3;
      uint32_t w = tb[0];
#pragma unroll
      for (int q = 1; q < 8; q++) w = (j >> 1) == (uint32_t)q ? tb[q] : w;
      const int d = (int)((w >> (16 * (j & 1))) & 0xFFFFu) - 0x8000;
      const int ib = d < 0 ? -d : d;
      const uint32_t* src =
          btab + (size_t)(BC16_BASE + j * BT16_ENTRIES + (ib > 0 ? ib - 1 : 0)) * BTAB_ROW_WORDS + 9 * part;
      uint32_t v9[9];
#pragma unroll
      for (int q = 0; q < 9; q++) v9[q] = src[q];
#pragma unroll
      for (int q = 0; q < 9; q++) brows[j * BTAB_ROW_WORDS + 9 * part + q] = v9[q];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    uint32_t v = r_bcomb16(x, sw, [&](int e) { return brows + ((e - BC16_BASE) >> 15) * BTAB_ROW_WORDS; });
    CMTV_STAMP(1);
    __syncthreads();  // 1: k
    CMTV_STAMP(2);
    kcomb_half(v, 31);
    xb[t] = rp_to_cached(x, v, d2);
    CMTV_STAMP(3);
    __syncthreads();  // 2: [s]B + positions 31..16 of [k](-A)
    return;
  }
  if (wave == 1) {
    CMTV_STAMP(1);
    __syncthreads();  // 1: k
    CMTV_STAMP(2);
    uint32_t v = rp_identity(x);
    kcomb_half(v, 15);
    xa[t] = rp_to_cached(x, v, d2);
    CMTV_STAMP(3);
    __syncthreads();  // 2: positions 15..0 of [k](-A)
    return;
  }
  uint32_t sigw[8], sw[8];
  load_words(sigw, sgp, 2);
  load_words(sw, sgp + 8, 2);
  const uint32_t limb = reinterpret_cast<const uint16_t*>(sgp)[t & 15];
  bool r_ok;
  const uint32_t nr = r_decode_neg_r<MODE, kKeyedRowMidAt>(x, limb, sigw, r_ok, [&]() {
    CMTV_STAMP(1);
    __syncthreads();  // 1
    CMTV_STAMP(2);
  });
  CMTV_STAMP(3);
  __syncthreads();  // 2
  CMTV_STAMP(4);
  const bool s_ok = (sw[7] & 0xE0000000u) == 0 && sc_is_canonical(sw);
  const bool ok = kin && keys_ok[kid] != 0 && s_ok && r_ok;
  bool v_ok = r_keyed_join<MODE>(x, nr, xa[t], xb[t], ok);
  CMTV_STAMP(5);
  const bool active = s < n;
  v_ok = v_ok && active;
  if (t == 0 && active && out_valid) out_valid[s] = v_ok ? 1 : 0;
  if (out_bitmap && active) row_bitmap_add(slot, s, n, v_ok, out_bitmap, t);
}

// Comb of (negate ? -P : P) for n_keys encoded points; workgroup = key,
// thread = multiple d = 1..128. keys_ok[key] records whether P decoded.
__global__ __launch_bounds__(128) void k_comb_build(const uint32_t* __restrict__ keys_pk, uint8_t* __restrict__ keys_ok,
                                                    uint32_t* __restrict__ tabs, uint32_t* __restrict__ scratch,
                                                    int negate) {
  const uint32_t key = blockIdx.x;
  uint32_t w[8];
  load_words(w, keys_pk + 8 * (size_t)key, 2);
  ge_p3 A, nA;
  const bool ok = p3_frombytes(A, w);
  if (negate) {
    cached_neg_point(nA, A);
    A = nA;
  }
  if (threadIdx.x == 0 && keys_ok) keys_ok[key] = ok ? 1 : 0;
  DevCombScratch sc{scratch, gridDim.x * 128u, blockIdx.x * 128u + threadIdx.x};
  comb_build_column(tabs + (size_t)key * COMB_TABLE_WORDS, A, (int)threadIdx.x + 1, sc);
}

__global__ __launch_bounds__(64) void k_pubkey(uint32_t n, const uint32_t* __restrict__ seeds,
                                               const uint32_t* __restrict__ btab, uint32_t* __restrict__ out_pk) {
  const uint32_t gid = blockIdx.x * 64 + threadIdx.x;
  if (gid >= n) return;
  uint32_t sw[8], pkw[8];
  load_words(sw, seeds + 8 * (size_t)gid, 2);
  DevBTab bt{btab};
  pubkey_from_seed(pkw, sw, bt);
#pragma unroll
  for (int q = 0; q < 8; q++) out_pk[8 * (size_t)gid + q] = pkw[q];
}

__global__ __launch_bounds__(64) void k_sign(uint32_t n, const uint32_t* __restrict__ seeds,
                                             const uint32_t* __restrict__ key_idx, const uint8_t* __restrict__ msg,
                                             const uint32_t* __restrict__ off, const uint32_t* __restrict__ btab,
                                             uint32_t* __restrict__ out_sig) {
  const uint32_t gid = blockIdx.x * 64 + threadIdx.x;
  if (gid >= n) return;
  const uint32_t kid = key_idx ? key_idx[gid] : gid;
  uint32_t sw[8], sg[16];
  load_words(sw, seeds + 8 * (size_t)kid, 2);
  DevBTab bt{btab};
  const uint32_t m0 = off[gid], m1 = off[gid + 1];
  sign_one(sg, sw, msg + m0, m1 - m0, bt);
#pragma unroll
  for (int q = 0; q < 16; q++) out_sig[16 * (size_t)gid + q] = sg[q];
}

static inline unsigned blocks_for(uint32_t n) { return (n + 63) / 64; }

hipError_t launch_btab_init(uint32_t* d_rows, hipStream_t s) {
  hipLaunchKernelGGL(k_btab_init, dim3(blocks_for(BTAB_TOTAL_ROWS)), dim3(64), 0, s, d_rows);
  return hipGetLastError();
}

hipError_t launch_verify(uint32_t mode, uint32_t n, const void* pk, const void* sig, const void* msg,
                         const void* off, const uint32_t* btab, uint32_t* atab, void* valid, void* bitmap,
                         uint32_t kflags, hipStream_t s, const SbFuse* sb, const RowSlot* row_slot) {
  const SbFuse fz = sb ? *sb : SbFuse{};
  const uint32_t form = kflags & kFormMask;
  const uint32_t fw = (kflags & kLaunchForceWide) ? 1u : 0u;
  if (n == 0) return hipSuccess;
  auto pkp = static_cast<const uint32_t*>(pk);
  auto sgp = static_cast<const uint32_t*>(sig);
  auto mp = static_cast<const uint8_t*>(msg);
  auto op = static_cast<const uint32_t*>(off);
  auto vp = static_cast<uint8_t*>(valid);
  auto bp = static_cast<uint64_t*>(bitmap);
  const RowSlot rs = row_slot ? *row_slot : RowSlot{};
  const bool go = mode != MODE_ZIP215;
  if ((form == kFormRow4 || form == kFormRow) && (n > kRowMaxCap || (bp && !rs.words))) return hipErrorInvalidValue;
  if (form != kFormLane && form != kFormQuad && form != kFormOct2 && form != kFormRow && form != kFormRow4)
    return hipErrorInvalidValue;
  if (fz.tmpls && form == kFormLane) return hipErrorInvalidValue;
  switch (form) {
    case kFormRow4:  // one signature per 256-lane block (lo, A-hi, R-hi, the helper)
      if (go)
        hipLaunchKernelGGL(k_verify_row4_split<MODE_GO_STDLIB>, dim3(n), dim3(256), 0, s, n, pkp, sgp, mp, op, btab,
                           vp, bp, fw, fz, rs);
      else
        hipLaunchKernelGGL(k_verify_row4_split<MODE_ZIP215>, dim3(n), dim3(256), 0, s, n, pkp, sgp, mp, op, btab, vp,
                           bp, fw, fz, rs);
      break;
    case kFormRow:  // 3 signatures per 256-lane block (3 row waves + the helper)
      if (go)
        hipLaunchKernelGGL(k_verify_row_split<MODE_GO_STDLIB>, dim3((n + 2) / 3), dim3(256), 0, s, n, pkp, sgp, mp, op,
                           btab, vp, bp, fw, fz, rs);
      else
        hipLaunchKernelGGL(k_verify_row_split<MODE_ZIP215>, dim3((n + 2) / 3), dim3(256), 0, s, n, pkp, sgp, mp, op,
                           btab, vp, bp, fw, fz, rs);
      break;
    case kFormOct2:  // one 128-lane block (2 waves) = 8 signatures; whole groups of 8 blocks
      if (go)
        hipLaunchKernelGGL(k_verify_oct_split<MODE_GO_STDLIB>, dim3(((n + 63) / 64) * 8), dim3(128), 0, s, n, pkp, sgp,
                           mp, op, btab, vp, bp, fw, fz);
      else
        hipLaunchKernelGGL(k_verify_oct_split<MODE_ZIP215>, dim3(((n + 63) / 64) * 8), dim3(128), 0, s, n, pkp, sgp,
                           mp, op, btab, vp, bp, fw, fz);
      break;
    case kFormQuad: {
      // 48 signatures per 256-lane block; enough blocks for every 16-bit
      // slice of every bitmap word
      const uint32_t slices = 4 * ((n + 63) / 64);
      const dim3 grid((slices + 2) / 3), block(256);
      const RowSlot tg = row_slot ? *row_slot : RowSlot{};  // its tagged entries only
      if (go)
        hipLaunchKernelGGL(k_verify_quad_hs<MODE_GO_STDLIB>, grid, block, 0, s, n, pkp, sgp, mp, op, btab, vp, bp, fw,
                           fz, kflags >> 16, tg);
      else
        hipLaunchKernelGGL(k_verify_quad_hs<MODE_ZIP215>, grid, block, 0, s, n, pkp, sgp, mp, op, btab, vp, bp, fw, fz,
                           kflags >> 16, tg);
      break;
    }
    default:
      if (go)
        hipLaunchKernelGGL(k_verify<MODE_GO_STDLIB>, dim3(blocks_for(n)), dim3(64), 0, s, n, pkp, sgp, mp, op, btab,
                           atab, vp, bp);
      else
        hipLaunchKernelGGL(k_verify<MODE_ZIP215>, dim3(blocks_for(n)), dim3(64), 0, s, n, pkp, sgp, mp, op, btab, atab,
                           vp, bp);
  }
  return hipGetLastError();
}

hipError_t launch_comb_build(uint32_t n_keys, const void* keys_pk, uint8_t* keys_ok, uint32_t* tabs,
                             uint32_t* scratch, bool negate, hipStream_t s) {
  if (n_keys == 0) return hipSuccess;
  hipLaunchKernelGGL(k_comb_build, dim3(n_keys), dim3(128), 0, s, static_cast<const uint32_t*>(keys_pk), keys_ok, tabs,
                     scratch, negate ? 1 : 0);
  return hipGetLastError();
}

// Registered-key quads with two helper waves: 3 quad waves (48 signatures)
// run the 32 fixed-base comb additions, take k from the hash helper (wave 4,
// q_keyed_challenge; published through an LDS flag, not a barrier), run the
// 32 key-comb additions and take R at the one barrier; the decode helper
// (wave 3, q_keyed_decode_r) starts R's square-root chain at the first cycle,
// one lane per signature. With one helper hashing and then decoding, the
// hash + decode chain (~225k cycles) set the kernel time; now the longer of
// the decode (~140k) and the quads' 64 additions does. 5 waves on 4 SIMDs:
// the short hash helper shares one.
//
// The quads wait for the hash helper's flag for at most k_wait polls. The
// verdict never depends on that wait: a quad wave that stops waiting hashes
// its own signatures (q_keyed_challenge, the same k the helper computes) and
// counts itself in diag[kDiagLateK] (cmtv_stats.late_k_waves). k_wait = 0
// (the CMTV_FORCE_K_LATE test knob) skips the flag entirely, so every quad
// wave takes that path.
template <uint32_t MODE>
__global__ __launch_bounds__(320, 1) void k_verify_keyed_quad_split(
    uint32_t n, uint32_t n_keys, const uint32_t* __restrict__ key_idx, const uint32_t* __restrict__ sig,
    const uint8_t* __restrict__ msg, const uint32_t* __restrict__ off, const uint32_t* __restrict__ keys_pk,
    const uint8_t* __restrict__ keys_ok, const uint32_t* __restrict__ ktabs, uint8_t* __restrict__ out_valid, uint64_t* __restrict__ out_bitmap, uint32_t k_wait, uint32_t* __restrict__ diag,
    const uint32_t* __restrict__ btab, SbFuse sb, RowSlot tags) {
  CMTV_URGENT();
  const uint32_t wave = threadIdx.x >> 6, t = threadIdx.x & 63;
  const uint32_t base = blockIdx.x * 48;
  __shared__ uint32_t tks[48][9];
  __shared__ uint32_t sbm[48][kSbFuseMaxMsg / 4];  // fused sign-bytes
  __shared__ uint32_t rpt[48][31];  // R: x, y, t (10 words each), decode flag
  __shared__ uint32_t k_ready;
  CMTV_STAMP5(0);
  CMTV_HWID5();
  if (threadIdx.x == 0) k_ready = 0u;
  __syncthreads();  // the flag is clear before any wave can set or read it
  // probe slots: 0 entry; hash helper 3 = k published; decode helper 3 = R
  // decoded; quads 4 = k taken, 1 / 2 = before / after the barrier (the combs
  // done / R in hand), 5 = exit; every wave 2 = after the barrier
  if (wave >= 3) {
    const uint32_t s = base + (t < 48 ? t : 47);
    const uint32_t i = s < n ? s : n - 1;
    if (wave == 4) {
      // hash helper: k for all 48 signatures, published through k_ready so
      // the decode helper never waits on it
      const uint8_t* mp;
      uint32_t ml;
      helper_message(sb, i, msg, off, sbm[t < 48 ? t : 47], mp, ml);
      uint32_t kid = key_idx ? key_idx[i] : i;
      kid = kid < n_keys ? kid : 0;
      uint32_t tk[8];
      q_keyed_challenge(tk, keys_pk + 8 * (size_t)kid, sig + 16 * (size_t)i, mp, ml);
      if (t < 48)
#pragma unroll
        for (int j = 0; j < 8; j++) tks[t][j] = tk[j];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      if (t == 0) __hip_atomic_store(&k_ready, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      CMTV_STAMP5(3);
    } else {
      // decode helper: R from the first cycle, overlapping the quads' fixed-
      // base and key combs (the chain that bounded the one-helper form)
      ge_p3 R;
      const bool r_ok = q_keyed_decode_r<MODE>(R, sig + 16 * (size_t)i);
      if (t < 48) {
#pragma unroll
        for (int j = 0; j < 10; j++) {
          rpt[t][j] = R.X.v[j];
          rpt[t][10 + j] = R.Y.v[j];
          rpt[t][20 + j] = R.T.v[j];
        }
        rpt[t][30] = r_ok ? 1u : 0u;
      }
      CMTV_STAMP5(3);
    }
    __syncthreads();  // R (and k)
    CMTV_STAMP5(2);
    return;
  }
  const uint32_t ls = wave * 16 + (t >> 2);
  const uint32_t s = base + ls;
  const bool active = s < n;
  const uint32_t i = active ? s : n - 1;
  uint32_t kid = key_idx ? key_idx[i] : i;  // null: signature i is by key i (one commit)
  const bool kin = kid < n_keys;
  kid = kin ? kid : 0;
  DevQuad q;
  const int lane = (int)(t & 3);
  // [s]B over the B table's radix-2^16 comb (16 additions)
  bool v = q_verify_keyed_split<MODE, true>(
      q, kin && keys_ok[kid] != 0, sig + 16 * (size_t)i, ktabs + (size_t)kid * COMB_TABLE_WORDS, nullptr,
      [&](uint32_t tk[8]) {
        // the hash helper's flag, polled at most k_wait times (a wave never
        // spins forever)
        bool ready = false;
        for (uint32_t spins = 0; spins < k_wait; spins++) {
          ready = __hip_atomic_load(&k_ready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != 0u;
          if (ready) break;
          __builtin_amdgcn_s_sleep(2);
        }
        if (__builtin_expect(__ballot(ready) != __ballot(1), 0)) {
          // the helper's k did not arrive in time: hash this signature here
          // (identical k), so the wait bounds only the time, never the verdict;
          // fused sign-bytes are written again into the signature's slot (the
          // helper may be writing the same bytes there)
          const uint8_t* mp;
          uint32_t ml;
          helper_message(sb, i, msg, off, sbm[ls], mp, ml);
          q_keyed_challenge(tk, keys_pk + 8 * (size_t)kid, sig + 16 * (size_t)i, mp, ml);
          if (t == 0) atomicAdd(diag + kDiagLateK, 1u);
        } else {
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
#pragma unroll
          for (int j = 0; j < 8; j++) tk[j] = tks[ls][j];
        }
        CMTV_STAMP5(4);
      },
      [&](fe& rc, bool& r_ok) {
        CMTV_STAMP5(1);
        __syncthreads();
        CMTV_STAMP5(2);
        // this lane's coordinate: x, y, 1, t
        const uint32_t* p = rpt[ls] + 10 * (lane == 3 ? 2 : lane);
#pragma unroll
        for (int j = 0; j < 10; j++) rc.v[j] = lane == 2 ? (j == 0 ? 1u : 0u) : p[j];
        r_ok = rpt[ls][30] != 0;
      },
      DevBTabQ{btab});
  v = v && active;
  if (active && (t & 3) == 0 && out_valid) out_valid[s] = v ? 1 : 0;
  uint64_t x = __ballot(v && (t & 3) == 0) & 0x1111111111111111ull;
  x = (x | (x >> 3)) & 0x0303030303030303ull;
  x = (x | (x >> 6)) & 0x000F000F000F000Full;
  x = (x | (x >> 12)) & 0x000000FF000000FFull;
  x = (x | (x >> 24)) & 0xFFFFull;
  const uint32_t slice = blockIdx.x * 3 + wave;
  if (t == 0 && slice < 4 * ((n + 63) / 64)) {
    if (tags.tagged)  // a polled host call (kernels.h RowSlot): the slice with the call's tag
      __hip_atomic_store(tags.tagged + slice, ((uint64_t)tags.seq << 32) | x, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
    else if (out_bitmap)
      reinterpret_cast<uint16_t*>(out_bitmap)[slice] = (uint16_t)x;
  }
  CMTV_STAMP5(5);
}

hipError_t launch_verify_keyed(uint32_t mode, uint32_t n, uint32_t n_keys, const void* key_idx, const void* sig,
                               const void* msg, const void* off, const uint32_t* keys_pk, const uint8_t* keys_ok,
                               const uint32_t* ktabs, void* valid, void* bitmap, uint32_t form, uint32_t k_wait,
                               uint32_t* diag, uint32_t batch_kb, uint32_t* scr, const uint32_t* wtabs,
                               const uint32_t* btab, hipStream_t s, const RowSlot* row_slot, const SbFuse* sbp) {
  if (n == 0) return hipSuccess;
  const SbFuse sb = sbp ? *sbp : SbFuse{};
  // fused sign-bytes and identity keys only in the forms whose helper wave
  // hashes (row, quad)
  if ((sb.tmpls || !key_idx) && form == kKeyedLane) return hipErrorInvalidValue;
  if (form == kKeyedRow && (n > kRowMaxCap || (bitmap && !(row_slot && row_slot->words))))
    return hipErrorInvalidValue;
  auto ki = static_cast<const uint32_t*>(key_idx);
  auto sgp = static_cast<const uint32_t*>(sig);
  auto mp = static_cast<const uint8_t*>(msg);
  auto op = static_cast<const uint32_t*>(off);
  auto vp = static_cast<uint8_t*>(valid);
  auto bp = static_cast<uint64_t*>(bitmap);
  const bool go = mode != MODE_ZIP215;
  if (form == kKeyedRow) {
    // one signature per 256-lane block
    const RowSlot rs = row_slot ? *row_slot : RowSlot{};
    if (go)
      hipLaunchKernelGGL(k_verify_keyed_row_split<MODE_GO_STDLIB>, dim3(n), dim3(256), 0, s, n, n_keys, ki, sgp, mp,
                         op, keys_pk, keys_ok, ktabs, btab, vp, bp, rs, sb);
    else
      hipLaunchKernelGGL(k_verify_keyed_row_split<MODE_ZIP215>, dim3(n), dim3(256), 0, s, n, n_keys, ki, sgp, mp, op,
                         keys_pk, keys_ok, ktabs, btab, vp, bp, rs, sb);
    return hipGetLastError();
  }
  if (form == kKeyedQuad) {
    const uint32_t slices = 4 * ((n + 63) / 64);
    const dim3 grid((slices + 2) / 3), block(320);
    // row_slot here: only its tagged entries (16 signatures each) and seq
    const RowSlot tg = row_slot ? *row_slot : RowSlot{};
    if (go)
      hipLaunchKernelGGL(k_verify_keyed_quad_split<MODE_GO_STDLIB>, grid, block, 0, s, n, n_keys, ki, sgp, mp, op,
                         keys_pk, keys_ok, ktabs, vp, bp, k_wait, diag, btab, sb, tg);
    else
      hipLaunchKernelGGL(k_verify_keyed_quad_split<MODE_ZIP215>, grid, block, 0, s, n, n_keys, ki, sgp, mp, op,
                         keys_pk, keys_ok, ktabs, vp, bp, k_wait, diag, btab, sb, tg);
    return hipGetLastError();
  }
  if (form != kKeyedLane) return hipErrorInvalidValue;
  return launch_verify_keyed_lane(mode, n, n_keys, ki, sgp, mp, op, keys_pk, keys_ok, ktabs, vp, bp, batch_kb, scr,
                                  wtabs, btab, s);
}

hipError_t launch_pubkey(uint32_t n, const void* seeds, const uint32_t* btab, void* out_pk, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_pubkey, dim3(blocks_for(n)), dim3(64), 0, s, n, static_cast<const uint32_t*>(seeds), btab,
                     static_cast<uint32_t*>(out_pk));
  return hipGetLastError();
}

hipError_t launch_sign(uint32_t n, const void* seeds, const void* key_idx, const void* msg, const void* off,
                       const uint32_t* btab, void* out_sig, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_sign, dim3(blocks_for(n)), dim3(64), 0, s, n, static_cast<const uint32_t*>(seeds),
                     static_cast<const uint32_t*>(key_idx), static_cast<const uint8_t*>(msg),
                     static_cast<const uint32_t*>(off), btab, static_cast<uint32_t*>(out_sig));
  return hipGetLastError();
}

}  // namespace cmtv

#ifdef CMTV_PHASE_PROBE
// probe build only: copy the recorded stamps (n <= 4096 * 4 * 8 words)
extern "C" int cmtv_debug_phase_times(uint64_t* out, size_t n) {
  const size_t cap = sizeof(cmtv::g_phase) / sizeof(uint64_t);
  if (n > cap) n = cap;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(cmtv::g_phase), n * sizeof(uint64_t), 0, hipMemcpyDeviceToHost) ==
                 hipSuccess
             ? 0
             : -1;
}
#endif

