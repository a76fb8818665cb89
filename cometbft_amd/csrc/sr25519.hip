// sr25519.hip -- gfx950 kernel for sr25519 (schnorrkel / ristretto255) batch
// verification (BASELINE configs[4]; reference path
// /root/reference/crypto/sr25519/pubkey.go:34-60).
//
//   k_verify_sr25519_quad_hs: one signature per quad of lanes (sr25519_quad.h)
//     and a helper wave, half-size scalars and shared windows like the Ed25519
//     helper-summed quad kernel; the runtime uses it below the crossover
//   k_verify_sr25519: one signature per lane (sr25519.h): merlin transcript
//     (merlin.h: host-computed prefix sponge, chunked message, two-pass tail),
//     ristretto255 decoding of A and R, Straus [s]B - [k]A over the Ed25519
//     kernel's field, point formulas and fixed-base table, ristretto equality;
//     a wavefront ballot packs 64 verdicts into one bitmap word.
//
// Memory layout: inputs exactly as the Ed25519 kernels (pk n x 32 B, sig
// n x 64 B, msg flat bytes + (n+1) u32 offsets); the transcript's prefix
// sponge (SR_PREFIX_WORDS, merlin.h sr_prefix_state) is read with scalar
// loads; the sponge stays in registers and each lane's current
// STROBE block (42 words) gathers in LDS lane-interleaved (word w of lane l
// at word w*64 + l: conflict-free for any per-lane position).
#include <hip/hip_runtime.h>

#include "devtables.h"
#include "hs_helper.h"
#include "kernels.h"
#include "sr25519.h"
#include "sr25519_quad.h"

namespace cmtv {

// Phase probe (tools/phase_probe.py --sr): built only into a separate library
// with -DCMTV_PHASE_PROBE, as kernels.hip's; lane 0 of every wave of the
// first 4,096 workgroups of k_verify_sr25519_quad_hs records the shader clock
// (0 entry, 1/2 before/after barrier 1, 3/4 before/after the last barrier,
// 5 exit) and, in slot 6, the cycles it waited at the window barriers; the
// helper's slot 7 is the end of its merlin transcripts.
#ifdef CMTV_PHASE_PROBE
constexpr int kSrPhaseSlots = 8;
__device__ uint64_t g_phase_sr[4096 * 4 * kSrPhaseSlots];
#define CMTV_SR_STAMP(k)                                                                             \
  do {                                                                                               \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 4096)                                                \
      g_phase_sr[((size_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * kSrPhaseSlots + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#define CMTV_SR_STAMP_VAL(k, val)                                                                    \
  do {                                                                                               \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 4096)                                                \
      g_phase_sr[((size_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * kSrPhaseSlots + (k)] = (val);       \
  } while (0)
#define CMTV_SR_CLOCK() __builtin_amdgcn_s_memtime()
#else
#define CMTV_SR_STAMP(k) ((void)0)
#define CMTV_SR_STAMP_VAL(k, val) ((void)0)
#define CMTV_SR_CLOCK() 0ull
#endif

// The STROBE block buffer of one lane in LDS (42 words, lane-interleaved)
struct LdsStrobeState {
  uint32_t* __restrict__ lds;
  uint32_t lane;
  __device__ __forceinline__ void store(int i, uint32_t x) { lds[i * 64 + lane] = x; }
  __device__ __forceinline__ uint32_t load(int i) const { return lds[i * 64 + lane]; }
};

__global__ __launch_bounds__(64, 2) void k_verify_sr25519(uint32_t n, const uint32_t* __restrict__ pk,
                                                          const uint32_t* __restrict__ sig,
                                                          const uint8_t* __restrict__ msg,
                                                          const uint32_t* __restrict__ off,
                                                          const uint32_t* __restrict__ btab,
                                                          uint32_t* __restrict__ atab,
                                                          const uint32_t* __restrict__ prog, int nops,
                                                          uint8_t* __restrict__ out_valid,
                                                          uint64_t* __restrict__ out_bitmap) {
  __shared__ uint32_t st_lds[STROBE_BLOCK_WORDS * 64];
  const uint32_t gid = blockIdx.x * 64 + threadIdx.x;
  const bool active = gid < n;
  const uint32_t i = active ? gid : n - 1;
  const uint32_t m0 = off[i], m1 = off[i + 1];
  DevATab at{atab, gridDim.x * 64u, gid};
  DevBTab bt{btab};
  LdsStrobeState st{st_lds, threadIdx.x};
  bool v = sr_verify_one(pk + 8 * (size_t)i, sig + 16 * (size_t)i, msg + m0, m1 - m0, prog, nops, st, at, bt);
  v = v && active;
  if (active && out_valid) out_valid[gid] = v ? 1 : 0;
  const uint64_t mask = __ballot(v);
  if (threadIdx.x == 0 && out_bitmap) out_bitmap[gid >> 6] = mask;
}

// The helper-summed form (kernels.hip k_verify_quad_hs, hs_helper.h): the
// helper runs the merlin transcripts (STROBE block buffers in the LDS the window ring
// takes over afterwards), the quads build both tables before barrier 1, then
// the helper sums every window's two table entries and the quads add one
// point per window (sr25519_quad.h q_verify_sr_hs).
__global__ __launch_bounds__(256, 1) void k_verify_sr25519_quad_hs(
    uint32_t n, const uint32_t* __restrict__ pk, const uint32_t* __restrict__ sig, const uint8_t* __restrict__ msg,
    const uint32_t* __restrict__ off, const uint32_t* __restrict__ btab, const uint32_t* __restrict__ prog, int nops,
    uint8_t* __restrict__ out_valid, uint64_t* __restrict__ out_bitmap, uint32_t force_wide, uint32_t hs_tune) {
  __builtin_amdgcn_s_setprio(2);  // a latency form (kernels.hip CMTV_URGENT)
  const uint32_t wave = threadIdx.x >> 6, t = threadIdx.x & 63;
  const uint32_t base = blockIdx.x * 48;
  const int comb_pre = hs_comb_pre(hs_tune, kHsCombPreSr);
  __shared__ uint32_t prep[48][SIG_PREP_WORDS + 1];
  __shared__ uint2 tab_lds[3][kHsTabU2];
  // the helper's STROBE block buffers (42 x 64 words), then the 2-slot window ring
  __shared__ uint2 xbuf[2 * kHsSlotU2];
  static_assert(sizeof(xbuf) >= STROBE_BLOCK_WORDS * 64 * 4, "ring must cover the STROBE blocks");
  CMTV_SR_STAMP(0);
  if (wave == 3) {
    const uint32_t s = base + (t < 48 ? t : 47);
    const uint32_t i = s < n ? s : n - 1;
    const uint32_t m0 = off[i], m1 = off[i + 1];
    LdsStrobeState st{reinterpret_cast<uint32_t*>(xbuf), t};
    SigPrep p;
    sr_prepare(p, pk + 8 * (size_t)i, sig + 16 * (size_t)i, msg + m0, m1 - m0, prog, nops, st, force_wide != 0,
               [] { CMTV_SR_STAMP(7); });
    const int W = hs_workgroup_windows(p.flags, t);
    p.flags |= (uint32_t)W << 16;
    if (t < 48) sig_prep_store(prep[t], p);
    BComb16 bc;
    bc.init(p.u);
    const DevBTab bt{btab};
#pragma unroll 1
    for (int k = 0; k < comb_pre; k++) bc.step(bt);
    CMTV_SR_STAMP(1);
    __syncthreads();  // 1: the scalars; the tables are built
    CMTV_SR_STAMP(2);
    uint64_t hwait = 0;
    hs_helper_windows(p, W, bc, &tab_lds[0][0], xbuf, t, [] { return (uint64_t)CMTV_SR_CLOCK(); }, hwait);
    CMTV_SR_STAMP_VAL(6, hwait);
    CMTV_SR_STAMP(3);
    __syncthreads();  // B: [u]B
    CMTV_SR_STAMP(4);
    return;
  }
  const uint32_t ls = wave * 16 + (t >> 2);
  const uint32_t s = base + ls;
  const bool active = s < n;
  const uint32_t i = active ? s : n - 1;
  DevQuad q;
  DevBTabQ bt{btab};
  DevATabQ ta{tab_lds[wave], t}, tr{tab_lds[wave] + 9 * 5 * 64, t};
  uint64_t qwait = 0;  // probe build: cycles this quad wave waits at the window barriers
  (void)qwait;
  bool v = q_verify_sr_hs(
      q, pk + 8 * (size_t)i, sig + 16 * (size_t)i, bt, ta, tr, 16 - comb_pre,
      [&](SigPrep& p) {
        CMTV_SR_STAMP(1);
        __syncthreads();
        CMTV_SR_STAMP(2);
        sig_prep_load(p, prep[ls]);
      },
      [&](int win, fe& c) {
        const uint64_t c0 = CMTV_SR_CLOCK();
        __syncthreads();
        qwait += CMTV_SR_CLOCK() - c0;
        hs_slot_load(xbuf + (win & 1) * kHsSlotU2, wave, t, c);
      },
      [&](fe& c) {
        CMTV_SR_STAMP(3);
        __syncthreads();
        CMTV_SR_STAMP(4);
        hs_slot_load(xbuf + kHsSlotU2, wave, t, c);
      });
  CMTV_SR_STAMP(5);
  CMTV_SR_STAMP_VAL(6, qwait);
  v = v && active;
  if (active && (t & 3) == 0 && out_valid) out_valid[s] = v ? 1 : 0;
  uint64_t x = __ballot(v && (t & 3) == 0) & 0x1111111111111111ull;
  x = (x | (x >> 3)) & 0x0303030303030303ull;
  x = (x | (x >> 6)) & 0x000F000F000F000Full;
  x = (x | (x >> 12)) & 0x000000FF000000FFull;
  x = (x | (x >> 24)) & 0xFFFFull;
  const uint32_t slice = blockIdx.x * 3 + wave;
  if (t == 0 && out_bitmap && slice < 4 * ((n + 63) / 64)) reinterpret_cast<uint16_t*>(out_bitmap)[slice] = (uint16_t)x;
}

hipError_t launch_verify_sr25519(uint32_t n, const void* pk, const void* sig, const void* msg, const void* off,
                                 const uint32_t* btab, uint32_t* atab, const uint32_t* prog, int nops, void* valid,
                                 void* bitmap, uint32_t kflags, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint32_t form = kflags & kFormMask;
  if (form == kFormQuad) {
    const uint32_t slices = 4 * ((n + 63) / 64);
    hipLaunchKernelGGL(k_verify_sr25519_quad_hs, dim3((slices + 2) / 3), dim3(256), 0, s, n,
                       static_cast<const uint32_t*>(pk), static_cast<const uint32_t*>(sig),
                       static_cast<const uint8_t*>(msg), static_cast<const uint32_t*>(off), btab, prog, nops,
                       static_cast<uint8_t*>(valid), static_cast<uint64_t*>(bitmap),
                       (kflags & kLaunchForceWide) ? 1u : 0u, kflags >> 16);
    return hipGetLastError();
  }
  if (form != kFormLane) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_verify_sr25519, dim3((n + 63) / 64), dim3(64), 0, s, n, static_cast<const uint32_t*>(pk),
                     static_cast<const uint32_t*>(sig), static_cast<const uint8_t*>(msg),
                     static_cast<const uint32_t*>(off), btab, atab, prog, nops, static_cast<uint8_t*>(valid),
                     static_cast<uint64_t*>(bitmap));
  return hipGetLastError();
}

}  // namespace cmtv

#ifdef CMTV_PHASE_PROBE
// probe build only: copy the recorded stamps (n <= 4096 * 4 * 8 words)
extern "C" int cmtv_debug_phase_times_sr(uint64_t* out, size_t n) {
  const size_t cap = sizeof(cmtv::g_phase_sr) / sizeof(uint64_t);
  if (n > cap) n = cap;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(cmtv::g_phase_sr), n * sizeof(uint64_t), 0, hipMemcpyDeviceToHost) ==
                 hipSuccess
             ? 0
             : -1;
}
#endif
