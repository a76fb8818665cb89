// keyed_lane.hip -- the one-signature-per-lane registered-key kernels
// (keyed.h) and the builders of the wide (radix-2^16) key combs.
//
//   k_verify_keyed<MODE, COMB>          one signature per lane, final check per lane
//   k_verify_keyed_batch<MODE, KB, COMB> KB signatures per lane sharing one inversion
//   k_wide_bases / k_wide_build         the wide combs of a key set
//
// COMB selects the tables: kCombWideDma = the radix-2^16 combs (32 additions;
// the key rows come from HBM, 64 MiB per key) with each addition's two rows
// staged into LDS one addition ahead by LDS-DMA (global_load_lds_dwordx4), so
// the HBM latency of the next rows overlaps the current addition instead of
// stalling it (profiles/r03_c3w_pmc_sq.txt: read by plain loads, the wide
// kernel waited on memory 38 % of its wave cycles at two waves per SIMD, the
// register file being full); kCombMixed = the keys' radix-256 combs (MALL-
// resident 512 KiB each) with B over the B table's radix-2^16 comb (48
// additions: keyed.h keyed_comb_mixed), for key sets without wide combs. (The
// plain-load wide form and the all-radix-256 form, 64 additions, were retired
// in round 5: no dispatch reached them.)
#include <hip/hip_runtime.h>

#include "devtables.h"
#include "kernels.h"
#include "keyed.h"

#ifndef CMTV_KEYED_WAVES_PER_EU
#define CMTV_KEYED_WAVES_PER_EU 2
#endif

namespace cmtv {

enum { kCombWideDma = 2, kCombMixed = 3 };

// ---------------------------------------------------------------- LDS staging
//
// A table row's three niels coordinates (10 words each, CSTRIDE bytes apart:
// 40 in a comb row, 48 in a B-table row) are copied by 9 LDS-DMA pieces of
// 16 bytes per lane into this wave's stage, piece-major: piece (3c + p) of
// lane l at stage word (3c + p) * 256 + 4 l. Piece 3c + 2 carries the
// coordinate's last two words (and two words of what follows in the row, which
// stay unread). One stage = 9 KiB per wave.
constexpr uint32_t kStageWords = 9 * 256;

// Issue the 9 pieces of `row` into the stage at LDS byte address lds. The
// loads are inline asm, outside the compiler's s_waitcnt bookkeeping: the
// caller waits for them with stage_wait<N>() (N = pieces issued after them).
// Before the first piece, this wave's earlier reads of the stage must be done
// (lgkmcnt(0)): the DMA overwrites it.
template <uint32_t CSTRIDE>
__device__ __forceinline__ void stage_row(uint32_t lds, const uint32_t* row) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  const char* g = reinterpret_cast<const char*>(row);
#pragma unroll
  for (uint32_t c = 0; c < 3; c++)
#pragma unroll
    for (uint32_t p = 0; p < 3; p++) {
      uint32_t keep;
      const char* src = g + c * CSTRIDE + 16 * p;
      asm volatile(
          "s_mov_b32 %0, m0\n\t"
          "s_mov_b32 m0, %2\n\t"
          "s_nop 0\n\t"
          "global_load_lds_dwordx4 %1, off\n\t"
          "s_mov_b32 m0, %0"
          : "=&s"(keep)
          : "v"(src), "s"(lds + (3 * c + p) * 1024u)
          : "memory");
    }
}

// Wait until at most N of this wave's vector-memory operations are
// outstanding (in issue order: everything older than the N youngest is done).
template <int N>
__device__ __forceinline__ void stage_wait() {
  if (N == 9)
    asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
  else
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// A staged row as an ge_add_table source (e is the row already staged).
struct LdsRow {
  const uint32_t* w;  // stage + 4 * lane
  __device__ __forceinline__ void load_fe(int, int c, fe& r) const {
    const uint32_t* p = w + c * 768;
    const uint4 a = *reinterpret_cast<const uint4*>(p);
    const uint4 b = *reinterpret_cast<const uint4*>(p + 256);
    const uint2 d = *reinterpret_cast<const uint2*>(p + 512);
    r.v[0] = a.x; r.v[1] = a.y; r.v[2] = a.z; r.v[3] = a.w;
    r.v[4] = b.x; r.v[5] = b.y; r.v[6] = b.z; r.v[7] = b.w;
    r.v[8] = d.x; r.v[9] = d.y;
  }
};

__device__ __forceinline__ const uint32_t* wide_row(const uint32_t* wtab, int j, int d) {
  const int i = d < 0 ? -d : d;
  return wtab + ((size_t)j * WIDE_ENTRIES + (i > 0 ? i - 1 : 0)) * COMB_ROW_WORDS;
}
__device__ __forceinline__ const uint32_t* bc16_row(const uint32_t* btab, int j, int d) {
  const int i = d < 0 ? -d : d;
  return btab + (size_t)(BC16_BASE + j * BT16_ENTRIES + (i > 0 ? i - 1 : 0)) * BTAB_ROW_WORDS;
}

// keyed_comb_wide with the rows staged: A row of position j-1 is issued
// right after the A addition of position j has read its stage, the B row
// likewise, so each row has one whole position (two additions) to arrive.
// stage: this wave's 2 x kStageWords of LDS (A, B).
__device__ __forceinline__ bool keyed_comb_wide_dma(ge_p3& acc, const uint32_t* key_pk, bool key_ok,
                                                    const uint32_t* sig_ptr, const uint8_t* msg, uint32_t mlen,
                                                    const uint32_t* wtab, const uint32_t* btab, uint32_t* stage) {
  uint32_t kLo[8], kHi[8], sLo[8], sHi[8];
  const bool ok = keyed_wide_digits(kLo, kHi, sLo, sHi, key_pk, key_ok, sig_ptr, msg, mlen);
  const uint32_t ldsA = (uint32_t)reinterpret_cast<uintptr_t>(stage);
  const uint32_t ldsB = ldsA + kStageWords * 4u;
  const uint32_t lane = threadIdx.x & 63;
  const LdsRow ra{stage + 4 * lane}, rb{stage + kStageWords + 4 * lane};
  int dA = (int)sc_shift_out(kHi, 16) - 0x8000;
  int dB = (int)sc_shift_out(sHi, 16) - 0x8000;
  stage_row<40>(ldsA, wide_row(wtab, WIDE_POSITIONS - 1, dA));
  stage_row<48>(ldsB, bc16_row(btab, WIDE_POSITIONS - 1, dB));
  p3_identity(acc);
  ge_efgh t;
#pragma unroll 1
  for (int j = WIDE_POSITIONS - 1; j >= 0; j--) {
    stage_wait<9>();  // A row j (B row j's 9 pieces may still be in flight)
    ge_add_table<false>(t, acc, ra, 0, dA < 0, dA == 0);
    efgh_to_p3(acc, t);
    if (j > 0) {
      dA = (int)(j > 8 ? sc_shift_out(kHi, 16) : sc_shift_out(kLo, 16)) - 0x8000;
      stage_row<40>(ldsA, wide_row(wtab, j - 1, dA));
      stage_wait<9>();  // B row j (A row j-1 in flight)
    } else {
      stage_wait<0>();
    }
    ge_add_table<false>(t, acc, rb, 0, dB < 0, dB == 0);
    efgh_to_p3(acc, t);
    if (j > 0) {
      dB = (int)(j > 8 ? sc_shift_out(sHi, 16) : sc_shift_out(sLo, 16)) - 0x8000;
      stage_row<48>(ldsB, bc16_row(btab, j - 1, dB));
    }
  }
  return ok;
}

// keyed.h keyed_comb_mixed with the table rows fetched one addition ahead:
// each addition's three niels coordinates (its row of the key's radix-256
// comb or of B's radix-2^16 comb, both MALL / HBM resident) are loaded into
// registers while the previous addition computes, so the load latency hides
// behind it instead of stalling every addition (the plain form waits on
// memory ~22 % of its wave cycles, profiles/r05_pmc_sq.txt). Same additions
// in the same order, so the same R' (the batched kernels' parity tests).
struct PfRow {
  fe c0, c1, c2;
  bool neg, ident;
};
struct PfRowTab {  // a fetched row as an ge_add_table source
  const PfRow& r;
  __device__ __forceinline__ void load_fe(int, int c, fe& q) const {
#pragma unroll
    for (int i = 0; i < 10; i++) q.v[i] = c == 0 ? r.c0.v[i] : (c == 1 ? r.c1.v[i] : r.c2.v[i]);
  }
};

__device__ __forceinline__ bool keyed_comb_mixed_pf(ge_p3& acc, const uint32_t* key_pk, bool key_ok,
                                                    const uint32_t* sig_ptr, const uint8_t* msg, uint32_t mlen,
                                                    const uint32_t* __restrict__ ktab,
                                                    const uint32_t* __restrict__ btab) {
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 8; i++) w[i] = sig_ptr[8 + i];  // S
  const bool ok = key_ok && (w[7] & 0xE0000000u) == 0 && sc_is_canonical(w);
  uint32_t sLo[8], sHi[8], tk[8];
  hs_digits65536(sLo, sHi, w);
  uint32_t h[16], k[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    w[i] = sig_ptr[i];  // R
    w[8 + i] = key_pk[i];
  }
  sha512_prefixed<16>(h, w, msg, mlen);
  sc_reduce512(k, h);
  sc_bias(tk, k, 0x80808080u);
  // the additions in keyed_comb_mixed's order: A position j = 31..0, and
  // after each odd j the B position j >> 1
  int j = COMB_WINDOWS - 1;
  bool next_b = false;
  auto fetch = [&](PfRow& r) {
    if (!next_b) {
      const int d = (int)sc_shift_out(tk, 8) - 128;
      const int i = d < 0 ? -d : d;
      const DevCombWindow win{ktab + ((size_t)j * COMB_ENTRIES + (i > 0 ? i - 1 : 0)) * COMB_ROW_WORDS};
      win.load_fe(0, 0, r.c0);
      win.load_fe(0, 1, r.c1);
      win.load_fe(0, 2, r.c2);
      r.neg = d < 0;
      r.ident = i == 0;
      if (j & 1)
        next_b = true;
      else
        j--;
    } else {
      const int jb = j >> 1;
      const int d = (int)(jb >= 8 ? sc_shift_out(sHi, 16) : sc_shift_out(sLo, 16)) - 0x8000;
      const int i = d < 0 ? -d : d;
      const DevBTab bt{btab + (size_t)(BC16_BASE + jb * BT16_ENTRIES + (i > 0 ? i - 1 : 0)) * BTAB_ROW_WORDS};
      bt.load_fe(0, 0, r.c0);
      bt.load_fe(0, 1, r.c1);
      bt.load_fe(0, 2, r.c2);
      r.neg = d < 0;
      r.ident = i == 0;
      next_b = false;
      j--;
    }
  };
  constexpr int kSteps = COMB_WINDOWS + COMB_WINDOWS / 2;  // 48
  static_assert(kSteps % 2 == 0, "ping-pong over pairs of additions");
  p3_identity(acc);
  ge_efgh t;
  PfRow r0, r1;
  fetch(r0);
#pragma unroll 1
  for (int st = 0; st < kSteps; st += 2) {
    fetch(r1);
    ge_add_table<false>(t, acc, PfRowTab{r0}, 0, r0.neg, r0.ident);
    efgh_to_p3(acc, t);
    if (st + 2 < kSteps) fetch(r0);
    ge_add_table<false>(t, acc, PfRowTab{r1}, 0, r1.neg, r1.ident);
    efgh_to_p3(acc, t);
  }
  return ok;
}

// R' = [s]B - [k]A of one signature by registered key kid over the tables
// COMB selects: ktabs = the key combs (wide for kCombWideDma, else radix-256),
// btab = the B table, whose BC16 blocks are B's radix-2^16 comb.
template <int COMB>
__device__ __forceinline__ bool keyed_comb_dev(ge_p3& acc, uint32_t kid, bool key_ok,
                                               const uint32_t* __restrict__ keys_pk, const uint32_t* sig_ptr,
                                               const uint8_t* msg, uint32_t mlen, const uint32_t* __restrict__ ktabs,
                                               const uint32_t* __restrict__ btab, uint32_t* stage) {
  if (COMB == kCombWideDma)
    return keyed_comb_wide_dma(acc, keys_pk + 8 * (size_t)kid, key_ok, sig_ptr, msg, mlen,
                               ktabs + (size_t)kid * WIDE_TABLE_WORDS, btab, stage);
  return keyed_comb_mixed_pf(acc, keys_pk + 8 * (size_t)kid, key_ok, sig_ptr, msg, mlen,
                             ktabs + (size_t)kid * COMB_TABLE_WORDS, btab);
}

// this wave's LDS stage (kCombWideDma only; one wave per workgroup)
#define CMTV_KEYED_STAGE                                                          \
  __shared__ uint32_t stage_[COMB == kCombWideDma ? 2 * kStageWords : 1];

// One signature per lane by registered key key_idx[i] (keyed.h). An index
// outside the key set yields an invalid verdict, never an out-of-bounds read.
template <uint32_t MODE, int COMB>
__global__ __launch_bounds__(64, CMTV_KEYED_WAVES_PER_EU) void k_verify_keyed(
    uint32_t n, uint32_t n_keys, const uint32_t* __restrict__ key_idx, const uint32_t* __restrict__ sig,
    const uint8_t* __restrict__ msg, const uint32_t* __restrict__ off, const uint32_t* __restrict__ keys_pk,
    const uint8_t* __restrict__ keys_ok, const uint32_t* __restrict__ ktabs, const uint32_t* __restrict__ btab,
    uint8_t* __restrict__ out_valid, uint64_t* __restrict__ out_bitmap) {
  CMTV_KEYED_STAGE
  const uint32_t gid = blockIdx.x * 64 + threadIdx.x;
  const bool active = gid < n;
  const uint32_t i = active ? gid : n - 1;
  const uint32_t m0 = off[i], m1 = off[i + 1];
  uint32_t kid = key_idx[i];
  const bool kin = kid < n_keys;
  kid = kin ? kid : 0;
  ge_p3 acc;
  const bool ok = keyed_comb_dev<COMB>(acc, kid, kin && keys_ok[kid] != 0, keys_pk, sig + 16 * (size_t)i, msg + m0,
                                       m1 - m0, ktabs, btab, stage_);
  bool v = check_R<MODE>(acc, sig + 16 * (size_t)i) && ok;
  v = v && active;
  if (active && out_valid) out_valid[gid] = v ? 1 : 0;
  const uint64_t mask = __ballot(v);
  if (threadIdx.x == 0 && out_bitmap) out_bitmap[gid >> 6] = mask;
}

// Registered-key verification with KB signatures per lane sharing one field
// inversion (Montgomery's trick: one 265-operation inversion and 3 (KB - 1)
// products instead of KB inversions):
//   GO_STDLIB: the final encode needs 1/Z of every R' (check_R_go_zi);
//   ZIP215:    the coset check (verify_core.h zip_coset) replaces decoding R
//              (a square-root chain per signature); the sign of the one
//              matching coset point's x needs 1/Z of that point.
// Signature s = gid + r * lanes (round r), so every round of a wave covers 64
// consecutive signatures and one bitmap word. Per signature the lane scratch
// holds (word-major, coalesced) Go: R'.X, R'.Y, Z, prefix product; ZIP: x
// numerator, -, Z, prefix product. A Z of 0 (possible only from an
// undecodable key's comb, whose verdicts are false anyway) enters the product
// as 1 so it cannot spoil the lane's other signatures. Verdicts equal
// verify_keyed<MODE>'s.
template <uint32_t MODE, int KB, int COMB>
__global__ __launch_bounds__(64, CMTV_KEYED_WAVES_PER_EU) void k_verify_keyed_batch(
    uint32_t n, uint32_t n_keys, const uint32_t* __restrict__ key_idx, const uint32_t* __restrict__ sig,
    const uint8_t* __restrict__ msg, const uint32_t* __restrict__ off, const uint32_t* __restrict__ keys_pk,
    const uint8_t* __restrict__ keys_ok, const uint32_t* __restrict__ ktabs, const uint32_t* __restrict__ btab,
    uint32_t* __restrict__ scr, uint8_t* __restrict__ out_valid, uint64_t* __restrict__ out_bitmap) {
  CMTV_KEYED_STAGE
  const uint32_t lanes = gridDim.x * 64u, gid = blockIdx.x * 64u + threadIdx.x;
  DevCombScratch sc{scr, lanes, gid};  // slot j: 10 words at [(j * 10 + i) * lanes + gid]
  uint32_t okbits = 0;  // per round: bit 0 ok, bits 1-2 the ZIP coset state
#pragma unroll 1
  for (int r = 0; r < KB; r++) {
    const uint32_t s = gid + (uint32_t)r * lanes;
    const bool active = s < n;
    const uint32_t i = active ? s : n - 1;
    const uint32_t m0 = off[i], m1 = off[i + 1];
    uint32_t kid = key_idx[i];
    const bool kin = kid < n_keys;
    kid = kin ? kid : 0;
    ge_p3 acc;
    bool ok = keyed_comb_dev<COMB>(acc, kid, kin && keys_ok[kid] != 0, keys_pk, sig + 16 * (size_t)i, msg + m0,
                                   m1 - m0, ktabs, btab, stage_);
    fe z, xn;
    uint32_t state = 0;
    if (MODE == MODE_ZIP215) {
      uint32_t rw[8];
      load_words(rw, sig + 16 * (size_t)i, 2);  // R
      state = zip_coset(xn, z, acc, rw);
    } else {
      z = acc.Z;
    }
    const bool zbad = fe_iszero(z);
    {
      fe one;
      fe_1(one);
      fe_select(z, z, one, zbad);
    }
    ok = ok && !zbad && active;
    okbits |= ((ok ? 1u : 0u) | (state << 1)) << (3 * r);
    // the running product goes through the scratch too, so nothing but
    // okbits stays live across the combs (their register budget is full)
    fe prod;
    if (r == 0) {
      prod = z;
    } else {
      sc.load(4 * (r - 1) + 3, prod);
      fe_mul(prod, prod, z);
    }
    if (MODE == MODE_ZIP215) {
      sc.store(4 * r + 0, xn);
    } else {
      sc.store(4 * r + 0, acc.X);
      sc.store(4 * r + 1, acc.Y);
    }
    sc.store(4 * r + 2, z);
    sc.store(4 * r + 3, prod);
  }
  fe inv;
  {
    fe prod;
    sc.load(4 * (KB - 1) + 3, prod);
    fe_invert(inv, prod);
  }
#pragma unroll 1
  for (int r = KB - 1; r >= 0; r--) {
    const uint32_t s = gid + (uint32_t)r * lanes;
    const bool active = s < n;
    const uint32_t i = active ? s : n - 1;
    fe z, zi;
    sc.load(4 * r + 2, z);
    if (r > 0) {
      fe pre;
      sc.load(4 * (r - 1) + 3, pre);
      fe_mul(zi, inv, pre);  // 1 / Z_r
      fe_mul(inv, inv, z);   // 1 / (Z_0 ... Z_{r-1})
    } else {
      zi = inv;
    }
    uint32_t rw[8];
    load_words(rw, sig + 16 * (size_t)i, 2);  // R
    const uint32_t bits = okbits >> (3 * r);
    bool v;
    if (MODE == MODE_ZIP215) {
      fe xn;
      sc.load(4 * r + 0, xn);
      v = zip_coset_finish((bits >> 1) & 3u, xn, zi, rw[7]);
    } else {
      fe X, Y;
      sc.load(4 * r + 0, X);
      sc.load(4 * r + 1, Y);
      v = check_R_go_zi(X, Y, zi, rw);
    }
    v = v && (bits & 1u) != 0;
    if (active && out_valid) out_valid[s] = v ? 1 : 0;
    const uint64_t mask = __ballot(v);
    const uint32_t word = s >> 6;
    if (threadIdx.x == 0 && out_bitmap && word < (n + 63) / 64) out_bitmap[word] = mask;
  }
}

template <int COMB>
static void launch_lane(uint32_t mode, uint32_t n, uint32_t n_keys, const uint32_t* ki, const uint32_t* sgp,
                        const uint8_t* mp, const uint32_t* op, const uint32_t* keys_pk, const uint8_t* keys_ok,
                        const uint32_t* tabs, const uint32_t* bsrc, uint8_t* vp, uint64_t* bp, uint32_t batch_kb,
                        uint32_t* scr, hipStream_t s) {
  if (batch_kb >= 4 && scr) {
    // batch_kb signatures per lane sharing one inversion (k_verify_keyed_batch)
    const dim3 grid((n + 64 * batch_kb - 1) / (64 * batch_kb)), block(64);
    if (mode == MODE_ZIP215 && batch_kb >= 8)
      hipLaunchKernelGGL((k_verify_keyed_batch<MODE_ZIP215, 8, COMB>), grid, block, 0, s, n, n_keys, ki, sgp, mp, op,
                         keys_pk, keys_ok, tabs, bsrc, scr, vp, bp);
    else if (mode == MODE_ZIP215)
      hipLaunchKernelGGL((k_verify_keyed_batch<MODE_ZIP215, 4, COMB>), grid, block, 0, s, n, n_keys, ki, sgp, mp, op,
                         keys_pk, keys_ok, tabs, bsrc, scr, vp, bp);
    else if (batch_kb >= 8)
      hipLaunchKernelGGL((k_verify_keyed_batch<MODE_GO_STDLIB, 8, COMB>), grid, block, 0, s, n, n_keys, ki, sgp, mp,
                         op, keys_pk, keys_ok, tabs, bsrc, scr, vp, bp);
    else
      hipLaunchKernelGGL((k_verify_keyed_batch<MODE_GO_STDLIB, 4, COMB>), grid, block, 0, s, n, n_keys, ki, sgp, mp,
                         op, keys_pk, keys_ok, tabs, bsrc, scr, vp, bp);
    return;
  }
  const dim3 grid((n + 63) / 64), block(64);
  if (mode == MODE_ZIP215)
    hipLaunchKernelGGL((k_verify_keyed<MODE_ZIP215, COMB>), grid, block, 0, s, n, n_keys, ki, sgp, mp, op, keys_pk,
                       keys_ok, tabs, bsrc, vp, bp);
  else
    hipLaunchKernelGGL((k_verify_keyed<MODE_GO_STDLIB, COMB>), grid, block, 0, s, n, n_keys, ki, sgp, mp, op,
                       keys_pk, keys_ok, tabs, bsrc, vp, bp);
}

hipError_t launch_verify_keyed_lane(uint32_t mode, uint32_t n, uint32_t n_keys, const uint32_t* ki,
                                    const uint32_t* sgp, const uint8_t* mp, const uint32_t* op,
                                    const uint32_t* keys_pk, const uint8_t* keys_ok, const uint32_t* ktabs,
                                    uint8_t* vp, uint64_t* bp, uint32_t batch_kb, uint32_t* scr,
                                    const uint32_t* wtabs, const uint32_t* btab, hipStream_t s) {
  if (n == 0) return hipSuccess;
  if (!btab) return hipErrorInvalidValue;
  if (wtabs)
    launch_lane<kCombWideDma>(mode, n, n_keys, ki, sgp, mp, op, keys_pk, keys_ok, wtabs, btab, vp, bp, batch_kb, scr,
                              s);
  else
    launch_lane<kCombMixed>(mode, n, n_keys, ki, sgp, mp, op, keys_pk, keys_ok, ktabs, btab, vp, bp, batch_kb, scr, s);
  return hipGetLastError();
}

// ---------------------------------------------------------------- wide comb build

// Position bases 2^(16j) (-A) of the wide combs (keyed.h), thread = (key, j):
// 16 j doublings of -A, stored as extended points (40 words).
__global__ __launch_bounds__(64) void k_wide_bases(uint32_t n_keys, const uint32_t* __restrict__ keys_pk,
                                                   uint32_t* __restrict__ bases) {
  const uint32_t gid = blockIdx.x * 64 + threadIdx.x;
  if (gid >= n_keys * WIDE_POSITIONS) return;
  const uint32_t key = gid / WIDE_POSITIONS, j = gid % WIDE_POSITIONS;
  uint32_t w[8];
  load_words(w, keys_pk + 8 * (size_t)key, 2);
  ge_p3 A, P;
  (void)p3_frombytes(A, w);  // an undecodable key's rows are never trusted (keys_ok)
  cached_neg_point(P, A);
  if (j > 0) {
    ge_p2 q;
    ge_efgh t;
    p3_to_p2(q, P);
#pragma unroll 1
    for (uint32_t r = 0; r < 16 * j; r++) {
      p2_dbl(t, q);
      efgh_to_p2(q, t);
    }
    efgh_to_p3(P, t);
  }
  uint32_t* o = bases + (size_t)gid * 40;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    o[i] = P.X.v[i];
    o[10 + i] = P.Y.v[i];
    o[20 + i] = P.Z.v[i];
    o[30 + i] = P.T.v[i];
  }
}

// Wide comb rows, thread = (key = blockIdx.y, position j, run b): rows
// 64 b .. 64 b + 63 of position j (wide_build_run).
__global__ __launch_bounds__(64) void k_wide_build(const uint32_t* __restrict__ bases, uint32_t* __restrict__ tabs,
                                                   uint32_t* __restrict__ scratch) {
  constexpr uint32_t kRuns = WIDE_ENTRIES / WIDE_RUN;
  const uint32_t key = blockIdx.y, tid = blockIdx.x * 64 + threadIdx.x;
  const uint32_t j = tid / kRuns, b = tid % kRuns;
  const uint32_t* pb = bases + ((size_t)key * WIDE_POSITIONS + j) * 40;
  ge_p3 P;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    P.X.v[i] = pb[i];
    P.Y.v[i] = pb[10 + i];
    P.Z.v[i] = pb[20 + i];
    P.T.v[i] = pb[30 + i];
  }
  const uint32_t per_key = gridDim.x * 64u;
  DevCombScratch sc{scratch, gridDim.y * per_key, key * per_key + tid};
  wide_build_run(tabs + (size_t)key * WIDE_TABLE_WORDS + (size_t)j * WIDE_ENTRIES * COMB_ROW_WORDS, P,
                 (int)(b * WIDE_RUN), sc);
}

static_assert(kWideTableWords == WIDE_TABLE_WORDS, "kernels.h / keyed.h wide comb size");
static_assert(kWideScratchWordsPerKey == (size_t)WIDE_POSITIONS * (WIDE_ENTRIES / WIDE_RUN) * WIDE_RUN * 10,
              "wide build scratch: WIDE_RUN prefix products per thread");

hipError_t launch_wide_build(uint32_t n_keys, const void* keys_pk, uint32_t* tabs, uint32_t* bases,
                             uint32_t* scratch, hipStream_t s) {
  if (n_keys == 0) return hipSuccess;
  hipLaunchKernelGGL(k_wide_bases, dim3((n_keys * WIDE_POSITIONS + 63) / 64), dim3(64), 0, s, n_keys,
                     static_cast<const uint32_t*>(keys_pk), bases);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_wide_build, dim3(WIDE_POSITIONS * (WIDE_ENTRIES / WIDE_RUN) / 64, n_keys), dim3(64), 0, s,
                     bases, tabs, scratch);
  return hipGetLastError();
}

}  // namespace cmtv
