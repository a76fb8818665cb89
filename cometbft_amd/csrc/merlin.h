// merlin.h -- the sr25519 verification transcript: merlin (STROBE-128 over
// Keccak-f[1600]) as go-schnorrkel v1.0.0 drives it from
// /root/reference/crypto/sr25519/pubkey.go:34-60:
//
//   t = merlin.NewTranscript("SigningContext")       dom-sep
//   t.AppendMessage("", {})                          NewSigningContext([]byte{}, msg)
//   t.AppendMessage("sign-bytes", msg)
//   t.AppendMessage("proto-name", "Schnorr-sig")     PublicKey.Verify
//   t.AppendMessage("sign:pk", pk)
//   t.AppendMessage("sign:R", R)
//   k = t.ExtractBytes("sign:c", 64)  (mod L by the caller)
//
// GPU layout. Everything before the message length is the same for every
// signature (STROBE's initial permutation, "Merlin v1.0", the dom-sep /
// signing-context / "sign-bytes" headers), so the host runs it once
// (sr_prefix_state, a plain byte-level STROBE) and the device starts from
// that sponge (the "program": 50 state words, pos, pos_begin). Then:
//   1. LE32(mlen), the begin_op header and the message, 4-byte chunks in one
//      rolled loop (the wave's longest message; shorter ones absorb nothing
//      for the extra trips) with the Keccak-f at pos == R inside it;
//   2. the tail -- "proto-name" ... "sign:c" and the PRF header, 136 bytes
//      with pk and R -- as straight-line code. 136 < R, so the tail meets
//      the block end at most once: it is emitted twice, pass 0 writing the
//      bytes that fall in the current block and pass 1 those past its end,
//      each pass followed by its Keccak-f (the block's, then the PRF's), in
//      a two-trip loop: one more Keccak call site, no branch per chunk.
// begin_op's pos_begin bytes in the tail follow from the stream positions
// (an F between two headers resets it), so both passes compute the same
// values. A taken branch costs an instruction fetch and one wave per SIMD
// hides none of it: the per-chunk work is selects and a store.
//
// The sponge (25 x u64) stays in registers; the bytes of the current STROBE
// block gather into block words -- the partial word in a register, every
// chunk stored to a per-lane block buffer through the State policy (LDS on
// the device, lane-interleaved; a plain array on the host) -- and are XORed
// into the sponge once, at the block's run_f:
//   void store(int i, uint32_t w);   block word i (bytes 4i..4i+3), 0..41
//   uint32_t load(int i) const;
#pragma once
#include <stdint.h>

#include "keccak.h"

#ifndef CMTV_HD
#define CMTV_HD __host__ __device__ __forceinline__
#endif

namespace cmtv {

constexpr int STROBE_R = 166;
constexpr int STROBE_BLOCK_WORDS = 42;  // R + 2 bytes: the block with its padding
constexpr uint32_t SF_I = 1, SF_A = 2, SF_C = 4, SF_T = 8, SF_M = 16, SF_K = 32;
// the device program: the sponge after the constant prefix
constexpr int SR_PREFIX_WORDS = 52;  // 50 state words, pos, pos_begin

// ---- host: the constant prefix, byte by byte ------------------------------
struct HostStrobe {
  uint64_t a[25] = {};
  int pos = 0, pos_begin = 0;
  void xor_byte(int p, uint32_t b) { a[p >> 3] ^= (uint64_t)(b & 0xFF) << (8 * (p & 7)); }
  void run_f() {
    xor_byte(pos, (uint32_t)pos_begin);
    xor_byte(pos + 1, 0x04);
    xor_byte(STROBE_R + 1, 0x80);
    keccak_f1600(a);
    pos = 0;
    pos_begin = 0;
  }
  void absorb(uint32_t b) {
    xor_byte(pos++, b);
    if (pos == STROBE_R) run_f();
  }
  void begin(uint32_t flags) {  // begin_op, not "more"
    const int old = pos_begin;
    pos_begin = pos + 1;
    absorb((uint32_t)old);
    absorb(flags);
  }
  void lit(const char* s) {
    for (; *s; s++) absorb((uint8_t)*s);
  }
  void lit_u32(uint32_t v) {
    for (int i = 0; i < 4; i++) absorb(v >> (8 * i));
  }
};

// merlin.NewTranscript("SigningContext"), AppendMessage("", {}), and the
// "sign-bytes" label of AppendMessage("sign-bytes", msg): the sponge the
// device program starts from. Returns SR_PREFIX_WORDS.
inline int sr_prefix_state(uint32_t out[SR_PREFIX_WORDS]) {
  HostStrobe s;
  // Strobe128::new("Merlin v1.0"): [1, R+2, 1, 0, 1, 96] || "STROBEv1.0.2", F
  s.a[0] = 0x545360010001A801ull;
  s.a[1] = 0x302E317645424F52ull;
  s.a[2] = 0x000000000000322Eull;
  keccak_f1600(s.a);
  s.begin(SF_M | SF_A);  // meta_ad("Merlin v1.0")
  s.lit("Merlin v1.0");
  // AppendMessage(label, m): meta_ad(label), meta_ad(LE32(len), more), ad(m)
  s.begin(SF_M | SF_A);
  s.lit("dom-sep");
  s.lit_u32(14);
  s.begin(SF_A);
  s.lit("SigningContext");
  s.begin(SF_M | SF_A);
  s.lit_u32(0);
  s.begin(SF_A);
  s.begin(SF_M | SF_A);
  s.lit("sign-bytes");
  for (int i = 0; i < 25; i++) {
    out[2 * i] = (uint32_t)s.a[i];
    out[2 * i + 1] = (uint32_t)(s.a[i] >> 32);
  }
  out[50] = (uint32_t)s.pos;
  out[51] = (uint32_t)s.pos_begin;
  return SR_PREFIX_WORDS;
}

// Word i of the program. On the device the index is a constant, so the word
// comes through the scalar cache (a constant-address-space load).
CMTV_HD uint32_t sr_word(const uint32_t* prog, int i) {
#if defined(__HIP_DEVICE_COMPILE__)
  const __attribute__((address_space(4))) uint32_t* c =
      (const __attribute__((address_space(4))) uint32_t*)(reinterpret_cast<uintptr_t>(prog));
  return c[i];
#else
  return prog[i];
#endif
}

CMTV_HD uint32_t sr_bytes_mask(int n) { return n >= 4 ? 0xFFFFFFFFu : (1u << (8 * n)) - 1u; }

// The sponge as the device keeps it: the permutation state, the STROBE
// position and begin offset, and the current block's bytes (words
// [wlo, pos/4] in the block buffer, the partial one also in acc).
template <class Blk>
struct StrobeSponge {
  uint64_t a[25];
  int pos, pos_begin, wlo;
  uint32_t acc;
  Blk& blk;

  // n (0..4) bytes v (bytes past n zero) at pos, pos + n <= R + 2. The word
  // is stored complete or not (a later put stores it again), so no branch.
  CMTV_HD void put(uint32_t v, int n) {
    const int f = pos & 3;
    const uint64_t t = (uint64_t)acc | ((uint64_t)v << (8 * f));
    blk.store(pos >> 2, (uint32_t)t);
    acc = f + n >= 4 ? (uint32_t)(t >> 32) : (uint32_t)t;
    pos += n;
  }
  // STROBE run_f with pos_begin pb: pad, fold the block into the state,
  // permute
  CMTV_HD void run_f(int pb) {
    put((uint32_t)pb | 0x0400u, 2);         // pos_begin at pos, 0x04 at pos + 1
    if (pos & 3) blk.store(pos >> 2, acc);  // a word the pad began
    const int whi = (pos + 3) >> 2;
    // every word is read (the loads issue back to back); the ones outside
    // [wlo, whi) are stale and masked off
#pragma unroll
    for (int i = 0; i < 21; i++) {
      const uint32_t l = blk.load(2 * i), h = blk.load(2 * i + 1);
      const uint32_t lo = 2 * i >= wlo && 2 * i < whi ? l : 0u;
      const uint32_t hi = 2 * i + 1 >= wlo && 2 * i + 1 < whi ? h : 0u;
      a[i] ^= (uint64_t)lo | ((uint64_t)hi << 32);
    }
    a[20] ^= 0x80ull << 56;  // 0x80 at R + 1
    keccak_f1600(a);
    pos = 0;
    pos_begin = 0;
    wlo = 0;
    acc = 0;
  }
  // k (0..4) bytes of v, the F at pos == R
  CMTV_HD void absorb(uint32_t v, int k) {
    const int room = STROBE_R - pos;  // >= 1
    const int n1 = k < room ? k : room;
    put(v & sr_bytes_mask(n1), n1);
    if (k >= room) run_f(pos_begin);
    const int n2 = k > room ? k - room : 0;
    put(room < 4 ? (v >> (8 * room)) & sr_bytes_mask(n2) : 0u, n2);
  }
};

// One pass over the tail: the bytes at stream positions [lo, lo + R) (pass 0:
// the current block, from the tail's start; pass 1: past its end) go to the
// sponge's block, in order; begin_op headers track pos_begin from the
// positions.
template <class Blk>
struct SrTailPass {
  StrobeSponge<Blk>& sp;
  int lo;        // R * pass
  int P;         // stream position of the next byte (the current block's origin)
  int hdr_p;     // position of the last header's first byte
  int pb;        // the pos_begin the next header absorbs
  int cross_pb;  // pos_begin at the block end (the F between the passes)

  CMTV_HD void bytes(uint32_t v, int k) {
    int s = lo - P, e = lo + STROBE_R - P;
    s = s < 0 ? 0 : s > k ? k : s;
    e = e < 0 ? 0 : e > k ? k : e;
    const int n = e - s;
    sp.put(s < 4 ? (v >> (8 * s)) & sr_bytes_mask(n) : 0u, n);
    P += k;
  }
  // begin_op(flags): absorb [pos_begin, flags], pos_begin = pos + 1; the
  // block-end F resets it
  CMTV_HD void hdr(uint32_t flags) {
    const bool f_between = hdr_p < STROBE_R && P >= STROBE_R;
    const uint32_t v = (uint32_t)(f_between ? 0 : pb);
    cross_pb = P < STROBE_R ? P + 1 : cross_pb;
    hdr_p = P;
    pb = (P < STROBE_R ? P : P - STROBE_R) + 1;
    bytes(v | (flags << 8), 2);
  }
  template <int N>
  CMTV_HD void lit(const char (&s)[N]) {
#pragma unroll
    for (int i = 0; i < N - 1; i += 4) {
      uint32_t w = 0;
#pragma unroll
      for (int j = 0; j < 4; j++) w |= i + j < N - 1 ? (uint32_t)(uint8_t)s[i + j] << (8 * j) : 0u;
      bytes(w, N - 1 - i < 4 ? N - 1 - i : 4);
    }
  }
  CMTV_HD void u32(uint32_t v) { bytes(v, 4); }
  // AppendMessage(label, <len bytes>): meta_ad(label), meta_ad(LE32(len),
  // more), then begin_op(A) of ad(message)
  template <int N>
  CMTV_HD void header(const char (&label)[N], uint32_t len) {
    hdr(SF_M | SF_A);
    lit(label);
    u32(len);
    hdr(SF_A);
  }
};

// Runs the transcript; out = the 64 challenge bytes as 16 little-endian
// words. prog: the SR_PREFIX_WORDS of sr_prefix_state. pk / R: 8
// little-endian words each; msg: mlen bytes at any alignment. On the device
// every lane of the wave calls it together (cross-lane maximum and vote).
template <class State>
CMTV_HD void sr_transcript(uint32_t out[16], State& st, const uint32_t* prog, int nprog, const uint8_t* msg,
                           uint32_t mlen, const uint32_t pk[8], const uint32_t R[8]) {
  (void)nprog;
  StrobeSponge<State> sp{{}, 0, 0, 0, 0u, st};
#pragma unroll
  for (int i = 0; i < 25; i++) sp.a[i] = (uint64_t)sr_word(prog, 2 * i) | ((uint64_t)sr_word(prog, 2 * i + 1) << 32);
  sp.pos = (int)sr_word(prog, 50);
  sp.pos_begin = (int)sr_word(prog, 51);
  sp.wlo = sp.pos >> 2;  // the words below hold prefix bytes already in the state

  // ---- 1. LE32(mlen), begin_op(A), the message
  const uint32_t sh = (uint32_t)((uintptr_t)msg & 3);
  const uint32_t* mw = reinterpret_cast<const uint32_t*>(msg - sh);  // keeps msg's address space
  const uint32_t mlast = mlen ? (sh + mlen - 1) >> 2 : 0;             // last word holding a message byte
  const uint32_t mchunks = (mlen + 3) >> 2;
  uint32_t mtrips = mchunks;  // the wave's longest message
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const uint32_t x = (uint32_t)__shfl_xor((int)mtrips, o);
    mtrips = x > mtrips ? x : mtrips;
  }
  // every lane holds the maximum; say so, or the trip count turns divergent
  mtrips = __builtin_amdgcn_readfirstlane(mtrips);
#endif
  uint32_t mv0 = 0, mv1 = 0, mv2 = 0, mv3 = 0;  // the message's chunks 4g .. 4g+3, fetched at chunk 4g
#pragma unroll 1
  for (uint32_t t = 0; t < mtrips + 2; t++) {
    const uint32_t j = t - 2;  // message chunk (t >= 2)
    if (t >= 2 && (j & 3) == 0 && j < mchunks) {
      // five words (independent loads, one wait) -> four chunks
      const uint32_t g0 = mw[j < mlast ? j : mlast], g1 = mw[j + 1 < mlast ? j + 1 : mlast],
                     g2 = mw[j + 2 < mlast ? j + 2 : mlast], g3 = mw[j + 3 < mlast ? j + 3 : mlast],
                     g4 = mw[j + 4 < mlast ? j + 4 : mlast];
      const uint32_t b = 8 * sh;
      mv0 = sh ? (uint32_t)((((uint64_t)g1 << 32) | g0) >> b) : g0;
      mv1 = sh ? (uint32_t)((((uint64_t)g2 << 32) | g1) >> b) : g1;
      mv2 = sh ? (uint32_t)((((uint64_t)g3 << 32) | g2) >> b) : g2;
      mv3 = sh ? (uint32_t)((((uint64_t)g4 << 32) | g3) >> b) : g3;
    }
    const uint32_t cq = j & 3;
    const uint32_t vm = cq == 0 ? mv0 : cq == 1 ? mv1 : cq == 2 ? mv2 : mv3;
    const uint32_t left = t >= 2 && j < mchunks ? mlen - 4 * j : 0u;
    const uint32_t vh = (uint32_t)sp.pos_begin | (SF_A << 8);  // begin_op(A): [pos_begin, A]
    sp.pos_begin = t == 1 ? sp.pos + 1 : sp.pos_begin;
    const uint32_t v = t == 0 ? mlen : t == 1 ? vh : vm;
    const int k = t == 0 ? 4 : t == 1 ? 2 : (int)(left < 4 ? left : 4);
    sp.absorb(v, k);
  }

  // ---- 2. the tail, two passes
  const int P0 = sp.pos, pb0 = sp.pos_begin;
  constexpr int kTail = 136;
  const bool crossed = P0 + kTail >= STROBE_R;
  bool any = crossed;
#if defined(__HIP_DEVICE_COMPILE__)
  any = __any(crossed);
#endif
#pragma unroll 1
  for (int r = 0; r < 2; r++) {
    SrTailPass<State> tp{sp, STROBE_R * r, P0, -1, pb0, 0};
    tp.header("proto-name", 11);
    tp.lit("Schnorr-sig");
    tp.header("sign:pk", 32);
#pragma unroll
    for (int i = 0; i < 8; i++) tp.u32(pk[i]);
    tp.header("sign:R", 32);
#pragma unroll
    for (int i = 0; i < 8; i++) tp.u32(R[i]);
    // ExtractBytes("sign:c", 64): meta_ad(label), meta_ad(LE32(64), more),
    // begin_op(I|A|C), then the F unless the header ended a block
    tp.hdr(SF_M | SF_A);
    tp.lit("sign:c");
    tp.u32(64);
    tp.hdr(SF_I | SF_A | SF_C);
    // pass 0: the block-end F (crossed) or the PRF's; pass 1: the PRF's,
    // unless the header ended exactly at the block end
    const bool prf_reset = tp.hdr_p < STROBE_R && tp.P >= STROBE_R;  // the block end came after it began
    const int prf_pb = prf_reset ? 0 : tp.pb;
    const bool do_f = r == 0 ? true : crossed && tp.P != STROBE_R;
    const int pad_pb = r == 0 && crossed ? tp.cross_pb : prf_pb;
    if (do_f) sp.run_f(pad_pb);
    if (!any) break;
  }
#pragma unroll
  for (int i = 0; i < 8; i++) {
    out[2 * i] = (uint32_t)sp.a[i];
    out[2 * i + 1] = (uint32_t)(sp.a[i] >> 32);
  }
}

// Host state policy: the block words in a plain array.
struct ArrayStrobeState {
  uint32_t w[STROBE_BLOCK_WORDS];
  void store(int i, uint32_t x) { w[i] = x; }
  uint32_t load(int i) const { return w[i]; }
};

}  // namespace cmtv
