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
// GPU layout: everything but the message, its length, pk and R is constant,
// so the transcript is a fixed program of absorb descriptors -- each one
// chunk of at most 4 bytes (a literal, a begin_op header, LE32(mlen), a key
// word, a message chunk) or a forced F -- built once on the host
// (sr_build_program) and run by one rolled loop per lane: a single Keccak
// call site however many STROBE operations the transcript has. The
// descriptor stream is the same for every lane (scalar loads; the value is
// picked by selects, not branches -- a taken branch costs an instruction
// fetch, and one wave per SIMD hides none of it); only the message's chunk
// count differs per lane (the loop runs the wave's longest message, shorter
// ones absorb nothing for the extra chunks).
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

// Descriptors: two u32 words, (data, type | bytes << 4 | index << 8).
constexpr uint32_t SD_LIT = 0;    // absorb the data's low k bytes
constexpr uint32_t SD_HDR = 1;    // begin_op(flags = data): absorb [pos_begin, flags], pos_begin = pos + 1
constexpr uint32_t SD_MLEN = 2;   // absorb LE32(mlen)
constexpr uint32_t SD_MSG = 3;    // absorb the message (one chunk per loop trip)
constexpr uint32_t SD_KEYW = 4;   // absorb word index of pk (0..7) or R (8..15)
constexpr uint32_t SD_INIT = 5;   // STROBE-128 initial state, F without padding
constexpr uint32_t SD_FORCE = 6;  // PRF: F unless the header ended a block; 64 output bytes = state[0..63]
constexpr uint32_t SD_STATE = 7;  // resume: data = pos | pos_begin << 16, then 25 (lo, hi) state pairs
constexpr int SR_STATE_DESCS = 26;
constexpr int SR_PROGRAM_MAX = 128;  // descriptors, either form
constexpr int SR_PROGRAM_WORDS = 2 * SR_PROGRAM_MAX;

// Host: the descriptor program, literal bytes packed 4 to a chunk.
struct SrProgramBuilder {
  uint32_t* w;
  int n = 0;
  uint32_t pend = 0;
  int npend = 0;
  void put(uint32_t data, uint32_t type, uint32_t k = 0, uint32_t idx = 0) {
    w[2 * n] = data;
    w[2 * n + 1] = type | (k << 4) | (idx << 8);
    n++;
  }
  void flush() {
    if (npend) put(pend, SD_LIT, (uint32_t)npend);
    pend = 0;
    npend = 0;
  }
  void byte(uint32_t b) {
    pend |= (b & 0xFF) << (8 * npend);
    if (++npend == 4) flush();
  }
  void lit(const char* s) {
    for (; *s; s++) byte((uint8_t)*s);
  }
  void lit_u32(uint32_t v) {
    for (int i = 0; i < 4; i++) byte(v >> (8 * i));
  }
  void op(uint32_t type, uint32_t data = 0, uint32_t k = 0, uint32_t idx = 0) {
    flush();
    put(data, type, k, idx);
  }
  void hdr(uint32_t flags) { op(SD_HDR, flags, 2); }
  // merlin AppendMessage(label, <message given by the following ops>)
  void append_header(const char* label) {
    hdr(SF_M | SF_A);  // meta_ad(label, false)
    lit(label);
  }
};

// The whole verification transcript (see the header comment). Returns the
// descriptor count.
inline int sr_build_program(uint32_t w[SR_PROGRAM_WORDS]) {
  SrProgramBuilder b{w};
  b.op(SD_INIT);
  b.hdr(SF_M | SF_A);  // Strobe128::new -> meta_ad("Merlin v1.0")
  b.lit("Merlin v1.0");
  b.append_header("dom-sep");
  b.lit_u32(14);  // meta_ad(LE32(len), more = true)
  b.hdr(SF_A);
  b.lit("SigningContext");
  b.append_header("");  // AppendMessage("", context = {})
  b.lit_u32(0);
  b.hdr(SF_A);
  b.append_header("sign-bytes");
  b.op(SD_MLEN, 0, 4);
  b.hdr(SF_A);
  b.op(SD_MSG);
  b.append_header("proto-name");
  b.lit_u32(11);
  b.hdr(SF_A);
  b.lit("Schnorr-sig");
  b.append_header("sign:pk");
  b.lit_u32(32);
  b.hdr(SF_A);
  for (uint32_t i = 0; i < 8; i++) b.op(SD_KEYW, 0, 4, i);
  b.append_header("sign:R");
  b.lit_u32(32);
  b.hdr(SF_A);
  for (uint32_t i = 0; i < 8; i++) b.op(SD_KEYW, 0, 4, 8 + i);
  b.append_header("sign:c");  // ExtractBytes("sign:c", 64)
  b.lit_u32(64);
  b.hdr(SF_I | SF_A | SF_C);
  b.op(SD_FORCE);
  return b.n;
}

// Word i of the program. On the device the index is wave-uniform, so the
// word comes through the scalar cache (a constant-address-space load).
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

// The sponge as the interpreter keeps it: the permutation state, the STROBE
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
  // STROBE run_f: pad (unless INIT), fold the block into the state, permute
  CMTV_HD void run_f(bool pad) {
    int whi = wlo;
    if (pad) {
      put((uint32_t)pos_begin | 0x0400u, 2);  // pos_begin at pos, 0x04 at pos + 1
      if (pos & 3) blk.store(pos >> 2, acc);   // a word the pad began
      whi = (pos + 3) >> 2;
    }
    // every word is read (the loads issue back to back); the ones outside
    // [wlo, whi) are stale and masked off
#pragma unroll
    for (int i = 0; i < 21; i++) {
      const uint32_t l = blk.load(2 * i), h = blk.load(2 * i + 1);
      const uint32_t lo = 2 * i >= wlo && 2 * i < whi ? l : 0u;
      const uint32_t hi = 2 * i + 1 >= wlo && 2 * i + 1 < whi ? h : 0u;
      a[i] ^= (uint64_t)lo | ((uint64_t)hi << 32);
    }
    if (pad) a[20] ^= 0x80ull << 56;  // 0x80 at R + 1
    keccak_f1600(a);
    pos = 0;
    pos_begin = 0;
    wlo = 0;
    acc = 0;
  }
  // k (0..4) bytes of v, the F at pos == R; force: an F regardless
  CMTV_HD void absorb(uint32_t v, int k, bool force, bool pad) {
    const int room = STROBE_R - pos;  // >= 1
    const int n1 = k < room ? k : room;
    put(v & sr_bytes_mask(n1), n1);
    if (force || k >= room) run_f(pad);
    const int n2 = k > room ? k - room : 0;
    put(room < 4 ? (v >> (8 * room)) & sr_bytes_mask(n2) : 0u, n2);
  }
};

// The sponge after a program prefix, for sr_build_device_program.
struct StrobeSnapshot {
  uint32_t w[50];
  int pos, pos_begin;
};

// Runs the program; out = the 64 challenge bytes as 16 little-endian words.
// pk / R: 8 little-endian words each; msg: mlen bytes at any alignment. On
// the device every lane of the wave calls it together (the wave's longest
// message is a cross-lane maximum).
template <class State>
CMTV_HD void sr_transcript(uint32_t out[16], State& st, const uint32_t* prog, int ndesc, const uint8_t* msg,
                           uint32_t mlen, const uint32_t pk[8], const uint32_t R[8],
                           StrobeSnapshot* snap = nullptr) {
  StrobeSponge<State> sp{{}, 0, 0, 0, 0u, st};
  // message read as aligned words (the per-lane offset is arbitrary)
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
  // every lane holds the maximum; say so, or the descriptor index that
  // follows it turns divergent (vector loads)
  mtrips = __builtin_amdgcn_readfirstlane(mtrips);
#endif
  uint32_t mv0 = 0, mv1 = 0, mv2 = 0, mv3 = 0;  // the message's chunks 4g .. 4g+3, fetched at chunk 4g
  uint32_t kw[16];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    kw[i] = pk[i];
    kw[8 + i] = R[i];
  }
  int d = 0;
  uint32_t j = 0;  // message chunk
#pragma unroll 1
  while (d < ndesc) {
    const uint32_t data = sr_word(prog, 2 * d), ctl = sr_word(prog, 2 * d + 1);
    const uint32_t type = ctl & 15;
    if (type == SD_STATE) {
      // the precomputed sponge after the transcript's constant prefix
#pragma unroll
      for (int i = 0; i < 25; i++)
        sp.a[i] = (uint64_t)sr_word(prog, 2 * d + 2 + 2 * i) | ((uint64_t)sr_word(prog, 2 * d + 3 + 2 * i) << 32);
      sp.pos = (int)(data & 0xFFFF);
      sp.pos_begin = (int)(data >> 16);
      sp.wlo = sp.pos >> 2;
      sp.acc = 0;
      d += SR_STATE_DESCS;
      continue;
    }
    if (type == SD_INIT) {
#pragma unroll
      for (int i = 0; i < 25; i++) sp.a[i] = 0;
      // [1, R+2, 1, 0, 1, 96] || "STROBEv1.0.2"
      sp.a[0] = 0x545360010001A801ull;
      sp.a[1] = 0x302E317645424F52ull;
      sp.a[2] = 0x000000000000322Eull;
    }
    int k = (int)((ctl >> 4) & 15);
    if (type == SD_MSG) {
      if ((j & 3) == 0 && j < mchunks) {
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
      const uint32_t left = j < mchunks ? mlen - 4 * j : 0u;
      k = (int)(left < 4 ? left : 4);
    }
    const uint32_t cq = j & 3;
    const uint32_t vm = cq == 0 ? mv0 : cq == 1 ? mv1 : cq == 2 ? mv2 : mv3;
    const uint32_t vh = (uint32_t)sp.pos_begin | (data << 8);
    const uint32_t v = type == SD_HDR    ? vh
                       : type == SD_MLEN ? mlen
                       : type == SD_KEYW ? kw[ctl >> 8]
                       : type == SD_MSG  ? vm
                                         : data;
    sp.pos_begin = type == SD_HDR ? sp.pos + 1 : sp.pos_begin;
    const bool force = type == SD_INIT || (type == SD_FORCE && sp.pos != 0);
    sp.absorb(v, k, force, type != SD_INIT);
    if (type == SD_FORCE) break;
    const bool more = type == SD_MSG && j + 1 < mtrips;
    j = more ? j + 1 : 0;
    d += more ? 0 : 1;
  }
  if (snap) {  // host: the sponge with the pending block folded in (no F)
    uint32_t blkw[STROBE_BLOCK_WORDS] = {};
    for (int i = sp.wlo; i < (sp.pos >> 2); i++) blkw[i] = st.load(i);
    if ((sp.pos >> 2) < STROBE_BLOCK_WORDS) blkw[sp.pos >> 2] = sp.acc;  // the partial word
    for (int i = 0; i < 25; i++) {
      snap->w[2 * i] = (uint32_t)sp.a[i] ^ (2 * i < STROBE_BLOCK_WORDS ? blkw[2 * i] : 0u);
      snap->w[2 * i + 1] = (uint32_t)(sp.a[i] >> 32) ^ (2 * i + 1 < STROBE_BLOCK_WORDS ? blkw[2 * i + 1] : 0u);
    }
    snap->pos = sp.pos;
    snap->pos_begin = sp.pos_begin;
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

// The device's form of the program: everything before the first descriptor
// that reads the input (the message length) is the same for every signature
// -- STROBE's initial permutation, "Merlin v1.0", the "dom-sep" / signing
// context / "sign-bytes" headers -- so the host runs it once (the same
// interpreter, stopped there) and the device program starts with an
// SD_STATE descriptor that loads the resulting sponge, its position and
// begin offset, then the remaining descriptors. One Keccak-f and ~70
// absorbed bytes fewer per signature; the same challenge
// (tests/host/srcheck.cpp computes it both ways).
inline int sr_build_device_program(uint32_t out[SR_PROGRAM_WORDS]) {
  uint32_t full[SR_PROGRAM_WORDS];
  const int nd = sr_build_program(full);
  int k = 0;
  while (k < nd && (full[2 * k + 1] & 15) != SD_MLEN) k++;
  ArrayStrobeState st{};
  uint32_t scratch[16];
  StrobeSnapshot snap;
  const uint32_t zero[8] = {};
  sr_transcript(scratch, st, full, k, nullptr, 0, zero, zero, &snap);
  if (snap.pos >= 65536 || snap.pos_begin >= 65536 || SR_STATE_DESCS + nd - k > SR_PROGRAM_MAX) return -1;
  int n = 0;
  out[n++] = (uint32_t)snap.pos | ((uint32_t)snap.pos_begin << 16);
  out[n++] = SD_STATE;
  for (int i = 0; i < 50; i++) out[n++] = snap.w[i];
  for (int i = 2 * k; i < 2 * nd; i++) out[n++] = full[i];
  return n / 2;
}

}  // namespace cmtv
