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
// so the transcript is a fixed byte-code program (built once on the host,
// sr_build_program) interpreted by one rolled loop per lane. That keeps a
// single Keccak call site in the kernel however many STROBE operations the
// transcript has. The 200-byte sponge state is byte-addressed through a State
// policy (LDS on the device, lane-interleaved words; a plain array on the host):
//   void xor_byte(int pos, uint32_t b);   byte pos of the state ^= b
//   uint32_t word(int i) const;           little-endian state word i (0..49)
//   void set_word(int i, uint32_t w);
#pragma once
#include <stdint.h>

#include "keccak.h"

#ifndef CMTV_HD
#define CMTV_HD __host__ __device__ __forceinline__
#endif

namespace cmtv {

constexpr int STROBE_R = 166;
constexpr uint32_t SF_I = 1, SF_A = 2, SF_C = 4, SF_T = 8, SF_M = 16, SF_K = 32;

// program opcodes (16-bit)
constexpr uint32_t SOP_LIT = 0x000;    // absorb literal byte (low 8 bits)
constexpr uint32_t SOP_BEGIN = 0x100;  // STROBE begin_op(flags = low 8 bits), not "more"
constexpr uint32_t SOP_MLEN = 0x200;   // absorb byte (low bits) of LE32(mlen)
constexpr uint32_t SOP_MSG = 0x300;    // absorb the whole message
constexpr uint32_t SOP_PK = 0x400;     // absorb the 32 key bytes
constexpr uint32_t SOP_R = 0x500;      // absorb the 32 R bytes
constexpr uint32_t SOP_INIT = 0x600;   // STROBE-128 initial state + F
constexpr uint32_t SOP_PRF64 = 0x700;  // begin_op(I|A|C) (+ forced F): 64 output bytes = state[0..63]
constexpr int SR_PROGRAM_MAX = 160;

// Host: append a STROBE/merlin operation sequence to the program.
struct SrProgramBuilder {
  uint16_t* ops;
  int n = 0;
  void op(uint32_t o) { ops[n++] = (uint16_t)o; }
  void lit(const char* s) {
    for (; *s; s++) op(SOP_LIT | (uint8_t)*s);
  }
  void lit_u32(uint32_t v) {
    for (int i = 0; i < 4; i++) op(SOP_LIT | ((v >> (8 * i)) & 0xFF));
  }
  // merlin AppendMessage(label, <message given by the callback ops>)
  void append_header(const char* label) {
    op(SOP_BEGIN | SF_M | SF_A);  // meta_ad(label, false)
    lit(label);
  }
};

// The whole verification transcript (see the header comment). Returns the
// opcode count.
inline int sr_build_program(uint16_t ops[SR_PROGRAM_MAX]) {
  SrProgramBuilder b{ops};
  b.op(SOP_INIT);
  b.op(SOP_BEGIN | SF_M | SF_A);  // Strobe128::new -> meta_ad("Merlin v1.0")
  b.lit("Merlin v1.0");
  b.append_header("dom-sep");
  b.lit_u32(14);  // meta_ad(LE32(len), more = true)
  b.op(SOP_BEGIN | SF_A);
  b.lit("SigningContext");
  b.append_header("");  // AppendMessage("", context = {})
  b.lit_u32(0);
  b.op(SOP_BEGIN | SF_A);
  b.append_header("sign-bytes");
  for (int i = 0; i < 4; i++) b.op(SOP_MLEN | i);
  b.op(SOP_BEGIN | SF_A);
  b.op(SOP_MSG);
  b.append_header("proto-name");
  b.lit_u32(11);
  b.op(SOP_BEGIN | SF_A);
  b.lit("Schnorr-sig");
  b.append_header("sign:pk");
  b.lit_u32(32);
  b.op(SOP_BEGIN | SF_A);
  b.op(SOP_PK);
  b.append_header("sign:R");
  b.lit_u32(32);
  b.op(SOP_BEGIN | SF_A);
  b.op(SOP_R);
  b.append_header("sign:c");  // ExtractBytes("sign:c", 64)
  b.lit_u32(64);
  b.op(SOP_PRF64);
  return b.n;
}

// Runs the program; out = the 64 challenge bytes as 16 little-endian words.
// pk / R: 8 little-endian words each; msg: mlen bytes at any alignment.
// The Keccak-f call is the single one in the loop (STROBE run_f).
template <class State>
CMTV_HD void sr_transcript(uint32_t out[16], State& st, const uint16_t* prog, int nops, const uint8_t* msg,
                           uint32_t mlen, const uint32_t pk[8], const uint32_t R[8]) {
  int pos = 0, pos_begin = 0;
  // message read as aligned words (the per-lane offset is arbitrary)
  const uintptr_t addr = (uintptr_t)msg;
  const uint32_t sh = (uint32_t)(addr & 3);
  const uint32_t* mw = (const uint32_t*)(addr - sh);
  int ip = 0;        // program counter
  uint32_t sub = 0;  // byte index inside a multi-byte op (MSG / PK / R) or BEGIN's second byte
  uint32_t mword = 0;
#pragma unroll 1
  for (;;) {
    const uint32_t o = prog[ip];
    const uint32_t kind = o & 0xF00;
    uint32_t byte = o & 0xFF;
    bool absorb = true, next = true, force_f = false;
    if (kind == SOP_INIT) {
#pragma unroll
      for (int i = 0; i < 50; i++) st.set_word(i, 0u);
      // [1, R+2, 1, 0, 1, 96] || "STROBEv1.0.2"
      st.set_word(0, 0x0001A801u);
      st.set_word(1, 0x54536001u);
      st.set_word(2, 0x45424F52u);
      st.set_word(3, 0x302E3176u);
      st.set_word(4, 0x0000322Eu);
      absorb = false;
      force_f = true;
    } else if (kind == SOP_BEGIN) {
      // absorb [old pos_begin, flags]; pos_begin = pos + 1 before the first
      if (sub == 0) {
        byte = (uint32_t)pos_begin;
        pos_begin = pos + 1;
        next = false;
        sub = 1;
      } else {
        sub = 0;
      }
    } else if (kind == SOP_MLEN) {
      byte = (mlen >> (8 * byte)) & 0xFF;
    } else if (kind == SOP_MSG) {
      if (sub >= mlen) {
        absorb = false;
        sub = 0;
      } else {
        const uint32_t q = sub + sh;
        if (sub == 0 || (q & 3) == 0) mword = mw[q >> 2];
        byte = (mword >> (8 * (q & 3))) & 0xFF;
        sub++;
        next = false;
      }
    } else if (kind == SOP_PK || kind == SOP_R) {
      const uint32_t* w = kind == SOP_PK ? pk : R;
      uint32_t x = 0;
#pragma unroll
      for (int i = 0; i < 8; i++) x = (sub >> 2) == (uint32_t)i ? w[i] : x;
      byte = (x >> (8 * (sub & 3))) & 0xFF;
      sub++;
      next = sub == 32;
      if (next) sub = 0;
    } else if (kind == SOP_PRF64) {
      // begin_op(I|A|C): header bytes, then F unless the header ended a block
      if (sub == 0) {
        byte = (uint32_t)pos_begin;
        pos_begin = pos + 1;
        next = false;
        sub = 1;
      } else if (sub == 1) {
        byte = SF_I | SF_A | SF_C;
        next = false;
        sub = 2;
      } else {
        absorb = false;
        force_f = pos != 0;
        next = false;
        sub = 3;
      }
    }
    if (absorb) {
      st.xor_byte(pos, byte);
      pos++;
      force_f = pos == STROBE_R;
    }
    if (force_f) {  // run_f
      if (kind != SOP_INIT) {
        st.xor_byte(pos, (uint32_t)pos_begin);
        st.xor_byte(pos + 1, 0x04u);
        st.xor_byte(STROBE_R + 1, 0x80u);
      }
      uint64_t a[25];
#pragma unroll
      for (int i = 0; i < 25; i++) a[i] = (uint64_t)st.word(2 * i) | ((uint64_t)st.word(2 * i + 1) << 32);
      keccak_f1600(a);
#pragma unroll
      for (int i = 0; i < 25; i++) {
        st.set_word(2 * i, (uint32_t)a[i]);
        st.set_word(2 * i + 1, (uint32_t)(a[i] >> 32));
      }
      pos = 0;
      pos_begin = 0;
    }
    if (kind == SOP_PRF64 && sub == 3) break;
    if (next) ip++;
    if (ip >= nops) break;  // malformed program guard
  }
#pragma unroll
  for (int i = 0; i < 16; i++) out[i] = st.word(i);
}

// Host state policy: a plain 50-word array.
struct ArrayStrobeState {
  uint32_t w[50];
  void xor_byte(int pos, uint32_t b) { w[pos >> 2] ^= (b & 0xFF) << (8 * (pos & 3)); }
  uint32_t word(int i) const { return w[i]; }
  void set_word(int i, uint32_t x) { w[i] = x; }
};

}  // namespace cmtv
