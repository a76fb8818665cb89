// sha512.h -- per-lane SHA-512 over (prefix || message) for gfx950.
//
// The Ed25519 challenge k = SHA-512(R || A || M) (Go crypto/ed25519 Verify,
// reference call site /root/reference/crypto/ed25519/ed25519.go:154) and the
// RFC 8032 signing hashes all have the shape "32- or 64-byte prefix held in
// registers, then a message in global memory". The padded stream is produced
// on the fly, 64-bit word by 64-bit word; 64-bit rotates lower to
// v_alignbit_b32 pairs. Two 128-byte compressions cover a commit vote
// (64 + 109..161 bytes).
#pragma once
#include <stdint.h>

#ifndef CMTV_HD
#define CMTV_HD __host__ __device__ __forceinline__
#endif

namespace cmtv {

// round constants: a global table (the compression's rolled loop indexes it
// with a wave-uniform round number: scalar loads)
#ifdef __HIP_DEVICE_COMPILE__
static __constant__ uint64_t g_sha512_K[80] = {
      0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL, 0xe9b5dba58189dbbcULL,
      0x3956c25bf348b538ULL, 0x59f111f1b605d019ULL, 0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL,
      0xd807aa98a3030242ULL, 0x12835b0145706fbeULL, 0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL,
      0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL, 0xc19bf174cf692694ULL,
      0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL, 0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL,
      0x2de92c6f592b0275ULL, 0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL,
      0x983e5152ee66dfabULL, 0xa831c66d2db43210ULL, 0xb00327c898fb213fULL, 0xbf597fc7beef0ee4ULL,
      0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL, 0x06ca6351e003826fULL, 0x142929670a0e6e70ULL,
      0x27b70a8546d22ffcULL, 0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL, 0x53380d139d95b3dfULL,
      0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL, 0x92722c851482353bULL,
      0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL, 0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL,
      0xd192e819d6ef5218ULL, 0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL,
      0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL, 0x2748774cdf8eeb99ULL, 0x34b0bcb5e19b48a8ULL,
      0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL, 0x5b9cca4f7763e373ULL, 0x682e6ff3d6b2b8a3ULL,
      0x748f82ee5defb2fcULL, 0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL,
      0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL, 0xc67178f2e372532bULL,
      0xca273eceea26619cULL, 0xd186b8c721c0c207ULL, 0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL,
      0x06f067aa72176fbaULL, 0x0a637dc5a2c898a6ULL, 0x113f9804bef90daeULL, 0x1b710b35131c471bULL,
      0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL, 0x431d67c49c100d4cULL,
      0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL, 0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL};
#else
static const uint64_t g_sha512_K[80] = {
      0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL, 0xe9b5dba58189dbbcULL,
      0x3956c25bf348b538ULL, 0x59f111f1b605d019ULL, 0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL,
      0xd807aa98a3030242ULL, 0x12835b0145706fbeULL, 0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL,
      0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL, 0xc19bf174cf692694ULL,
      0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL, 0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL,
      0x2de92c6f592b0275ULL, 0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL,
      0x983e5152ee66dfabULL, 0xa831c66d2db43210ULL, 0xb00327c898fb213fULL, 0xbf597fc7beef0ee4ULL,
      0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL, 0x06ca6351e003826fULL, 0x142929670a0e6e70ULL,
      0x27b70a8546d22ffcULL, 0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL, 0x53380d139d95b3dfULL,
      0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL, 0x92722c851482353bULL,
      0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL, 0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL,
      0xd192e819d6ef5218ULL, 0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL,
      0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL, 0x2748774cdf8eeb99ULL, 0x34b0bcb5e19b48a8ULL,
      0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL, 0x5b9cca4f7763e373ULL, 0x682e6ff3d6b2b8a3ULL,
      0x748f82ee5defb2fcULL, 0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL,
      0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL, 0xc67178f2e372532bULL,
      0xca273eceea26619cULL, 0xd186b8c721c0c207ULL, 0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL,
      0x06f067aa72176fbaULL, 0x0a637dc5a2c898a6ULL, 0x113f9804bef90daeULL, 0x1b710b35131c471bULL,
      0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL, 0x431d67c49c100d4cULL,
      0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL, 0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL};
#endif

CMTV_HD uint64_t sha512_k(int i) { return g_sha512_K[i]; }

CMTV_HD uint64_t rotr64(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }

#ifdef __HIP_DEVICE_COMPILE__
// (lo, hi) halves as one 64-bit value by a bit cast of a 2-vector, so LLVM
// keeps them a register pair: the ((uint64_t)hi << 32) | lo form made it split
// every following 64-bit add into "+ lo" and "+ (hi << 32)" plus moves
typedef uint32_t sha_u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint64_t sha_pair(uint32_t lo, uint32_t hi) {
  sha_u32x2 v = {lo, hi};
  return __builtin_bit_cast(uint64_t, v);
}
#endif

// x >>> n and x >> n for the compression's constant n: on the device as
// v_alignbit_b32 pairs on the 32-bit halves (the generic 64-bit form lowers
// to two 64-bit shifts and two ORs, and hides the three-way XORs from
// v_xor3_b32 -- ~1.8x the instructions of a round, which is the helper
// wave's whole cost: one wave per SIMD issues one instruction per ~4 cycles)
CMTV_HD uint64_t sha_rotr(uint64_t x, int n) {
#ifdef __HIP_DEVICE_COMPILE__
  uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  if (n >= 32) {
    const uint32_t t = lo;
    lo = hi;
    hi = t;
    n -= 32;
  }
  if (n == 0) return sha_pair(lo, hi);
  const uint32_t nlo = __builtin_amdgcn_alignbit(hi, lo, n), nhi = __builtin_amdgcn_alignbit(lo, hi, n);
  return sha_pair(nlo, nhi);
#else
  return rotr64(x, n);
#endif
}
CMTV_HD uint64_t sha_shr(uint64_t x, int n) {
#ifdef __HIP_DEVICE_COMPILE__
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  return sha_pair(__builtin_amdgcn_alignbit(hi, lo, n), hi >> n);
#else
  return x >> n;
#endif
}

// Three-input bitwise functions of 64-bit words as one v_bitop3_b32 per
// 32-bit half on gfx950 (truth tables: a^b^c = 0x96, majority = 0xE8,
// choose a ? b : c = 0xCA). LLVM forms neither v_xor3 nor bitop3 from the
// 64-bit expressions (the listing had 18 v_xor_b32 and 8 and/or per round).
CMTV_HD uint64_t sha_bitop3(uint64_t a, uint64_t b, uint64_t c, int tt) {
#ifdef __HIP_DEVICE_COMPILE__
  uint32_t lo, hi;
  switch (tt) {
    case 0x96:
      lo = __builtin_amdgcn_bitop3_b32((uint32_t)a, (uint32_t)b, (uint32_t)c, 0x96);
      hi = __builtin_amdgcn_bitop3_b32((uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32), 0x96);
      break;
    case 0xE8:
      lo = __builtin_amdgcn_bitop3_b32((uint32_t)a, (uint32_t)b, (uint32_t)c, 0xE8);
      hi = __builtin_amdgcn_bitop3_b32((uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32), 0xE8);
      break;
    default:
      lo = __builtin_amdgcn_bitop3_b32((uint32_t)a, (uint32_t)b, (uint32_t)c, 0xCA);
      hi = __builtin_amdgcn_bitop3_b32((uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32), 0xCA);
      break;
  }
  return sha_pair(lo, hi);
#else
  if (tt == 0x96) return a ^ b ^ c;
  if (tt == 0xE8) return (a & b) | (a & c) | (b & c);
  return (a & b) | (~a & c);
#endif
}
CMTV_HD uint64_t sha_xor3(uint64_t a, uint64_t b, uint64_t c) { return sha_bitop3(a, b, c, 0x96); }

// one round on the rotating state (a..h named by the caller's order)
CMTV_HD void sha512_round(uint64_t a, uint64_t b, uint64_t c, uint64_t& d, uint64_t e, uint64_t f, uint64_t g,
                          uint64_t& h, uint64_t kw) {
  const uint64_t S1 = sha_xor3(sha_rotr(e, 14), sha_rotr(e, 18), sha_rotr(e, 41));
  const uint64_t ch = sha_bitop3(e, f, g, 0xCA);
  const uint64_t t1 = h + S1 + ch + kw;
  const uint64_t S0 = sha_xor3(sha_rotr(a, 28), sha_rotr(a, 34), sha_rotr(a, 39));
  const uint64_t maj = sha_bitop3(a, b, c, 0xE8);
  d += t1;
  h = t1 + S0 + maj;
}

// 16 rounds from round r0 on: the state's names rotate by one per round, so
// after 16 (a multiple of 8) they are back in place; SCHED: w[j] becomes
// schedule word r0 + j first
template <bool SCHED>
CMTV_HD void sha512_rounds16(uint64_t& a, uint64_t& b, uint64_t& c, uint64_t& d, uint64_t& e, uint64_t& f,
                             uint64_t& g, uint64_t& h, uint64_t w[16], int r0) {
#pragma unroll
  for (int j = 0; j < 16; j++) {
    if (SCHED) {
      const uint64_t w15 = w[(j + 1) & 15], w2 = w[(j + 14) & 15];
      const uint64_t s0 = sha_xor3(sha_rotr(w15, 1), sha_rotr(w15, 8), sha_shr(w15, 7));
      const uint64_t s1 = sha_xor3(sha_rotr(w2, 19), sha_rotr(w2, 61), sha_shr(w2, 6));
      w[j] += s0 + w[(j + 9) & 15] + s1;
    }
    const uint64_t kw = sha512_k(r0 + j) + w[j];
    switch (j & 7) {
      case 0: sha512_round(a, b, c, d, e, f, g, h, kw); break;
      case 1: sha512_round(h, a, b, c, d, e, f, g, kw); break;
      case 2: sha512_round(g, h, a, b, c, d, e, f, kw); break;
      case 3: sha512_round(f, g, h, a, b, c, d, e, kw); break;
      case 4: sha512_round(e, f, g, h, a, b, c, d, kw); break;
      case 5: sha512_round(d, e, f, g, h, a, b, c, kw); break;
      case 6: sha512_round(c, d, e, f, g, h, a, b, kw); break;
      default: sha512_round(b, c, d, e, f, g, h, a, kw); break;
    }
  }
}

// The compression function: rounds 0..15 on the block's words, then four
// rolled passes of 16 with the message schedule (a rolled loop keeps the
// code ~1.5k instructions: the helper waves share the instruction cache with
// the row waves' field products)
CMTV_HD void sha512_compress(uint64_t st[8], uint64_t w[16]) {
  uint64_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
  sha512_rounds16<false>(a, b, c, d, e, f, g, h, w, 0);
#pragma unroll 1
  for (int r = 16; r < 80; r += 16) sha512_rounds16<true>(a, b, c, d, e, f, g, h, w, r);
  st[0] += a; st[1] += b; st[2] += c; st[3] += d;
  st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

// The word an empty, 4-byte aligned message "loads" (sha512_prefixed): a
// zero of our own in global memory on the device, so the load stays an
// unconditional global load next to the real ones.
#ifdef __HIP_DEVICE_COMPILE__
static __device__ uint32_t g_sha512_no_word;
#else
static const uint32_t g_sha512_no_word = 0u;
#endif

CMTV_HD uint32_t funnel_bytes(uint32_t hi, uint32_t lo, uint32_t sh) {
#ifdef __HIP_DEVICE_COMPILE__
  // the intrinsic keeps hi and lo separate values: the 64-bit form lets the
  // compiler fuse two adjacent array words into one 64-bit access, which
  // pins sha512_prefixed's word array in scratch
  return __builtin_amdgcn_alignbyte(hi, lo, sh);
#else
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * sh));
#endif
}

// SHA-512(prefix[0 .. 4*PW) || msg[0 .. mlen)); prefix as little-endian byte
// words. Output: 64 digest bytes as 16 little-endian 32-bit words.
//
// The message is read with 4-byte aligned loads and re-aligned in registers
// (the per-lane message offset has arbitrary alignment); only words holding
// at least one message byte are read, so nothing past msg[mlen-1]'s 4-byte
// word is touched.
template <int PW>
CMTV_HD void sha512_prefixed(uint32_t out[16], const uint32_t pre[PW], const uint8_t* msg, uint32_t mlen) {
  static_assert(PW % 2 == 0 && PW <= 16, "prefix must be whole 64-bit words inside block 0");
  constexpr uint32_t PB = 4 * PW;
  uint64_t st[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                    0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                    0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
  const uint32_t total = PB + mlen;
  const uint32_t nblocks = (total + 17 + 127) / 128;
  const uint64_t bitlen = (uint64_t)total * 8;
  const uint32_t sh = (uint32_t)((uintptr_t)msg & 3);
  // aligned base (pointer arithmetic keeps msg's address space: global loads)
  const uint32_t* mw = reinterpret_cast<const uint32_t*>(msg - sh);
  const uint32_t nwords = (sh + mlen + 3) / 4;         // aligned words holding message bytes
  // A block's aligned message words are all loaded before any is used (mv
  // below), so the loads go out together and are waited for once -- a load
  // under a per-lane branch costs a full memory round trip each. An index past
  // the message's last word re-reads that word (the 4-byte word holding a
  // message byte lies in the message's page) and is masked; an empty aligned
  // message, with no word to read at all, reads g_sha512_no_word.
  const uint32_t jmax = nwords ? nwords - 1 : 0u;
  const uint32_t* mb = nwords ? mw : &g_sha512_no_word;
  // little-endian stream word at byte position pos (pos % 4 == 0, pos >= PB),
  // branch-free: message bytes, then the 0x80 pad byte, then zeros
  auto tail_word = [&](uint32_t pos, uint32_t lo, uint32_t hi) -> uint32_t {
    const uint32_t v = funnel_bytes(hi, lo, sh);
    const int r = (int)total - (int)pos;  // message bytes left in this word
    const uint32_t rr = r < 0 ? 0u : (r > 4 ? 4u : (uint32_t)r);
    const uint32_t keep = (uint32_t)((1ull << (8 * rr)) - 1u);
    const uint32_t pad = (r >= 0 && r < 4) ? (0x80u << (8 * rr)) : 0u;
    return (v & keep) | pad;
  };
  auto be64 = [](uint32_t lo_word, uint32_t hi_word) -> uint64_t {
    return ((uint64_t)__builtin_bswap32(lo_word) << 32) | __builtin_bswap32(hi_word);
  };
#pragma unroll 1
  for (uint32_t b = 0; b < nblocks; b++) {
    // mv[k] = aligned message word j0 + k, j0 = (128 b - PB) / 4: the tail
    // word at block offset off is funnel(mv[off/4], mv[off/4 + 1]); block 0's
    // negative indices are the prefix's (loaded clamped, never used)
    const int j0 = (int)(b * 32) - (int)(PB / 4);
    uint32_t mv[33];
#pragma unroll
    for (int k = 0; k < 33; k++) {
      const uint32_t j = (uint32_t)(j0 + k);  // negative (block 0's prefix) -> huge: masked
      mv[k] = mb[j < nwords ? j : jmax];
    }
#pragma unroll
    for (int k = 0; k < 33; k++) mv[k] = (uint32_t)(j0 + k) < nwords ? mv[k] : 0u;
    uint64_t w[16];
#pragma unroll
    for (int t = 0; t < 16; t++) {
      uint32_t lw[2];
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const uint32_t off = 8 * t + 4 * h;  // byte offset inside the block
        if (b == 0 && off < PB)
          lw[h] = pre[off / 4];
        else
          lw[h] = tail_word(b * 128 + off, mv[off / 4], mv[off / 4 + 1]);
      }
      uint64_t word = be64(lw[0], lw[1]);
      if (b == nblocks - 1 && t == 15) word = bitlen;
      w[t] = word;
    }
    sha512_compress(st, w);
  }
#pragma unroll
  for (int i = 0; i < 8; i++) {
    // digest bytes are big-endian per 64-bit state word
    const uint64_t v = st[i];
    const uint32_t hi = (uint32_t)(v >> 32), lo = (uint32_t)v;
    out[2 * i] = __builtin_bswap32(hi);
    out[2 * i + 1] = __builtin_bswap32(lo);
  }
}

}  // namespace cmtv
