/*
 * cmtv_oracle.c -- CPU oracle (TEST INFRASTRUCTURE ONLY).
 *
 * A plain-C restatement of the Ed25519 verification that CometBFT runs on its
 * commit-verification path, in both verdict modes:
 *
 *   MODE_GO_STDLIB (0): Go 1.19 crypto/ed25519.Verify, reached from
 *       /root/reference/crypto/ed25519/ed25519.go:148-155 (PubKey.VerifySignature)
 *       via golang.org/x/crypto v0.5.0 (go.mod:37), an alias of the Go
 *       standard library for Go >= 1.13 (toolchain go.mod:3). The Go code is not
 *       in /root/reference; this file restates its published structure:
 *         - sig length / sig[63]&224 checks          (ed25519.go Verify)
 *         - Point.SetBytes(A): y taken mod p, x=0 with sign accepted
 *         - k = SHA-512(R || A || M) mod L           (Scalar.SetUniformBytes)
 *         - S < L                                    (Scalar.SetCanonicalBytes)
 *         - R' = [S]B - [k]A, wNAF(5) for A, wNAF(8) for B
 *                                                    (VarTimeDoubleScalarBaseMult)
 *         - bytes.Equal(sig[:32], R'.Bytes())
 *       Field arithmetic in radix 2^51 like Go's field.Element.
 *   MODE_ZIP215 (1): same up to R'; R decoded with the same rules as A;
 *       accept iff [8](R' - R) == identity.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library; the product (cometbft_amd/) never links it. It is checked
 * against the Python big-int restatement (oracle/ed25519_ref.py), the RFC 8032
 * vectors and libsodium (honest signatures) in tests/test_oracle.py.
 *
 * Exports (C ABI, see oracle/cmtv_oracle.h):
 *   oracle_verify_batch, oracle_verify_one, oracle_pubkey_from_seed,
 *   oracle_sign, oracle_sign_batch
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;

/* ------------------------------------------------------------------ SHA-512 */

static const uint64_t K512[80] = {
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

#define ROR64(x, n) (((x) >> (n)) | ((x) << (64 - (n))))

typedef struct {
  uint64_t h[8];
  uint8_t buf[128];
  size_t buflen;
  uint64_t total;
} sha512_ctx;

static void sha512_block(uint64_t h[8], const uint8_t *p) {
  uint64_t w[80];
  for (int i = 0; i < 16; i++) {
    uint64_t v = 0;
    for (int j = 0; j < 8; j++) v = (v << 8) | p[8 * i + j];
    w[i] = v;
  }
  for (int i = 16; i < 80; i++) {
    uint64_t s0 = ROR64(w[i - 15], 1) ^ ROR64(w[i - 15], 8) ^ (w[i - 15] >> 7);
    uint64_t s1 = ROR64(w[i - 2], 19) ^ ROR64(w[i - 2], 61) ^ (w[i - 2] >> 6);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  uint64_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  for (int i = 0; i < 80; i++) {
    uint64_t S1 = ROR64(e, 14) ^ ROR64(e, 18) ^ ROR64(e, 41);
    uint64_t ch = (e & f) ^ (~e & g);
    uint64_t t1 = hh + S1 + ch + K512[i] + w[i];
    uint64_t S0 = ROR64(a, 28) ^ ROR64(a, 34) ^ ROR64(a, 39);
    uint64_t maj = (a & b) ^ (a & c) ^ (b & c);
    uint64_t t2 = S0 + maj;
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

static void sha512_init(sha512_ctx *c) {
  static const uint64_t iv[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                                 0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                                 0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
  memcpy(c->h, iv, sizeof iv);
  c->buflen = 0;
  c->total = 0;
}

static void sha512_update(sha512_ctx *c, const uint8_t *p, size_t n) {
  c->total += n;
  while (n > 0) {
    size_t take = 128 - c->buflen;
    if (take > n) take = n;
    memcpy(c->buf + c->buflen, p, take);
    c->buflen += take; p += take; n -= take;
    if (c->buflen == 128) { sha512_block(c->h, c->buf); c->buflen = 0; }
  }
}

static void sha512_final(sha512_ctx *c, uint8_t out[64]) {
  uint64_t bits = c->total * 8;
  uint8_t pad = 0x80;
  sha512_update(c, &pad, 1);
  uint8_t z = 0;
  while (c->buflen != 112) sha512_update(c, &z, 1);
  uint8_t len[16] = {0};
  for (int i = 0; i < 8; i++) len[15 - i] = (uint8_t)(bits >> (8 * i));
  sha512_update(c, len, 16);
  for (int i = 0; i < 8; i++)
    for (int j = 0; j < 8; j++) out[8 * i + j] = (uint8_t)(c->h[i] >> (56 - 8 * j));
}

/* ------------------------------------------------------- GF(2^255-19), 2^51 */

typedef struct { uint64_t l[5]; } fe;
#define MASK51 ((1ULL << 51) - 1)

static void fe_carry(fe *h) {
  uint64_t c;
  c = h->l[0] >> 51; h->l[0] &= MASK51; h->l[1] += c;
  c = h->l[1] >> 51; h->l[1] &= MASK51; h->l[2] += c;
  c = h->l[2] >> 51; h->l[2] &= MASK51; h->l[3] += c;
  c = h->l[3] >> 51; h->l[3] &= MASK51; h->l[4] += c;
  c = h->l[4] >> 51; h->l[4] &= MASK51; h->l[0] += 19 * c;
}

static void fe_0(fe *h) { memset(h, 0, sizeof *h); }
static void fe_1(fe *h) { fe_0(h); h->l[0] = 1; }

static void fe_add(fe *h, const fe *f, const fe *g) {
  for (int i = 0; i < 5; i++) h->l[i] = f->l[i] + g->l[i];
  fe_carry(h);
}

/* f - g + 2p keeps limbs non-negative for carried inputs */
static void fe_sub(fe *h, const fe *f, const fe *g) {
  h->l[0] = (f->l[0] + 0xFFFFFFFFFFFDAULL) - g->l[0];
  h->l[1] = (f->l[1] + 0xFFFFFFFFFFFFEULL) - g->l[1];
  h->l[2] = (f->l[2] + 0xFFFFFFFFFFFFEULL) - g->l[2];
  h->l[3] = (f->l[3] + 0xFFFFFFFFFFFFEULL) - g->l[3];
  h->l[4] = (f->l[4] + 0xFFFFFFFFFFFFEULL) - g->l[4];
  fe_carry(h);
}

static void fe_neg(fe *h, const fe *f) { fe z; fe_0(&z); fe_sub(h, &z, f); }

static void fe_mul(fe *h, const fe *f, const fe *g) {
  const uint64_t *a = f->l, *b = g->l;
  uint64_t b1_19 = b[1] * 19, b2_19 = b[2] * 19, b3_19 = b[3] * 19, b4_19 = b[4] * 19;
  u128 r0 = (u128)a[0] * b[0] + (u128)a[1] * b4_19 + (u128)a[2] * b3_19 + (u128)a[3] * b2_19 + (u128)a[4] * b1_19;
  u128 r1 = (u128)a[0] * b[1] + (u128)a[1] * b[0] + (u128)a[2] * b4_19 + (u128)a[3] * b3_19 + (u128)a[4] * b2_19;
  u128 r2 = (u128)a[0] * b[2] + (u128)a[1] * b[1] + (u128)a[2] * b[0] + (u128)a[3] * b4_19 + (u128)a[4] * b3_19;
  u128 r3 = (u128)a[0] * b[3] + (u128)a[1] * b[2] + (u128)a[2] * b[1] + (u128)a[3] * b[0] + (u128)a[4] * b4_19;
  u128 r4 = (u128)a[0] * b[4] + (u128)a[1] * b[3] + (u128)a[2] * b[2] + (u128)a[3] * b[1] + (u128)a[4] * b[0];
  uint64_t c;
  r1 += (uint64_t)(r0 >> 51); uint64_t l0 = (uint64_t)r0 & MASK51;
  r2 += (uint64_t)(r1 >> 51); uint64_t l1 = (uint64_t)r1 & MASK51;
  r3 += (uint64_t)(r2 >> 51); uint64_t l2 = (uint64_t)r2 & MASK51;
  r4 += (uint64_t)(r3 >> 51); uint64_t l3 = (uint64_t)r3 & MASK51;
  c = (uint64_t)(r4 >> 51); uint64_t l4 = (uint64_t)r4 & MASK51;
  l0 += c * 19;
  c = l0 >> 51; l0 &= MASK51; l1 += c;
  h->l[0] = l0; h->l[1] = l1; h->l[2] = l2; h->l[3] = l3; h->l[4] = l4;
}

static void fe_sq(fe *h, const fe *f) { fe_mul(h, f, f); }

static void fe_sqn(fe *h, const fe *f, int n) {
  fe_sq(h, f);
  for (int i = 1; i < n; i++) fe_sq(h, h);
}

/* y = bytes with bit 255 ignored; value may be >= p (non-canonical accepted) */
static void fe_frombytes(fe *h, const uint8_t s[32]) {
  uint64_t w[4];
  for (int i = 0; i < 4; i++) {
    uint64_t v = 0;
    for (int j = 7; j >= 0; j--) v = (v << 8) | s[8 * i + j];
    w[i] = v;
  }
  h->l[0] = w[0] & MASK51;
  h->l[1] = ((w[0] >> 51) | (w[1] << 13)) & MASK51;
  h->l[2] = ((w[1] >> 38) | (w[2] << 26)) & MASK51;
  h->l[3] = ((w[2] >> 25) | (w[3] << 39)) & MASK51;
  h->l[4] = (w[3] >> 12) & MASK51;
}

static void fe_tobytes(uint8_t s[32], const fe *f) {
  fe h = *f;
  fe_carry(&h);
  fe_carry(&h);
  /* now h < 2^255 + small; compute h mod p canonically */
  uint64_t q = (h.l[0] + 19) >> 51;
  q = (h.l[1] + q) >> 51;
  q = (h.l[2] + q) >> 51;
  q = (h.l[3] + q) >> 51;
  q = (h.l[4] + q) >> 51;
  h.l[0] += 19 * q;
  uint64_t c;
  c = h.l[0] >> 51; h.l[0] &= MASK51; h.l[1] += c;
  c = h.l[1] >> 51; h.l[1] &= MASK51; h.l[2] += c;
  c = h.l[2] >> 51; h.l[2] &= MASK51; h.l[3] += c;
  c = h.l[3] >> 51; h.l[3] &= MASK51; h.l[4] += c;
  h.l[4] &= MASK51;
  uint64_t w0 = h.l[0] | (h.l[1] << 51);
  uint64_t w1 = (h.l[1] >> 13) | (h.l[2] << 38);
  uint64_t w2 = (h.l[2] >> 26) | (h.l[3] << 25);
  uint64_t w3 = (h.l[3] >> 39) | (h.l[4] << 12);
  uint64_t w[4] = {w0, w1, w2, w3};
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 8; j++) s[8 * i + j] = (uint8_t)(w[i] >> (8 * j));
}

static int fe_iszero(const fe *f) {
  uint8_t s[32]; fe_tobytes(s, f);
  uint8_t r = 0;
  for (int i = 0; i < 32; i++) r |= s[i];
  return r == 0;
}

static int fe_isneg(const fe *f) { uint8_t s[32]; fe_tobytes(s, f); return s[0] & 1; }

static int fe_equal(const fe *f, const fe *g) {
  uint8_t a[32], b[32]; fe_tobytes(a, f); fe_tobytes(b, g);
  return memcmp(a, b, 32) == 0;
}

/* z^(2^250 - 1) and helpers, standard addition chain */
static void fe_pow2_250m1(fe *out, fe *z11, const fe *z) {
  fe t0, t1, t2, z2, z9;
  fe_sq(&z2, z);                 /* 2 */
  fe_sqn(&t0, &z2, 2);           /* 8 */
  fe_mul(&z9, &t0, z);           /* 9 */
  fe_mul(z11, &z9, &z2);         /* 11 */
  fe_sq(&t0, z11);               /* 22 */
  fe_mul(&t0, &t0, &z9);         /* 2^5 - 1 */
  fe_sqn(&t1, &t0, 5);
  fe_mul(&t0, &t1, &t0);         /* 2^10 - 1 */
  fe_sqn(&t1, &t0, 10);
  fe_mul(&t1, &t1, &t0);         /* 2^20 - 1 */
  fe_sqn(&t2, &t1, 20);
  fe_mul(&t1, &t2, &t1);         /* 2^40 - 1 */
  fe_sqn(&t1, &t1, 10);
  fe_mul(&t0, &t1, &t0);         /* 2^50 - 1 */
  fe_sqn(&t1, &t0, 50);
  fe_mul(&t1, &t1, &t0);         /* 2^100 - 1 */
  fe_sqn(&t2, &t1, 100);
  fe_mul(&t1, &t2, &t1);         /* 2^200 - 1 */
  fe_sqn(&t1, &t1, 50);
  fe_mul(out, &t1, &t0);         /* 2^250 - 1 */
}

static void fe_invert(fe *out, const fe *z) {
  fe t, z11;
  fe_pow2_250m1(&t, &z11, z);
  fe_sqn(&t, &t, 5);             /* 2^255 - 2^5 */
  fe_mul(out, &t, &z11);         /* 2^255 - 21 = p - 2 */
}

static void fe_pow22523(fe *out, const fe *z) {
  fe t, z11;
  fe_pow2_250m1(&t, &z11, z);
  fe_sqn(&t, &t, 2);             /* 2^252 - 4 */
  fe_mul(out, &t, z);            /* 2^252 - 3 = (p-5)/8 */
}

static fe FE_D, FE_D2, FE_SQRTM1;

/* --------------------------------------------------------------- points */

typedef struct { fe X, Y, Z, T; } ge_p3;
typedef struct { fe X, Y, Z; } ge_p2;
typedef struct { fe X, Y, Z, T; } ge_p1p1;
typedef struct { fe YplusX, YminusX, Z, T2d; } ge_cached;
typedef struct { fe yplusx, yminusx, xy2d; } ge_precomp;

static void p1p1_to_p2(ge_p2 *r, const ge_p1p1 *p) {
  fe_mul(&r->X, &p->X, &p->T); fe_mul(&r->Y, &p->Y, &p->Z); fe_mul(&r->Z, &p->Z, &p->T);
}
static void p1p1_to_p3(ge_p3 *r, const ge_p1p1 *p) {
  fe_mul(&r->X, &p->X, &p->T); fe_mul(&r->Y, &p->Y, &p->Z);
  fe_mul(&r->Z, &p->Z, &p->T); fe_mul(&r->T, &p->X, &p->Y);
}
static void p3_to_p2(ge_p2 *r, const ge_p3 *p) { r->X = p->X; r->Y = p->Y; r->Z = p->Z; }
static void p3_to_cached(ge_cached *r, const ge_p3 *p) {
  fe_add(&r->YplusX, &p->Y, &p->X); fe_sub(&r->YminusX, &p->Y, &p->X);
  r->Z = p->Z; fe_mul(&r->T2d, &p->T, &FE_D2);
}
static void p3_0(ge_p3 *h) { fe_0(&h->X); fe_1(&h->Y); fe_1(&h->Z); fe_0(&h->T); }

/* dbl-2008-hwcd for a = -1 */
static void p2_dbl(ge_p1p1 *r, const ge_p2 *p) {
  fe t0;
  fe_sq(&r->X, &p->X);
  fe_sq(&r->Z, &p->Y);
  fe_sq(&r->T, &p->Z); fe_add(&r->T, &r->T, &r->T);
  fe_add(&r->Y, &p->X, &p->Y);
  fe_sq(&t0, &r->Y);
  fe_add(&r->Y, &r->Z, &r->X);
  fe_sub(&r->Z, &r->Z, &r->X);
  fe_sub(&r->X, &t0, &r->Y);
  fe_sub(&r->T, &r->T, &r->Z);
}
static void p3_dbl(ge_p1p1 *r, const ge_p3 *p) { ge_p2 q; p3_to_p2(&q, p); p2_dbl(r, &q); }

static void ge_add(ge_p1p1 *r, const ge_p3 *p, const ge_cached *q) {
  fe t0;
  fe_add(&r->X, &p->Y, &p->X);
  fe_sub(&r->Y, &p->Y, &p->X);
  fe_mul(&r->Z, &r->X, &q->YplusX);
  fe_mul(&r->Y, &r->Y, &q->YminusX);
  fe_mul(&r->T, &q->T2d, &p->T);
  fe_mul(&r->X, &p->Z, &q->Z);
  fe_add(&t0, &r->X, &r->X);
  fe_sub(&r->X, &r->Z, &r->Y);
  fe_add(&r->Y, &r->Z, &r->Y);
  fe_add(&r->Z, &t0, &r->T);
  fe_sub(&r->T, &t0, &r->T);
}
static void ge_sub(ge_p1p1 *r, const ge_p3 *p, const ge_cached *q) {
  fe t0;
  fe_add(&r->X, &p->Y, &p->X);
  fe_sub(&r->Y, &p->Y, &p->X);
  fe_mul(&r->Z, &r->X, &q->YminusX);
  fe_mul(&r->Y, &r->Y, &q->YplusX);
  fe_mul(&r->T, &q->T2d, &p->T);
  fe_mul(&r->X, &p->Z, &q->Z);
  fe_add(&t0, &r->X, &r->X);
  fe_sub(&r->X, &r->Z, &r->Y);
  fe_add(&r->Y, &r->Z, &r->Y);
  fe_sub(&r->Z, &t0, &r->T);
  fe_add(&r->T, &t0, &r->T);
}
static void ge_madd(ge_p1p1 *r, const ge_p3 *p, const ge_precomp *q) {
  fe t0;
  fe_add(&r->X, &p->Y, &p->X);
  fe_sub(&r->Y, &p->Y, &p->X);
  fe_mul(&r->Z, &r->X, &q->yplusx);
  fe_mul(&r->Y, &r->Y, &q->yminusx);
  fe_mul(&r->T, &q->xy2d, &p->T);
  fe_add(&t0, &p->Z, &p->Z);
  fe_sub(&r->X, &r->Z, &r->Y);
  fe_add(&r->Y, &r->Z, &r->Y);
  fe_add(&r->Z, &t0, &r->T);
  fe_sub(&r->T, &t0, &r->T);
}
static void ge_msub(ge_p1p1 *r, const ge_p3 *p, const ge_precomp *q) {
  fe t0;
  fe_add(&r->X, &p->Y, &p->X);
  fe_sub(&r->Y, &p->Y, &p->X);
  fe_mul(&r->Z, &r->X, &q->yminusx);
  fe_mul(&r->Y, &r->Y, &q->yplusx);
  fe_mul(&r->T, &q->xy2d, &p->T);
  fe_add(&t0, &p->Z, &p->Z);
  fe_sub(&r->X, &r->Z, &r->Y);
  fe_add(&r->Y, &r->Z, &r->Y);
  fe_sub(&r->Z, &t0, &r->T);
  fe_add(&r->T, &t0, &r->T);
}

static void p3_tobytes(uint8_t s[32], const ge_p3 *h) {
  fe recip, x, y;
  fe_invert(&recip, &h->Z);
  fe_mul(&x, &h->X, &recip);
  fe_mul(&y, &h->Y, &recip);
  fe_tobytes(s, &y);
  s[31] ^= (uint8_t)(fe_isneg(&x) << 7);
}

/* Go 1.19 Point.SetBytes + field.Element.SqrtRatio. Returns 0 on success. */
static int p3_frombytes(ge_p3 *h, const uint8_t s[32]) {
  fe u, v, v3, v7, r, check, y2, uneg, t;
  fe_frombytes(&h->Y, s);
  fe_1(&h->Z);
  fe_sq(&y2, &h->Y);
  fe one; fe_1(&one);
  fe_sub(&u, &y2, &one);             /* u = y^2 - 1 */
  fe_mul(&v, &y2, &FE_D);
  fe_add(&v, &v, &one);              /* v = d y^2 + 1 */
  fe_sq(&v3, &v); fe_mul(&v3, &v3, &v);    /* v^3 */
  fe_sq(&v7, &v3); fe_mul(&v7, &v7, &v);   /* v^7 */
  fe_mul(&t, &u, &v7);
  fe_pow22523(&t, &t);               /* (u v^7)^((p-5)/8) */
  fe_mul(&r, &u, &v3);
  fe_mul(&r, &r, &t);                /* r = u v^3 (u v^7)^((p-5)/8) */
  fe_sq(&check, &r); fe_mul(&check, &check, &v);
  fe_neg(&uneg, &u);
  int correct = fe_equal(&check, &u);
  int flipped = fe_equal(&check, &uneg);
  if (!correct && !flipped) return -1;
  if (flipped) fe_mul(&r, &r, &FE_SQRTM1);
  if (fe_isneg(&r)) fe_neg(&r, &r);  /* Absolute(): non-negative root */
  if (s[31] >> 7) fe_neg(&r, &r);    /* x = 0 stays 0 */
  h->X = r;
  fe_mul(&h->T, &h->X, &h->Y);
  return 0;
}

/* ------------------------------------------------------------ scalars mod L */

static const uint64_t L64[4] = {0x5812631a5cf5d3edULL, 0x14def9dea2f79cd6ULL, 0ULL, 0x1000000000000000ULL};
/* delta = L - 2^252 */
static const uint64_t DELTA[2] = {0x5812631a5cf5d3edULL, 0x14def9dea2f79cd6ULL};

/* x (nw 64-bit words, little-endian) := x mod L, result in r[4]. Folding
 * 2^252 == -delta (mod L) while keeping every intermediate non-negative. */
static void big_mod_l(uint64_t r[4], const uint64_t *x, int nw) {
  uint64_t a[9] = {0};
  memcpy(a, x, (size_t)nw * 8);
  for (int round = 0; round < 4; round++) {
    /* split a = h * 2^252 + l */
    uint64_t h[6] = {0}, l[4];
    for (int i = 0; i < 6; i++) {
      uint64_t lo = (i + 3 < 9) ? a[i + 3] >> 60 : 0;
      uint64_t hi = (i + 4 < 9) ? a[i + 4] << 4 : 0;
      h[i] = lo | hi;
    }
    l[0] = a[0]; l[1] = a[1]; l[2] = a[2]; l[3] = a[3] & 0x0FFFFFFFFFFFFFFFULL;
    int hz = 1;
    for (int i = 0; i < 6; i++) if (h[i]) hz = 0;
    if (hz) break;
    /* hd = h * delta (8 words) */
    uint64_t hd[8] = {0};
    for (int i = 0; i < 6; i++) {
      u128 c = 0;
      for (int j = 0; j < 2; j++) {
        c += (u128)h[i] * DELTA[j] + hd[i + j];
        hd[i + j] = (uint64_t)c;
        c >>= 64;
      }
      for (int k = i + 2; k < 8 && c; k++) { c += hd[k]; hd[k] = (uint64_t)c; c >>= 64; }
    }
    /* m = L * 2^sh with 2^sh * L >= h * delta (delta < 2^125, L > 2^252) */
    int hbits = 0;
    for (int i = 5; i >= 0; i--)
      if (h[i]) { hbits = 64 * i + 64 - __builtin_clzll(h[i]); break; }
    int sh = hbits + 125 - 252 + 1;
    if (sh < 0) sh = 0;
    uint64_t m[9] = {0};
    {
      int ws = sh / 64, bs = sh % 64;
      for (int i = 0; i < 4; i++) {
        u128 v = (u128)L64[i] << bs;
        m[i + ws] |= (uint64_t)v;
        if (i + ws + 1 < 9) m[i + ws + 1] |= (uint64_t)(v >> 64);
      }
    }
    /* a = l + m - hd */
    u128 c = 0;
    uint64_t na[9];
    for (int i = 0; i < 9; i++) {
      c += (u128)(i < 4 ? l[i] : 0) + m[i];
      na[i] = (uint64_t)c;
      c >>= 64;
    }
    uint64_t borrow = 0;
    for (int i = 0; i < 9; i++) {
      uint64_t sub = (i < 8 ? hd[i] : 0);
      u128 t = (u128)na[i] - sub - borrow;
      na[i] = (uint64_t)t;
      borrow = (uint64_t)(t >> 64) & 1;
    }
    memcpy(a, na, sizeof na);
  }
  /* a < 2^253ish now: subtract L while a >= L */
  for (;;) {
    int ge = 1;
    for (int i = 8; i >= 4; i--) if (a[i]) goto sub;
    for (int i = 3; i >= 0; i--) {
      if (a[i] > L64[i]) break;
      if (a[i] < L64[i]) { ge = 0; break; }
    }
    if (!ge) break;
  sub: {
      uint64_t borrow = 0;
      for (int i = 0; i < 9; i++) {
        u128 t = (u128)a[i] - (i < 4 ? L64[i] : 0) - borrow;
        a[i] = (uint64_t)t;
        borrow = (uint64_t)(t >> 64) & 1;
      }
    }
  }
  memcpy(r, a, 32);
}

static void bytes_to_words(uint64_t *w, const uint8_t *b, int nw) {
  for (int i = 0; i < nw; i++) {
    uint64_t v = 0;
    for (int j = 7; j >= 0; j--) v = (v << 8) | b[8 * i + j];
    w[i] = v;
  }
}

static void words_to_bytes(uint8_t *b, const uint64_t *w, int nw) {
  for (int i = 0; i < nw; i++)
    for (int j = 0; j < 8; j++) b[8 * i + j] = (uint8_t)(w[i] >> (8 * j));
}

/* SetUniformBytes */
static void sc_reduce64(uint8_t out[32], const uint8_t in[64]) {
  uint64_t w[8], r[4];
  bytes_to_words(w, in, 8);
  big_mod_l(r, w, 8);
  words_to_bytes(out, r, 4);
}

/* SetCanonicalBytes acceptance: s < L */
static int sc_is_canonical(const uint8_t s[32]) {
  uint64_t w[4];
  bytes_to_words(w, s, 4);
  for (int i = 3; i >= 0; i--) {
    if (w[i] < L64[i]) return 1;
    if (w[i] > L64[i]) return 0;
  }
  return 0; /* equal to L */
}

/* (a*b + c) mod L for signing */
static void sc_muladd(uint8_t out[32], const uint8_t a[32], const uint8_t b[32], const uint8_t c[32]) {
  uint64_t wa[4], wb[4], wc[4], prod[9] = {0}, r[4];
  bytes_to_words(wa, a, 4); bytes_to_words(wb, b, 4); bytes_to_words(wc, c, 4);
  for (int i = 0; i < 4; i++) {
    u128 carry = 0;
    for (int j = 0; j < 4; j++) {
      carry += (u128)wa[i] * wb[j] + prod[i + j];
      prod[i + j] = (uint64_t)carry;
      carry >>= 64;
    }
    prod[i + 4] += (uint64_t)carry;
  }
  u128 carry = 0;
  for (int i = 0; i < 9; i++) {
    carry += (u128)prod[i] + (i < 4 ? wc[i] : 0);
    prod[i] = (uint64_t)carry;
    carry >>= 64;
  }
  big_mod_l(r, prod, 9);
  words_to_bytes(out, r, 4);
}

/* width-w NAF of a 256-bit scalar (Go scalar.go nonAdjacentForm) */
static void slide_naf(int8_t naf[256], const uint8_t s[32], int w) {
  uint64_t digits[5] = {0};
  bytes_to_words(digits, s, 4);
  int width = 1 << w, windowMask = width - 1;
  memset(naf, 0, 256);
  int pos = 0;
  int carry = 0;
  while (pos < 256) {
    int idx = pos / 64, bit = pos % 64;
    uint64_t bitBuf;
    if (bit < 64 - w) bitBuf = digits[idx] >> bit;
    else bitBuf = (digits[idx] >> bit) | (digits[idx + 1] << (64 - bit));
    int window = carry + (int)(bitBuf & (uint64_t)windowMask);
    if ((window & 1) == 0) { pos += 1; continue; }
    if (window < width / 2) { carry = 0; naf[pos] = (int8_t)window; }
    else { carry = 1; naf[pos] = (int8_t)(window - width); }
    pos += w;
  }
}

/* basepoint wNAF(8) table: odd multiples B, 3B, ..., 127B (64 entries) */
static ge_precomp BTAB[64];
static ge_p3 GE_B;
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static void to_precomp(ge_precomp *r, const ge_p3 *p) {
  fe zi, x, y;
  fe_invert(&zi, &p->Z);
  fe_mul(&x, &p->X, &zi);
  fe_mul(&y, &p->Y, &zi);
  fe_add(&r->yplusx, &y, &x);
  fe_sub(&r->yminusx, &y, &x);
  fe_mul(&r->xy2d, &x, &y);
  fe_mul(&r->xy2d, &r->xy2d, &FE_D2);
}

static void init_constants(void) {
  /* d = -121665/121666 */
  fe num, den, deni;
  fe_0(&num); num.l[0] = 121665; fe_neg(&num, &num);
  fe_0(&den); den.l[0] = 121666;
  fe_invert(&deni, &den);
  fe_mul(&FE_D, &num, &deni);
  fe_add(&FE_D2, &FE_D, &FE_D);
  /* sqrt(-1) = 2^((p-1)/4) */
  fe two; fe_0(&two); two.l[0] = 2;
  /* (p-1)/4 = 2^253 - 5 = (2^252-3)*2 + 1 : 2^((p-5)/8 * 2 + 1) */
  fe t; fe_pow22523(&t, &two); fe_sq(&t, &t); fe_mul(&FE_SQRTM1, &t, &two);
  /* B: y = 4/5, x even */
  static const uint8_t by[32] = {0x58, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66,
                                 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66,
                                 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66};
  p3_frombytes(&GE_B, by);
  ge_p3 cur = GE_B, b2;
  ge_p1p1 t1;
  p3_dbl(&t1, &GE_B); p1p1_to_p3(&b2, &t1);
  ge_cached b2c; p3_to_cached(&b2c, &b2);
  for (int i = 0; i < 64; i++) {
    to_precomp(&BTAB[i], &cur);
    ge_add(&t1, &cur, &b2c); p1p1_to_p3(&cur, &t1);
  }
}

/* r = [a]A + [b]B, variable time (Go VarTimeDoubleScalarBaseMult structure) */
static void double_scalarmult_vartime(ge_p3 *out, const uint8_t a[32], const ge_p3 *A, const uint8_t b[32]) {
  int8_t anaf[256], bnaf[256];
  slide_naf(anaf, a, 5);
  slide_naf(bnaf, b, 8);
  ge_cached Ai[8];
  ge_p3 A2, cur = *A;
  ge_p1p1 t;
  p3_dbl(&t, A); p1p1_to_p3(&A2, &t);
  ge_cached a2c; p3_to_cached(&a2c, &A2);
  for (int i = 0; i < 8; i++) {
    p3_to_cached(&Ai[i], &cur);
    ge_add(&t, &cur, &a2c); p1p1_to_p3(&cur, &t);
  }
  int i = 255;
  while (i >= 0 && !anaf[i] && !bnaf[i]) i--;
  ge_p2 r;
  ge_p3 u;
  fe_0(&r.X); fe_1(&r.Y); fe_1(&r.Z);
  if (i < 0) { p3_0(out); return; }
  for (; i >= 0; i--) {
    p2_dbl(&t, &r);
    if (anaf[i] > 0) { p1p1_to_p3(&u, &t); ge_add(&t, &u, &Ai[anaf[i] / 2]); }
    else if (anaf[i] < 0) { p1p1_to_p3(&u, &t); ge_sub(&t, &u, &Ai[(-anaf[i]) / 2]); }
    if (bnaf[i] > 0) { p1p1_to_p3(&u, &t); ge_madd(&t, &u, &BTAB[bnaf[i] / 2]); }
    else if (bnaf[i] < 0) { p1p1_to_p3(&u, &t); ge_msub(&t, &u, &BTAB[(-bnaf[i]) / 2]); }
    if (i == 0) { p1p1_to_p3(out, &t); return; }
    p1p1_to_p2(&r, &t);
  }
}

/* -------------------------------------------------------------- verify */

int oracle_verify_one(const uint8_t *pk, const uint8_t *msg, size_t mlen, const uint8_t *sig, int mode) {
  pthread_once(&g_once, init_constants);
  if (sig[63] & 224) return 0;
  ge_p3 A;
  if (p3_frombytes(&A, pk) != 0) return 0;
  if (!sc_is_canonical(sig + 32)) return 0;
  uint8_t h[64], k[32];
  sha512_ctx c;
  sha512_init(&c);
  sha512_update(&c, sig, 32);
  sha512_update(&c, pk, 32);
  sha512_update(&c, msg, mlen);
  sha512_final(&c, h);
  sc_reduce64(k, h);
  /* R' = [k](-A) + [s]B */
  ge_p3 negA = A;
  fe_neg(&negA.X, &A.X);
  fe_neg(&negA.T, &A.T);
  ge_p3 Rp;
  double_scalarmult_vartime(&Rp, k, &negA, sig + 32);
  if (mode == 0) {
    uint8_t enc[32];
    p3_tobytes(enc, &Rp);
    return memcmp(enc, sig, 32) == 0;
  }
  ge_p3 R;
  if (p3_frombytes(&R, sig) != 0) return 0;
  ge_cached Rc;
  p3_to_cached(&Rc, &R);
  ge_p1p1 t;
  ge_sub(&t, &Rp, &Rc);
  ge_p2 q;
  p1p1_to_p2(&q, &t);
  p2_dbl(&t, &q); p1p1_to_p2(&q, &t);
  p2_dbl(&t, &q); p1p1_to_p2(&q, &t);
  p2_dbl(&t, &q); p1p1_to_p2(&q, &t);
  return fe_iszero(&q.X) && fe_equal(&q.Y, &q.Z);
}

typedef struct {
  size_t lo, hi;
  const uint8_t *pk, *sig, *msg;
  const uint32_t *off;
  int mode;
  uint8_t *out;
} job_t;

static void *worker(void *arg) {
  job_t *j = (job_t *)arg;
  for (size_t i = j->lo; i < j->hi; i++)
    j->out[i] = (uint8_t)oracle_verify_one(j->pk + 32 * i, j->msg + j->off[i], j->off[i + 1] - j->off[i],
                                           j->sig + 64 * i, j->mode);
  return NULL;
}

/* Batch verdicts; msg_off has n+1 entries. nthreads <= 0 -> 1. */
void oracle_verify_batch(size_t n, const uint8_t *pk, const uint8_t *sig, const uint8_t *msg,
                         const uint32_t *msg_off, int mode, uint8_t *out, int nthreads) {
  pthread_once(&g_once, init_constants);
  if (nthreads <= 1 || n < 2) {
    job_t j = {0, n, pk, sig, msg, msg_off, mode, out};
    worker(&j);
    return;
  }
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  job_t jobs[256];
  for (int t = 0; t < nthreads; t++) {
    jobs[t] = (job_t){n * t / nthreads, n * (t + 1) / nthreads, pk, sig, msg, msg_off, mode, out};
    pthread_create(&th[t], NULL, worker, &jobs[t]);
  }
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
}

/* --------------------------------------------------------- keygen / sign */

static void scalarmult_base(ge_p3 *out, const uint8_t s[32]) {
  uint8_t zero[32] = {0};
  double_scalarmult_vartime(out, zero, &GE_B, s);
}

void oracle_pubkey_from_seed(const uint8_t seed[32], uint8_t pk[32]) {
  pthread_once(&g_once, init_constants);
  uint8_t h[64];
  sha512_ctx c;
  sha512_init(&c); sha512_update(&c, seed, 32); sha512_final(&c, h);
  h[0] &= 248; h[31] &= 127; h[31] |= 64;
  ge_p3 A;
  scalarmult_base(&A, h);
  p3_tobytes(pk, &A);
}

void oracle_sign(const uint8_t seed[32], const uint8_t *msg, size_t mlen, uint8_t sig[64]) {
  pthread_once(&g_once, init_constants);
  uint8_t h[64], pk[32], rh[64], r[32], kh[64], k[32];
  sha512_ctx c;
  sha512_init(&c); sha512_update(&c, seed, 32); sha512_final(&c, h);
  h[0] &= 248; h[31] &= 127; h[31] |= 64;
  ge_p3 A, R;
  scalarmult_base(&A, h);
  p3_tobytes(pk, &A);
  sha512_init(&c); sha512_update(&c, h + 32, 32); sha512_update(&c, msg, mlen); sha512_final(&c, rh);
  sc_reduce64(r, rh);
  scalarmult_base(&R, r);
  p3_tobytes(sig, &R);
  sha512_init(&c); sha512_update(&c, sig, 32); sha512_update(&c, pk, 32); sha512_update(&c, msg, mlen);
  sha512_final(&c, kh);
  sc_reduce64(k, kh);
  /* a is h[0:32] as a 255-bit integer (may exceed L; sc_muladd reduces) */
  sc_muladd(sig + 32, k, h, r);
}

typedef struct {
  size_t lo, hi;
  const uint8_t *seeds, *msg;
  const uint32_t *off;
  const uint32_t *key_idx;
  uint8_t *sig;
} sjob_t;

static void *sworker(void *arg) {
  sjob_t *j = (sjob_t *)arg;
  for (size_t i = j->lo; i < j->hi; i++) {
    size_t kid = j->key_idx ? j->key_idx[i] : i;
    oracle_sign(j->seeds + 32 * kid, j->msg + j->off[i], j->off[i + 1] - j->off[i], j->sig + 64 * i);
  }
  return NULL;
}

/* sig[i] = Sign(seeds[key_idx ? key_idx[i] : i], msg_i) */
void oracle_sign_batch(size_t n, const uint8_t *seeds, const uint32_t *key_idx, const uint8_t *msg,
                       const uint32_t *msg_off, uint8_t *sig, int nthreads) {
  pthread_once(&g_once, init_constants);
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  sjob_t jobs[256];
  for (int t = 0; t < nthreads; t++) {
    jobs[t] = (sjob_t){n * t / nthreads, n * (t + 1) / nthreads, seeds, msg, msg_off, key_idx, sig};
    pthread_create(&th[t], NULL, sworker, &jobs[t]);
  }
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
}

/* ================================================================ sr25519
 * schnorrkel / merlin / ristretto255 restatement (go-schnorrkel v1.0.0,
 * gtank/merlin v0.1.1, gtank/ristretto255 v0.1.2), reached from
 * /root/reference/crypto/sr25519/pubkey.go:34-60. Same semantics as
 * oracle/sr25519_ref.py (the Python restatement, pinned against published
 * vectors in tests/test_sr25519_oracle.py); this C copy is the fast checker
 * and the CPU baseline for the sr25519 kernel. */

static const uint64_t KECCAK_RC[24] = {
    0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808AULL, 0x8000000080008000ULL,
    0x000000000000808BULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
    0x000000000000008AULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000AULL,
    0x000000008000808BULL, 0x800000000000008BULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
    0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800AULL, 0x800000008000000AULL,
    0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};
/* rotation of lane x + 5y */
static const int KECCAK_ROT[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43,
                                   25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};

static uint64_t rol64(uint64_t x, int n) { return n ? (x << n) | (x >> (64 - n)) : x; }

static void keccak_f1600(uint64_t a[25]) {
  for (int rnd = 0; rnd < 24; rnd++) {
    uint64_t c[5], d[5], b[25];
    for (int x = 0; x < 5; x++) c[x] = a[x] ^ a[x + 5] ^ a[x + 10] ^ a[x + 15] ^ a[x + 20];
    for (int x = 0; x < 5; x++) d[x] = c[(x + 4) % 5] ^ rol64(c[(x + 1) % 5], 1);
    for (int i = 0; i < 25; i++) a[i] ^= d[i % 5];
    for (int x = 0; x < 5; x++)
      for (int y = 0; y < 5; y++) b[y + 5 * ((2 * x + 3 * y) % 5)] = rol64(a[x + 5 * y], KECCAK_ROT[x + 5 * y]);
    for (int y = 0; y < 5; y++)
      for (int x = 0; x < 5; x++)
        a[x + 5 * y] = b[x + 5 * y] ^ (~b[(x + 1) % 5 + 5 * y] & b[(x + 2) % 5 + 5 * y]);
    a[0] ^= KECCAK_RC[rnd];
  }
}

enum { STROBE_R = 166, SF_I = 1, SF_A = 2, SF_C = 4, SF_T = 8, SF_M = 16, SF_K = 32 };
typedef struct {
  uint64_t st[25]; /* little-endian byte view below (x86 host) */
  int pos, pos_begin, cur_flags;
} strobe_t;

static uint8_t *sbytes(strobe_t *s) { return (uint8_t *)s->st; }

static void strobe_run_f(strobe_t *s) {
  sbytes(s)[s->pos] ^= (uint8_t)s->pos_begin;
  sbytes(s)[s->pos + 1] ^= 0x04;
  sbytes(s)[STROBE_R + 1] ^= 0x80;
  keccak_f1600(s->st);
  s->pos = 0;
  s->pos_begin = 0;
}
static void strobe_absorb(strobe_t *s, const uint8_t *p, size_t n) {
  for (size_t i = 0; i < n; i++) {
    sbytes(s)[s->pos++] ^= p[i];
    if (s->pos == STROBE_R) strobe_run_f(s);
  }
}
static void strobe_squeeze(strobe_t *s, uint8_t *out, size_t n) {
  for (size_t i = 0; i < n; i++) {
    out[i] = sbytes(s)[s->pos];
    sbytes(s)[s->pos++] = 0;
    if (s->pos == STROBE_R) strobe_run_f(s);
  }
}
static void strobe_begin_op(strobe_t *s, int flags, int more) {
  if (more) return; /* callers only continue an op with the same flags */
  uint8_t hdr[2] = {(uint8_t)s->pos_begin, (uint8_t)flags};
  s->pos_begin = s->pos + 1;
  s->cur_flags = flags;
  strobe_absorb(s, hdr, 2);
  if ((flags & (SF_C | SF_K)) && s->pos != 0) strobe_run_f(s);
}
static void strobe_meta_ad(strobe_t *s, const uint8_t *p, size_t n, int more) {
  strobe_begin_op(s, SF_M | SF_A, more);
  strobe_absorb(s, p, n);
}
static void strobe_ad(strobe_t *s, const uint8_t *p, size_t n, int more) {
  strobe_begin_op(s, SF_A, more);
  strobe_absorb(s, p, n);
}
static void transcript_append(strobe_t *s, const char *label, const uint8_t *m, size_t n) {
  uint8_t len[4] = {(uint8_t)n, (uint8_t)(n >> 8), (uint8_t)(n >> 16), (uint8_t)(n >> 24)};
  strobe_meta_ad(s, (const uint8_t *)label, strlen(label), 0);
  strobe_meta_ad(s, len, 4, 1);
  strobe_ad(s, m, n, 0);
}
static void transcript_challenge(strobe_t *s, const char *label, uint8_t *out, size_t n) {
  uint8_t len[4] = {(uint8_t)n, (uint8_t)(n >> 8), (uint8_t)(n >> 16), (uint8_t)(n >> 24)};
  strobe_meta_ad(s, (const uint8_t *)label, strlen(label), 0);
  strobe_meta_ad(s, len, 4, 1);
  strobe_begin_op(s, SF_I | SF_A | SF_C, 0);
  strobe_squeeze(s, out, n);
}
static void transcript_init(strobe_t *s, const char *label) {
  memset(s, 0, sizeof *s);
  static const uint8_t hdr[6] = {1, STROBE_R + 2, 1, 0, 1, 96};
  memcpy(sbytes(s), hdr, 6);
  memcpy(sbytes(s) + 6, "STROBEv1.0.2", 12);
  keccak_f1600(s->st);
  strobe_meta_ad(s, (const uint8_t *)"Merlin v1.0", 11, 0);
  transcript_append(s, "dom-sep", (const uint8_t *)label, strlen(label));
}

/* merlin.NewTranscript("SigningContext") + AppendMessage("", ctx={}) +
 * AppendMessage("sign-bytes", msg) + proto-name / sign:pk / sign:R, then
 * 64 challenge bytes reduced mod L */
static void sr_challenge(uint8_t k[32], const uint8_t pk[32], const uint8_t R[32], const uint8_t *msg, size_t mlen) {
  strobe_t s;
  transcript_init(&s, "SigningContext");
  transcript_append(&s, "", NULL, 0);
  transcript_append(&s, "sign-bytes", msg, mlen);
  transcript_append(&s, "proto-name", (const uint8_t *)"Schnorr-sig", 11);
  transcript_append(&s, "sign:pk", pk, 32);
  transcript_append(&s, "sign:R", R, 32);
  uint8_t kb[64];
  transcript_challenge(&s, "sign:c", kb, 64);
  sc_reduce64(k, kb);
}

/* the verifier's challenge k for n (pk, R, msg) triples (test-vector
 * generation: tests/golden/make_wide.py searches messages for k values the
 * product's half-size-scalar split handles on its wide fallback) */
void oracle_sr25519_challenge_batch(size_t n, const uint8_t *pk, const uint8_t *R, const uint8_t *msg,
                                    const uint32_t *off, uint8_t *out_k) {
  for (size_t i = 0; i < n; i++)
    sr_challenge(out_k + 32 * i, pk + 32 * i, R + 32 * i, msg + off[i], off[i + 1] - off[i]);
}

/* RFC 9496 SQRT_RATIO_M1: r = |sqrt(u/v)| or |sqrt(i u/v)|; returns was_square */
static int fe_sqrt_ratio_m1(fe *r, const fe *u, const fe *v) {
  fe v3, v7, t, check, nu, nui;
  fe_sq(&v3, v); fe_mul(&v3, &v3, v);
  fe_sq(&v7, &v3); fe_mul(&v7, &v7, v);
  fe_mul(&t, u, &v7);
  fe_pow22523(&t, &t);
  fe_mul(&t, &t, &v3);
  fe_mul(r, &t, u);
  fe_sq(&check, r); fe_mul(&check, &check, v);
  fe_neg(&nu, u);
  fe_mul(&nui, &nu, &FE_SQRTM1);
  const int correct = fe_equal(&check, u), flipped = fe_equal(&check, &nu), flipped_i = fe_equal(&check, &nui);
  if (flipped || flipped_i) fe_mul(r, r, &FE_SQRTM1);
  if (fe_isneg(r)) fe_neg(r, r);
  return correct || flipped;
}

/* RFC 9496 4.3.1 DECODE; 0 on success */
static int ristretto_decode(ge_p3 *h, const uint8_t in[32]) {
  fe s;
  uint8_t chk[32];
  fe_frombytes(&s, in);
  fe_tobytes(chk, &s);
  if ((in[31] & 0x80) || memcmp(chk, in, 32) != 0) return -1; /* non-canonical */
  if (in[0] & 1) return -1;                                     /* negative */
  fe ss, u1, u2, u2sq, v, t, one, invsqrt, den_x, den_y;
  fe_1(&one);
  fe_sq(&ss, &s);
  fe_sub(&u1, &one, &ss);
  fe_add(&u2, &one, &ss);
  fe_sq(&u2sq, &u2);
  fe_sq(&t, &u1); fe_mul(&t, &t, &FE_D); fe_neg(&t, &t);
  fe_sub(&v, &t, &u2sq);
  fe_mul(&t, &v, &u2sq);
  const int was_square = fe_sqrt_ratio_m1(&invsqrt, &one, &t);
  fe_mul(&den_x, &invsqrt, &u2);
  fe_mul(&den_y, &invsqrt, &den_x); fe_mul(&den_y, &den_y, &v);
  fe_add(&t, &s, &s); fe_mul(&h->X, &t, &den_x);
  if (fe_isneg(&h->X)) fe_neg(&h->X, &h->X);
  fe_mul(&h->Y, &u1, &den_y);
  fe_1(&h->Z);
  fe_mul(&h->T, &h->X, &h->Y);
  if (!was_square || fe_isneg(&h->T) || fe_iszero(&h->Y)) return -1;
  return 0;
}

static fe FE_INVSQRT_A_MINUS_D;
static pthread_once_t sr_once = PTHREAD_ONCE_INIT;
static void sr_init(void) {
  pthread_once(&g_once, init_constants);
  fe one, amd;
  fe_1(&one);
  fe_neg(&amd, &one);
  fe_sub(&amd, &amd, &FE_D); /* a - d = -1 - d */
  fe_sqrt_ratio_m1(&FE_INVSQRT_A_MINUS_D, &one, &amd);
}

/* RFC 9496 4.3.2 ENCODE */
static void ristretto_encode(uint8_t out[32], const ge_p3 *p) {
  fe u1, u2, t, invsqrt, den1, den2, zinv, ix, iy, ench, x, y, deninv, one;
  fe_1(&one);
  fe_add(&u1, &p->Z, &p->Y);
  fe_sub(&t, &p->Z, &p->Y);
  fe_mul(&u1, &u1, &t);
  fe_mul(&u2, &p->X, &p->Y);
  fe_sq(&t, &u2); fe_mul(&t, &t, &u1);
  fe_sqrt_ratio_m1(&invsqrt, &one, &t);
  fe_mul(&den1, &invsqrt, &u1);
  fe_mul(&den2, &invsqrt, &u2);
  fe_mul(&zinv, &den1, &den2); fe_mul(&zinv, &zinv, &p->T);
  fe_mul(&ix, &p->X, &FE_SQRTM1);
  fe_mul(&iy, &p->Y, &FE_SQRTM1);
  fe_mul(&ench, &den1, &FE_INVSQRT_A_MINUS_D);
  fe_mul(&t, &p->T, &zinv);
  if (fe_isneg(&t)) { x = iy; y = ix; deninv = ench; }
  else { x = p->X; y = p->Y; deninv = den2; }
  fe_mul(&t, &x, &zinv);
  if (fe_isneg(&t)) fe_neg(&y, &y);
  fe_sub(&t, &p->Z, &y);
  fe_mul(&t, &deninv, &t);
  if (fe_isneg(&t)) fe_neg(&t, &t);
  fe_tobytes(out, &t);
}

/* sr25519.PubKey.VerifySignature for a 32-byte key and 64-byte signature */
int oracle_sr25519_verify_one(const uint8_t *pk, const uint8_t *msg, size_t mlen, const uint8_t *sig) {
  pthread_once(&sr_once, sr_init);
  ge_p3 A, R, Rp;
  if (ristretto_decode(&A, pk) != 0) return 0;
  if (!(sig[63] & 0x80)) return 0;
  if (ristretto_decode(&R, sig) != 0) return 0;
  uint8_t s[32], k[32];
  memcpy(s, sig + 32, 32);
  s[31] &= 0x7f;
  if (!sc_is_canonical(s)) return 0;
  sr_challenge(k, pk, sig, msg, mlen);
  ge_p3 negA = A;
  fe_neg(&negA.X, &A.X);
  fe_neg(&negA.T, &A.T);
  double_scalarmult_vartime(&Rp, k, &negA, s);
  fe l, r;
  fe_mul(&l, &Rp.X, &R.Y); fe_mul(&r, &Rp.Y, &R.X);
  if (fe_equal(&l, &r)) return 1;
  fe_mul(&l, &Rp.Y, &R.Y); fe_mul(&r, &Rp.X, &R.X);
  return fe_equal(&l, &r);
}

static void *sr_worker(void *arg) {
  job_t *j = (job_t *)arg;
  for (size_t i = j->lo; i < j->hi; i++)
    j->out[i] = (uint8_t)oracle_sr25519_verify_one(j->pk + 32 * i, j->msg + j->off[i], j->off[i + 1] - j->off[i],
                                                   j->sig + 64 * i);
  return NULL;
}

void oracle_sr25519_verify_batch(size_t n, const uint8_t *pk, const uint8_t *sig, const uint8_t *msg,
                                 const uint32_t *msg_off, uint8_t *out, int nthreads) {
  pthread_once(&sr_once, sr_init);
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  job_t jobs[256];
  for (int t = 0; t < nthreads; t++) {
    jobs[t] = (job_t){n * t / nthreads, n * (t + 1) / nthreads, pk, sig, msg, msg_off, 0, out};
    pthread_create(&th[t], NULL, sr_worker, &jobs[t]);
  }
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
}

/* MiniSecretKey.ExpandEd25519 -> (key = clamp(h[0:32]) / 8, nonce = h[32:64]) */
static void sr_expand(uint8_t key[32], uint8_t nonce[32], const uint8_t mini[32]) {
  uint8_t h[64];
  sha512_ctx c;
  sha512_init(&c); sha512_update(&c, mini, 32); sha512_final(&c, h);
  h[0] &= 248; h[31] &= 63; h[31] |= 64;
  for (int i = 0; i < 32; i++) key[i] = (uint8_t)((h[i] >> 3) | (i < 31 ? h[i + 1] << 5 : 0));
  memcpy(nonce, h + 32, 32);
}

void oracle_sr25519_pubkey(const uint8_t mini[32], uint8_t pk[32]) {
  pthread_once(&sr_once, sr_init);
  uint8_t key[32], nonce[32];
  sr_expand(key, nonce, mini);
  ge_p3 A;
  scalarmult_base(&A, key);
  ristretto_encode(pk, &A);
}

/* SecretKey.Sign with the deterministic witness of oracle/sr25519_ref.py:
 * r = SHA-512("cmtverify/sr25519-witness" || nonce || msg) mod L */
void oracle_sr25519_sign(const uint8_t mini[32], const uint8_t *msg, size_t mlen, uint8_t sig[64]) {
  pthread_once(&sr_once, sr_init);
  uint8_t key[32], nonce[32], pk[32], rh[64], r[32], k[32];
  sr_expand(key, nonce, mini);
  ge_p3 P;
  scalarmult_base(&P, key);
  ristretto_encode(pk, &P);
  sha512_ctx c;
  sha512_init(&c);
  sha512_update(&c, (const uint8_t *)"cmtverify/sr25519-witness", 25);
  sha512_update(&c, nonce, 32);
  sha512_update(&c, msg, mlen);
  sha512_final(&c, rh);
  sc_reduce64(r, rh);
  scalarmult_base(&P, r);
  ristretto_encode(sig, &P);
  sr_challenge(k, pk, sig, msg, mlen);
  sc_muladd(sig + 32, k, key, r);
  sig[63] |= 0x80;
}

void oracle_sr25519_sign_batch(size_t n, const uint8_t *minis, const uint32_t *key_idx, const uint8_t *msg,
                               const uint32_t *msg_off, uint8_t *sig) {
  for (size_t i = 0; i < n; i++) {
    size_t kid = key_idx ? key_idx[i] : i;
    oracle_sr25519_sign(minis + 32 * kid, msg + msg_off[i], msg_off[i + 1] - msg_off[i], sig + 64 * i);
  }
}
