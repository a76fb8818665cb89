"""CPU oracle (TEST INFRASTRUCTURE ONLY) -- big-integer restatement of the
sr25519 (schnorrkel over ristretto255) verification on the reference's
sr25519 key path.

Nothing in the product (`cometbft_amd/`) may import this module. It is used by
`tests/`, by the golden generator `tests/golden/make_sr25519_corpus.py` and by
bench.py's cpu_baseline leg only.

What it restates
----------------
  /root/reference/crypto/sr25519/pubkey.go:34-60   PubKey.VerifySignature
     len(sig) != 64 -> false; the key bytes are copied into a [32]byte (short
     keys zero-padded, long ones truncated); PublicKey.Decode (ristretto255);
     NewSigningContext([]byte{}, msg); Signature.Decode; PublicKey.Verify.
  /root/reference/crypto/sr25519/privkey.go:22-60  PrivKey.Sign / PubKey
     (MiniSecretKey -> ExpandEd25519 -> Sign), used here only to make test data.
The algorithms live in third-party modules that are NOT in /root/reference
(go.mod:7,19,162): github.com/ChainSafe/go-schnorrkel v1.0.0,
github.com/gtank/merlin v0.1.1 (STROBE-128 over Keccak-f[1600]) and
github.com/gtank/ristretto255 v0.1.2 (RFC 9496 ristretto255). Their published
behaviour, restated below:

  Signature.Decode(in[64]):  in[63] & 0x80 == 0 -> error ("not marked");
                             R = ristretto255 Decode(in[0:32]) (non-canonical,
                             negative or non-square -> error);
                             in[63] &= 0x7f; S = Scalar.Decode(in[32:64])
                             (non-canonical S >= L -> error)
  PublicKey.Decode(pk[32]):  ristretto255 Decode
  PublicKey.Verify(sig, t):  t.AppendMessage("proto-name", "Schnorr-sig")
                             t.AppendMessage("sign:pk", pk bytes)
                             t.AppendMessage("sign:R", R bytes)
                             k = Scalar.FromUniformBytes(t.ExtractBytes("sign:c", 64))
                             R' = [S]B - [k]A ;  return R'.Equal(R)
  NewSigningContext(ctx, m): t = merlin.NewTranscript("SigningContext")
                             t.AppendMessage("", ctx); t.AppendMessage("sign-bytes", m)

Parity status: no Go toolchain and no network, so the reference cannot run
here. The restatement is pinned by published vectors of its building blocks
(tests/test_sr25519_oracle.py): the ristretto255 encodings of [0..15]B
(RFC 9496 appendix A.1), the merlin "simple transcript" challenge of
gtank/merlin's own test, and Keccak-f[1600] through hashlib's SHA3-256. The
end-to-end sr25519 verdicts are otherwise "parity unpinned" (SURVEY.md 8c):
no reference test holds a fixed sr25519 vector (crypto/sr25519/sr25519_test.go
only round-trips random keys).
"""
from __future__ import annotations

import hashlib

P = 2**255 - 19
L = 2**252 + 27742317777372353535851937790883648493
D = (-121665 * pow(121666, P - 2, P)) % P
SQRT_M1 = pow(2, (P - 1) // 4, P)

# --------------------------------------------------------------------------
# Keccak-f[1600] (FIPS 202)
_RC = [
    0x0000000000000001, 0x0000000000008082, 0x800000000000808A, 0x8000000080008000,
    0x000000000000808B, 0x0000000080000001, 0x8000000080008081, 0x8000000000008009,
    0x000000000000008A, 0x0000000000000088, 0x0000000080008009, 0x000000008000000A,
    0x000000008000808B, 0x800000000000008B, 0x8000000000008089, 0x8000000000008003,
    0x8000000000008002, 0x8000000000000080, 0x000000000000800A, 0x800000008000000A,
    0x8000000080008081, 0x8000000000008080, 0x0000000080000001, 0x8000000080008008,
]
# rotation offsets r[x][y]
_ROT = [
    [0, 36, 3, 41, 18],
    [1, 44, 10, 45, 2],
    [62, 6, 43, 15, 61],
    [28, 55, 25, 21, 56],
    [27, 20, 39, 8, 14],
]
_M64 = (1 << 64) - 1


def _rol(x: int, n: int) -> int:
    return ((x << n) | (x >> (64 - n))) & _M64 if n else x


def keccak_f1600(state: bytearray) -> None:
    """In-place permutation of a 200-byte state (lane (x, y) = bytes 8(x+5y)..)."""
    a = [int.from_bytes(state[8 * i: 8 * i + 8], "little") for i in range(25)]
    for rnd in range(24):
        c = [a[x] ^ a[x + 5] ^ a[x + 10] ^ a[x + 15] ^ a[x + 20] for x in range(5)]
        d = [c[(x - 1) % 5] ^ _rol(c[(x + 1) % 5], 1) for x in range(5)]
        a = [a[i] ^ d[i % 5] for i in range(25)]
        b = [0] * 25
        for x in range(5):
            for y in range(5):
                b[y + 5 * ((2 * x + 3 * y) % 5)] = _rol(a[x + 5 * y], _ROT[x][y])
        a = [b[i] ^ ((~b[(i % 5 + 1) % 5 + 5 * (i // 5)]) & b[(i % 5 + 2) % 5 + 5 * (i // 5)]) for i in range(25)]
        a[0] ^= _RC[rnd]
    for i in range(25):
        state[8 * i: 8 * i + 8] = a[i].to_bytes(8, "little")


def sha3_256(data: bytes) -> bytes:
    """SHA3-256 on keccak_f1600 (only to pin the permutation against hashlib)."""
    rate = 136
    st = bytearray(200)
    msg = bytearray(data) + b"\x06"
    msg += b"\x00" * (-len(msg) % rate)
    msg[-1] |= 0x80
    for off in range(0, len(msg), rate):
        for i in range(rate):
            st[i] ^= msg[off + i]
        keccak_f1600(st)
    return bytes(st[:32])


# --------------------------------------------------------------------------
# STROBE-128 as used by merlin (gtank/merlin strobe.go, merlin strobe.rs)
STROBE_R = 166
FLAG_I, FLAG_A, FLAG_C, FLAG_T, FLAG_M, FLAG_K = 1, 2, 4, 8, 16, 32


class Strobe128:
    def __init__(self, protocol_label: bytes):
        st = bytearray(200)
        st[0:6] = bytes([1, STROBE_R + 2, 1, 0, 1, 96])
        st[6:18] = b"STROBEv1.0.2"
        keccak_f1600(st)
        self.st = st
        self.pos = 0
        self.pos_begin = 0
        self.cur_flags = 0
        self.meta_ad(protocol_label, False)

    def copy(self) -> "Strobe128":
        c = Strobe128.__new__(Strobe128)
        c.st = bytearray(self.st)
        c.pos, c.pos_begin, c.cur_flags = self.pos, self.pos_begin, self.cur_flags
        return c

    def _run_f(self):
        self.st[self.pos] ^= self.pos_begin
        self.st[self.pos + 1] ^= 0x04
        self.st[STROBE_R + 1] ^= 0x80
        keccak_f1600(self.st)
        self.pos = 0
        self.pos_begin = 0

    def _absorb(self, data: bytes):
        for b in data:
            self.st[self.pos] ^= b
            self.pos += 1
            if self.pos == STROBE_R:
                self._run_f()

    def _squeeze(self, n: int) -> bytes:
        out = bytearray()
        for _ in range(n):
            out.append(self.st[self.pos])
            self.st[self.pos] = 0
            self.pos += 1
            if self.pos == STROBE_R:
                self._run_f()
        return bytes(out)

    def _begin_op(self, flags: int, more: bool):
        if more:
            assert self.cur_flags == flags
            return
        assert flags & FLAG_T == 0
        old_begin = self.pos_begin
        self.pos_begin = self.pos + 1
        self.cur_flags = flags
        self._absorb(bytes([old_begin, flags]))
        if flags & (FLAG_C | FLAG_K) and self.pos != 0:
            self._run_f()

    def meta_ad(self, data: bytes, more: bool):
        self._begin_op(FLAG_M | FLAG_A, more)
        self._absorb(data)

    def ad(self, data: bytes, more: bool):
        self._begin_op(FLAG_A, more)
        self._absorb(data)

    def prf(self, n: int, more: bool) -> bytes:
        self._begin_op(FLAG_I | FLAG_A | FLAG_C, more)
        return self._squeeze(n)


class Transcript:
    """merlin.Transcript (gtank/merlin v0.1.1 merlin.go)."""

    def __init__(self, label: bytes):
        self.s = Strobe128(b"Merlin v1.0")
        self.append_message(b"dom-sep", label)

    def copy(self) -> "Transcript":
        c = Transcript.__new__(Transcript)
        c.s = self.s.copy()
        return c

    def append_message(self, label: bytes, message: bytes):
        self.s.meta_ad(label, False)
        self.s.meta_ad(len(message).to_bytes(4, "little"), True)
        self.s.ad(message, False)

    def extract_bytes(self, label: bytes, n: int) -> bytes:
        self.s.meta_ad(label, False)
        self.s.meta_ad(n.to_bytes(4, "little"), True)
        return self.s.prf(n, False)


def signing_context(context: bytes, msg: bytes) -> Transcript:
    """go-schnorrkel NewSigningContext (sign.go)."""
    t = Transcript(b"SigningContext")
    t.append_message(b"", context)
    t.append_message(b"sign-bytes", msg)
    return t


# --------------------------------------------------------------------------
# edwards25519 / ristretto255 (RFC 9496 section 4)
def _inv(x: int) -> int:
    return pow(x, P - 2, P)


def _is_neg(x: int) -> bool:
    return (x % P) & 1 == 1


def _abs(x: int) -> int:
    x %= P
    return P - x if x & 1 else x


INVSQRT_A_MINUS_D = None  # filled below


def sqrt_ratio_m1(u: int, v: int):
    """RFC 9496 SQRT_RATIO_M1: (was_square, r) with r non-negative."""
    u %= P
    v %= P
    v3 = v * v % P * v % P
    v7 = v3 * v3 % P * v % P
    r = u * v3 % P * pow(u * v7 % P, (P - 5) // 8, P) % P
    check = v * r % P * r % P
    correct = check == u
    flipped = check == (-u) % P
    flipped_i = check == (-u * SQRT_M1) % P
    if flipped or flipped_i:
        r = r * SQRT_M1 % P
    r = _abs(r)
    return (correct or flipped), r


INVSQRT_A_MINUS_D = sqrt_ratio_m1(1, (-1 - D) % P)[1]

IDENTITY = (0, 1, 1, 0)
_BY = 4 * _inv(5) % P


def _recover_bx():
    u = (_BY * _BY - 1) % P
    v = (D * _BY * _BY + 1) % P
    ok, x = sqrt_ratio_m1(u, v)
    assert ok
    return x  # non-negative (even): the RFC 8032 base point


_BX = _recover_bx()
B = (_BX, _BY, 1, _BX * _BY % P)


def point_add(p1, p2):
    X1, Y1, Z1, T1 = p1
    X2, Y2, Z2, T2 = p2
    A = (Y1 - X1) * (Y2 - X2) % P
    Bv = (Y1 + X1) * (Y2 + X2) % P
    C = 2 * D * T1 * T2 % P
    Dv = 2 * Z1 * Z2 % P
    E, F, G, H = Bv - A, Dv - C, Dv + C, Bv + A
    return (E * F % P, G * H % P, F * G % P, E * H % P)


def point_neg(p):
    X, Y, Z, T = p
    return ((-X) % P, Y, Z, (-T) % P)


def scalar_mult(k: int, p):
    q = IDENTITY
    while k > 0:
        if k & 1:
            q = point_add(q, p)
        p = point_add(p, p)
        k >>= 1
    return q


def ristretto_decode(b: bytes):
    """RFC 9496 4.3.1 DECODE (gtank/ristretto255 Element.Decode); None on error."""
    if len(b) != 32:
        return None
    s = int.from_bytes(b, "little")
    if s >= P or s & 1:  # non-canonical (incl. bit 255) or negative
        return None
    ss = s * s % P
    u1 = (1 - ss) % P
    u2 = (1 + ss) % P
    u2_sqr = u2 * u2 % P
    v = (-(D * u1 % P * u1) - u2_sqr) % P
    was_square, invsqrt = sqrt_ratio_m1(1, v * u2_sqr % P)
    den_x = invsqrt * u2 % P
    den_y = invsqrt * den_x % P * v % P
    x = _abs(2 * s * den_x)
    y = u1 * den_y % P
    t = x * y % P
    if not was_square or _is_neg(t) or y == 0:
        return None
    return (x, y, 1, t)


def ristretto_encode(p) -> bytes:
    """RFC 9496 4.3.2 ENCODE."""
    x0, y0, z0, t0 = p
    u1 = (z0 + y0) * (z0 - y0) % P
    u2 = x0 * y0 % P
    _, invsqrt = sqrt_ratio_m1(1, u1 * u2 % P * u2 % P)
    den1 = invsqrt * u1 % P
    den2 = invsqrt * u2 % P
    z_inv = den1 * den2 % P * t0 % P
    ix0 = x0 * SQRT_M1 % P
    iy0 = y0 * SQRT_M1 % P
    enchanted = den1 * INVSQRT_A_MINUS_D % P
    rotate = _is_neg(t0 * z_inv)
    if rotate:
        x, y, den_inv = iy0, ix0, enchanted
    else:
        x, y, den_inv = x0, y0, den2
    if _is_neg(x * z_inv):
        y = (-y) % P
    s = _abs(den_inv * (z0 - y))
    return s.to_bytes(32, "little")


def ristretto_equal(p1, p2) -> bool:
    """RFC 9496 4.3.3 EQUALS: x1 y2 == y1 x2 or y1 y2 == x1 x2."""
    X1, Y1, _, _ = p1
    X2, Y2, _, _ = p2
    return (X1 * Y2 - Y1 * X2) % P == 0 or (Y1 * Y2 - X1 * X2) % P == 0


# --------------------------------------------------------------------------
# schnorrkel (go-schnorrkel v1.0.0)
SIGNATURE_SIZE = 64
PUBKEY_SIZE = 32


def challenge(t: Transcript, pk: bytes, r: bytes) -> int:
    """The verifier's k: proto-name, sign:pk, sign:R, then 64 challenge bytes
    reduced mod L (Scalar.FromUniformBytes)."""
    t = t.copy()
    t.append_message(b"proto-name", b"Schnorr-sig")
    t.append_message(b"sign:pk", pk)
    t.append_message(b"sign:R", r)
    return int.from_bytes(t.extract_bytes(b"sign:c", 64), "little") % L


def verify(pub: bytes, msg: bytes, sig: bytes) -> bool:
    """sr25519.PubKey.VerifySignature (crypto/sr25519/pubkey.go:34-60)."""
    if len(sig) != SIGNATURE_SIZE:
        return False
    p = (bytes(pub) + b"\x00" * 32)[:32]  # copy(p[:], pubKey) into a zeroed [32]byte
    A = ristretto_decode(p)
    if A is None:
        return False
    if sig[63] & 0x80 == 0:
        return False
    R = ristretto_decode(sig[:32])
    if R is None:
        return False
    s = int.from_bytes(sig[32:63] + bytes([sig[63] & 0x7F]), "little")
    if s >= L:
        return False
    k = challenge(signing_context(b"", msg), p, sig[:32])
    Rp = point_add(scalar_mult(s, B), point_neg(scalar_mult(k, A)))
    return ristretto_equal(Rp, R)


def expand_mini(mini: bytes):
    """MiniSecretKey.ExpandEd25519: h = SHA-512(mini); key = clamp(h[:32]) / 8
    (divideScalarByCofactor); nonce = h[32:]."""
    h = hashlib.sha512(mini).digest()
    key = bytearray(h[:32])
    key[0] &= 248
    key[31] &= 63
    key[31] |= 64
    return int.from_bytes(key, "little") >> 3, h[32:]


def pubkey_from_mini(mini: bytes) -> bytes:
    """sr25519.PrivKey.PubKey (crypto/sr25519/privkey.go:43-60)."""
    a, _ = expand_mini(mini)
    return ristretto_encode(scalar_mult(a, B))


def sign(mini: bytes, msg: bytes, nonce_seed: bytes = b"") -> bytes:
    """SecretKey.Sign with a deterministic witness r (go-schnorrkel draws r at
    random; any r gives a valid signature): R = [r]B, s = k a + r, sig[63] |= 0x80."""
    a, nonce = expand_mini(mini)
    pk = ristretto_encode(scalar_mult(a, B))
    r = int.from_bytes(hashlib.sha512(b"cmtverify/sr25519-witness" + nonce + nonce_seed + msg).digest(), "little") % L
    Rb = ristretto_encode(scalar_mult(r, B))
    k = challenge(signing_context(b"", msg), pk, Rb)
    s = (k * a + r) % L
    sb = bytearray(s.to_bytes(32, "little"))
    sb[31] |= 0x80
    return Rb + bytes(sb)
