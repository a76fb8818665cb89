"""CPU oracle (TEST INFRASTRUCTURE ONLY) -- big-integer restatement of the
Ed25519 verification semantics on CometBFT's commit-verification path.

Nothing in the product (`cometbft_amd/`) may import this module. It is used
only by `tests/`, `__graft_entry__.smoke()` (as the checker) and by the golden
corpus generator `tests/golden/make_corpus.py`.

What it restates
----------------
The reference verifies a commit signature through
  /root/reference/crypto/ed25519/ed25519.go:148-155  PubKey.VerifySignature
    -> golang.org/x/crypto/ed25519.Verify (x/crypto v0.5.0, go.mod:37) which,
       for Go >= 1.13, is an alias of the Go 1.19 standard library
       crypto/ed25519.Verify (toolchain pin go.mod:3, DOCKER/Dockerfile:3).
That dependency is NOT in /root/reference; its published algorithm is:

  Verify(pub, msg, sig):
    len(pub) != 32                    -> panic("ed25519: bad public key length")
    len(sig) != 64 or sig[63]&224!=0  -> false
    A = Point.SetBytes(pub)           (y mod p accepted non-canonical; x=0 with
                                       sign bit accepted; no sqrt -> false)
    k = SHA-512(sig[:32] || pub || msg)  mod L     (Scalar.SetUniformBytes)
    S = Scalar.SetCanonicalBytes(sig[32:])          (S >= L -> false)
    R' = VarTimeDoubleScalarBaseMult(k, -A, S)      (= [S]B - [k]A)
    return sig[:32] == R'.Bytes()                   (cofactorless; canonical)

MODE_ZIP215 (north-star / upstream curve25519-voi semantics) shares every step
up to R' and replaces the last line with: decode R with the same rules as A
(failure -> false) and accept iff [8](R' - R) is the identity.

Parity status: the Go-mode restatement is pinned by honest-signature
agreement with libsodium 1.0.18 / OpenSSL 3 (independent RFC 8032 code) and by
the RFC 8032 section 7.1 vectors; edge-case verdicts (non-canonical encodings,
small/mixed order, s >= L) are pinned only by this restatement of the published
Go algorithm -- no reference test exercises them.
"""
from __future__ import annotations

import hashlib

P = 2**255 - 19
L = 2**252 + 27742317777372353535851937790883648493
D = (-121665 * pow(121666, P - 2, P)) % P
SQRT_M1 = pow(2, (P - 1) // 4, P)

MODE_GO_STDLIB = 0
MODE_ZIP215 = 1


def _inv(x: int) -> int:
    return pow(x, P - 2, P)


# Base point B (RFC 8032 5.1): y = 4/5, x even.
_BY = (4 * _inv(5)) % P


def _recover_x(y: int, sign: int):
    """Go 1.19 Point.SetBytes x recovery (edwards25519.go SetBytes +
    field.Element.SqrtRatio): returns None when (y^2-1)/(dy^2+1) is not a
    square; otherwise the root whose low bit equals `sign` -- except that
    x == 0 is returned for either sign (the x=0/sign=1 encoding is accepted)."""
    u = (y * y - 1) % P
    v = (D * y * y + 1) % P
    # r = (u v^3) (u v^7)^((p-5)/8)
    r = (u * pow(v, 3, P) * pow(u * pow(v, 7, P), (P - 5) // 8, P)) % P
    check = (v * r * r) % P
    if check == u:
        pass
    elif check == (-u) % P:
        r = (r * SQRT_M1) % P
    else:
        return None
    if r & 1:  # Absolute(): choose the non-negative (even) root
        r = P - r
    if sign:
        r = (-r) % P
    return r


_BX = _recover_x(_BY, 0)

# Extended coordinates (X, Y, Z, T), x = X/Z, y = Y/Z, xy = T/Z.
IDENTITY = (0, 1, 1, 0)
B = (_BX, _BY, 1, (_BX * _BY) % P)


def point_add(p1, p2):
    """Unified addition for a=-1 twisted Edwards (HWCD 2008, add-2008-hwcd-3);
    complete on edwards25519."""
    X1, Y1, Z1, T1 = p1
    X2, Y2, Z2, T2 = p2
    a = ((Y1 - X1) * (Y2 - X2)) % P
    b = ((Y1 + X1) * (Y2 + X2)) % P
    c = (2 * D * T1 * T2) % P
    d = (2 * Z1 * Z2) % P
    e, f, g, h = b - a, d - c, d + c, b + a
    return ((e * f) % P, (g * h) % P, (f * g) % P, (e * h) % P)


def point_neg(p):
    X, Y, Z, T = p
    return ((-X) % P, Y, Z, (-T) % P)


def point_double(p):
    return point_add(p, p)


def scalar_mult(k: int, p):
    q = IDENTITY
    while k > 0:
        if k & 1:
            q = point_add(q, p)
        p = point_double(p)
        k >>= 1
    return q


def point_equal(p1, p2) -> bool:
    X1, Y1, Z1, _ = p1
    X2, Y2, Z2, _ = p2
    return (X1 * Z2 - X2 * Z1) % P == 0 and (Y1 * Z2 - Y2 * Z1) % P == 0


def is_identity(p) -> bool:
    X, Y, Z, _ = p
    return X % P == 0 and (Y - Z) % P == 0


def encode_point(p) -> bytes:
    """Go Point.Bytes(): canonical y, sign bit = low bit of canonical x."""
    X, Y, Z, _ = p
    zi = _inv(Z)
    x, y = (X * zi) % P, (Y * zi) % P
    return (y | ((x & 1) << 255)).to_bytes(32, "little")


def decode_point(b: bytes):
    """Go 1.19 Point.SetBytes: y = bytes mod 2^255 taken mod p (non-canonical
    accepted), returns None when no square root exists."""
    if len(b) != 32:
        return None
    v = int.from_bytes(b, "little")
    sign = v >> 255
    y = (v & ((1 << 255) - 1)) % P
    x = _recover_x(y, sign)
    if x is None:
        return None
    return (x, y, 1, (x * y) % P)


def sha512(data: bytes) -> bytes:
    return hashlib.sha512(data).digest()


def scalar_from_hash(h: bytes) -> int:
    """Scalar.SetUniformBytes: 64-byte little-endian integer mod L."""
    return int.from_bytes(h, "little") % L


class BadPublicKeyLength(Exception):
    """Stands in for Go's panic("ed25519: bad public key length: N")."""


def verify(pub: bytes, msg: bytes, sig: bytes, mode: int = MODE_GO_STDLIB) -> bool:
    """Single-signature verdict in the given mode (see module docstring).

    The tendermint wrapper's own length check (crypto/ed25519/ed25519.go:150)
    and Go's (sig[63]&224, s<L) are both applied."""
    if len(pub) != 32:
        raise BadPublicKeyLength(f"ed25519: bad public key length: {len(pub)}")
    if len(sig) != 64 or sig[63] & 224:
        return False
    A = decode_point(pub)
    if A is None:
        return False
    k = scalar_from_hash(sha512(sig[:32] + pub + msg))
    s = int.from_bytes(sig[32:], "little")
    if s >= L:
        return False
    Rp = point_add(scalar_mult(s, B), point_neg(scalar_mult(k, A)))
    if mode == MODE_GO_STDLIB:
        return encode_point(Rp) == sig[:32]
    R = decode_point(sig[:32])
    if R is None:
        return False
    diff = point_add(Rp, point_neg(R))
    for _ in range(3):
        diff = point_double(diff)
    return is_identity(diff)


# --- RFC 8032 key generation and signing (deterministic; equals Go's Sign) ---

def expand_seed(seed: bytes):
    h = sha512(seed)
    a = int.from_bytes(h[:32], "little")
    a &= (1 << 254) - 8
    a |= 1 << 254
    return a, h[32:]


def pubkey_from_seed(seed: bytes) -> bytes:
    a, _ = expand_seed(seed)
    return encode_point(scalar_mult(a, B))


def sign(seed: bytes, msg: bytes) -> bytes:
    a, prefix = expand_seed(seed)
    A = encode_point(scalar_mult(a, B))
    r = scalar_from_hash(sha512(prefix + msg))
    R = encode_point(scalar_mult(r, B))
    k = scalar_from_hash(sha512(R + A + msg))
    s = (r + k * a) % L
    return R + s.to_bytes(32, "little")


def gen_priv_key_from_secret(secret: bytes) -> bytes:
    """crypto/ed25519/ed25519.go:122 GenPrivKeyFromSecret: seed = SHA-256(secret);
    returns the 32-byte seed (the Go PrivKey is seed || pubkey)."""
    return hashlib.sha256(secret).digest()
