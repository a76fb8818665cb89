"""Generate the Ed25519 edge-case corpus (tests/golden/corpus.json).

Every vector holds (pk, sig, msg) and BOTH verdicts computed by the big-int
oracle `oracle/ed25519_ref.py`:
  go     -- Go 1.19 stdlib semantics (this reference, crypto/ed25519/ed25519.go:148-155)
  zip215 -- ZIP-215 cofactored semantics (north-star / upstream voi)

Categories follow SURVEY.md section 8(d) C4. Honest signatures are cross-checked
against libsodium when it is loadable. Deterministic: seeded by SEED.

    python tests/golden/make_corpus.py  [--out tests/golden/corpus.json]
"""
from __future__ import annotations

import argparse
import ctypes
import hashlib
import json
import os
import random
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from oracle import ed25519_ref as E  # noqa: E402
from oracle import signbytes as SB  # noqa: E402

SEED = 20250205
P, L = E.P, E.L


def enc_y(y: int, sign: int) -> bytes:
    return (y | (sign << 255)).to_bytes(32, "little")


def torsion_points():
    """The 8 points of the order-8 subgroup, [i]T8 for i = 0..7."""
    rng = random.Random(1)
    while True:
        y = rng.randrange(P)
        pt = E.decode_point(enc_y(y, 0))
        if pt is None:
            continue
        t = E.scalar_mult(L, pt)
        t4 = E.point_double(E.point_double(t))
        if not E.is_identity(t4):  # order exactly 8
            break
    pts, q = [], E.IDENTITY
    for _ in range(8):
        pts.append(q)
        q = E.point_add(q, t)
    return pts


def affine(pt):
    X, Y, Z, _ = pt
    zi = pow(Z, P - 2, P)
    return (X * zi) % P, (Y * zi) % P


def small_order_encodings(tors):
    """All 32-byte strings that Go's SetBytes decodes to a small-order point:
    canonical, non-canonical y (y+p < 2^255), and x=0 with the sign bit."""
    encs = []
    for pt in tors:
        x, y = affine(pt)
        ys = [y] + ([y + P] if y + P < 2**255 else [])
        for yy in ys:
            for sign in (0, 1):
                b = enc_y(yy, sign)
                d = E.decode_point(b)
                if d is not None and E.point_equal(d, pt):
                    encs.append(b)
    return sorted(set(encs))


class Gen:
    def __init__(self):
        self.rng = random.Random(SEED)
        self.vecs = []
        self.sodium = None
        try:
            so = ctypes.CDLL("/opt/conda/lib/libsodium.so")
            so.sodium_init()
            self.sodium = so
        except OSError:
            pass

    def rbytes(self, n):
        return bytes(self.rng.getrandbits(8) for _ in range(n))

    def add(self, cat, pk, msg, sig):
        go = E.verify(pk, msg, sig, E.MODE_GO_STDLIB)
        z = E.verify(pk, msg, sig, E.MODE_ZIP215)
        self.vecs.append({"cat": cat, "pk": pk.hex(), "msg": msg.hex(), "sig": sig.hex(),
                          "go": int(go), "zip215": int(z)})
        return go, z

    def sodium_check(self, pk, msg, sig, expect):
        if self.sodium is None:
            return
        ok = self.sodium.crypto_sign_verify_detached(sig, msg, ctypes.c_ulonglong(len(msg)), pk) == 0
        assert ok == expect, "libsodium disagrees on an honest vector"

    def msg(self):
        kind = self.rng.randrange(4)
        if kind == 0:  # a commit vote sign-bytes message
            h = self.rng.randrange(1, 10**6)
            bid = (hashlib.sha256(b"block%d" % h).digest(), 1, hashlib.sha256(b"parts%d" % h).digest())
            return SB.vote_sign_bytes("cmtverify-bench", 2, h, self.rng.randrange(3), bid,
                                      1672531200 + h, self.rng.randrange(10**9))
        if kind == 1:  # SHA-512 block boundaries for R||A||M (64-byte prefix)
            return self.rbytes(self.rng.choice([0, 1, 47, 48, 49, 111, 112, 175, 176, 177, 239, 240]))
        return self.rbytes(self.rng.randrange(0, 300))

    def keypair(self):
        seed = self.rbytes(32)
        return seed, E.pubkey_from_seed(seed)

    def run(self):
        rng = self.rng
        tors = torsion_points()
        so_encs = small_order_encodings(tors)
        assert len(so_encs) == 14, len(so_encs)

        # 1. honest signatures (+ libsodium cross-check)
        for _ in range(160):
            seed, pk = self.keypair()
            m = self.msg()
            sig = E.sign(seed, m)
            go, z = self.add("honest", pk, m, sig)
            assert go and z
            self.sodium_check(pk, m, sig, True)

        # 2. single bit flips of sig / msg / pk
        for _ in range(160):
            seed, pk = self.keypair()
            m = self.msg()
            sig = bytearray(E.sign(seed, m))
            where = rng.randrange(3)
            if where == 0:
                i = rng.randrange(64)
                sig[i] ^= 1 << rng.randrange(8)
            elif where == 1 and m:
                mm = bytearray(m)
                mm[rng.randrange(len(mm))] ^= 1 << rng.randrange(8)
                m = bytes(mm)
            else:
                pkb = bytearray(pk)
                pkb[rng.randrange(32)] ^= 1 << rng.randrange(8)
                pk = bytes(pkb)
            self.add("bitflip", pk, m, bytes(sig))

        # 3. s >= L and high bits of sig[63]
        for _ in range(40):
            seed, pk = self.keypair()
            m = self.msg()
            sig = E.sign(seed, m)
            R, s = sig[:32], int.from_bytes(sig[32:], "little")
            for s2 in (s + L, L, L + 1, 2**253 - 1, L - 1, 2**252 + rng.randrange(2**252)):
                if s2 < 2**256:
                    self.add("s_range", pk, m, R + s2.to_bytes(32, "little"))
            for bit in (0x20, 0x40, 0x80):
                sb = bytearray(sig)
                sb[63] |= bit
                self.add("s_highbits", pk, m, bytes(sb))
        self.add("s_range", pk, m, R + (2**256 - 1).to_bytes(32, "little"))

        # 4. ZIP-215 small-order matrix: every small-order encoding as A and R, s = 0
        m0 = b"Zcash"
        for a in so_encs:
            for r in so_encs:
                self.add("small_order_s0", a, m0, r + bytes(32))

        # 5. small-order A with a Go-valid construction: R = [s]B - [t]A, k = t mod ord
        for a in so_encs:
            A = E.decode_point(a)
            for _ in range(3):
                m = self.msg()
                for _try in range(256):
                    s = rng.randrange(L)  # R only depends on t mod ord(A): re-pick s too
                    sB = E.scalar_mult(s, E.B)
                    t = rng.randrange(8)
                    Rp = E.point_add(sB, E.point_neg(E.scalar_mult(t, A)))
                    R = E.encode_point(Rp)
                    k = E.scalar_from_hash(E.sha512(R + a + m))
                    if E.point_equal(E.scalar_mult(k, A), E.scalar_mult(t, A)):
                        break
                else:
                    raise AssertionError("no Go-valid small-order-A construction found")
                self.add("small_order_A", a, m, R + s.to_bytes(32, "little"))

        # 6. mixed-order A = [a]B + T (cofactorless/cofactored split)
        for i in range(96):
            T = tors[1 + i % 7]
            a = rng.randrange(1, L)
            Ap = E.point_add(E.scalar_mult(a, E.B), T)
            pk = E.encode_point(Ap)
            m = self.msg()
            r = rng.randrange(1, L)
            R = E.encode_point(E.scalar_mult(r, E.B))
            k = E.scalar_from_hash(E.sha512(R + pk + m))
            s = (r + k * a) % L
            self.add("mixed_order_A", pk, m, R + s.to_bytes(32, "little"))

        # 7. mixed-order R = [r]B + T with an honest key
        for i in range(56):
            seed, pk = self.keypair()
            a, _ = E.expand_seed(seed)
            T = tors[1 + i % 7]
            m = self.msg()
            r = rng.randrange(1, L)
            R = E.encode_point(E.point_add(E.scalar_mult(r, E.B), T))
            k = E.scalar_from_hash(E.sha512(R + pk + m))
            s = (r + k * a) % L
            self.add("mixed_order_R", pk, m, R + s.to_bytes(32, "little"))

        # 8. small-order R (canonical and non-canonical encodings), s = k*a
        for r_enc in so_encs:
            for _ in range(3):
                seed, pk = self.keypair()
                a, _ = E.expand_seed(seed)
                m = self.msg()
                k = E.scalar_from_hash(E.sha512(r_enc + pk + m))
                s = (k * a) % L
                self.add("small_order_R", pk, m, r_enc + s.to_bytes(32, "little"))

        # 9. non-canonical R encoding of an honest R (only possible for y < 19)
        #    and x=0-with-sign-bit A (identity, order-2 point) with s = r
        for a in so_encs:
            A = E.decode_point(a)
            for _ in range(2):
                m = self.msg()
                r = rng.randrange(1, L)
                R = E.encode_point(E.scalar_mult(r, E.B))
                k = E.scalar_from_hash(E.sha512(R + a + m))
                # choose s so that [s]B = R + [k]A holds exactly when [k]A = O
                self.add("small_order_A_s_eq_r", a, m, R + r.to_bytes(32, "little"))

        # 10. non-canonical y (y+p, y in [0,18]) that decode, as A and as R
        noncanon = []
        for y in range(19):
            for sign in (0, 1):
                b = enc_y(y + P, sign)
                if E.decode_point(b) is not None:
                    noncanon.append(b)
        for b in noncanon:
            for _ in range(4):
                seed, pk = self.keypair()
                m = self.msg()
                sig = E.sign(seed, m)
                self.add("noncanonical_A", b, m, sig)
                a, _ = E.expand_seed(seed)
                k = E.scalar_from_hash(E.sha512(b + pk + m))
                # [s]B - [k]A = [s - k a]B; pick s so R' = R_point (unknown dlog
                # of R_point) is impossible -> exercise decode + both checks
                self.add("noncanonical_R", pk, m, b + ((k * a + rng.randrange(L)) % L).to_bytes(32, "little"))

        # 11. off-curve A / R (no square root) and y >= p that does not decode
        off = []
        while len(off) < 24:
            y = rng.randrange(P)
            b = enc_y(y, rng.randrange(2))
            if E.decode_point(b) is None:
                off.append(b)
        for b in off[:12]:
            seed, pk = self.keypair()
            m = self.msg()
            self.add("offcurve_A", b, m, E.sign(seed, m))
        for b in off[12:]:
            seed, pk = self.keypair()
            m = self.msg()
            sig = E.sign(seed, m)
            self.add("offcurve_R", pk, m, b + sig[32:])

        # 12. degenerate all-zero / all-ones inputs and random garbage
        for pk in (bytes(32), b"\xff" * 32, b"\x01" + bytes(31)):
            for sig in (bytes(64), b"\xff" * 64, b"\x01" + bytes(63)):
                self.add("degenerate", pk, b"", sig)
        for _ in range(40):
            self.add("random", self.rbytes(32), self.msg(), self.rbytes(64))

        return self.vecs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(os.path.dirname(__file__), "corpus.json"))
    args = ap.parse_args()
    vecs = Gen().run()
    cats = {}
    for v in vecs:
        c = cats.setdefault(v["cat"], [0, 0, 0])
        c[0] += 1
        c[1] += v["go"]
        c[2] += v["zip215"]
    doc = {
        "generator": "tests/golden/make_corpus.py (seed %d) using oracle/ed25519_ref.py" % SEED,
        "modes": {"go": "Go 1.19 crypto/ed25519.Verify (cofactorless)", "zip215": "ZIP-215 (cofactored)"},
        "summary": {k: {"n": v[0], "go_valid": v[1], "zip215_valid": v[2]} for k, v in sorted(cats.items())},
        "vectors": vecs,
    }
    with open(args.out, "w") as f:
        json.dump(doc, f, indent=0, separators=(",", ":"))
    print(json.dumps(doc["summary"], indent=1))
    print("total", len(vecs))


if __name__ == "__main__":
    main()
