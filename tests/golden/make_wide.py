"""Generate tests/golden/wide_vectors.json: signatures whose challenge k makes
the product's half-size-scalar split (cometbft_amd/csrc/halfscalar.h) leave
its common 34-window schedule: pairs of 135-146 bits take 35, 36 or 37
windows (~5.5e-5, ~3e-6 and ~3e-7 of random k), and the window count is
shared by the whole wave. (Beyond 146 bits the split falls back to k1 = k,
k2 = 1 over 64 windows; no k can be searched for that -- ~1e-10 -- so the
GPU tests force that schedule with the CMTV_FORCE_WIDE knob instead.)

The window count only changes the cost of a verification, never its
verdict, and random test data almost never reaches the larger ones.
Here the message is searched instead: R (and so the nonce r) is fixed, the
CanonicalVote timestamp nanos of the message vary, and k = H(R || A || M) is
classified by the host build of halfscalar.h (tests/host/halfcheck.cpp, the
device source compiled for the CPU). s is then r + k a mod L, so the
signature is valid by construction; the verdicts themselves come from the
oracles (oracle/ed25519_ref.py and oracle/liboracle.so in both Ed25519 modes,
oracle/sr25519_ref.py and liboracle.so for sr25519) and must agree.

Categories (every vector takes >= 35 windows; "windows" records how many):
  ed25519:
    honest        valid in both modes
    s_flip        honest with one bit of s flipped: invalid in both modes
    mixed_R       R = [r]B + T8 (T8 of order 8): Go-invalid (cofactorless),
                  ZIP-215-valid (cofactored)
    mixed_A       A = [a]B + T8, R = [r]B, s = r + k a: Go-invalid unless
                  8 | k, ZIP-215-valid
  sr25519:
    honest, s_flip

Deterministic (fixed seeds).  python tests/golden/make_wide.py
"""
from __future__ import annotations

import hashlib
import json
import os
import struct
import subprocess
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, ROOT)
from oracle import coracle  # noqa: E402
from oracle import ed25519_ref as E  # noqa: E402
from oracle import signbytes as SB  # noqa: E402
from oracle import sr25519_ref as S  # noqa: E402

L = E.L
CHAIN_ID = "cmtverify-wide"
BLOCK_ID = (hashlib.sha256(b"wide-block").digest(), 1, hashlib.sha256(b"wide-parts").digest())
# an order-8 point (canonical encoding), checked below
T8_ENC = bytes.fromhex("26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc05")
BATCH = 20000


def halfcheck_bin() -> str:
    src = os.path.join(ROOT, "tests", "host", "halfcheck.cpp")
    out = os.path.join(ROOT, "build", "halfcheck")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", out, src], check=True)
    return out


def windows(binary: str, ks: list[int]) -> list[int]:
    """the half-scalar window count of each k (64 = the wide fallback)"""
    buf = struct.pack("<I", len(ks)) + b"".join(k.to_bytes(32, "little") for k in ks)
    out = subprocess.run([binary], input=buf, capture_output=True, check=True).stdout
    return [(out[130 * j + 64] >> 2) + 32 for j in range(len(ks))]


def message(height: int, nanos: int) -> bytes:
    return SB.vote_sign_bytes(CHAIN_ID, SB.PRECOMMIT, height, 0, BLOCK_ID, 1_700_000_000 + height, nanos)


def search(binary: str, kfn, height: int, want: dict, budget: int = 60 * BATCH):
    """messages M (by timestamp nanos) whose challenge kfn(M) takes W
    windows, for W -> count in `want` (W = 35 also accepts more); returns
    [(M, k, W)] -- classes not found within `budget` tries are skipped"""
    found, nanos, need = [], 0, dict(want)
    while any(v > 0 for v in need.values()) and nanos < budget:
        msgs = [message(height, nanos + j) for j in range(BATCH)]
        ks = kfn(msgs)
        for m, k, w in zip(msgs, ks, windows(binary, ks)):
            cls = w if w in need else (35 if 35 < w < 64 and 35 in need else None)
            if cls is not None and need[cls] > 0:
                found.append((m, k, w))
                need[cls] -= 1
        nanos += BATCH
    return found


def ed_vectors(binary: str) -> list[dict]:
    T8 = E.decode_point(T8_ENC)
    assert T8 is not None and not E.is_identity(E.scalar_mult(4, T8))
    assert E.is_identity(E.scalar_mult(8, T8))
    out = []
    for i in range(3):
        seed = hashlib.sha256(b"cmtverify/wide/%d" % i).digest()
        a, _ = E.expand_seed(seed)
        A_pt = E.scalar_mult(a, E.B)
        A = E.encode_point(A_pt)
        r = int.from_bytes(hashlib.sha512(b"cmtverify/wide-nonce/%d" % i).digest(), "little") % L
        rB = E.scalar_mult(r, E.B)
        Rh = E.encode_point(rB)
        Rm = E.encode_point(E.point_add(rB, T8))
        Am = E.encode_point(E.point_add(A_pt, T8))

        def kfn(R, Ab):
            return lambda msgs: [E.scalar_from_hash(E.sha512(R + Ab + m)) for m in msgs]

        want = {35: 2, 36: 1, 37: 1} if i == 0 else {35: 2}
        budget = 400 * BATCH if i == 0 else 60 * BATCH
        for m, k, w in search(binary, kfn(Rh, A), 1000 + i, want, budget):
            s = (r + k * a) % L
            sig = Rh + s.to_bytes(32, "little")
            out.append({"cat": "honest", "pk": A, "sig": sig, "msg": m, "windows": w})
            flip = bytearray(sig)
            flip[32 + (k % 31)] ^= 1 << (k % 8)
            out.append({"cat": "s_flip", "pk": A, "sig": bytes(flip), "msg": m, "windows": w})
        for m, k, w in search(binary, kfn(Rm, A), 2000 + i, {35: 1}):
            s = (r + k * a) % L
            out.append({"cat": "mixed_R", "pk": A, "sig": Rm + s.to_bytes(32, "little"), "msg": m, "windows": w})
        for m, k, w in search(binary, kfn(Rh, Am), 3000 + i, {35: 1}):
            s = (r + k * a) % L
            out.append({"cat": "mixed_A", "pk": Am, "sig": Rh + s.to_bytes(32, "little"), "msg": m, "windows": w})
    # verdicts: the Python restatement and the C oracle must agree
    for v in out:
        v["go"] = int(E.verify(v["pk"], v["msg"], v["sig"], E.MODE_GO_STDLIB))
        v["zip215"] = int(E.verify(v["pk"], v["msg"], v["sig"], E.MODE_ZIP215))
    pk = np.array([np.frombuffer(v["pk"], np.uint8) for v in out])
    sig = np.array([np.frombuffer(v["sig"], np.uint8) for v in out])
    m, off = coracle.pack_msgs([v["msg"] for v in out])
    for mode, key in ((0, "go"), (1, "zip215")):
        c = coracle.verify_batch(pk, sig, m, off, mode)
        assert [int(x) for x in c] == [v[key] for v in out], key
    return out


def sr_vectors(binary: str) -> list[dict]:
    out = []
    for i in range(2):
        mini = hashlib.sha256(b"cmtverify/wide-sr/%d" % i).digest()
        a, _ = S.expand_mini(mini)
        pk = S.ristretto_encode(S.scalar_mult(a, S.B))
        r = int.from_bytes(hashlib.sha512(b"cmtverify/wide-sr-nonce/%d" % i).digest(), "little") % L
        R = S.ristretto_encode(S.scalar_mult(r, S.B))

        def kfn(msgs):
            mm, off = coracle.pack_msgs(msgs)
            n = len(msgs)
            ks = coracle.sr25519_challenges(np.tile(np.frombuffer(pk, np.uint8), (n, 1)),
                                            np.tile(np.frombuffer(R, np.uint8), (n, 1)), mm, off)
            return [int.from_bytes(k.tobytes(), "little") for k in ks]

        for m, k, w in search(binary, kfn, 4000 + i, {35: 2}):
            assert k == S.challenge(S.signing_context(b"", m), pk, R)
            sb = bytearray(((k * a + r) % L).to_bytes(32, "little"))
            sb[31] |= 0x80
            sig = R + bytes(sb)
            out.append({"cat": "honest", "pk": pk, "sig": sig, "msg": m, "windows": w})
            flip = bytearray(sig)
            flip[32 + (k % 30)] ^= 1 << (k % 8)
            out.append({"cat": "s_flip", "pk": pk, "sig": bytes(flip), "msg": m, "windows": w})
    for v in out:
        v["valid"] = int(S.verify(v["pk"], v["msg"], v["sig"]))
    pk = np.array([np.frombuffer(v["pk"], np.uint8) for v in out])
    sig = np.array([np.frombuffer(v["sig"], np.uint8) for v in out])
    m, off = coracle.pack_msgs([v["msg"] for v in out])
    c = coracle.sr25519_verify_batch(pk, sig, m, off)
    assert [int(x) for x in c] == [v["valid"] for v in out]
    return out


def main():
    binary = halfcheck_bin()
    ed = ed_vectors(binary)
    sr = sr_vectors(binary)
    hx = lambda v: {k: (x.hex() if isinstance(x, bytes) else x) for k, x in v.items()}  # noqa: E731
    doc = {"generator": "tests/golden/make_wide.py",
           "note": "every vector's challenge takes >= 35 half-scalar windows (halfscalar.h); 'windows' records it",
           "ed25519": [hx(v) for v in ed], "sr25519": [hx(v) for v in sr]}
    path = os.path.join(ROOT, "tests", "golden", "wide_vectors.json")
    with open(path, "w") as f:
        json.dump(doc, f, indent=1)
    print(f"wrote {path}: {len(ed)} ed25519, {len(sr)} sr25519 vectors")


if __name__ == "__main__":
    main()
