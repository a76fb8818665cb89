"""Generate the sr25519 edge-case corpus (tests/golden/sr25519_corpus.json).

Every vector holds (pk, sig, msg) and the verdict of
sr25519.PubKey.VerifySignature (/root/reference/crypto/sr25519/pubkey.go:34-60)
computed by the big-int restatement `oracle/sr25519_ref.py`, cross-checked at
generation time against the C restatement (oracle/liboracle.so). Also holds
the published vectors that pin the restatement (ristretto255 RFC 9496 A.1
multiples of B, the merlin simple-transcript challenge, one schnorrkel
verification vector) so the CPU tests need neither the generator nor the
network.

Categories:
  honest          valid signatures, message lengths 0..300 (incl. the 42 / 116 /
                  161-byte CanonicalVote sizes)
  bitflip         one flipped bit in R, s or the message
  no_marker       valid signature with the schnorrkel marker bit (sig[63] & 0x80) cleared
  s_range         s >= L with the marker set (s + L, L, 2^255 - 1, ...)
  pk_encoding     non-canonical / negative / non-square / bit-255 public keys
  r_encoding      the same encodings in R
  identity_pk     the all-zero key (the identity) with s = r: valid
  rfc_bad         RFC 9496 A.2-style invalid encodings as pk and as R
  random          random bytes

    python tests/golden/make_sr25519_corpus.py [--out tests/golden/sr25519_corpus.json]
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import random
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from oracle import coracle as C  # noqa: E402
from oracle import sr25519_ref as S  # noqa: E402
from oracle import signbytes as SB  # noqa: E402

SEED = 25519
P, L = S.P, S.L

RISTRETTO_MULTIPLES = [  # RFC 9496 appendix A.1: encodings of [i]B, i = 0..8
    "0000000000000000000000000000000000000000000000000000000000000000",
    "e2f2ae0a6abc4e71a884a961c500515f58e30b6aa582dd8db6a65945e08d2d76",
    "6a493210f7499cd17fecb510ae0cea23a110e8d5b901f8acadd3095c73a3b919",
    "94741f5d5d52755ece4f23f044ee27d5d1ea1e2bd196b462166b16152a9d0259",
    "da80862773358b466ffadfe0b3293ab3d9fd53c5ea6c955358f568322daf6a57",
    "e882b131016b52c1d3337080187cf768423efccbb517bb495ab812c4160ff44e",
    "f64746d3c92b13050ed8d80236a7f0007c3b3f962f5ba793d19a601ebb1df403",
    "44f53520926ec81fbd5a387845beb7df85a96a24ece18738bdcfa6a7822a176d",
    "903293d8f2287ebe10e2374dc1a53e0bc887e592699f02d077d5263cdd55601c",
]
MERLIN_SIMPLE = {  # gtank/merlin merlin_test.go TestSimpleTranscript
    "label": "test protocol", "msg_label": "some label", "msg": "some data",
    "challenge_label": "challenge",
    "challenge": "d5a21972d0d5fe320c0d263fac7fffb8145aa640af6e9bca177c03c7efcf0615",
}
SCHNORRKEL_VECTOR = {  # a schnorrkel-rs signature carried in go-schnorrkel's tests
    "context": "substrate", "msg": "this is a message",
    "pk": "46ebddef8cd9bb167dc30878d7113b7e168e6f0646beffd77d69d39bad76b47a",
    "sig": "4e172314444b8f820bb54c22e95076f220ed25373e5c178234aa6c211d29271244b947e3ff3418ff6b45fd1df1140c8cbff69fc58ee6dc96df70936a2bb74b82",
}
RFC_BAD = [  # invalid ristretto255 encodings (non-canonical, negative, non-square, ...)
    "00ffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff",
    "ffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff7f",
    "f3ffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff7f",
    "edffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff7f",
    "0100000000000000000000000000000000000000000000000000000000000000",
    "01ffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff7f",
    "ed57ffd8c914fb201471d1c3d245ce3c746fcbe63a3679d51b6a516ebebe0e20",
    "c34c4e1826e5d403b78e246e88aa051c36ccf0aafebffe137d148a2bf9104562",
    "c940e5a4404157cfb1628b108db051a8d439e1a421394ec4ebccb9ec92a8ac78",
    "47cfc5497c53dc8e61c91d17fd626ffb1c49e2bca94eed052281b510b1117a24",
    "f1c6165d33367351b0da8f6e4511010c68174a03b6581212c71c0e1d026c3c72",
    "87260f7a2f12495118360f02c26a470f450dadf34a413d21042b43b9d93e1309",
    "26948d35ca62e643e26a83177332e6b6afeb9d08e4268b650f1f5bbd8d81d371",
    "4eac077a713c57b4f4397629a4145982c661f48044dd3f96427d40b147d9742f",
    "de6a7b00deadc788eb6b6c8d20c0ae96c2f2019078fa604fee5b87d6e989ad7b",
    "bcab477be20861e01e4a0e295284146a510150d9817763caf1a6f4b422d67042",
    "2a292df7e32cababbd9de088d1d1abec9fc0440f637ed2fba145094dc14bea08",
    "f4a9e534fc0d216c44b218fa0c42d99635a0127ee2e53c712f70609649fdff22",
    "8268436f8c4126196cf64b3c7ddbda90746a378625f9813dd9b8457077256731",
    "2810e5cbc2cc4d4eece54f61c6f69758e289aa7ab440b3cbeaa21995c2f4232b",
]


def vote_msgs(rng: random.Random):
    """CanonicalVote sign-bytes of the three sizes the commit path produces."""
    out = []
    for h, chain, rnd, nil in [(1000, "cmtverify-bench", 0, False), (7, "c" * 50, 3, False), (9, "x", 0, True)]:
        bid = None if nil else (hashlib.sha256(b"block%d" % h).digest(), 1, hashlib.sha256(b"parts%d" % h).digest())
        out.append(SB.vote_sign_bytes(chain, 2, h, rnd, bid, 1672531200 + h, rng.randrange(10**9)))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(os.path.dirname(__file__), "sr25519_corpus.json"))
    args = ap.parse_args()
    rng = random.Random(SEED)
    vecs = []

    def add(cat, pk, msg, sig):
        vecs.append({"cat": cat, "pk": bytes(pk).hex(), "msg": bytes(msg).hex(), "sig": bytes(sig).hex()})

    minis = [bytes(rng.randrange(256) for _ in range(32)) for _ in range(24)]
    pks = [S.pubkey_from_mini(m) for m in minis]
    msgs = vote_msgs(rng) + [bytes(rng.randrange(256) for _ in range(n)) for n in
                             [0, 1, 31, 32, 33, 63, 64, 65, 100, 127, 128, 129, 160, 165, 166, 167, 200, 255, 256, 300]]
    honest = []
    for i, m in enumerate(msgs):
        for j in range(3):
            k = (i * 3 + j) % len(minis)
            sig = S.sign(minis[k], m, nonce_seed=bytes([j]))
            honest.append((pks[k], m, sig))
            add("honest", pks[k], m, sig)
    for pk, m, sig in honest[:40]:
        b = rng.randrange(64 * 8 + max(len(m), 1) * 8)
        s2, m2 = bytearray(sig), bytearray(m)
        if b < 512:
            s2[b // 8] ^= 1 << (b % 8)
        elif m2:
            b -= 512
            m2[b // 8 % len(m2)] ^= 1 << (b % 8)
        else:
            s2[0] ^= 2
        add("bitflip", pk, m2, s2)
    for pk, m, sig in honest[:12]:
        s2 = bytearray(sig)
        s2[63] &= 0x7F
        add("no_marker", pk, m, s2)
    for pk, m, sig in honest[:12]:
        s = int.from_bytes(sig[32:63] + bytes([sig[63] & 0x7F]), "little")
        for s_bad in (s + L, L, 2**255 - 1, L + 1, 2**253):
            sb = bytearray(s_bad.to_bytes(32, "little"))
            sb[31] |= 0x80
            add("s_range", pk, m, sig[:32] + bytes(sb))
    # encodings of public keys and R
    enc_cases = []
    for pk in pks[:8]:
        v = int.from_bytes(pk, "little")
        if v + P < 2**256:
            enc_cases.append(((v + P) % 2**256).to_bytes(32, "little"))  # non-canonical
        enc_cases.append((v | (1 << 255)).to_bytes(32, "little"))        # bit 255
        enc_cases.append((P - v).to_bytes(32, "little"))                 # negative (odd)
    for _ in range(16):  # random even canonical values: mostly non-square / invalid
        v = rng.randrange(P) & ~1
        enc_cases.append(v.to_bytes(32, "little"))
    enc_cases += [bytes.fromhex(h) for h in RFC_BAD]
    for j, e in enumerate(enc_cases):
        pk, m, sig = honest[j % len(honest)]
        add("pk_encoding" if j < len(enc_cases) - len(RFC_BAD) else "rfc_bad", e, m, sig)
        add("r_encoding" if j < len(enc_cases) - len(RFC_BAD) else "rfc_bad", pk, m, e + sig[32:])
    # the identity key: R' = [s]B, valid with s = r
    for i in range(4):
        m = msgs[i]
        r = rng.randrange(1, L)
        Rb = S.ristretto_encode(S.scalar_mult(r, S.B))
        sb = bytearray(r.to_bytes(32, "little"))
        sb[31] |= 0x80
        add("identity_pk", bytes(32), m, Rb + bytes(sb))
    for _ in range(16):
        add("random", bytes(rng.randrange(256) for _ in range(32)), msgs[rng.randrange(len(msgs))],
            bytes(rng.randrange(256) for _ in range(64)))

    # verdicts: Python restatement, cross-checked against the C restatement
    for v in vecs:
        v["valid"] = int(S.verify(bytes.fromhex(v["pk"]), bytes.fromhex(v["msg"]), bytes.fromhex(v["sig"])))
    pk = np.array([np.frombuffer(bytes.fromhex(v["pk"]), np.uint8) for v in vecs])
    sig = np.array([np.frombuffer(bytes.fromhex(v["sig"]), np.uint8) for v in vecs])
    m, off = C.pack_msgs([bytes.fromhex(v["msg"]) for v in vecs])
    cv = C.sr25519_verify_batch(pk, sig, m, off)
    bad = [i for i, v in enumerate(vecs) if v["valid"] != int(cv[i])]
    assert not bad, ("C and Python restatements disagree", bad[:10])

    summary = {}
    for v in vecs:
        s = summary.setdefault(v["cat"], {"n": 0, "valid": 0})
        s["n"] += 1
        s["valid"] += v["valid"]
    doc = {
        "generator": "tests/golden/make_sr25519_corpus.py (oracle/sr25519_ref.py)",
        "pins": {"ristretto255_multiples": RISTRETTO_MULTIPLES, "merlin_simple": MERLIN_SIMPLE,
                 "schnorrkel_vector": SCHNORRKEL_VECTOR},
        "summary": summary,
        "vectors": vecs,
    }
    with open(args.out, "w") as f:
        json.dump(doc, f, indent=0)
    print(json.dumps(summary))


if __name__ == "__main__":
    main()
