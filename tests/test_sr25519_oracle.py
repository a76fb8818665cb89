"""sr25519 (configs[4]) on the CPU: the oracle pinned against published
vectors, the C and Python restatements against the committed corpus, and the
GPU kernel's source (cometbft_amd/csrc/sr25519.h) host-compiled and run over
the same corpus.

Reference path: /root/reference/crypto/sr25519/pubkey.go:34-60 (VerifySignature)
over go-schnorrkel v1.0.0 / gtank/merlin v0.1.1 / gtank/ristretto255 v0.1.2.
The reference's own test (crypto/sr25519/sr25519_test.go:13-31) is a random
sign / verify / one-bit-flip round trip; test_reference_round_trip mirrors it.
"""
import hashlib
import json
import os
import struct
import subprocess

import numpy as np
import pytest

from tests.host import hostbuild

from oracle import coracle as C
from oracle import sr25519_ref as S

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden", "sr25519_corpus.json")
SRC = os.path.join(ROOT, "tests", "host", "srcheck.cpp")
BIN = os.path.join(ROOT, "build", "srcheck")


@pytest.fixture(scope="module")
def doc():
    with open(GOLDEN) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def vectors(doc):
    vecs = doc["vectors"]
    pk = np.array([np.frombuffer(bytes.fromhex(v["pk"]), np.uint8) for v in vecs])
    sig = np.array([np.frombuffer(bytes.fromhex(v["sig"]), np.uint8) for v in vecs])
    msgs = [bytes.fromhex(v["msg"]) for v in vecs]
    valid = np.array([v["valid"] for v in vecs], np.uint8)
    return {"pk": pk, "sig": sig, "msgs": msgs, "valid": valid, "cats": [v["cat"] for v in vecs]}


@pytest.fixture(scope="module")
def srcheck():
    return hostbuild.build(SRC, BIN, ["-std=c++17"])


def test_keccak_matches_sha3():
    for m in [b"", b"abc", bytes(range(256)) * 3]:
        assert S.sha3_256(m) == hashlib.sha3_256(m).digest()


def test_merlin_simple_transcript(doc):
    v = doc["pins"]["merlin_simple"]
    t = S.Transcript(v["label"].encode())
    t.append_message(v["msg_label"].encode(), v["msg"].encode())
    assert t.extract_bytes(v["challenge_label"].encode(), 32).hex() == v["challenge"]


def test_ristretto_multiples_of_base(doc):
    for i, h in enumerate(doc["pins"]["ristretto255_multiples"]):
        assert S.ristretto_encode(S.scalar_mult(i, S.B)).hex() == h
        p = S.ristretto_decode(bytes.fromhex(h))
        assert p is not None and S.ristretto_equal(p, S.scalar_mult(i, S.B))


def test_schnorrkel_vector(doc):
    """A signature produced by the Rust schnorrkel implementation (context
    "substrate") verifies under the restated transcript and equation."""
    v = doc["pins"]["schnorrkel_vector"]
    pk, sig = bytes.fromhex(v["pk"]), bytes.fromhex(v["sig"])
    A, R = S.ristretto_decode(pk), S.ristretto_decode(sig[:32])
    s = int.from_bytes(sig[32:63] + bytes([sig[63] & 0x7F]), "little")
    k = S.challenge(S.signing_context(v["context"].encode(), v["msg"].encode()), pk, sig[:32])
    Rp = S.point_add(S.scalar_mult(s, S.B), S.point_neg(S.scalar_mult(k, A)))
    assert S.ristretto_equal(Rp, R)
    k2 = S.challenge(S.signing_context(b"", v["msg"].encode()), pk, sig[:32])
    Rp2 = S.point_add(S.scalar_mult(s, S.B), S.point_neg(S.scalar_mult(k2, A)))
    assert not S.ristretto_equal(Rp2, R)  # the context is bound into k


def test_python_oracle_matches_corpus(vectors):
    got = [int(S.verify(vectors["pk"][i].tobytes(), vectors["msgs"][i], vectors["sig"][i].tobytes()))
           for i in range(len(vectors["msgs"]))]
    assert got == list(vectors["valid"])


def test_c_oracle_matches_corpus(vectors):
    m, off = C.pack_msgs(vectors["msgs"])
    got = C.sr25519_verify_batch(vectors["pk"], vectors["sig"], m, off, nthreads=4)
    assert np.array_equal(got, vectors["valid"])


def test_corpus_covers_the_equality_path(vectors):
    """Honest signatures where R' != R as points but R' == R as ristretto
    elements (they differ by 4-torsion): an exact point comparison would
    reject them, so the kernel's ristretto Equal is exercised."""
    n_torsion = 0
    for i, c in enumerate(vectors["cats"]):
        if c != "honest":
            continue
        pk, sig, msg = vectors["pk"][i].tobytes(), vectors["sig"][i].tobytes(), vectors["msgs"][i]
        A, R = S.ristretto_decode(pk), S.ristretto_decode(sig[:32])
        s = int.from_bytes(sig[32:63] + bytes([sig[63] & 0x7F]), "little")
        k = S.challenge(S.signing_context(b"", msg), pk, sig[:32])
        Rp = S.point_add(S.scalar_mult(s, S.B), S.point_neg(S.scalar_mult(k, A)))
        X1, Y1, Z1, _ = Rp
        X2, Y2, Z2, _ = R
        exact = (X1 * Z2 - X2 * Z1) % S.P == 0 and (Y1 * Z2 - Y2 * Z1) % S.P == 0
        n_torsion += not exact
    assert n_torsion > 0


def test_reference_round_trip():
    """crypto/sr25519/sr25519_test.go:13-31: sign a random 128-byte message,
    verify twice, flip one bit of the signature, verify fails."""
    rng = np.random.default_rng(13)
    mini = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    msg = rng.integers(0, 256, 128, dtype=np.uint8).tobytes()
    pk = S.pubkey_from_mini(mini)
    sig = bytearray(S.sign(mini, msg))
    assert S.verify(pk, msg, bytes(sig)) and S.verify(pk, msg, bytes(sig))
    sig[7] ^= 0x01
    assert not S.verify(pk, msg, bytes(sig))


def test_key_and_signature_lengths():
    """pubkey.go:36-48: len(sig) != 64 -> false; the key is copied into a
    zeroed [32]byte (a short key is zero-padded, a long one truncated)."""
    rng = np.random.default_rng(14)
    mini = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    pk = S.pubkey_from_mini(mini)
    sig = S.sign(mini, b"m")
    assert S.verify(pk, b"m", sig)
    assert not S.verify(pk, b"m", sig[:63]) and not S.verify(pk, b"m", sig + b"\0")
    assert S.verify(pk + b"trailing", b"m", sig)
    assert S.verify(b"", b"m", S.sign(b"\0" * 32, b"m")) == S.verify(bytes(32), b"m", S.sign(b"\0" * 32, b"m"))


def _srcheck_input(vectors, idx):
    buf = [struct.pack("<I", len(idx))]
    for i in idx:
        m = vectors["msgs"][i]
        buf.append(vectors["pk"][i].tobytes() + vectors["sig"][i].tobytes() + struct.pack("<I", len(m)) + m)
    return b"".join(buf)


def _run_srcheck(binary, vectors, idx, arg=None):
    out = subprocess.run([binary] + ([arg] if arg else []), input=_srcheck_input(vectors, idx), capture_output=True,
                         check=True, timeout=600).stdout
    return out


def test_device_transcript_matches_oracle(srcheck, vectors):
    """merlin.h's byte-code transcript (host build) == the Python merlin."""
    idx = list(range(0, len(vectors["msgs"]), 7))
    out = _run_srcheck(srcheck, vectors, idx, "challenge")
    for j, i in enumerate(idx):
        pk, sig, msg = vectors["pk"][i].tobytes(), vectors["sig"][i].tobytes(), vectors["msgs"][i]
        t = S.signing_context(b"", msg)
        t.append_message(b"proto-name", b"Schnorr-sig")
        t.append_message(b"sign:pk", pk)
        t.append_message(b"sign:R", sig[:32])
        assert out[64 * j: 64 * (j + 1)] == t.extract_bytes(b"sign:c", 64), i


def test_device_transcript_every_length(srcheck):
    """The chunked transcript at every message length 0..340: every position
    the 4-byte chunks, the headers and the key words can meet the STROBE
    block end (R = 166) at, against the Python merlin (srcheck also checks
    the device program -- precomputed prefix -- against the full one)."""
    rng = np.random.default_rng(7)
    lens = list(range(0, 341))
    pks = [rng.integers(0, 256, 32, dtype=np.uint8).tobytes() for _ in lens]
    sigs = [rng.integers(0, 256, 64, dtype=np.uint8).tobytes() for _ in lens]
    msgs = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in lens]
    buf = [struct.pack("<I", len(lens))]
    for pk, sig, m in zip(pks, sigs, msgs):
        buf += [pk, sig, struct.pack("<I", len(m)), m]
    out = subprocess.run([srcheck, "challenge"], input=b"".join(buf), capture_output=True, check=True,
                         timeout=600).stdout
    for j, (pk, sig, m) in enumerate(zip(pks, sigs, msgs)):
        t = S.signing_context(b"", m)
        t.append_message(b"proto-name", b"Schnorr-sig")
        t.append_message(b"sign:pk", pk)
        t.append_message(b"sign:R", sig[:32])
        assert out[64 * j: 64 * (j + 1)] == t.extract_bytes(b"sign:c", 64), len(m)


def test_device_pipeline_matches_corpus(srcheck, vectors):
    """sr25519.h (the kernel's source, host build with bound checks) over the
    whole corpus."""
    idx = list(range(len(vectors["msgs"])))
    got = np.frombuffer(_run_srcheck(srcheck, vectors, idx), np.uint8)
    bad = np.nonzero(got != vectors["valid"])[0]
    assert bad.size == 0, [(int(i), vectors["cats"][int(i)]) for i in bad[:10]]


QSRC = os.path.join(ROOT, "tests", "host", "quadcheck.cpp")
QBIN = os.path.join(ROOT, "build", "quadcheck")


def test_quad_pipeline_matches_corpus(vectors):
    """sr25519_quad.h (the quad kernel's source: half-size scalars, E[4]
    final check), four host threads in lockstep for the DPP exchanges, over
    every non-honest vector and a slice of the honest ones."""
    hostbuild.build(QSRC, QBIN, ["-std=c++20", "-pthread"])
    cats = vectors["cats"]
    idx = [i for i, c in enumerate(cats) if c != "honest"] + [i for i, c in enumerate(cats) if c == "honest"][::3]
    got = np.frombuffer(_run_srcheck(QBIN, vectors, sorted(idx), "sr"), np.uint8)
    exp = vectors["valid"][sorted(idx)]
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, [(sorted(idx)[int(i)], cats[sorted(idx)[int(i)]]) for i in bad[:10]]


def test_split_quad_pipeline_matches_corpus(vectors):
    """the split kernel's order (k_verify_sr25519_quad_split) --
    tables before the scalars (q_tables_early, R's table of -R), the
    transcript and [u]B from the helper's code, a negative k2 flipping R's
    digits at lookup (q_straus_prep_b<true, true>) -- over the whole corpus,
    with both signs of k2 represented. Every radix-16 digit value, including
    dR = 0 and dR = -8, occurs in the corpus' ~10k windows."""
    hostbuild.build(QSRC, QBIN, ["-std=c++20", "-pthread"])
    idx = list(range(len(vectors["cats"])))
    buf = _srcheck_input(vectors, idx)
    r = subprocess.run([QBIN, "sr2"], input=buf, capture_output=True, check=True, timeout=600)
    got = np.frombuffer(r.stdout, np.uint8)
    bad = np.nonzero(got != vectors["valid"])[0]
    assert bad.size == 0, [(int(i), vectors["cats"][int(i)]) for i in bad[:10]]
    neg = int(r.stderr.decode().split("k2_neg ")[1].split()[0])
    assert 0.2 * len(idx) < neg < 0.8 * len(idx), neg


def test_helper_summed_quad_pipeline_matches_corpus(vectors):
    """k_verify_sr25519_quad_hs's path (sr25519_quad.h q_verify_sr_hs on
    quad.h q_hs_straus): both tables of extended points before the scalars,
    every window's two entries summed as the helper wave does
    (h_window_addend over the four lane threads' tables), window counts raised
    by 0-2 and the helper's share of [u]B varied, over the whole corpus."""
    hostbuild.build(QSRC, QBIN, ["-std=c++20", "-pthread"])
    idx = list(range(len(vectors["cats"])))
    buf = _srcheck_input(vectors, idx)
    r = subprocess.run([QBIN, "sr3"], input=buf, capture_output=True, check=True, timeout=600)
    got = np.frombuffer(r.stdout, np.uint8)
    bad = np.nonzero(got != vectors["valid"])[0]
    assert bad.size == 0, [(int(i), vectors["cats"][int(i)]) for i in bad[:10]]
