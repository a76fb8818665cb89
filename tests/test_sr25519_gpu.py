"""GPU parity for sr25519 (configs[4]): libcmtverify's k_verify_sr25519_quad
(batches up to the quad crossover) and k_verify_sr25519 (lane) verdicts vs the
oracle, bit-exact.

Oracle: tests/golden/sr25519_corpus.json (verdicts of oracle/sr25519_ref.py,
pinned in tests/test_sr25519_oracle.py) and the C restatement in
oracle/liboracle.so for the seeded batches.
"""
import json
import os

import numpy as np
import pytest

from oracle import coracle
from cometbft_amd import Sr25519BatchVerifier, Sr25519PubKey, pack_messages

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def srcorpus():
    with open(os.path.join(ROOT, "tests", "golden", "sr25519_corpus.json")) as f:
        vecs = json.load(f)["vectors"]
    pk = np.array([np.frombuffer(bytes.fromhex(v["pk"]), np.uint8) for v in vecs])
    sig = np.array([np.frombuffer(bytes.fromhex(v["sig"]), np.uint8) for v in vecs])
    msgs = [bytes.fromhex(v["msg"]) for v in vecs]
    return pk, sig, msgs, np.array([v["valid"] for v in vecs], np.uint8), [v["cat"] for v in vecs]


@pytest.mark.parametrize("kernel", ["quad", "lane"])
def test_corpus_bit_exact(gpu_ctx, gpu_ctx_lane, srcorpus, kernel):
    gpu_ctx = {"quad": gpu_ctx, "lane": gpu_ctx_lane}[kernel]
    pk, sig, msgs, exp, cats = srcorpus
    m, off = pack_messages(msgs)
    valid, words = gpu_ctx.verify_sr25519(pk, sig, m, off, bitmap=True)
    bad = np.nonzero(valid != exp)[0]
    assert bad.size == 0, [(cats[i], int(valid[i]), int(exp[i])) for i in bad[:20]]
    bits = np.unpackbits(words.view(np.uint8), bitorder="little")[: len(exp)]
    assert np.array_equal(bits, exp)


def _honest(n, seed, nkeys=None, msg_len=None):
    rng = np.random.default_rng(seed)
    nkeys = nkeys or n
    minis = rng.integers(0, 256, (nkeys, 32), dtype=np.uint8)
    kidx = (np.arange(n) % nkeys).astype(np.uint32)
    lens = rng.integers(0, 260, n) if msg_len is None else np.full(n, msg_len)
    msgs = [rng.integers(0, 256, int(l), dtype=np.uint8).tobytes() for l in lens]
    m, off = coracle.pack_msgs(msgs)
    sig = coracle.sr25519_sign_batch(minis, m, off, key_idx=kidx)
    pk = coracle.sr25519_pubkeys(minis)[kidx]
    return pk, sig, m, off, msgs


@pytest.mark.parametrize("kernel", ["quad", "lane"])
@pytest.mark.parametrize("n", [1, 15, 16, 17, 63, 64, 65, 1000])
def test_ragged_sizes_honest_and_flipped(gpu_ctx, gpu_ctx_lane, n, kernel):
    gpu_ctx = {"quad": gpu_ctx, "lane": gpu_ctx_lane}[kernel]
    pk, sig, m, off, _ = _honest(n, 500 + n, nkeys=min(n, 50))
    rng = np.random.default_rng(n)
    sig = sig.copy()
    flip = rng.random(n) < 0.3
    rows = np.nonzero(flip)[0]
    sig[rows, rng.integers(0, 64, rows.size)] ^= (1 << rng.integers(0, 8, rows.size)).astype(np.uint8)
    exp = coracle.sr25519_verify_batch(pk, sig, m, off, nthreads=8)
    got = gpu_ctx.verify_sr25519(pk, sig, m, off)
    assert np.array_equal(got, exp)
    assert exp[~flip].all()


@pytest.mark.parametrize("kernel", ["quad", "lane"])
def test_commit_sized_batch(gpu_ctx, gpu_ctx_lane, kernel):
    """A 10k-signature batch of 116-byte messages over 150 keys (the commit
    shape), all valid, plus a 1% corrupted copy."""
    gpu_ctx = {"quad": gpu_ctx, "lane": gpu_ctx_lane}[kernel]
    pk, sig, m, off, _ = _honest(10000, 7, nkeys=150, msg_len=116)
    assert gpu_ctx.verify_sr25519(pk, sig, m, off).all()
    sig2 = sig.copy()
    sig2[::100, 40] ^= 1
    exp = coracle.sr25519_verify_batch(pk, sig2, m, off, nthreads=16)
    assert np.array_equal(gpu_ctx.verify_sr25519(pk, sig2, m, off), exp)
    assert exp.sum() == 10000 - 100


@pytest.mark.parametrize("kernel", ["quad", "lane"])
def test_long_and_mixed_message_lengths(gpu_ctx, gpu_ctx_lane, kernel):
    """merlin.h runs a wave's message loop for its longest message and the
    136-byte tail in two passes around the STROBE block end: waves mixing
    empty, short and multi-block messages (up to 2,000 bytes, several F's in
    the message loop), the tail starting at every block position, honest and
    flipped, against the C oracle."""
    gpu_ctx = {"quad": gpu_ctx, "lane": gpu_ctx_lane}[kernel]
    rng = np.random.default_rng(31)
    n = 640
    minis = rng.integers(0, 256, (32, 32), dtype=np.uint8)
    kidx = (np.arange(n) % 32).astype(np.uint32)
    lens = np.where(np.arange(n) % 7 == 0, rng.integers(600, 2000, n), rng.integers(0, 400, n))
    lens[::13] = 0
    msgs = [rng.integers(0, 256, int(l), dtype=np.uint8).tobytes() for l in lens]
    m, off = coracle.pack_msgs(msgs)
    sig = coracle.sr25519_sign_batch(minis, m, off, key_idx=kidx).copy()
    pk = coracle.sr25519_pubkeys(minis)[kidx]
    sig[1::5, 50] ^= 0x10
    exp = coracle.sr25519_verify_batch(pk, sig, m, off, nthreads=8)
    assert np.array_equal(gpu_ctx.verify_sr25519(pk, sig, m, off), exp)
    assert exp.sum() == n - len(range(1, n, 5))


def test_device_buffers_match_host_path(gpu_ctx):
    import torch

    pk, sig, m, off, _ = _honest(777, 8, nkeys=20)
    sig = sig.copy()
    sig[::5, 3] ^= 4
    exp = gpu_ctx.verify_sr25519(pk, sig, m, off)
    dev = torch.device("cuda:0")
    d = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in
         {"pk": pk, "sig": sig, "m": m, "off": off.view(np.int32)}.items()}
    d_valid = torch.zeros(777, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    gpu_ctx.verify_sr25519_device(777, d["pk"].data_ptr(), d["sig"].data_ptr(), d["m"].data_ptr(),
                                  d["off"].data_ptr(), d_valid.data_ptr(), 0, s)
    torch.cuda.synchronize()
    assert np.array_equal(d_valid.cpu().numpy(), exp)


def test_pubkey_and_batch_mirror(gpu_ctx):
    """Sr25519PubKey.verify_signature / Sr25519BatchVerifier follow
    pubkey.go:34-60's length rules: a 63-byte signature is false, a key
    longer than 32 bytes is truncated."""
    pk, sig, m, off, msgs = _honest(3, 9)
    k = Sr25519PubKey(pk[0].tobytes())
    assert k.verify_signature(msgs[0], sig[0].tobytes(), ctx=gpu_ctx)
    assert not k.verify_signature(msgs[0], sig[0].tobytes()[:63], ctx=gpu_ctx)
    assert Sr25519PubKey(pk[0].tobytes() + b"xx").verify_signature(msgs[0], sig[0].tobytes(), ctx=gpu_ctx)
    bv = Sr25519BatchVerifier(gpu_ctx)
    for i in range(3):
        bv.add(pk[i].tobytes(), msgs[i], sig[i].tobytes())
    bv.add(pk[0].tobytes(), msgs[0], sig[0].tobytes()[:10])
    ok, res = bv.verify()
    assert not ok and res == [True, True, True, False]


@pytest.mark.parametrize("n", [49152, 49153])
def test_default_dispatch_at_the_sr25519_crossover(gpu_ctx, n):
    """the default context on both sides of sr25519's quad / lane
    crossover (49,152 since the round-5 transcript, as Ed25519's; 40,000 in
    round 4), 1% flipped signatures, verdict bytes and bitmap against the C
    restatement of go-schnorrkel."""
    rng = np.random.default_rng(n)
    pk, sig, m, off, _ = _honest(n, n, nkeys=512, msg_len=116)
    sig = sig.copy()
    for i in np.nonzero(rng.random(n) < 0.01)[0]:
        sig[i, rng.integers(0, 64)] ^= 1 << rng.integers(0, 8)
    exp = coracle.sr25519_verify_batch(pk, sig, m, off, nthreads=16)
    assert (exp == 0).sum() > n // 200
    got, words = gpu_ctx.verify_sr25519(pk, sig, m, off, bitmap=True)
    assert np.array_equal(got, exp), np.nonzero(got != exp)[0][:10]
    bits = np.unpackbits(words.view(np.uint8), bitorder="little")
    assert np.array_equal(bits[:n], exp) and not bits[n:].any()
