"""GPU parity: libcmtverify verdicts vs the oracle, bit-exact, both modes.

Oracle: tests/golden/corpus.json (verdicts from oracle/ed25519_ref.py, pinned
in tests/test_oracle.py) and the C restatement oracle/liboracle.so.
"""
import hashlib

import numpy as np
import pytest

from oracle import coracle
from cometbft_amd import MODE_GO_STDLIB, MODE_ZIP215, pack_messages
from conftest import ED_FORMS

pytestmark = pytest.mark.gpu


def _cat_report(cats, got, exp):
    bad = np.nonzero(got != exp)[0]
    return [(cats[i], int(got[i]), int(exp[i])) for i in bad[:20]]


@pytest.mark.parametrize("kernel", ED_FORMS)
@pytest.mark.parametrize("mode,key", [(MODE_GO_STDLIB, "go"), (MODE_ZIP215, "zip215")])
def test_corpus_bit_exact(form_ctx, corpus, mode, key, kernel):
    ctx = form_ctx(kernel)
    msg, off = pack_messages(corpus["msgs"])
    valid, words = ctx.verify(corpus["pk"], corpus["sig"], msg, off, mode, bitmap=True)
    exp = corpus[key]
    assert np.array_equal(valid, exp), _cat_report(corpus["cats"], valid, exp)
    bits = np.unpackbits(words.view(np.uint8), bitorder="little")[: len(exp)]
    assert np.array_equal(bits, exp)


def _honest(n, seed, msg_len=None):
    rng = np.random.default_rng(seed)
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    if msg_len is None:
        lens = rng.integers(0, 260, n)
    else:
        lens = np.full(n, msg_len)
    msgs = [rng.integers(0, 256, int(l), dtype=np.uint8).tobytes() for l in lens]
    m, off = coracle.pack_msgs(msgs)
    sig = coracle.sign_batch(seeds, m, off, nthreads=8)
    pk = coracle.pubkeys_from_seeds(seeds)
    return seeds, pk, sig, m, off


def test_device_keygen_and_signing_match_oracle(gpu_ctx):
    seeds, pk, sig, m, off = _honest(300, 1)
    assert np.array_equal(gpu_ctx.pubkeys(seeds), pk)
    assert np.array_equal(gpu_ctx.sign(seeds, m, off), sig)


def test_bench_signer_matches_oracle_at_commit_scale(gpu_ctx):
    """The bench's workloads are signed by the device (k_sign): pin it byte
    for byte against the C oracle's RFC 8032 signer at the 10k-commit shape
    (10,000 CanonicalVote-sized messages over 1,000 keys), so the bench's
    verdict check is not self-consistency only."""
    n, nk = 10_000, 1_000
    rng = np.random.default_rng(2024)
    seeds = rng.integers(0, 256, (nk, 32), dtype=np.uint8)
    kidx = rng.integers(0, nk, n).astype(np.uint32)
    msgs = [rng.integers(0, 256, 110 + int(rng.integers(0, 12)), dtype=np.uint8).tobytes() for _ in range(n)]
    m, off = coracle.pack_msgs(msgs)
    assert np.array_equal(gpu_ctx.pubkeys(seeds), coracle.pubkeys_from_seeds(seeds))
    dev = gpu_ctx.sign(seeds, m, off, key_idx=kidx)
    ref = coracle.sign_batch(seeds, m, off, key_idx=kidx, nthreads=8)
    assert np.array_equal(dev, ref), np.nonzero((dev != ref).any(axis=1))[0][:10]


@pytest.mark.parametrize("kernel", ED_FORMS)
@pytest.mark.parametrize("n", [1, 2, 3, 4, 15, 16, 17, 63, 64, 65, 127, 769, 1000])
def test_ragged_sizes_honest_and_flipped(form_ctx, n, kernel):
    gpu_ctx = form_ctx(kernel)
    seeds, pk, sig, m, off = _honest(n, 100 + n)
    rng = np.random.default_rng(n)
    sig = sig.copy()
    flip = rng.random(n) < 0.3
    for i in np.nonzero(flip)[0]:
        sig[i, rng.integers(0, 64)] ^= 1 << rng.integers(0, 8)
    for mode in (MODE_GO_STDLIB, MODE_ZIP215):
        exp = coracle.verify_batch(pk, sig, m, off, mode, nthreads=8)
        got, words = gpu_ctx.verify(pk, sig, m, off, mode, bitmap=True)
        assert np.array_equal(got, exp)
        bits = np.unpackbits(words.view(np.uint8), bitorder="little")
        assert np.array_equal(bits[:n], exp) and not bits[n:].any()


def test_empty_batch(gpu_ctx):
    v = gpu_ctx.verify(np.zeros((0, 32), np.uint8), np.zeros((0, 64), np.uint8), np.zeros(0, np.uint8),
                       np.zeros(1, np.uint32))
    assert v.shape == (0,)
