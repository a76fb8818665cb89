"""crypto.BatchVerifier mirror, PubKey.VerifySignature and large-batch
properties on the GPU.

Mirrors /root/reference/crypto/ed25519/ed25519_test.go:13-30
(TestSignAndValidateEd25519: sign, verify, flip one bit, reject)."""
import numpy as np
import pytest

from cometbft_amd import MODE_GO_STDLIB, MODE_ZIP215, BatchVerifier, PubKey, pack_messages
from cometbft_amd import parallel as P
from oracle import coracle
from oracle import ed25519_ref as E

pytestmark = pytest.mark.gpu


def test_sign_and_validate_ed25519(gpu_ctx):
    rng = np.random.default_rng(5)
    seed = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    msg = rng.integers(0, 256, 128, dtype=np.uint8).tobytes()
    pk = PubKey(E.pubkey_from_seed(seed))
    sig = bytearray(E.sign(seed, msg))
    assert pk.verify_signature(msg, bytes(sig), ctx=gpu_ctx)
    sig[7] ^= 0x01
    assert not pk.verify_signature(msg, bytes(sig), ctx=gpu_ctx)
    assert not pk.verify_signature(msg, bytes(sig[:63]), ctx=gpu_ctx)
    with pytest.raises(ValueError, match="bad public key length: 31"):
        PubKey(bytes(pk)[:31]).verify_signature(msg, E.sign(seed, msg), ctx=gpu_ctx)


@pytest.mark.parametrize("mode", [MODE_GO_STDLIB, MODE_ZIP215])
def test_batch_verifier_mixed(gpu_ctx, corpus, mode):
    bv = BatchVerifier(gpu_ctx, mode)
    idx = list(range(0, len(corpus["msgs"]), 3))
    for i in idx:
        bv.add(bytes(corpus["pk"][i]), corpus["msgs"][i], bytes(corpus["sig"][i]))
    # malformed entries are accepted by Add and come back invalid
    bv.add(bytes(corpus["pk"][0]), b"x", bytes(63))
    bv.add(bytes(31), b"x", bytes(64))
    ok, verdicts = bv.verify()
    key = "go" if mode == MODE_GO_STDLIB else "zip215"
    exp = [bool(corpus[key][i]) for i in idx] + [False, False]
    assert verdicts == exp and ok is False
    assert bv.bad_key_index == len(idx) + 1


def test_batch_verifier_all_valid_and_empty(gpu_ctx):
    bv = BatchVerifier(gpu_ctx)
    assert bv.verify() == (False, [])
    for i in range(10):
        seed = bytes([i]) * 32
        bv.add(E.pubkey_from_seed(seed), b"m%d" % i, E.sign(seed, b"m%d" % i))
    assert bv.verify() == (True, [True] * 10)
    bv.reset()
    assert len(bv) == 0


def test_large_batch_properties(gpu_ctx):
    """300k signatures over 512 keys (blocksync shape): every honest signature
    accepted, exactly the corrupted ones rejected; bitmap popcount matches;
    a random sample agrees with the oracle in both modes."""
    n, nk = 300_000, 512
    rng = np.random.default_rng(99)
    seeds = rng.integers(0, 256, (nk, 32), dtype=np.uint8)
    kidx = rng.integers(0, nk, n).astype(np.uint32)
    msgs = [b"h%07d-%s" % (i, b"x" * int(i % 97)) for i in range(n)]
    m, off = pack_messages(msgs)
    sig = gpu_ctx.sign(seeds, m, off, key_idx=kidx)
    pk = gpu_ctx.pubkeys(seeds)[kidx]
    bad = rng.random(n) < 0.01
    sig[bad, 33] ^= 0x04
    for mode in (MODE_GO_STDLIB, MODE_ZIP215):
        valid, words = gpu_ctx.verify(pk, sig, m, off, mode, bitmap=True)
        assert np.array_equal(valid == 0, bad)
        assert int(np.unpackbits(words.view(np.uint8)).sum()) == int((~bad).sum())
        sample = rng.choice(n, 2000, replace=False)
        sample.sort()
        sub_m = [msgs[i] for i in sample]
        sm, so = coracle.pack_msgs(sub_m)
        exp = coracle.verify_batch(pk[sample], sig[sample], sm, so, mode, nthreads=8)
        assert np.array_equal(valid[sample], exp)


@pytest.mark.parametrize("n", [4097, 12287, 12289, 20000, 39999])
def test_multi_round_quad_split_sizes(gpu_ctx, n):
    """The helper-wave quad kernel past one round (256 workgroups x 48) and at
    the oct / quad crossover: 1% corrupted, exactly those rejected, the bitmap
    tail clear, a sample against the oracle in both modes."""
    nk = 300
    rng = np.random.default_rng(n)
    seeds = rng.integers(0, 256, (nk, 32), dtype=np.uint8)
    kidx = rng.integers(0, nk, n).astype(np.uint32)
    msgs = [b"r%06d-%s" % (i, b"y" * int(i % 53)) for i in range(n)]
    m, off = pack_messages(msgs)
    sig = gpu_ctx.sign(seeds, m, off, key_idx=kidx)
    pk = gpu_ctx.pubkeys(seeds)[kidx]
    bad = rng.random(n) < 0.01
    sig[bad, 40] ^= 0x10
    for mode in (MODE_GO_STDLIB, MODE_ZIP215):
        valid, words = gpu_ctx.verify(pk, sig, m, off, mode, bitmap=True)
        assert np.array_equal(valid == 0, bad)
        bits = np.unpackbits(words.view(np.uint8), bitorder="little")
        assert np.array_equal(bits[:n], valid) and not bits[n:].any()
        sample = np.sort(rng.choice(n, 600, replace=False))
        sm, so = coracle.pack_msgs([msgs[i] for i in sample])
        exp = coracle.verify_batch(pk[sample], sig[sample], sm, so, mode, nthreads=8)
        assert np.array_equal(valid[sample], exp)


def test_verify_sharded_single_rank(gpu_ctx):
    n = 5000
    rng = np.random.default_rng(1)
    seeds = rng.integers(0, 256, (64, 32), dtype=np.uint8)
    kidx = (np.arange(n) % 64).astype(np.uint32)
    msgs = [b"commit-%d" % i for i in range(n)]
    m, off = pack_messages(msgs)
    sig = gpu_ctx.sign(seeds, m, off, key_idx=kidx)
    pk = gpu_ctx.pubkeys(seeds)[kidx]
    sig[17, 2] ^= 1
    words = P.verify_sharded(gpu_ctx, pk, sig, m, off, MODE_GO_STDLIB, world=1, rank=0)
    v = P.unpack_bitmap(words.cpu().numpy().view(np.uint64), n)
    assert v.sum() == n - 1 and v[17] == 0


@pytest.mark.parametrize("n", [49152, 49153])
def test_default_dispatch_at_the_quad_lane_crossover(gpu_ctx, n):
    """The default context on both sides of kQuadMax (49,152: four
    rounds of the helper-summed quad kernel; one more signature takes the lane
    kernel), Go mode, 1% flipped signatures, verdict bytes and bitmap against
    the oracle."""
    rng = np.random.default_rng(n)
    seeds = rng.integers(0, 256, (512, 32), dtype=np.uint8)
    kidx = (np.arange(n) % 512).astype(np.uint32)
    msgs = [rng.integers(0, 256, 120, dtype=np.uint8).tobytes() for _ in range(n)]
    m, off = coracle.pack_msgs(msgs)
    sig = coracle.sign_batch(seeds, m, off, key_idx=kidx, nthreads=8).copy()
    pk = coracle.pubkeys_from_seeds(seeds)[kidx]
    for i in np.nonzero(rng.random(n) < 0.01)[0]:
        sig[i, rng.integers(0, 64)] ^= 1 << rng.integers(0, 8)
    exp = coracle.verify_batch(pk, sig, m, off, MODE_GO_STDLIB, nthreads=8)
    got, words = gpu_ctx.verify(pk, sig, m, off, MODE_GO_STDLIB, bitmap=True)
    assert np.array_equal(got, exp)
    bits = np.unpackbits(words.view(np.uint8), bitorder="little")
    assert np.array_equal(bits[:n], exp) and not bits[n:].any()
