"""GPU parity at BASELINE.json's own sizes (the bench workloads, checked here
rather than only timed):

  configs[1]  one 10,000-validator commit: the raw batch (quad kernel, the
              default dispatch for n <= 49,152) and cmtv_verify_commit /
              VerifyCommitLight (templated sign-bytes + replay) with ~1% of
              the signatures bit-flipped, both verdict modes, against the C
              oracle's verdicts and a Python replay of the reference loop
              (types/validator_set.go:667-765).
  configs[2]  the replay shape at >= 1M signatures: 7,000 commits x 150
              validators through cmtv_register_keys +
              cmtv_verify_ed25519_indexed (the registered-key LANE kernel,
              the default dispatch above 36,864), 1% bit-flipped: exactly the
              flipped ones must be rejected, the packed bitmap must agree, and
              a 2,000-signature sample must match the C oracle in both modes.

Signatures are made by the device signer (k_sign, RFC 8032 deterministic);
each test first pins that signer against the C oracle's on a sample, so the
verdict checks are not a self-consistency loop.
"""
import numpy as np
import pytest

from oracle import coracle
from cometbft_amd import MODE_GO_STDLIB, MODE_ZIP215, pack_messages
from cometbft_amd import testutil as TU
from cometbft_amd import types as T

pytestmark = pytest.mark.gpu


def _err(fn):
    try:
        fn()
    except Exception as e:  # noqa: BLE001 -- the reference's returned error
        return e
    return None


def _replay_verify_commit(valid, powers, light):
    """types/validator_set.go:685-713 (full) / 740-764 (light) over per-index
    verdicts, all flags BlockIDFlagCommit: the first bad index, or None."""
    needed = int(powers.sum()) * 2 // 3
    tally = 0
    for i, ok in enumerate(valid):
        if not ok:
            return i
        tally += int(powers[i])
        if light and tally > needed:
            return None
    return None if tally > needed else -1


@pytest.mark.parametrize("mode", [MODE_GO_STDLIB, MODE_ZIP215])
def test_configs1_10k_validator_commit(gpu_ctx, mode):
    n, h = 10_000, 1000
    sv = TU.make_validator_set(gpu_ctx, n)
    commit, msgs, sigs = TU.make_commit(gpu_ctx, sv, h)
    m, off = pack_messages(msgs)
    rng = np.random.default_rng(10_000 + mode)
    # the device signer and keygen against the oracle's, on a sample
    samp = rng.choice(n, 400, replace=False)
    assert np.array_equal(coracle.pubkeys_from_seeds(sv.seeds[samp]), sv.pubkeys[samp])
    sm, soff = coracle.pack_msgs([msgs[i] for i in samp])
    assert np.array_equal(coracle.sign_batch(sv.seeds[samp], sm, soff, nthreads=8), sigs[samp])
    # ~1% flipped, the first one late in the commit (index > 2/3 n) so that
    # VerifyCommitLight's early exit is exercised too
    flip = np.sort(rng.choice(np.arange(7000, n), 100, replace=False))
    bits = rng.integers(0, 512, flip.size)
    bad = sigs.copy()
    bad[flip, bits // 8] ^= (1 << (bits % 8)).astype(np.uint8)
    exp = coracle.verify_batch(sv.pubkeys, bad, m, off, mode, nthreads=8)
    assert exp.sum() == n - flip.size
    got, words = gpu_ctx.verify(sv.pubkeys, bad, m, off, mode, bitmap=True)
    assert np.array_equal(got, exp), np.nonzero(got != exp)[0][:10]
    assert np.array_equal(np.unpackbits(words.view(np.uint8), bitorder="little")[:n], exp)
    # through the commit path
    for i in flip:
        commit.signatures[int(i)].signature = bytes(bad[i])
    bid = TU.block_id_for_height(h)
    powers = np.array([v.voting_power for v in sv.valset.validators])
    want_full = _replay_verify_commit(exp, powers, light=False)
    want_light = _replay_verify_commit(exp, powers, light=True)
    assert want_full == int(flip[0]) and want_light is None
    err = _err(lambda: sv.valset.verify_commit(TU.CHAIN_ID, bid, h, commit, ctx=gpu_ctx, mode=mode))
    assert isinstance(err, T.ErrWrongSignature) and err.index == want_full
    assert _err(lambda: sv.valset.verify_commit_light(TU.CHAIN_ID, bid, h, commit, ctx=gpu_ctx, mode=mode)) is None


def test_configs2_keyed_replay_1m(gpu_ctx):
    n_vals, heights = 150, 7000
    n = n_vals * heights
    sv = TU.make_validator_set(gpu_ctx, n_vals)
    m, off = TU.replay_messages(1, heights, n_vals)
    kidx = np.tile(np.arange(n_vals, dtype=np.uint32), heights)
    sig = gpu_ctx.sign(sv.seeds, m, off, kidx)
    rng = np.random.default_rng(2)
    samp = np.sort(rng.choice(n, 2000, replace=False))
    smsgs = [m[off[i]:off[i + 1]].tobytes() for i in samp]
    sm, soff = coracle.pack_msgs(smsgs)
    assert np.array_equal(coracle.sign_batch(sv.seeds, sm, soff, key_idx=kidx[samp], nthreads=8), sig[samp])
    flip = rng.choice(n, n // 100, replace=False)
    bits = rng.integers(0, 512, flip.size)
    sig[flip, bits // 8] ^= (1 << (bits % 8)).astype(np.uint8)
    exp = np.ones(n, np.uint8)
    exp[flip] = 0
    ks = gpu_ctx.register_keys(sv.pubkeys)
    try:
        for mode in (MODE_GO_STDLIB, MODE_ZIP215):
            got, words = gpu_ctx.verify_indexed(ks, kidx, sig, m, off, mode, bitmap=True)
            assert np.array_equal(got, exp), np.nonzero(got != exp)[0][:10]
            assert int(np.unpackbits(words.view(np.uint8)).sum()) == n - flip.size
            samp2 = np.concatenate([samp, flip[:200]])
            o = coracle.verify_batch(sv.pubkeys[kidx[samp2]], sig[samp2],
                                     *coracle.pack_msgs([m[off[i]:off[i + 1]].tobytes() for i in samp2]),
                                     mode, nthreads=8)
            assert np.array_equal(o, got[samp2])
    finally:
        ks.free()
