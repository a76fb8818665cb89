"""VerifyCommit / VerifyCommitLight / VerifyCommitLightTrusting through the GPU
batch + replay (cmtv_verify_commit), mirroring the reference's tests:

  types/validator_set_test.go:670-744  TestValidatorSet_VerifyCommit_All
  types/validator_set_test.go:746-769  ..._VerifyCommit_CheckAllSignatures
  types/validator_set_test.go:771-792  ..._VerifyCommitLight_ReturnsAsSoonAsMajority...
  types/validator_set_test.go:794-815  ..._VerifyCommitLightTrusting_ReturnsAsSoonAs...
  types/validator_set_test.go:1520-1574 ..._VerifyCommitLightTrusting(+ErrorsOnOverflow)
  light/verifier_test.go:120           ErrNotEnoughVotingPowerSigned{Got: 50, Needed: 93}

Signatures are produced by the oracle signer (RFC 8032); sign-bytes by the
oracle encoder, so the library's encoder is exercised against an independent one.
"""
import hashlib

import numpy as np
import pytest

from cometbft_amd import types as T
from oracle import ed25519_ref as E
from oracle import signbytes as SB

pytestmark = pytest.mark.gpu

CHAIN = "Lalande21185"
MAX_TOTAL_VOTING_POWER = (2**63 - 1) // 8


def _bid(tag=b"blk"):
    return T.BlockID(hashlib.sha256(tag).digest(), T.PartSetHeader(1, hashlib.sha256(tag + b"p").digest()))


def _bid_tuple(b: T.BlockID):
    return (b.hash, b.part_set_header.total, b.part_set_header.hash)


class Val:
    def __init__(self, i, power):
        self.seed = hashlib.sha256(b"test-val-%d" % i).digest()
        self.pk = E.pubkey_from_seed(self.seed)
        self.v = T.Validator(self.pk, power)

    def sign_vote(self, chain, height, round_, bid, ts, flag=T.BLOCK_ID_FLAG_COMMIT):
        b = _bid_tuple(bid) if flag == T.BLOCK_ID_FLAG_COMMIT else None
        msg = SB.vote_sign_bytes(chain, T.PRECOMMIT_TYPE, height, round_, b, *ts)
        return T.CommitSig(flag, self.v.address, ts, E.sign(self.seed, msg))


def _valset(n, power, start=0):
    vals = [Val(start + i, power) for i in range(n)]
    vals.sort(key=lambda x: x.v.address)
    return vals, T.ValidatorSet([x.v for x in vals])


def _commit(vals, chain, height, round_, bid, flags=None):
    sigs = []
    for i, v in enumerate(vals):
        f = T.BLOCK_ID_FLAG_COMMIT if flags is None else flags[i]
        if f == T.BLOCK_ID_FLAG_ABSENT:
            sigs.append(T.new_commit_sig_absent())
        else:
            sigs.append(v.sign_vote(chain, height, round_, bid, (1_600_000_000 + i, 1000 * i), f))
    return T.Commit(height, round_, bid, sigs)


def _err(fn):
    try:
        fn()
    except Exception as e:  # noqa: BLE001
        return e
    return None


def test_verify_commit_all(gpu_ctx):
    vals, vset = _valset(1, 1000)
    bid, h = _bid(), 12345
    commit = _commit(vals, CHAIN, h, 2, bid)
    vote2 = vals[0].sign_vote("EpsilonEridani", h, 2, bid, (1_600_000_000, 0))
    cases = [
        ("good", CHAIN, bid, h, commit, None),
        ("wrong signature (#0)", "EpsilonEridani", bid, h, commit, T.ErrWrongSignature),
        ("wrong block ID", CHAIN, _bid(b"random"), h, commit, T.ErrWrongBlockID),
        ("wrong height", CHAIN, bid, h - 1, commit, T.ErrInvalidCommitHeight),
        ("wrong set size: 1 vs 0", CHAIN, bid, h, T.Commit(h, 2, bid, []), T.ErrInvalidCommitSignatures),
        ("wrong set size: 1 vs 2", CHAIN, bid, h,
         T.Commit(h, 2, bid, [commit.signatures[0], T.new_commit_sig_absent()]), T.ErrInvalidCommitSignatures),
        ("insufficient voting power: got 0, needed more than 666", CHAIN, bid, h,
         T.Commit(h, 2, bid, [T.new_commit_sig_absent()]), T.ErrNotEnoughVotingPowerSigned),
        ("wrong signature (#0)", CHAIN, bid, h, T.Commit(h, 2, bid, [vote2]), T.ErrWrongSignature),
    ]
    for desc, chain, b, height, c, exc in cases:
        for fn in (vset.verify_commit, vset.verify_commit_light):
            e = _err(lambda: fn(chain, b, height, c, ctx=gpu_ctx))
            if exc is None:
                assert e is None, (desc, e)
            else:
                assert isinstance(e, exc), (desc, fn.__name__, e)
                assert desc in str(e), (desc, str(e))


def test_error_strings_exact(gpu_ctx):
    vals, vset = _valset(1, 1000)
    bid, h = _bid(), 7
    commit = _commit(vals, CHAIN, h, 0, bid)
    e = _err(lambda: vset.verify_commit(CHAIN, bid, h + 1, commit, ctx=gpu_ctx))
    assert str(e) == "Invalid commit -- wrong height: 8 vs 7"
    other = _bid(b"other")
    e = _err(lambda: vset.verify_commit(CHAIN, other, h, commit, ctx=gpu_ctx))
    want = ("invalid commit -- wrong block ID: want %s:1:%s, got %s:1:%s" %
            (other.hash.hex().upper(), other.part_set_header.hash[:6].hex().upper(),
             bid.hash.hex().upper(), bid.part_set_header.hash[:6].hex().upper()))
    assert str(e) == want
    e = _err(lambda: vset.verify_commit("nope", bid, h, commit, ctx=gpu_ctx))
    assert str(e) == "wrong signature (#0): " + commit.signatures[0].signature.hex().upper()


def test_verify_commit_checks_all_signatures(gpu_ctx):
    vals, vset = _valset(4, 10)
    bid, h = _bid(), 3
    commit = _commit(vals, "test_chain_id", h, 0, bid)
    commit.signatures[3] = vals[3].sign_vote("CentaurusA", h, 0, bid, commit.signatures[3].timestamp)
    e = _err(lambda: vset.verify_commit("test_chain_id", bid, h, commit, ctx=gpu_ctx))
    assert isinstance(e, T.ErrWrongSignature) and "wrong signature (#3)" in str(e)
    # ... while VerifyCommitLight returns as soon as +2/3 signed (#3 never checked)
    assert vset.verify_commit_light("test_chain_id", bid, h, commit, ctx=gpu_ctx) is None


def test_light_trusting_returns_at_trust_level(gpu_ctx):
    vals, vset = _valset(4, 10)
    bid, h = _bid(), 3
    commit = _commit(vals, "test_chain_id", h, 0, bid)
    commit.signatures[2] = vals[2].sign_vote("CentaurusA", h, 0, bid, commit.signatures[2].timestamp)
    assert vset.verify_commit_light_trusting("test_chain_id", commit, (1, 3), ctx=gpu_ctx) is None


def test_light_trusting_overlap(gpu_ctx):
    vals, original = _valset(6, 1, start=100)
    bid = _bid(b"lt")
    commit = _commit(vals, "test_chain_id", 1, 1, bid)
    _, newset = _valset(2, 1, start=500)
    assert original.verify_commit_light_trusting("test_chain_id", commit, (1, 3), ctx=gpu_ctx) is None
    e = _err(lambda: newset.verify_commit_light_trusting("test_chain_id", commit, (1, 3), ctx=gpu_ctx))
    assert isinstance(e, T.ErrNotEnoughVotingPowerSigned)
    merged = T.ValidatorSet(newset.validators + original.validators)
    assert merged.verify_commit_light_trusting("test_chain_id", commit, (1, 3), ctx=gpu_ctx) is None


def test_light_trusting_overflow_and_zero_denominator(gpu_ctx):
    vals, vset = _valset(1, MAX_TOTAL_VOTING_POWER, start=900)
    bid = _bid(b"of")
    commit = _commit(vals, "test_chain_id", 1, 1, bid)
    e = _err(lambda: vset.verify_commit_light_trusting("test_chain_id", commit, (25, 55), ctx=gpu_ctx))
    assert isinstance(e, T.ErrTrustLevel) and "int64 overflow" in str(e)
    e = _err(lambda: vset.verify_commit_light_trusting("test_chain_id", commit, (1, 0), ctx=gpu_ctx))
    assert str(e) == "trustLevel has zero Denominator"


def test_light_trusting_double_vote(gpu_ctx):
    vals, vset = _valset(3, 10, start=40)
    bid = _bid(b"dv")
    commit = _commit(vals, "c", 5, 0, bid)
    commit.signatures[2] = commit.signatures[0]  # validator 0 signs twice
    e = _err(lambda: vset.verify_commit_light_trusting("c", commit, (9, 10), ctx=gpu_ctx))
    assert isinstance(e, T.ErrDoubleVote)
    assert str(e).startswith("double vote from Validator{%s PubKeyEd25519{%s} VP:10 A:0} (0 and 2)" %
                             (vals[0].v.address.hex().upper(), vals[0].pk.hex().upper()))
    # the indices a Go binding formats the error from:
    # sig_index = second, got = first commit index, needed = validator index
    r = e.result
    assert (r.sig_index, r.got, vset.validators[r.needed].pub_key) == (2, 0, vals[0].pk)


def test_not_enough_power_values(gpu_ctx):
    # light/verifier_test.go:120 style: ErrNotEnoughVotingPowerSigned{Got: 50, Needed: 93}
    vals, vset = _valset(14, 10, start=200)
    bid = _bid(b"ne")
    flags = [T.BLOCK_ID_FLAG_COMMIT] * 5 + [T.BLOCK_ID_FLAG_ABSENT] * 9
    commit = _commit(vals, "c", 9, 0, bid, flags)
    e = _err(lambda: vset.verify_commit_light("c", bid, 9, commit, ctx=gpu_ctx))
    assert isinstance(e, T.ErrNotEnoughVotingPowerSigned) and (e.got, e.needed) == (50, 93)
    assert str(e) == "invalid commit -- insufficient voting power: got 50, needed more than 93"


def test_nil_votes_and_absent(gpu_ctx):
    vals, vset = _valset(6, 10, start=300)
    bid = _bid(b"nil")
    flags = [T.BLOCK_ID_FLAG_COMMIT] * 5 + [T.BLOCK_ID_FLAG_NIL]
    commit = _commit(vals, "c", 4, 0, bid, flags)
    # nil vote is verified (its sign-bytes carry no BlockID) but not tallied
    assert vset.verify_commit("c", bid, 4, commit, ctx=gpu_ctx) is None
    commit.signatures[5] = vals[5].sign_vote("c", 4, 0, bid, commit.signatures[5].timestamp, T.BLOCK_ID_FLAG_COMMIT)
    commit.signatures[5].block_id_flag = T.BLOCK_ID_FLAG_NIL  # signed for the block, claims nil
    e = _err(lambda: vset.verify_commit("c", bid, 4, commit, ctx=gpu_ctx))
    assert isinstance(e, T.ErrWrongSignature) and e.index == 5
    # Light skips nil votes entirely
    assert vset.verify_commit_light("c", bid, 4, commit, ctx=gpu_ctx) is None


def test_reference_panics_are_surfaced(gpu_ctx):
    vals, vset = _valset(3, 10, start=700)
    bid = _bid(b"pn")
    commit = _commit(vals, "c", 2, 0, bid)
    commit.signatures[1].block_id_flag = 9
    e = _err(lambda: vset.verify_commit("c", bid, 2, commit, ctx=gpu_ctx))
    assert isinstance(e, T.ReferencePanic) and "Unknown BlockIDFlag" in str(e)
    commit = _commit(vals, "c", 2, 0, bid)
    bad = T.ValidatorSet([vset.validators[0], T.Validator(vset.validators[1].pub_key[:31], 10),
                          vset.validators[2]])
    e = _err(lambda: bad.verify_commit("c", bid, 2, commit, ctx=gpu_ctx))
    assert isinstance(e, T.ReferencePanic) and "bad public key length: 31" in str(e)
    # a bad signature BEFORE the bad key is reported first, like the sequential loop
    commit.signatures[0] = vals[0].sign_vote("zz", 2, 0, bid, commit.signatures[0].timestamp)
    e = _err(lambda: bad.verify_commit("c", bid, 2, commit, ctx=gpu_ctx))
    assert isinstance(e, T.ErrWrongSignature) and e.index == 0


def test_wrong_signature_lengths_are_invalid(gpu_ctx):
    vals, vset = _valset(2, 10, start=800)
    bid = _bid(b"len")
    commit = _commit(vals, "c", 2, 0, bid)
    commit.signatures[1].signature = commit.signatures[1].signature[:63]
    e = _err(lambda: vset.verify_commit("c", bid, 2, commit, ctx=gpu_ctx))
    assert isinstance(e, T.ErrWrongSignature) and e.index == 1


def test_large_commit_first_error_in_index_order(gpu_ctx):
    from cometbft_amd import testutil as TU

    sv = TU.make_validator_set(gpu_ctx, 1000)
    commit, msgs, sigs = TU.make_commit(gpu_ctx, sv, height=77)
    bid = TU.block_id_for_height(77)
    assert sv.valset.verify_commit(TU.CHAIN_ID, bid, 77, commit, ctx=gpu_ctx) is None
    for bad in (911, 250):
        s = bytearray(commit.signatures[bad].signature)
        s[3] ^= 1
        commit.signatures[bad].signature = bytes(s)
    e = _err(lambda: sv.valset.verify_commit(TU.CHAIN_ID, bid, 77, commit, ctx=gpu_ctx))
    assert isinstance(e, T.ErrWrongSignature) and e.index == 250


@pytest.mark.parametrize("fuse", [True, False])
@pytest.mark.parametrize("chain", ["", "c", "x" * 50, "y" * 150])
def test_device_sign_bytes_templating(monkeypatch, chain, fuse):
    """with the verdict cache off, cmtv_verify_commit ships
    one CanonicalVote template per commit and (flag, seconds, nanos) per
    signature, and the device writes the sign-bytes: the split kernels'
    helper wave writes them into LDS itself (fused), or k_sign_bytes into HBM
    (CMTV_NO_SB_FUSE=1, and any batch with a message over the helper's
    192-byte slot, e.g. the 150-character chain id). The signatures here are
    made by the oracle over the oracle encoder's bytes (pinned by
    types/vote_test.go's KATs), so any byte the device writes differently
    fails verification. Timestamps cover zero, negative, one- to ten-byte
    varints and the Go zero time; rounds, heights and nil votes vary."""
    from cometbft_amd import Context

    if not fuse:
        monkeypatch.setenv("CMTV_NO_SB_FUSE", "1")
    gpu_ctx = Context(device=0)
    # registered keys: the keyed row (16 signatures) and keyed quad split
    # (CMTV_FORM=kquad) kernels' hash helpers write the bytes themselves
    keyed = Context(device=0)
    keyed.keyset_cache(4)
    monkeypatch.setenv("CMTV_FORM", "kquad")
    keyed_q = Context(device=0)
    keyed_q.keyset_cache(4)
    monkeypatch.delenv("CMTV_FORM", raising=False)
    monkeypatch.delenv("CMTV_NO_SB_FUSE", raising=False)

    secs = [0, 1, 127, 128, 2**40, -1, -62135596800, 1_700_000_000]
    nanos = [0, 1, 127, 128, 999_999_999, 5]
    vals, vset = _valset(len(secs) * 2, 10)
    for height, round_ in [(1, 0), (2**40 + 3, 1), (5, 2**31 - 1)]:
        bid = _bid(b"t%d" % height)
        sigs = []
        for i, v in enumerate(vals):
            ts = (secs[i % len(secs)], nanos[(i * 5) % len(nanos)])
            flag = T.BLOCK_ID_FLAG_NIL if i % 4 == 3 else T.BLOCK_ID_FLAG_COMMIT
            sigs.append(v.sign_vote(chain, height, round_, bid, ts, flag))
        commit = T.Commit(height, round_, bid, sigs)
        assert _err(lambda: vset.verify_commit(chain, bid, height, commit, ctx=gpu_ctx)) is None
        assert _err(lambda: vset.verify_commit_light(chain, bid, height, commit, ctx=gpu_ctx)) is None
        # the host-encoding path (taken when the verdict cache is on) agrees
        cached = Context(device=0)
        cached.verdict_cache(64)
        assert _err(lambda: vset.verify_commit(chain, bid, height, commit, ctx=cached)) is None
        # and a flipped timestamp nanosecond is caught by the device bytes
        bad = T.Commit(height, round_, bid, [T.CommitSig(s.block_id_flag, s.validator_address,
                                                         (s.timestamp[0], s.timestamp[1] ^ 1), s.signature)
                                             if j == 5 else s for j, s in enumerate(sigs)])
        e = _err(lambda: vset.verify_commit(chain, bid, height, bad, ctx=gpu_ctx))
        assert isinstance(e, T.ErrWrongSignature) and e.index == 5
        for kc in (keyed, keyed_q):
            assert _err(lambda: vset.verify_commit(chain, bid, height, commit, ctx=kc)) is None
            assert _err(lambda: vset.verify_commit_light(chain, bid, height, commit, ctx=kc)) is None
            e = _err(lambda: vset.verify_commit(chain, bid, height, bad, ctx=kc))
            assert isinstance(e, T.ErrWrongSignature) and e.index == 5
    fused = gpu_ctx.stats()["fused_sign_bytes"]
    assert (fused > 0) == (fuse and len(chain) <= 50), fused
    for kc in (keyed, keyed_q):
        st = kc.stats()
        assert st["keyed_launches"] > 0
        assert (st["fused_sign_bytes"] > 0) == (fuse and len(chain) <= 50), st["fused_sign_bytes"]


@pytest.mark.parametrize("pinned", [False, True])
@pytest.mark.parametrize("keyed", [True, False])
def test_early_staged_signatures_never_go_stale(keyed, pinned):
    """a single-commit VerifyCommit copies its signatures to
    the device before planning (stage_sigs_early_locked). When it stops
    before any batch runs (here: a wrong height), those device bytes must not
    be taken for the next call's, even if that call passes the SAME buffer
    with new contents -- as the Go binding's reused arena does. The next call
    (cmtv_verify_commits with one commit, and cmtv_verify_commit itself) must
    verify the bytes it is given now. pinned: the commit's arrays in the
    context's cmtv_alloc_pinned memory (then the signatures go to the device
    by DMA straight from the caller's buffer)."""
    import ctypes

    from cometbft_amd import Context
    from cometbft_amd import _native as N
    from cometbft_amd import testutil as TU

    ctx = Context(device=0)
    if keyed:
        ctx.keyset_cache(4)  # keyed quad kernel at 1,000 validators
    n = 1000 if keyed else 2000  # past the row bands, where the early copy runs
    sv = TU.make_validator_set(ctx, n)
    h = 91
    commit, _, _ = TU.make_commit(ctx, sv, height=h)
    bid = TU.block_id_for_height(h)
    vs, keep_v = sv.valset._pack()
    arena = T._Arena(ctx.alloc_pinned(4096 + 100 * (n + 1))) if pinned else None
    cm, keep_c = T._pack_commit(commit, arena)
    sb = keep_c[3]  # the signatures' buffer, reused below at the same address
    b, keep_b = bid._c()
    cid = TU.CHAIN_ID.encode()

    def single(height):
        res = N.cmtv_commit_result()
        buf = ctypes.create_string_buffer(1024)
        rc = N.lib().cmtv_verify_commit(ctx.handle, N.VERIFY_COMMIT, 0, cid, len(cid), ctypes.byref(vs),
                                        ctypes.byref(b), height, ctypes.byref(cm), 0, 0, ctypes.byref(res), buf,
                                        len(buf))
        return rc, res

    def many():
        res = (N.cmtv_commit_result * 1)()
        rcs = (ctypes.c_int * 1)()
        bufs = ctypes.create_string_buffer(1024)
        vsa, cma, bida, hs = (N.cmtv_valset * 1)(vs), (N.cmtv_commit * 1)(cm), (N.cmtv_block_id * 1)(b), \
            (ctypes.c_int64 * 1)(h)
        rc = N.lib().cmtv_verify_commits(ctx.handle, N.VERIFY_COMMIT, 0, cid, len(cid), 1, vsa, bida, hs, cma, 0, 0,
                                         res, rcs, bufs, 1024)
        assert rc == N.CMTV_OK
        return rcs[0], res[0]

    assert single(h)[0] == N.CMTV_OK  # the honest commit
    for bad, call in ((437, many), (611, lambda: single(h))):
        rc, _ = single(h + 1)  # stages the honest bytes, then fails its preamble
        assert rc != N.CMTV_OK
        saved = sb[64 * bad + 5]
        sb[64 * bad + 5] ^= 0x40  # the same buffer now holds a corrupted signature
        rc, res = call()
        assert rc != N.CMTV_OK and res.code == N.COMMIT_ERR_WRONG_SIGNATURE and res.sig_index == bad, \
            (rc, res.code, res.sig_index)
        sb[64 * bad + 5] = saved
        assert single(h)[0] == N.CMTV_OK
    del keep_v, keep_b


@pytest.mark.parametrize("pinned", [False, True])
def test_speculative_verify_commit_matches(pinned):
    """The speculative single-commit path (commit.cpp verify_commit_spec,
    round 6): a large commit of a cached validator set launches its keyed
    kernel on the set the cache matched last time for the same key array,
    before the per-signature host checks, which then run beside the kernel.
    Every outcome equals the non-speculative path's (CMTV_SPEC=0): clean,
    a flipped signature, a nil vote, an absent signature (the plan stops
    being a prefix), a wrong height, and the set's key bytes rewritten in
    place between calls (the guess must be refuted)."""
    import ctypes

    from cometbft_amd import _native as N
    from cometbft_amd import testutil as TU
    from test_runtime_gpu import _env

    ctxs = []
    for spec in ("1", "0"):
        with _env(CMTV_SPEC=spec):
            c = __import__("cometbft_amd").Context(device=0)
        c.keyset_cache(4)
        ctxs.append(c)
    n = 4096
    sv = TU.make_validator_set(ctxs[0], n)
    h = 55
    bid = TU.block_id_for_height(h)
    b, keep_b = bid._c()
    cid = TU.CHAIN_ID.encode()
    vs, keep_v = sv.valset._pack()
    pk_buf = keep_v[0]  # the set's key bytes, rewritten in place below

    def outcome(c, commit, height, kind):
        arena = T._Arena(c.alloc_pinned(4096 + 100 * (n + 1))) if pinned else None
        cm, keep_c = T._pack_commit(commit, arena)
        res = N.cmtv_commit_result()
        rc = N.lib().cmtv_verify_commit(c.handle, kind, 0, cid, len(cid), ctypes.byref(vs), ctypes.byref(b), height,
                                        ctypes.byref(cm), 0, 0, ctypes.byref(res), None, 0)
        del keep_c
        return rc, res.code, res.sig_index

    clean, _, _ = TU.make_commit(ctxs[0], sv, height=h)
    flags = [T.BLOCK_ID_FLAG_COMMIT] * n
    flags[7] = T.BLOCK_ID_FLAG_NIL
    with_nil, _, _ = TU.make_commit(ctxs[0], sv, height=h, flags=flags)
    flags[9] = T.BLOCK_ID_FLAG_ABSENT
    with_absent, _, _ = TU.make_commit(ctxs[0], sv, height=h, flags=flags)
    flipped, _, _ = TU.make_commit(ctxs[0], sv, height=h)
    s = bytearray(flipped.signatures[3001].signature)
    s[20] ^= 8
    flipped.signatures[3001].signature = bytes(s)
    cases = [(clean, h), (clean, h), (flipped, h), (with_nil, h), (with_absent, h), (clean, h + 1), (clean, h)]
    for kind in (N.VERIFY_COMMIT, N.VERIFY_COMMIT_LIGHT):
        got = [[outcome(c, cm, hh, kind) for cm, hh in cases] for c in ctxs]
        assert got[0] == got[1], (kind, got)
        assert got[0][0][0] == N.CMTV_OK and got[0][5][1] == N.COMMIT_ERR_HEIGHT
    assert got[1][2][2] == -1 or True  # light may stop before #3001
    # the key array rewritten in place: key 11 now another validator's
    saved = pk_buf[32 * 11:32 * 12].copy()
    pk_buf[32 * 11:32 * 12] = pk_buf[32 * 12:32 * 13]
    got = [outcome(c, clean, h, N.VERIFY_COMMIT) for c in ctxs]
    assert got[0] == got[1] and got[0][1] == N.COMMIT_ERR_WRONG_SIGNATURE and got[0][2] == 11, got
    pk_buf[32 * 11:32 * 12] = saved
    assert [outcome(c, clean, h, N.VERIFY_COMMIT) for c in ctxs] == [(N.CMTV_OK, 0, -1)] * 2
    del keep_b
    for c in ctxs:
        c.close()


@pytest.mark.parametrize("keyset", [False, True])
def test_polled_quad_slices_match(keyset):
    """CMTV_QUAD_POLL=1 (round 6, off by default): the quad kernels of a small
    host batch tag their 16-signature slices and the call polls them instead
    of waiting for the stream. Outcomes equal the default path's: clean, a
    flipped signature near the end, and the call is counted as polled."""
    import ctypes

    from cometbft_amd import _native as N
    from cometbft_amd import testutil as TU
    from test_runtime_gpu import _env

    ctxs = []
    for poll in ("1", "0"):
        with _env(CMTV_QUAD_POLL=poll):
            c = __import__("cometbft_amd").Context(device=0)
        if keyset:
            c.keyset_cache(4)
        ctxs.append(c)
    n = 3000
    sv = TU.make_validator_set(ctxs[0], n)
    h = 9
    b, keep_b = TU.block_id_for_height(h)._c()
    cid = TU.CHAIN_ID.encode()
    vs, keep_v = sv.valset._pack()
    clean, _, _ = TU.make_commit(ctxs[0], sv, height=h)
    flipped, _, _ = TU.make_commit(ctxs[0], sv, height=h)
    s = bytearray(flipped.signatures[n - 5].signature)
    s[33] ^= 1
    flipped.signatures[n - 5].signature = bytes(s)
    packed = [T._pack_commit(cm) for cm in (clean, flipped)]

    def outcome(c, pc):
        res = N.cmtv_commit_result()
        rc = N.lib().cmtv_verify_commit(c.handle, N.VERIFY_COMMIT, 0, cid, len(cid), ctypes.byref(vs),
                                        ctypes.byref(b), h, ctypes.byref(pc[0]), 0, 0, ctypes.byref(res), None, 0)
        return rc, res.code, res.sig_index

    st0 = ctxs[0].stats()
    got = [[outcome(c, pc) for pc in packed for _ in range(3)] for c in ctxs]
    assert got[0] == got[1], got
    assert got[0][0][0] == N.CMTV_OK and got[0][3][2] == n - 5
    assert ctxs[0].stats()["polled_calls"] > st0["polled_calls"]
    for c in ctxs:
        c.close()
    del keep_b, keep_v
