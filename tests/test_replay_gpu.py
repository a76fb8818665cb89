"""Replay paths on the GPU:

  * cross-height batching -- cmtv_verify_commits: many commits, one device
    batch, each commit's reference loop replayed over its verdicts. Parity:
    per commit, the outcome (nil / error type / error string / index) equals
    cmtv_verify_commit's, which tests/test_commit_gpu.py pins to
    types/validator_set_test.go;
  * the verdict cache -- cmtv_verdict_cache: blocksync's VerifyCommitLight +
    VerifyCommit + VerifyCommit over the same commit
    (blockchain/v0/reactor.go:366-400, state/validation.go:93,
    state/execution.go:135) gives the same outcomes with and without the
    cache, and the two VerifyCommit calls launch no kernel.
"""
import numpy as np
import pytest

from cometbft_amd import Context
from cometbft_amd import testutil as TU
from cometbft_amd import types as T

pytestmark = pytest.mark.gpu

N_VALS = 40


def _outcome(fn):
    try:
        fn()
        return None
    except Exception as e:  # noqa: BLE001 -- the reference returns errors as values
        return (type(e).__name__, str(e), getattr(e, "index", None))


def _as_outcome(err):
    return None if err is None else (type(err).__name__, str(err), getattr(err, "index", None))


@pytest.fixture(scope="module")
def chain(gpu_ctx):
    """12 heights over one 40-validator set with assorted faults."""
    sv = TU.make_validator_set(gpu_ctx, N_VALS)
    items = []
    for h in range(100, 112):
        flags = [T.BLOCK_ID_FLAG_COMMIT] * N_VALS
        if h == 103:
            flags = [T.BLOCK_ID_FLAG_NIL if i % 3 == 0 else T.BLOCK_ID_FLAG_COMMIT for i in range(N_VALS)]
        if h == 104:
            flags = [T.BLOCK_ID_FLAG_ABSENT if i < 20 else T.BLOCK_ID_FLAG_COMMIT for i in range(N_VALS)]
        commit, _, _ = TU.make_commit(gpu_ctx, sv, h, flags=flags)
        if h == 105:  # a bad signature early: every kind fails on it
            s = bytearray(commit.signatures[2].signature)
            s[10] ^= 1
            commit.signatures[2].signature = bytes(s)
        if h == 106:  # a bad signature late: only VerifyCommit reaches it
            s = bytearray(commit.signatures[N_VALS - 1].signature)
            s[40] ^= 4
            commit.signatures[N_VALS - 1].signature = bytes(s)
        height = h + 1 if h == 107 else h  # wrong height
        bid = TU.block_id_for_height(h + 1000) if h == 108 else TU.block_id_for_height(h)  # wrong block ID
        items.append((sv.valset, bid, height, commit))
    return items


@pytest.mark.parametrize("kind", [0, 1, 2])
def test_cross_height_batch_equals_per_commit(gpu_ctx, chain, kind):
    per = []
    for vals, bid, height, commit in chain:
        if kind == 0:
            per.append(_outcome(lambda: vals.verify_commit(TU.CHAIN_ID, bid, height, commit, ctx=gpu_ctx)))
        elif kind == 1:
            per.append(_outcome(lambda: vals.verify_commit_light(TU.CHAIN_ID, bid, height, commit, ctx=gpu_ctx)))
        else:
            per.append(_outcome(lambda: vals.verify_commit_light_trusting(TU.CHAIN_ID, commit, ctx=gpu_ctx)))
    items = [(v, b if kind != 2 else None, h, c) for v, b, h, c in chain]
    got = [_as_outcome(e) for e in T.verify_commits(kind, TU.CHAIN_ID, items, ctx=gpu_ctx)]
    assert got == per
    # trusting ignores height / block ID, so only the early bad signature fails it
    assert sum(o is None for o in got) >= 5 and sum(o is not None for o in got) >= (1 if kind == 2 else 3)


def test_cross_height_batch_is_one_launch(gpu_ctx, chain):
    before = gpu_ctx.stats()
    T.verify_commits(0, TU.CHAIN_ID, chain, ctx=gpu_ctx)
    after = gpu_ctx.stats()
    assert after["calls"] - before["calls"] == 1


def _blocksync(ctx, chain):
    out = []
    for vals, bid, height, commit in chain:
        out.append(_outcome(lambda: vals.verify_commit_light(TU.CHAIN_ID, bid, height, commit, ctx=ctx)))
        out.append(_outcome(lambda: vals.verify_commit(TU.CHAIN_ID, bid, height, commit, ctx=ctx)))
        out.append(_outcome(lambda: vals.verify_commit(TU.CHAIN_ID, bid, height, commit, ctx=ctx)))
    return out


def test_verdict_cache_blocksync_pattern(chain):
    plain = Context(device=0)
    cached = Context(device=0)
    cached.verdict_cache(100_000)
    ref = _blocksync(plain, chain)
    before = cached.stats()
    got = _blocksync(cached, chain)
    after = cached.stats()
    assert got == ref
    # one device call per height (the light call, prefetching the rest); the
    # two VerifyCommit calls are served from the cache
    assert after["calls"] - before["calls"] <= len(chain)
    assert after["cache_hits"] - before["cache_hits"] > 0
    # a second pass is all hits
    calls = after["calls"]
    assert _blocksync(cached, chain) == ref
    assert cached.stats()["calls"] == calls


def test_verdict_cache_matches_full_key(gpu_ctx):
    """A cached verdict is only reused for identical (key, signature,
    message): the same signature under another message is verified again."""
    ctx = Context(device=0)
    ctx.verdict_cache(1000)
    sv = TU.make_validator_set(gpu_ctx, 8)
    msgs = TU.commit_messages(8, 500)
    from cometbft_amd import pack_messages

    m, off = pack_messages(msgs)
    sig = ctx.sign(sv.seeds, m, off)
    assert ctx.verify(sv.pubkeys, sig, m, off).all()
    msgs2 = [x[:-1] + bytes([x[-1] ^ 1]) for x in msgs]
    m2, off2 = pack_messages(msgs2)
    assert not ctx.verify(sv.pubkeys, sig, m2, off2).any()
    assert ctx.verify(sv.pubkeys, sig, m, off).all()
    assert ctx.verify(sv.pubkeys, sig, m, off, mode=1).all()  # mode is part of the key


def test_verdict_cache_eviction(chain):
    """A cache far smaller than the working set still gives exact outcomes."""
    plain = Context(device=0)
    tiny = Context(device=0)
    tiny.verdict_cache(7)
    assert _blocksync(tiny, chain) == _blocksync(plain, chain)
    assert tiny.stats()["cache_entries"] == 7


@pytest.mark.parametrize("kind", [0, 1, 2])
def test_keyset_cache_matches_plain(chain, kind):
    """cmtv_keyset_cache: commits of a registered validator set are verified
    by key index (keyed_quad.h / keyed.h) with outcomes identical to the
    generic path's, for single and cross-height calls."""
    plain = Context(device=0)
    keyed = Context(device=0)
    keyed.keyset_cache(4)

    def run(ctx):
        out = []
        for vals, bid, height, commit in chain:
            if kind == 0:
                out.append(_outcome(lambda: vals.verify_commit(TU.CHAIN_ID, bid, height, commit, ctx=ctx)))
            elif kind == 1:
                out.append(_outcome(lambda: vals.verify_commit_light(TU.CHAIN_ID, bid, height, commit, ctx=ctx)))
            else:
                out.append(_outcome(lambda: vals.verify_commit_light_trusting(TU.CHAIN_ID, commit, ctx=ctx)))
        items = [(v, b if kind != 2 else None, h, c) for v, b, h, c in chain]
        out += [_as_outcome(e) for e in T.verify_commits(kind, TU.CHAIN_ID, items, ctx=ctx)]
        return out

    assert run(keyed) == run(plain)


def test_keyset_cache_bad_key_in_set(gpu_ctx):
    """A validator set holding an undecodable key: that validator's signature
    is invalid on the keyed path exactly as on the generic one."""
    sv = TU.make_validator_set(gpu_ctx, 6)
    commit, _, _ = TU.make_commit(gpu_ctx, sv, 77)
    vals = sv.valset
    bad = T.ValidatorSet([T.Validator(v.pub_key, v.voting_power) for v in vals.validators])
    # y = 2 has no square root on edwards25519: the key does not decode
    bad.validators[3] = T.Validator((2).to_bytes(32, "little"), bad.validators[3].voting_power)
    plain = Context(device=0)
    keyed = Context(device=0)
    keyed.keyset_cache(2)
    bid = TU.block_id_for_height(77)
    a = _outcome(lambda: bad.verify_commit(TU.CHAIN_ID, bid, 77, commit, ctx=plain))
    b = _outcome(lambda: bad.verify_commit(TU.CHAIN_ID, bid, 77, commit, ctx=keyed))
    assert a == b and a is not None and a[0] == "ErrWrongSignature"
