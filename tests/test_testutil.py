"""Synthetic-workload generators (cometbft_amd/testutil.py) used by bench.py:
the vectorised configs[2] sign-bytes generator must reproduce the library's
CanonicalVote encoder (pinned by the types/vote_test.go KATs in test_abi.py)
byte for byte."""
import numpy as np
import pytest

from cometbft_amd import pack_messages
from cometbft_amd import testutil as TU


@pytest.mark.parametrize("h0,nh,nv", [(1, 3, 150), (99_998, 3, 150), (4095, 2, 7), (1000, 1, 1), (12_500, 5, 64)])
def test_replay_messages_match_encoder(h0, nh, nv):
    m, off = TU.replay_messages(h0, nh, nv, chunk=2)
    msgs = []
    for h in range(h0, h0 + nh):
        msgs += TU.commit_messages(nv, h)
    want_m, want_off = pack_messages(msgs)
    assert off.dtype == np.uint32 and off.shape == (nh * nv + 1,)
    assert np.array_equal(off, want_off.astype(np.uint32))
    assert np.array_equal(m, want_m)


class _FakeSigner:
    """ReplayChain's only device call is ctx.sign: a deterministic stand-in
    (the packing, not the signatures, is under test here)."""

    def sign(self, seeds, m, off, kidx):
        n = off.size - 1
        h = np.frombuffer(np.arange(n, dtype=np.uint64).tobytes() * 8, np.uint8)
        return h.reshape(8, n, 8).transpose(1, 0, 2).reshape(n, 64).copy()


def test_replay_chain_packing():
    """The cmtv_commit / cmtv_block_id arrays the chain hands to
    cmtv_verify_commits point at the right rows of its flat arrays, and
    expected() is the reference loop's first reachable flipped index."""
    import ctypes

    from cometbft_amd import _native as N
    from cometbft_amd.types import Validator, ValidatorSet

    nv, nh, h0 = 7, 40, 1000
    pks = [bytes([i + 1]) * 32 for i in range(nv)]
    sv = TU.SyntheticValidators(np.zeros((nv, 32), np.uint8), np.frombuffer(b"".join(pks), np.uint8).reshape(nv, 32),
                                ValidatorSet([Validator(pk, 10) for pk in pks]))
    ch = TU.ReplayChain(_FakeSigner(), sv, h0, nh, flip=0.05, seed=3)
    assert ch.flipped.size == int(nv * nh * 0.05)
    for c in (0, 17, nh - 1):
        cm = ch.cm_arr[c]
        h = h0 + c
        assert cm.height == h and cm.n_sigs == nv and ch.heights[c] == h
        sigs = np.ctypeslib.as_array(cm.sigs, (nv * 64,))
        assert np.array_equal(sigs, ch.sig[c * nv:(c + 1) * nv].reshape(-1))
        secs = np.ctypeslib.as_array(cm.ts_seconds, (nv,))
        assert np.all(secs == TU.EPOCH_2023 + h)
        nanos = np.ctypeslib.as_array(cm.ts_nanos, (nv,))
        assert [(int(s), int(n)) for s, n in zip(secs, nanos)] == [TU.timestamp(h, i) for i in range(nv)]
        want = TU.block_id_for_height(h)
        for b in (cm.block_id, ch.bid_arr[c]):
            assert ctypes.string_at(b.hash, b.hash_len) == want.hash
            assert ctypes.string_at(b.psh_hash, b.psh_hash_len) == want.part_set_header.hash
            assert b.psh_total == 1
        assert ch.vs_arr[c].n_vals == nv
        assert ctypes.string_at(ch.vs_arr[c].pubkeys, 32 * nv) == b"".join(pks)
    flipped = set(int(x) for x in ch.flipped)
    for kind, reach in ((N.VERIFY_COMMIT, nv), (N.VERIFY_COMMIT_LIGHT, 47 // 10 + 1),
                        (N.VERIFY_COMMIT_LIGHT_TRUSTING, 23 // 10 + 1)):
        exp = ch.expected(kind)
        for c in range(nh):
            bad = [i for i in range(reach) if c * nv + i in flipped]
            assert exp[c] == (bad[0] if bad else -1), (kind, c)
