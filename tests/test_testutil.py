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
