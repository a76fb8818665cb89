"""The varint-length identity cometbft_amd/csrc/commit_internal.h uvlen relies
on: ceil(bits / 7) (at least one byte) == ((bits + 6) * 37) >> 8 for every
bit width of a uint64 (1..64), and the message-length bound msg_len_bound
uses (a timestamp is at most 22 bytes: two field tags and two 10-byte
varints). CPU only."""


def test_uvlen_identity():
    for bits in range(1, 65):
        assert ((bits + 6) * 37) >> 8 == max(1, -(-bits // 7)), bits


def test_timestamp_bound():
    def uvlen(v):
        n = 1
        while v >= 0x80:
            v >>= 7
            n += 1
        return n

    worst = 0
    for sec in (0, 1, 127, 128, 2**40, 2**63 - 1, (-1) % 2**64, (-62135596800) % 2**64):
        for nanos in (0, 1, 999_999_999, (-5) % 2**64, (-(2**31)) % 2**64):
            tl = (1 + uvlen(sec) if sec else 0) + (1 + uvlen(nanos) if nanos else 0)
            worst = max(worst, tl)
    assert worst == 22
