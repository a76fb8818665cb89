"""CPU oracle (TEST INFRASTRUCTURE ONLY) -- restatement of CometBFT's vote
sign-bytes encoder, used to check the product's C++ encoder.

Follows:
  /root/reference/types/vote.go:93-101          VoteSignBytes
  /root/reference/types/canonical.go:18-65      CanonicalizeBlockID / CanonicalizeVote
  /root/reference/types/block.go:784-810        Commit.GetVote / VoteSignBytes
  /root/reference/libs/protoio/writer.go:93     MarshalDelimited (uvarint length prefix)
  /root/reference/proto/tendermint/types/canonical.pb.go:370-567
      CanonicalBlockID / CanonicalPartSetHeader / CanonicalVote MarshalToSizedBuffer
  gogoproto StdTimeMarshalTo = google.protobuf.Timestamp {1: seconds, 2: nanos}

Pinned by the known-answer vectors of types/vote_test.go:60-137
(tests/golden/signbytes_kat.json).
"""
from __future__ import annotations

import struct


def uvarint(v: int) -> bytes:
    v &= (1 << 64) - 1
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def _bytes_field(tag: int, b: bytes) -> bytes:
    return bytes([tag]) + uvarint(len(b)) + b


def timestamp(seconds: int, nanos: int) -> bytes:
    out = b""
    if seconds != 0:
        out += b"\x08" + uvarint(seconds)
    if nanos != 0:
        out += b"\x10" + uvarint(nanos)
    return out


def canonical_block_id(hash_: bytes, psh_total: int, psh_hash: bytes) -> bytes | None:
    """None when the BlockID IsZero() (types/block.go:1199) -> field omitted."""
    if len(hash_) == 0 and psh_total == 0 and len(psh_hash) == 0:
        return None
    psh = b""
    if psh_total != 0:
        psh += b"\x08" + uvarint(psh_total)
    if psh_hash:
        psh += _bytes_field(0x12, psh_hash)
    out = b""
    if hash_:
        out += _bytes_field(0x0A, hash_)
    out += _bytes_field(0x12, psh)
    return out


def canonical_vote(chain_id: str, vtype: int, height: int, round_: int,
                   block_id: tuple | None, ts_seconds: int, ts_nanos: int) -> bytes:
    out = b""
    if vtype != 0:
        out += b"\x08" + uvarint(vtype)
    if height != 0:
        out += b"\x11" + struct.pack("<q", height)
    if round_ != 0:
        out += b"\x19" + struct.pack("<q", round_)
    if block_id is not None:
        cb = canonical_block_id(*block_id)
        if cb is not None:
            out += _bytes_field(0x22, cb)
    out += _bytes_field(0x2A, timestamp(ts_seconds, ts_nanos))
    cid = chain_id.encode()
    if cid:
        out += _bytes_field(0x32, cid)
    return out


def vote_sign_bytes(chain_id: str, vtype: int, height: int, round_: int,
                    block_id: tuple | None, ts_seconds: int, ts_nanos: int) -> bytes:
    body = canonical_vote(chain_id, vtype, height, round_, block_id, ts_seconds, ts_nanos)
    return uvarint(len(body)) + body


# Go's zero time.Time{} is 0001-01-01T00:00:00Z = -62135596800 Unix seconds.
GO_ZERO_TIME_SECONDS = -62135596800

PRECOMMIT = 2
PREVOTE = 1
