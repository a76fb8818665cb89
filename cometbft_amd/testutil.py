"""Synthetic validator sets and commits (bench + tests), mirroring the
reference's fixtures:
  ed25519.GenPrivKeyFromSecret      /root/reference/crypto/ed25519/ed25519.go:122
  types.RandValidatorSet / MakeCommit /root/reference/types/validator_set.go:1027, test_util.go:12

Keys and signatures are produced by the device (cmtv_pubkeys_ed25519 /
cmtv_sign_ed25519 = RFC 8032 deterministic signing, identical to Go's Sign);
sign-bytes by the library's CanonicalVote encoder.

Workload definition:
  seed_i  = SHA-256("cmtverify/val/" || i), voting power 10, set sorted by address
  commit  = chain "cmtverify-bench", Precommit, round 0,
            BlockID{SHA-256("block"||h), PSH{1, SHA-256("parts"||h)}},
            timestamp 2023-01-01T00:00:00Z + h s + i us, all BlockIDFlagCommit
"""
from __future__ import annotations

import hashlib
from dataclasses import dataclass

import numpy as np

from .crypto import Context, pack_messages
from .types import (BLOCK_ID_FLAG_COMMIT, PRECOMMIT_TYPE, BlockID, Commit, CommitSig, PartSetHeader, Validator,
                    ValidatorSet, vote_sign_bytes)

CHAIN_ID = "cmtverify-bench"
EPOCH_2023 = 1672531200


def validator_seeds(n: int, offset: int = 0) -> np.ndarray:
    return np.array([np.frombuffer(hashlib.sha256(b"cmtverify/val/%d" % (offset + i)).digest(), np.uint8)
                     for i in range(n)], dtype=np.uint8).reshape(n, 32)


@dataclass
class SyntheticValidators:
    seeds: np.ndarray     # n x 32, in validator-set order
    pubkeys: np.ndarray   # n x 32
    valset: ValidatorSet


def make_validator_set(ctx: Context, n: int, power: int = 10, offset: int = 0) -> SyntheticValidators:
    seeds = validator_seeds(n, offset)
    pks = ctx.pubkeys(seeds)
    addrs = [hashlib.sha256(bytes(pk)).digest()[:20] for pk in pks]
    order = sorted(range(n), key=lambda i: addrs[i])  # equal power: NewValidatorSet sorts by address
    seeds, pks = seeds[order], pks[order]
    vals = ValidatorSet([Validator(bytes(pk), power) for pk in pks])
    return SyntheticValidators(seeds, pks, vals)


def block_id_for_height(h: int) -> BlockID:
    return BlockID(hashlib.sha256(b"block%d" % h).digest(),
                   PartSetHeader(1, hashlib.sha256(b"parts%d" % h).digest()))


def timestamp(h: int, i: int):
    us = i
    return EPOCH_2023 + h + us // 1_000_000, (us % 1_000_000) * 1000


def commit_messages(n: int, height: int, round_: int = 0, chain_id: str = CHAIN_ID, flags=None):
    """Sign-bytes for each validator index of a synthetic commit."""
    bid = block_id_for_height(height)
    msgs = []
    for i in range(n):
        f = BLOCK_ID_FLAG_COMMIT if flags is None else flags[i]
        b = bid if f == BLOCK_ID_FLAG_COMMIT else BlockID()
        msgs.append(vote_sign_bytes(chain_id, PRECOMMIT_TYPE, height, round_, b, *timestamp(height, i)))
    return msgs


def make_commit(ctx: Context, sv: SyntheticValidators, height: int, round_: int = 0, chain_id: str = CHAIN_ID,
                flags=None):
    """Returns (Commit, msgs, sig array) with every present validator signing."""
    n = len(sv.valset.validators)
    flags = [BLOCK_ID_FLAG_COMMIT] * n if flags is None else list(flags)
    msgs = commit_messages(n, height, round_, chain_id, flags)
    m, off = pack_messages(msgs)
    sigs = ctx.sign(sv.seeds, m, off)
    bid = block_id_for_height(height)
    css = []
    for i in range(n):
        if flags[i] == 1:  # absent
            css.append(CommitSig(1))
        else:
            css.append(CommitSig(flags[i], sv.valset.validators[i].address, timestamp(height, i), bytes(sigs[i])))
    return Commit(height, round_, bid, css), msgs, sigs


_TEMPLATE_HEIGHT = 1000


def _varint5(v: np.ndarray) -> np.ndarray:
    """5-byte protobuf varints of v (2^28 <= v < 2^35), shape (len(v), 5)."""
    v = v.astype(np.uint64)
    out = np.empty((v.shape[0], 5), np.uint8)
    for k in range(5):
        b = (v >> np.uint64(7 * k)) & np.uint64(0x7F)
        out[:, k] = (b | np.uint64(0x80 if k < 4 else 0)).astype(np.uint8)
    return out


def replay_messages(h0: int, n_heights: int, n_vals: int, chunk: int = 8192):
    """Sign-bytes of the synthetic commits at heights h0 .. h0+n_heights-1
    (n_vals validators each, all BlockIDFlagCommit), in (height, validator)
    order, as (msg u8, msg_off u32[n+1]) -- the same bytes as concatenating
    commit_messages(n_vals, h) over h (tests/test_testutil.py), built without
    calling the encoder per message so configs[2]'s 15M messages take seconds.
    Like pack_messages, msg carries one trailing zero byte.

    Across heights a validator's CanonicalVote differs only in the sfixed64
    height, the two 32-byte BlockID hashes and the timestamp's seconds (a
    5-byte varint for every height here), all at fixed offsets: the encoder's
    output at one template height is patched per height."""
    assert n_vals <= 1_000_000 and h0 >= 1 and EPOCH_2023 + h0 + n_heights < 2**35
    th = _TEMPLATE_HEIGHT
    tmpl = commit_messages(n_vals, th)
    tbid = block_id_for_height(th)
    lens = np.array([len(t) for t in tmpl], np.int64)
    lh = int(lens.sum())
    base = np.frombuffer(b"".join(tmpl), np.uint8)
    starts = np.concatenate([[0], np.cumsum(lens)[:-1]])

    def where(t: bytes, needle: bytes) -> int:
        p = t.find(needle)
        assert p >= 0 and t.find(needle, p + 1) < 0, "template field not unique"
        return p

    # per validator: byte offsets (in the height's block) of its height,
    # block hash, parts hash and seconds fields
    fields = []
    for i, t in enumerate(tmpl):
        sec, _ = timestamp(th, i)
        assert sec == EPOCH_2023 + th  # i < 1e6 microseconds
        s = int(starts[i])
        fields.append((s + where(t, int(th).to_bytes(8, "little")), s + where(t, tbid.hash),
                       s + where(t, tbid.part_set_header.hash), s + where(t, bytes(_varint5(np.array([sec]))[0]))))

    msg = np.zeros(n_heights * lh + 1, np.uint8)  # + pad byte, as pack_messages
    for c0 in range(0, n_heights, chunk):
        c1 = min(n_heights, c0 + chunk)
        hs = np.arange(h0 + c0, h0 + c1, dtype=np.int64)
        hb = hs.astype("<i8").view(np.uint8).reshape(-1, 8)
        bh = np.frombuffer(b"".join(hashlib.sha256(b"block%d" % h).digest() for h in hs), np.uint8).reshape(-1, 32)
        ph = np.frombuffer(b"".join(hashlib.sha256(b"parts%d" % h).digest() for h in hs), np.uint8).reshape(-1, 32)
        sb = _varint5(EPOCH_2023 + hs)
        blk = msg[c0 * lh:c1 * lh].reshape(c1 - c0, lh)
        blk[:] = base
        for fh, fb, fp, fs in fields:
            blk[:, fh:fh + 8] = hb
            blk[:, fb:fb + 32] = bh
            blk[:, fp:fp + 32] = ph
            blk[:, fs:fs + 5] = sb
    off = np.empty(n_heights * n_vals + 1, np.int64)
    off[:-1] = (np.arange(n_heights, dtype=np.int64)[:, None] * lh + starts[None, :]).reshape(-1)
    off[-1] = n_heights * lh
    assert off[-1] < 2**32
    return msg, off.astype(np.uint32)
