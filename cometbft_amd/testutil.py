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
