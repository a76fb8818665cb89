"""Python mirror of the reference's commit-verification types, backed by the
C++ replay + GPU batch in libcmtverify.so (cmtv_verify_commit).

Mirrors
  BlockID / PartSetHeader           /root/reference/types/block.go:1160-1245, part_set.go:103
  CommitSig / BlockIDFlag / Commit  /root/reference/types/block.go:575-810
  Validator / ValidatorSet          /root/reference/types/validator.go, validator_set.go
  VerifyCommit                      /root/reference/types/validator_set.go:667-714
  VerifyCommitLight                 /root/reference/types/validator_set.go:722-765
  VerifyCommitLightTrusting         /root/reference/types/validator_set.go:775-826
  ErrNotEnoughVotingPowerSigned     /root/reference/types/validator_set.go:856-863
  ErrInvalidCommitHeight/Signatures /root/reference/types/errors.go:15-41
  VoteSignBytes                     /root/reference/types/vote.go:93-101

Errors are raised as exceptions whose str() is the reference's error string;
the places where the reference panics raise ReferencePanic.
"""
from __future__ import annotations

import ctypes
import hashlib
from dataclasses import dataclass, field
from typing import Optional, Sequence

import numpy as np

from . import _native as N
from .crypto import MODE_GO_STDLIB, Context, default_context

BLOCK_ID_FLAG_ABSENT = 1
BLOCK_ID_FLAG_COMMIT = 2
BLOCK_ID_FLAG_NIL = 3
PRECOMMIT_TYPE = 2
PREVOTE_TYPE = 1
GO_ZERO_TIME_SECONDS = -62135596800  # time.Time{} as Unix seconds


class CommitError(Exception):
    code = -1


class ErrInvalidCommitSignatures(CommitError):
    code = N.COMMIT_ERR_SET_SIZE


class ErrInvalidCommitHeight(CommitError):
    code = N.COMMIT_ERR_HEIGHT


class ErrWrongBlockID(CommitError):
    code = N.COMMIT_ERR_BLOCK_ID


class ErrWrongSignature(CommitError):
    code = N.COMMIT_ERR_WRONG_SIGNATURE

    def __init__(self, msg, index):
        super().__init__(msg)
        self.index = index


class ErrNotEnoughVotingPowerSigned(CommitError):
    code = N.COMMIT_ERR_NOT_ENOUGH_POWER

    def __init__(self, msg, got, needed):
        super().__init__(msg)
        self.got = got
        self.needed = needed


class ErrDoubleVote(CommitError):
    code = N.COMMIT_ERR_DOUBLE_VOTE


class ErrTrustLevel(CommitError):
    code = N.COMMIT_ERR_TRUST_LEVEL


class ReferencePanic(Exception):
    """Raised where the reference Go code would panic."""


@dataclass
class PartSetHeader:
    total: int = 0
    hash: bytes = b""


@dataclass
class BlockID:
    hash: bytes = b""
    part_set_header: PartSetHeader = field(default_factory=PartSetHeader)

    def is_zero(self) -> bool:
        return len(self.hash) == 0 and self.part_set_header.total == 0 and len(self.part_set_header.hash) == 0

    def _c(self):
        h = (ctypes.c_uint8 * max(len(self.hash), 1)).from_buffer_copy(self.hash + b"\0")
        ph = (ctypes.c_uint8 * max(len(self.part_set_header.hash), 1)).from_buffer_copy(
            self.part_set_header.hash + b"\0")
        s = N.cmtv_block_id(hash=ctypes.cast(h, ctypes.POINTER(ctypes.c_uint8)), hash_len=len(self.hash),
                            psh_total=self.part_set_header.total,
                            psh_hash=ctypes.cast(ph, ctypes.POINTER(ctypes.c_uint8)),
                            psh_hash_len=len(self.part_set_header.hash))
        return s, (h, ph)


@dataclass
class CommitSig:
    block_id_flag: int
    validator_address: bytes = b""
    timestamp: tuple = (GO_ZERO_TIME_SECONDS, 0)  # (unix seconds, nanos)
    signature: bytes = b""

    def for_block(self) -> bool:
        return self.block_id_flag == BLOCK_ID_FLAG_COMMIT

    def absent(self) -> bool:
        return self.block_id_flag == BLOCK_ID_FLAG_ABSENT


def new_commit_sig_absent() -> CommitSig:
    return CommitSig(BLOCK_ID_FLAG_ABSENT)


@dataclass
class Commit:
    height: int
    round: int
    block_id: BlockID
    signatures: list

    def vote_sign_bytes(self, chain_id: str, val_idx: int) -> bytes:
        """Commit.VoteSignBytes (types/block.go:807)."""
        cs = self.signatures[val_idx]
        if cs.block_id_flag == BLOCK_ID_FLAG_COMMIT:
            bid = self.block_id
        elif cs.block_id_flag in (BLOCK_ID_FLAG_ABSENT, BLOCK_ID_FLAG_NIL):
            bid = BlockID()
        else:
            raise ReferencePanic(f"Unknown BlockIDFlag: {cs.block_id_flag}")
        return vote_sign_bytes(chain_id, PRECOMMIT_TYPE, self.height, self.round, bid, *cs.timestamp)


def vote_sign_bytes(chain_id: str, vote_type: int, height: int, round_: int, block_id: Optional[BlockID],
                    ts_seconds: int, ts_nanos: int) -> bytes:
    """VoteSignBytes (types/vote.go:93) through the library's encoder."""
    cid = chain_id.encode()
    bid = block_id or BlockID()
    cb, keep = bid._c()
    buf = (ctypes.c_uint8 * 512)()
    n = N.lib().cmtv_vote_sign_bytes(cid, len(cid), vote_type, height, round_, ctypes.byref(cb), ts_seconds,
                                     ts_nanos, buf, 512)
    if n < 0:
        raise N.CmtvError(int(n), "cmtv_vote_sign_bytes")
    if n > 512:
        buf = (ctypes.c_uint8 * n)()
        n = N.lib().cmtv_vote_sign_bytes(cid, len(cid), vote_type, height, round_, ctypes.byref(cb), ts_seconds,
                                         ts_nanos, buf, n)
    return bytes(buf[:n])


@dataclass
class Validator:
    pub_key: bytes
    voting_power: int
    proposer_priority: int = 0

    @property
    def address(self) -> bytes:
        """PubKey.Address(): SHA-256(pubkey)[:20] (crypto/ed25519/ed25519.go:136)."""
        return hashlib.sha256(self.pub_key).digest()[:20]


class ValidatorSet:
    def __init__(self, validators: Sequence[Validator]):
        self.validators = list(validators)
        self._packed = None

    def size(self) -> int:
        return len(self.validators)

    def total_voting_power(self) -> int:
        return sum(v.voting_power for v in self.validators)

    def _pack(self):
        if self._packed is None:
            vals = self.validators
            pks = b"".join(v.pub_key for v in vals)
            off = np.zeros(len(vals) + 1, np.uint32)
            off[1:] = np.cumsum([len(v.pub_key) for v in vals]) if vals else []
            pk = np.frombuffer(pks + b"\0", np.uint8).copy()
            vp = np.array([v.voting_power for v in vals] + [0], np.int64)
            pp = np.array([v.proposer_priority for v in vals] + [0], np.int64)
            ad = np.frombuffer(b"".join(v.address for v in vals) + b"\0", np.uint8).copy()
            self._packed = (pk, off, vp, pp, ad)
        pk, off, vp, pp, ad = self._packed
        s = N.cmtv_valset(n_vals=len(self.validators), pubkeys=_p8(pk), pk_off=_p32(off),
                          voting_power=vp.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), addrs=_p8(ad),
                          proposer_priority=pp.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)))
        return s, self._packed

    # ----------------------------------------------------------------- verify
    def verify_commit(self, chain_id: str, block_id: BlockID, height: int, commit: Commit,
                      ctx: Context | None = None, mode: int = MODE_GO_STDLIB):
        return _verify(self, N.VERIFY_COMMIT, chain_id, block_id, height, commit, 0, 0, ctx, mode)

    def verify_commit_light(self, chain_id: str, block_id: BlockID, height: int, commit: Commit,
                            ctx: Context | None = None, mode: int = MODE_GO_STDLIB):
        return _verify(self, N.VERIFY_COMMIT_LIGHT, chain_id, block_id, height, commit, 0, 0, ctx, mode)

    def verify_commit_light_trusting(self, chain_id: str, commit: Commit, trust_level=(1, 3),
                                     ctx: Context | None = None, mode: int = MODE_GO_STDLIB):
        num, den = trust_level
        return _verify(self, N.VERIFY_COMMIT_LIGHT_TRUSTING, chain_id, None, 0, commit, num, den, ctx, mode)


def _p8(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


def _p32(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))


class _Arena:
    """Carves arrays out of one pinned block (a cgo shim's argument arena in
    cmtv_alloc_pinned memory), 8-byte aligned."""

    def __init__(self, block):
        self.block, self.at = block, 0

    def put(self, a: np.ndarray) -> np.ndarray:
        a = np.ascontiguousarray(a)
        out = self.block.array(a.dtype, a.size, self.at).reshape(a.shape)
        out[...] = a
        self.at += (a.nbytes + 7) // 8 * 8
        return out


def _pack_commit(commit: Commit, arena: _Arena | None = None):
    sigs = commit.signatures
    n = len(sigs)
    flags = np.array([s.block_id_flag for s in sigs] + [0], np.uint8)
    ts_s = np.array([s.timestamp[0] for s in sigs] + [0], np.int64)
    ts_n = np.array([s.timestamp[1] for s in sigs] + [0], np.int32)
    sb = np.frombuffer(b"".join(s.signature for s in sigs) + b"\0", np.uint8).copy()
    so = np.zeros(n + 1, np.uint32)
    if n:
        so[1:] = np.cumsum([len(s.signature) for s in sigs])
    if arena is not None:  # per commit flags | secs | nanos | sig_off | sigs, as INTEGRATION.md's arena
        flags, ts_s, ts_n, so, sb = (arena.put(x) for x in (flags, ts_s, ts_n, so, sb))
    addrs = b"".join((s.validator_address + bytes(20))[:20] for s in sigs)
    ad = np.frombuffer(addrs + b"\0", np.uint8).copy()
    bid, keep = commit.block_id._c()
    c = N.cmtv_commit(height=commit.height, round=commit.round, block_id=bid, n_sigs=n, flags=_p8(flags),
                      ts_seconds=ts_s.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                      ts_nanos=ts_n.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), sigs=_p8(sb), sig_off=_p32(so),
                      val_addrs=_p8(ad))
    return c, (flags, ts_s, ts_n, sb, so, ad, keep)


def _verify(vals: ValidatorSet, kind, chain_id, block_id, height, commit, num, den, ctx, mode):
    ctx = ctx or default_context()
    vs, keep_v = vals._pack()
    cm, keep_c = _pack_commit(commit)
    if block_id is not None:
        bid, keep_b = block_id._c()
        bidp = ctypes.byref(bid)
    else:
        bidp, keep_b = None, None
    res = N.cmtv_commit_result()
    buf = ctypes.create_string_buffer(4096)
    cid = chain_id.encode()
    rc = N.lib().cmtv_verify_commit(ctx.handle, kind, mode, cid, len(cid), ctypes.byref(vs), bidp, height,
                                    ctypes.byref(cm), num, den, ctypes.byref(res), buf, len(buf))
    N.check(rc, "cmtv_verify_commit")
    err = _error_for(rc, res, buf.value.decode())
    if err is not None:
        raise err
    return None


def _error_for(rc, res, msg):
    """The exception the reference's VerifyCommit* would produce (None = nil)."""
    if rc == N.CMTV_OK:
        return None
    code = res.code
    if code == N.COMMIT_ERR_SET_SIZE:
        return ErrInvalidCommitSignatures(msg)
    if code == N.COMMIT_ERR_HEIGHT:
        return ErrInvalidCommitHeight(msg)
    if code == N.COMMIT_ERR_BLOCK_ID:
        return ErrWrongBlockID(msg)
    if code == N.COMMIT_ERR_WRONG_SIGNATURE:
        return ErrWrongSignature(msg, res.sig_index)
    if code == N.COMMIT_ERR_NOT_ENOUGH_POWER:
        return ErrNotEnoughVotingPowerSigned(msg, res.got, res.needed)
    if code == N.COMMIT_ERR_DOUBLE_VOTE:
        e = ErrDoubleVote(msg)
        e.result = N.cmtv_commit_result.from_buffer_copy(res)
        return e
    if code == N.COMMIT_ERR_TRUST_LEVEL:
        return ErrTrustLevel(msg)
    if code in (N.COMMIT_PANIC_BAD_PUBKEY, N.COMMIT_PANIC_UNKNOWN_FLAG):
        return ReferencePanic(msg)
    return CommitError(msg)


def verify_commits(kind: int, chain_id: str, items, ctx: Context | None = None, mode: int = MODE_GO_STDLIB,
                   trust_level=(1, 3)):
    """Cross-height batching (cmtv_verify_commits): items is a sequence of
    (ValidatorSet, BlockID | None, height, Commit). All their signatures go to
    the device in ONE batch; returns, per item, None (the reference's nil) or
    the exception its VerifyCommit* would have returned -- not raised, so one
    bad height does not hide the others."""
    if len(items) == 0:
        return []
    return PackedCommits(kind, chain_id, items, mode, trust_level).verify(ctx or default_context())


class PackedCommits:
    """The C arguments of one cmtv_verify_commits call, packed once (what a
    cgo shim holds when it calls the library); verify() makes the call."""

    def __init__(self, kind: int, chain_id: str, items, mode: int = MODE_GO_STDLIB, trust_level=(1, 3),
                 pinned: Context | None = None):
        """pinned: the commits' arrays in one cmtv_alloc_pinned block of that
        context (the direct, zero-copy chunks of cmtv_verify_commits there)."""
        n = len(items)
        keep = []
        arena = None
        if pinned is not None:
            nb = 4096 + sum(80 + 24 * (len(c.signatures) + 1) + sum(len(s.signature) for s in c.signatures)
                            for _, _, _, c in items)
            self.block = pinned.alloc_pinned(nb)
            arena = _Arena(self.block)
        vs_arr = (N.cmtv_valset * n)()
        cm_arr = (N.cmtv_commit * n)()
        bid_arr = (N.cmtv_block_id * n)()
        heights = (ctypes.c_int64 * n)()
        for c, (vals, block_id, height, commit) in enumerate(items):
            vs, kv = vals._pack()
            cm, kc = _pack_commit(commit, arena)
            vs_arr[c], cm_arr[c] = vs, cm
            keep += [kv, kc]
            if block_id is not None:
                bid, kb = block_id._c()
                bid_arr[c] = bid
                keep.append(kb)
            heights[c] = height
        self.n, self.kind, self.mode, self.cap = n, kind, mode, 1024
        self.cid = chain_id.encode()
        self.num, self.den = trust_level if kind == N.VERIFY_COMMIT_LIGHT_TRUSTING else (0, 0)
        self.vs_arr, self.cm_arr, self.heights, self._keep = vs_arr, cm_arr, heights, keep
        self.bid_arr = bid_arr if kind != N.VERIFY_COMMIT_LIGHT_TRUSTING else None
        self.res = (N.cmtv_commit_result * n)()
        self.rcs = (ctypes.c_int * n)()
        self.bufs = ctypes.create_string_buffer(n * self.cap)

    def call(self, ctx: Context) -> None:
        """The C call alone (results left in res / rcs / bufs)."""
        rc = N.lib().cmtv_verify_commits(ctx.handle, self.kind, self.mode, self.cid, len(self.cid), self.n,
                                         self.vs_arr, self.bid_arr, self.heights, self.cm_arr, self.num, self.den,
                                         self.res, self.rcs, self.bufs, self.cap)
        N.check(rc, "cmtv_verify_commits")

    def verify(self, ctx: Context):
        self.call(ctx)
        raw, cap = self.bufs.raw, self.cap
        out = []
        for c in range(self.n):
            msg = raw[c * cap: (c + 1) * cap].split(b"\0", 1)[0].decode()
            out.append(_error_for(self.rcs[c], self.res[c], msg))
        return out
