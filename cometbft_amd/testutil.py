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


class ReplayChain:
    """configs[2]'s input as a node's cgo shim hands it to cmtv_verify_commits:
    n_heights synthetic commits (heights h0 ..) of one validator set, every
    signature present (BlockIDFlagCommit), packed ONCE into flat arrays with one
    cmtv_commit / cmtv_valset / cmtv_block_id per height pointing into them
    (blockchain/v0/reactor.go:349-400, light/client.go:613-689 verify commit
    after commit of the same set). Signatures come from the device signer over
    replay_messages' sign-bytes; a fraction `flip` of them (seed, global
    indices) carry one flipped bit.

    expected(kind) gives, per height, the reference loop's outcome over these
    inputs (types/validator_set.go:685-713 / 740-764): the first flipped
    signature the loop reaches (-1 = nil error)."""

    def __init__(self, ctx: Context, sv: SyntheticValidators, h0: int, n_heights: int, flip: float = 0.01,
                 seed: int = 42, sign_heights: int = 8192, pinned: Context | None = None):
        import ctypes

        from . import _native as N

        n = len(sv.valset.validators)
        self.n_vals, self.n_heights, self.h0 = n, n_heights, h0
        total = n * n_heights
        # pinned: the commits' flags, timestamps and signatures in ONE
        # cmtv_alloc_pinned block of that context (a cgo shim's arena in
        # pinned memory: cmtv_verify_commits then DMAs them, no host pack)
        self.block = None
        if pinned is not None:
            nb = 256 + (n + 1 + 7) // 8 * 8 + 8 * total + (4 * (n + 1) + 7) // 8 * 8 + 64 * total
            self.block = pinned.alloc_pinned(nb)
            at = 0

            def carve(dtype, count):
                nonlocal at
                a = self.block.array(dtype, count, at)
                at += (count * np.dtype(dtype).itemsize + 7) // 8 * 8
                return a
            flags_a = carve(np.uint8, n + 1)
            secs_a = carve(np.int64, total).reshape(n_heights, n)
            nanos_a = carve(np.int32, n + 1)
            self.sig = carve(np.uint8, 64 * total).reshape(total, 64)
        else:
            self.sig = np.empty((total, 64), np.uint8)
        kidx = np.tile(np.arange(n, dtype=np.uint32), min(sign_heights, n_heights))
        for c0 in range(0, n_heights, sign_heights):
            hc = min(sign_heights, n_heights - c0)
            m, off = replay_messages(h0 + c0, hc, n)
            self.sig[c0 * n:(c0 + hc) * n] = ctx.sign(sv.seeds, m, off, kidx[:hc * n])
            del m, off
        rng = np.random.default_rng(seed)
        self.flipped = np.sort(rng.choice(total, int(total * flip), replace=False)) if flip > 0 else \
            np.zeros(0, np.int64)
        bit = rng.integers(0, 512, self.flipped.size)
        self.sig[self.flipped, bit // 8] ^= (1 << (bit % 8)).astype(np.uint8)
        # shared per-validator arrays (identical in every commit of the chain)
        self.flags = np.full(n + 1, BLOCK_ID_FLAG_COMMIT, np.uint8)
        self.sig_off = (np.arange(n + 1, dtype=np.uint32) * 64)
        ts = [timestamp(h0, i) for i in range(n)]
        assert all(s == EPOCH_2023 + h0 for s, _ in ts)  # n < 1e6: seconds = EPOCH + h
        self.nanos = np.array([ns for _, ns in ts] + [0], np.int32)
        self.secs = (EPOCH_2023 + h0 + np.arange(n_heights, dtype=np.int64))[:, None].repeat(n, 1)
        if self.block is not None:
            flags_a[:] = self.flags
            nanos_a[:] = self.nanos
            secs_a[:] = self.secs
            self.flags, self.nanos, self.secs = flags_a, nanos_a, secs_a
        self.addrs = np.frombuffer(b"".join(v.address for v in sv.valset.validators) + b"\0", np.uint8).copy()
        hs = range(h0, h0 + n_heights)
        self.bhash = np.frombuffer(b"".join(hashlib.sha256(b"block%d" % h).digest() for h in hs), np.uint8).reshape(
            n_heights, 32)
        self.phash = np.frombuffer(b"".join(hashlib.sha256(b"parts%d" % h).digest() for h in hs), np.uint8).reshape(
            n_heights, 32)
        self.heights = (ctypes.c_int64 * n_heights)(*range(h0, h0 + n_heights))
        vs, self._keep_vs = sv.valset._pack()
        self.vs_arr = (N.cmtv_valset * n_heights)()
        raw = np.frombuffer(self.vs_arr, np.uint8).reshape(n_heights, ctypes.sizeof(N.cmtv_valset))
        raw[:] = np.frombuffer(bytes(vs), np.uint8)
        # cmtv_commit / cmtv_block_id arrays, filled through numpy views at
        # the ctypes field offsets
        C, B = N.cmtv_commit, N.cmtv_block_id
        self.cm_arr = (C * n_heights)()
        self.bid_arr = (B * n_heights)()
        cm = np.frombuffer(self.cm_arr, np.uint8).reshape(n_heights, ctypes.sizeof(C))
        bd = np.frombuffer(self.bid_arr, np.uint8).reshape(n_heights, ctypes.sizeof(B))
        ar = np.arange(n_heights, dtype=np.uint64)

        def put(rows, off, vals, dt):
            w = np.dtype(dt).itemsize
            rows[:, off:off + w] = np.ascontiguousarray(np.asarray(vals).astype(dt)).view(np.uint8).reshape(-1, w)

        def ptr(a):
            return np.uint64(a.ctypes.data)

        for rows, boff in ((cm, C.block_id.offset), (bd, 0)):
            put(rows, boff + B.hash.offset, ptr(self.bhash) + 32 * ar, np.uint64)
            put(rows, boff + B.hash_len.offset, np.full(n_heights, 32), np.uint32)
            put(rows, boff + B.psh_total.offset, np.ones(n_heights), np.uint32)
            put(rows, boff + B.psh_hash.offset, ptr(self.phash) + 32 * ar, np.uint64)
            put(rows, boff + B.psh_hash_len.offset, np.full(n_heights, 32), np.uint32)
        put(cm, C.height.offset, np.arange(h0, h0 + n_heights), np.int64)
        put(cm, C.round.offset, np.zeros(n_heights), np.int32)
        put(cm, C.n_sigs.offset, np.full(n_heights, n), np.uint32)
        put(cm, C.flags.offset, np.full(n_heights, ptr(self.flags)), np.uint64)
        put(cm, C.ts_seconds.offset, ptr(self.secs) + 8 * n * ar, np.uint64)
        put(cm, C.ts_nanos.offset, np.full(n_heights, ptr(self.nanos)), np.uint64)
        put(cm, C.sigs.offset, ptr(self.sig) + 64 * n * ar, np.uint64)
        put(cm, C.sig_off.offset, np.full(n_heights, ptr(self.sig_off)), np.uint64)
        put(cm, C.val_addrs.offset, np.full(n_heights, ptr(self.addrs)), np.uint64)
        self.res = (N.cmtv_commit_result * n_heights)()
        self.rcs = (ctypes.c_int * n_heights)()

    def call(self, ctx: Context, kind: int, mode: int = 0, msg_bufs=None, msg_cap: int = 0) -> None:
        """One cmtv_verify_commits over the whole chain (results in res / rcs)."""
        from . import _native as N

        cid = CHAIN_ID.encode()
        rc = N.lib().cmtv_verify_commits(ctx.handle, kind, mode, cid, len(cid), self.n_heights, self.vs_arr,
                                         self.bid_arr, self.heights, self.cm_arr, 1, 3, self.res, self.rcs, msg_bufs,
                                         msg_cap)
        N.check(rc, "cmtv_verify_commits")

    def expected(self, kind: int) -> np.ndarray:
        """Per height: the index of the first flipped signature the reference
        loop reaches, -1 when it returns nil. VerifyCommit visits every
        signature; VerifyCommitLight (and LightTrusting at 1/3 over the same
        set) stops once the tally exceeds the threshold (equal powers: after
        floor(needed / power) + 1 signatures)."""
        from . import _native as N

        n = self.n_vals
        power = 10
        total = power * n
        if kind == N.VERIFY_COMMIT:
            reach = n
        elif kind == N.VERIFY_COMMIT_LIGHT:
            reach = min(n, (total * 2 // 3) // power + 1)
        else:
            reach = min(n, (total * 1 // 3) // power + 1)
        first = np.full(self.n_heights, -1, np.int64)
        h = self.flipped // n
        i = self.flipped % n
        sel = i < reach
        h, i = h[sel], i[sel]
        # flipped is sorted: the first entry per height is its lowest index
        uh, at = np.unique(h, return_index=True)
        first[uh] = i[at]
        return first

    def outcome(self) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
        """(rcs, codes, sig_index) of the last call, as arrays."""
        rcs = np.ctypeslib.as_array(self.rcs).copy()
        res = np.frombuffer(self.res, np.uint8).reshape(self.n_heights, -1)
        from . import _native as N

        code = res[:, N.cmtv_commit_result.code.offset:N.cmtv_commit_result.code.offset + 4].copy().view(np.int32)[:, 0]
        si = res[:, N.cmtv_commit_result.sig_index.offset:N.cmtv_commit_result.sig_index.offset + 4].copy().view(
            np.int32)[:, 0]
        return rcs, code, si
