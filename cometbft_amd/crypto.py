"""Python mirror of the reference's crypto boundary for Ed25519, backed by the
gfx950 verifier in libcmtverify.so.

Reference interfaces mirrored
  crypto.PubKey.VerifySignature(msg, sig) bool      /root/reference/crypto/crypto.go:25
  ed25519.PubKey.VerifySignature                    /root/reference/crypto/ed25519/ed25519.go:148-155
  crypto.BatchVerifier {Add, Verify}                upstream CometBFT v0.38 (not in this v0.34 tree;
                                                    see SURVEY.md section 8b and INTEGRATION.md)
  ed25519.NewBatchVerifier()                        upstream, same

Every verdict is computed on the GPU. There is no CPU fallback in this package.
"""
from __future__ import annotations

import ctypes
import threading
from typing import Sequence

import numpy as np

from . import _native as N

MODE_GO_STDLIB = N.MODE_GO_STDLIB
MODE_ZIP215 = N.MODE_ZIP215

PUBKEY_SIZE = 32     # crypto/ed25519/ed25519.go:24
SIGNATURE_SIZE = 64  # crypto/ed25519/ed25519.go:28


def _u8(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


class Context:
    """A verification context (cmtv_open / cmtv_open_devices): per device a
    stream, fixed-base tables and staging buffers.

    devices=None opens one device (`device`, -1 = the current one); a list of
    HIP ordinals opens one context over all of them (batches are sharded and
    their verdict bitmaps all-gathered over RCCL); devices=[] takes the list
    from CMTVERIFY_DEVICES, or every visible gfx950 device."""

    def __init__(self, device: int = -1, default_mode: int = MODE_GO_STDLIB, devices: Sequence[int] | None = None):
        L = N.lib()
        cfg = N.cmtv_config(device=device, default_mode=default_mode, flags=0, reserved=0)
        h = ctypes.c_void_p()
        if devices is None:
            N.check(L.cmtv_open(ctypes.byref(cfg), ctypes.byref(h)), "cmtv_open")
        else:
            arr = (ctypes.c_int32 * max(len(devices), 1))(*devices)
            N.check(L.cmtv_open_devices(ctypes.byref(cfg), arr, len(devices), ctypes.byref(h)), "cmtv_open_devices")
        self._h = h
        self.default_mode = default_mode

    @property
    def n_devices(self) -> int:
        return N.lib().cmtv_device_count(self._h)

    def device_ordinal(self, g: int) -> int:
        return N.lib().cmtv_device_ordinal(self._h, g)

    def device_stream(self, g: int) -> int:
        return N.lib().cmtv_device_stream(self._h, g) or 0

    def sync(self) -> None:
        N.check(N.lib().cmtv_sync(self._h), "cmtv_sync")

    def verify_sharded_device(self, n_shard: Sequence[int], d_pk, d_sig, d_msg, d_off, mode: int, d_bitmap_all,
                              d_valid=None, keys: "KeySet | None" = None) -> int:
        """cmtv_verify_ed25519[_indexed]_sharded_device: shard g's device
        pointers (ints) on the context's g-th device (d_pk holds key indices
        when `keys` is given); returns W, the bitmap words per shard. The
        gathered bitmap on every device is G x W words. Non-blocking."""
        G = len(n_shard)
        vp = ctypes.c_void_p
        arr = lambda xs: (vp * G)(*[vp(x) if x else None for x in xs])  # noqa: E731
        ns = (ctypes.c_size_t * G)(*n_shard)
        w = ctypes.c_size_t(0)
        dv = arr(d_valid) if d_valid is not None else None
        if keys is None:
            rc = N.lib().cmtv_verify_ed25519_sharded_device(self._h, ns, arr(d_pk), arr(d_sig), arr(d_msg), arr(d_off),
                                                            mode, dv, arr(d_bitmap_all), ctypes.byref(w))
        else:
            rc = N.lib().cmtv_verify_ed25519_indexed_sharded_device(self._h, keys.handle, ns, arr(d_pk), arr(d_sig),
                                                                    arr(d_msg), arr(d_off), mode, dv,
                                                                    arr(d_bitmap_all), ctypes.byref(w))
        N.check(rc, "cmtv_verify_ed25519_sharded_device")
        return w.value

    def verify_multi_device(self, n_dev: Sequence[int], d_pk, d_sig, d_msg, d_off, mode: int, d_bitmap,
                            d_valid=None) -> None:
        """cmtv_verify_ed25519_multi_device: device g verifies its own batch
        (pointers as ints on the context's g-th device) into its own
        ceil(n_dev[g] / 64) bitmap words; no exchange. Non-blocking."""
        G = len(n_dev)
        vp = ctypes.c_void_p
        arr = lambda xs: (vp * G)(*[vp(x) if x else None for x in xs])  # noqa: E731
        ns = (ctypes.c_size_t * G)(*n_dev)
        dv = arr(d_valid) if d_valid is not None else None
        rc = N.lib().cmtv_verify_ed25519_multi_device(self._h, ns, arr(d_pk), arr(d_sig), arr(d_msg), arr(d_off), mode,
                                                      dv, arr(d_bitmap))
        N.check(rc, "cmtv_verify_ed25519_multi_device")

    @property
    def handle(self):
        return self._h

    def close(self):
        if self._h:
            N.lib().cmtv_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def stream(self) -> int:
        return N.lib().cmtv_stream(self._h) or 0

    def stats(self) -> dict:
        st = N.cmtv_stats()
        N.check(N.lib().cmtv_stats_get(self._h, ctypes.byref(st)), "cmtv_stats_get")
        return {k: getattr(st, k) for k, _ in st._fields_ if k != "reserved"}

    def device_stats(self) -> list:
        """cmtv_device_stats_get for every device of the context: ordinal,
        failed (retired after a HIP error), calls, signatures, launches and
        summed kernel milliseconds on that device."""
        out = []
        for g in range(self.n_devices):
            st = N.cmtv_device_stats()
            N.check(N.lib().cmtv_device_stats_get(self._h, g, ctypes.byref(st)), "cmtv_device_stats_get")
            out.append({k: getattr(st, k) for k, _ in st._fields_})
        return out

    def alloc_pinned(self, nbytes: int) -> "PinnedBlock":
        """cmtv_alloc_pinned: page-locked host memory of this context, the
        zero-copy source of cmtv_verify_commits' direct chunks; .array(dtype,
        count, offset) views it as numpy."""
        return PinnedBlock(self, nbytes)

    def keyset_cache(self, max_sets: int) -> None:
        """cmtv_keyset_cache: registered key sets of up to max_sets validator
        sets for cmtv_verify_commit(s) (0 = off)."""
        N.check(N.lib().cmtv_keyset_cache(self._h, max_sets), "cmtv_keyset_cache")

    def verdict_cache(self, max_entries: int) -> None:
        """cmtv_verdict_cache: keep the last max_entries verdicts (0 = off)."""
        N.check(N.lib().cmtv_verdict_cache(self._h, max_entries), "cmtv_verdict_cache")

    # -------------------------------------------------------------- batches
    def verify(self, pk: np.ndarray, sig: np.ndarray, msg: np.ndarray, msg_off: np.ndarray,
               mode: int | None = None, bitmap: bool = False):
        """Verdicts for n signatures held in host arrays (pk n x 32, sig n x 64,
        flat msg bytes + n+1 uint32 offsets). Returns uint8[n] (and the uint64
        bitmap when bitmap=True)."""
        mode = self.default_mode if mode is None else mode
        pk = np.ascontiguousarray(pk, dtype=np.uint8).reshape(-1, 32)
        sig = np.ascontiguousarray(sig, dtype=np.uint8).reshape(-1, 64)
        n = pk.shape[0]
        if sig.shape[0] != n or len(msg_off) != n + 1:
            raise ValueError("pk / sig / msg_off sizes disagree")
        msg = np.ascontiguousarray(msg, dtype=np.uint8)
        if msg.size == 0:
            msg = np.zeros(1, np.uint8)
        off = np.ascontiguousarray(msg_off, dtype=np.uint32)
        valid = np.zeros(max(n, 1), np.uint8)
        words = np.zeros(max((n + 63) // 64, 1), np.uint64)
        rc = N.lib().cmtv_verify_ed25519(self._h, n, _u8(pk), _u8(sig), _u8(msg),
                                         off.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), mode, _u8(valid),
                                         words.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)))
        N.check(rc, "cmtv_verify_ed25519")
        if bitmap:
            return valid[:n], words[: (n + 63) // 64]
        return valid[:n]

    def verify_device(self, n: int, d_pk: int, d_sig: int, d_msg: int, d_off: int, mode: int,
                      d_valid: int = 0, d_bitmap: int = 0, stream: int = 0) -> None:
        """Enqueue verification over device-resident buffers (raw pointers) on
        `stream` (a hipStream_t handle; 0 = the null stream, which is what
        torch's default stream reports)."""
        rc = N.lib().cmtv_verify_ed25519_device(self._h, n, d_pk, d_sig, d_msg, d_off, mode, d_valid or None,
                                                d_bitmap or None, ctypes.c_void_p(stream) if stream else None)
        N.check(rc, "cmtv_verify_ed25519_device")

    # -------------------------------------------------------------- sr25519
    def verify_sr25519(self, pk: np.ndarray, sig: np.ndarray, msg: np.ndarray, msg_off: np.ndarray,
                       bitmap: bool = False):
        """sr25519 verdicts (crypto/sr25519/pubkey.go:34-60) for n 32-byte keys
        and 64-byte signatures in host arrays; layout as verify()."""
        pk = np.ascontiguousarray(pk, dtype=np.uint8).reshape(-1, 32)
        sig = np.ascontiguousarray(sig, dtype=np.uint8).reshape(-1, 64)
        n = pk.shape[0]
        if sig.shape[0] != n or len(msg_off) != n + 1:
            raise ValueError("pk / sig / msg_off sizes disagree")
        msg = np.ascontiguousarray(msg, dtype=np.uint8)
        if msg.size == 0:
            msg = np.zeros(1, np.uint8)
        off = np.ascontiguousarray(msg_off, dtype=np.uint32)
        valid = np.zeros(max(n, 1), np.uint8)
        words = np.zeros(max((n + 63) // 64, 1), np.uint64)
        rc = N.lib().cmtv_verify_sr25519(self._h, n, _u8(pk), _u8(sig), _u8(msg),
                                         off.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), _u8(valid),
                                         words.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)))
        N.check(rc, "cmtv_verify_sr25519")
        if bitmap:
            return valid[:n], words[: (n + 63) // 64]
        return valid[:n]

    def verify_sr25519_device(self, n: int, d_pk: int, d_sig: int, d_msg: int, d_off: int, d_valid: int = 0,
                              d_bitmap: int = 0, stream: int = 0) -> None:
        """Enqueue sr25519 verification over device-resident buffers."""
        rc = N.lib().cmtv_verify_sr25519_device(self._h, n, d_pk, d_sig, d_msg, d_off, d_valid or None,
                                                d_bitmap or None, ctypes.c_void_p(stream) if stream else None)
        N.check(rc, "cmtv_verify_sr25519_device")

    # -------------------------------------------------------------- registered keys
    def register_keys(self, pk: np.ndarray, wide: bool = False) -> "KeySet":
        """Decode n 32-byte keys once and build their combs on the device
        (cmtv_register_keys); verify_indexed then needs no decompression of
        A and no doublings. 512 KiB of HBM per key; wide=True also builds the
        radix-2^16 combs (CMTV_KEYS_WIDE, 64 MiB per key) that halve the
        additions of large batches."""
        return KeySet(self, pk, wide)

    def verify_indexed(self, keys: "KeySet", key_idx: np.ndarray, sig: np.ndarray, msg: np.ndarray,
                       msg_off: np.ndarray, mode: int | None = None, bitmap: bool = False):
        """Verdicts for n signatures, signature i by registered key key_idx[i];
        same verdicts as verify(keys.pk[key_idx], ...)."""
        mode = self.default_mode if mode is None else mode
        key_idx = np.ascontiguousarray(key_idx, dtype=np.uint32).reshape(-1)
        sig = np.ascontiguousarray(sig, dtype=np.uint8).reshape(-1, 64)
        n = key_idx.shape[0]
        if sig.shape[0] != n or len(msg_off) != n + 1:
            raise ValueError("key_idx / sig / msg_off sizes disagree")
        msg = np.ascontiguousarray(msg, dtype=np.uint8)
        if msg.size == 0:
            msg = np.zeros(1, np.uint8)
        off = np.ascontiguousarray(msg_off, dtype=np.uint32)
        valid = np.zeros(max(n, 1), np.uint8)
        words = np.zeros(max((n + 63) // 64, 1), np.uint64)
        u32p = ctypes.POINTER(ctypes.c_uint32)
        rc = N.lib().cmtv_verify_ed25519_indexed(self._h, keys.handle, n, key_idx.ctypes.data_as(u32p), _u8(sig),
                                                 _u8(msg), off.ctypes.data_as(u32p), mode, _u8(valid),
                                                 words.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)))
        N.check(rc, "cmtv_verify_ed25519_indexed")
        if bitmap:
            return valid[:n], words[: (n + 63) // 64]
        return valid[:n]

    def verify_indexed_device(self, keys: "KeySet", n: int, d_key_idx: int, d_sig: int, d_msg: int, d_off: int,
                              mode: int, d_valid: int = 0, d_bitmap: int = 0, stream: int = 0) -> None:
        rc = N.lib().cmtv_verify_ed25519_indexed_device(self._h, keys.handle, n, d_key_idx, d_sig, d_msg, d_off,
                                                        mode, d_valid or None, d_bitmap or None,
                                                        ctypes.c_void_p(stream) if stream else None)
        N.check(rc, "cmtv_verify_ed25519_indexed_device")

    # -------------------------------------------------------------- test data
    def pubkeys(self, seeds: np.ndarray) -> np.ndarray:
        seeds = np.ascontiguousarray(seeds, dtype=np.uint8).reshape(-1, 32)
        out = np.zeros_like(seeds)
        N.check(N.lib().cmtv_pubkeys_ed25519(self._h, seeds.shape[0], _u8(seeds), _u8(out)), "cmtv_pubkeys_ed25519")
        return out

    def sign(self, seeds: np.ndarray, msg: np.ndarray, msg_off: np.ndarray, key_idx=None) -> np.ndarray:
        seeds = np.ascontiguousarray(seeds, dtype=np.uint8).reshape(-1, 32)
        off = np.ascontiguousarray(msg_off, dtype=np.uint32)
        n = len(off) - 1
        msg = np.ascontiguousarray(msg, dtype=np.uint8)
        if msg.size == 0:
            msg = np.zeros(1, np.uint8)
        out = np.zeros((max(n, 1), 64), np.uint8)
        kp = None
        if key_idx is not None:
            key_idx = np.ascontiguousarray(key_idx, dtype=np.uint32)
            kp = key_idx.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))
        rc = N.lib().cmtv_sign_ed25519(self._h, n, _u8(seeds), kp, _u8(msg),
                                       off.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), _u8(out))
        N.check(rc, "cmtv_sign_ed25519")
        return out[:n]


class KeySet:
    """Registered public keys (cmtv_keyset): per-key combs resident in HBM."""

    def __init__(self, ctx: Context, pk: np.ndarray, wide: bool = False):
        pk = np.ascontiguousarray(pk, dtype=np.uint8).reshape(-1, 32)
        h = ctypes.c_void_p()
        flags = N.CMTV_KEYS_WIDE if wide else 0
        N.check(N.lib().cmtv_register_keys_ex(ctx.handle, pk.shape[0], _u8(pk), flags, ctypes.byref(h)),
                "cmtv_register_keys_ex")
        self.wide = wide
        self._h = h
        self.ctx = ctx  # keeps the context alive while the key set is
        self.pk = pk.copy()

    @property
    def handle(self):
        return self._h

    def __len__(self):
        return N.lib().cmtv_keyset_len(self._h)

    def free(self):
        if self._h:
            N.lib().cmtv_keyset_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


_default_ctx = None
_default_lock = threading.Lock()


class PinnedBlock:
    """A cmtv_alloc_pinned block; freed by free() or with its context."""

    def __init__(self, ctx: Context, nbytes: int):
        p = ctypes.c_void_p()
        N.check(N.lib().cmtv_alloc_pinned(ctx.handle, nbytes, ctypes.byref(p)), "cmtv_alloc_pinned")
        self._ctx, self.ptr, self.nbytes = ctx, p.value, nbytes
        self._buf = (ctypes.c_uint8 * nbytes).from_address(p.value)

    def array(self, dtype, count: int, offset: int = 0) -> np.ndarray:
        dt = np.dtype(dtype)
        assert offset % dt.itemsize == 0 and offset + count * dt.itemsize <= self.nbytes
        return np.frombuffer(self._buf, dt, count, offset)

    def free(self) -> None:
        if self.ptr and self._ctx.handle:
            N.check(N.lib().cmtv_free_pinned(self._ctx.handle, self.ptr), "cmtv_free_pinned")
        self.ptr = None


def default_context() -> Context:
    global _default_ctx
    with _default_lock:
        if _default_ctx is None:
            _default_ctx = Context()
        return _default_ctx


def pack_messages(msgs: Sequence[bytes]):
    off = np.zeros(len(msgs) + 1, dtype=np.uint32)
    if msgs:
        off[1:] = np.cumsum([len(m) for m in msgs], dtype=np.uint64).astype(np.uint32)
    buf = np.frombuffer(b"".join(msgs) + b"\0", dtype=np.uint8).copy()
    return buf, off


class PubKey(bytes):
    """ed25519.PubKey (crypto/ed25519/ed25519.go:133): raw 32 bytes."""

    def verify_signature(self, msg: bytes, sig: bytes, ctx: Context | None = None,
                         mode: int = MODE_GO_STDLIB) -> bool:
        """PubKey.VerifySignature (ed25519.go:148-155) as a batch of one on the
        GPU. Wrong-length keys raise like Go's panic; wrong-length signatures
        return False."""
        if len(sig) != SIGNATURE_SIZE:
            return False
        if len(self) != PUBKEY_SIZE:
            raise ValueError(f"ed25519: bad public key length: {len(self)}")
        ctx = ctx or default_context()
        m, off = pack_messages([bytes(msg)])
        v = ctx.verify(np.frombuffer(bytes(self), np.uint8), np.frombuffer(bytes(sig), np.uint8), m, off, mode)
        return bool(v[0])


class Sr25519PubKey(bytes):
    """sr25519.PubKey (crypto/sr25519/pubkey.go:21): raw key bytes."""

    def verify_signature(self, msg: bytes, sig: bytes, ctx: Context | None = None) -> bool:
        """PubKey.VerifySignature (pubkey.go:34-60) as a batch of one on the
        GPU: len(sig) != 64 -> False; the key is copied into a zeroed 32-byte
        array (shorter keys zero-padded, longer ones truncated) as Go's copy()
        does."""
        if len(sig) != SIGNATURE_SIZE:
            return False
        key = (bytes(self) + bytes(PUBKEY_SIZE))[:PUBKEY_SIZE]
        ctx = ctx or default_context()
        m, off = pack_messages([bytes(msg)])
        v = ctx.verify_sr25519(np.frombuffer(key, np.uint8), np.frombuffer(bytes(sig), np.uint8), m, off)
        return bool(v[0])


class Sr25519BatchVerifier:
    """Batch form of sr25519 PubKey.VerifySignature with the BatchVerifier
    shape (add / verify -> (bool, list[bool])); every verdict comes from the
    GPU kernel, entries with a wrong signature length are invalid."""

    def __init__(self, ctx: Context | None = None):
        self.ctx = ctx or default_context()
        self.reset()

    def __len__(self):
        return len(self._msgs)

    def reset(self):
        self._pk, self._sig, self._msgs, self._len_ok = [], [], [], []

    def add(self, key: bytes, msg: bytes, sig: bytes) -> None:
        self._pk.append((bytes(key) + bytes(PUBKEY_SIZE))[:PUBKEY_SIZE])
        self._len_ok.append(len(sig) == SIGNATURE_SIZE)
        self._sig.append(bytes(sig) if len(sig) == SIGNATURE_SIZE else bytes(SIGNATURE_SIZE))
        self._msgs.append(bytes(msg))

    def verify(self):
        n = len(self._msgs)
        if n == 0:
            return True, []
        m, off = pack_messages(self._msgs)
        pk = np.frombuffer(b"".join(self._pk), np.uint8)
        sig = np.frombuffer(b"".join(self._sig), np.uint8)
        v = self.ctx.verify_sr25519(pk, sig, m, off)
        out = [bool(x) and ok for x, ok in zip(v, self._len_ok)]
        return all(out), out


class BatchVerifier:
    """crypto.BatchVerifier (upstream v0.38): Add(key, msg, sig) then
    Verify() -> (bool, list[bool]). Malformed entries are accepted by add() and
    come back invalid; a wrong-length key is also reported by bad_key_index so
    a caller replaying the reference loop can raise at the same index."""

    def __init__(self, ctx: Context | None = None, mode: int = MODE_GO_STDLIB):
        self.ctx = ctx or default_context()
        self.mode = mode
        h = ctypes.c_void_p()
        N.check(N.lib().cmtv_batch_new(self.ctx.handle, mode, ctypes.byref(h)), "cmtv_batch_new")
        self._h = h
        self.bad_key_index = -1

    def __del__(self):
        try:
            if self._h:
                N.lib().cmtv_batch_free(self._h)
                self._h = None
        except Exception:
            pass

    def __len__(self):
        return N.lib().cmtv_batch_len(self._h)

    def add(self, key: bytes, msg: bytes, sig: bytes) -> None:
        k = np.frombuffer(bytes(key) + b"\0", np.uint8)
        m = np.frombuffer(bytes(msg) + b"\0", np.uint8)
        s = np.frombuffer(bytes(sig) + b"\0", np.uint8)
        N.check(N.lib().cmtv_batch_add(self._h, _u8(k), len(key), _u8(m), len(msg), _u8(s), len(sig)),
                "cmtv_batch_add")

    def verify(self):
        n = len(self)
        out = np.zeros(max(n, 1), np.uint8)
        ok = ctypes.c_int(0)
        bad = ctypes.c_int64(-1)
        N.check(N.lib().cmtv_batch_verify(self._h, _u8(out), ctypes.byref(ok), ctypes.byref(bad)),
                "cmtv_batch_verify")
        self.bad_key_index = bad.value
        return bool(ok.value), [bool(x) for x in out[:n]]

    def reset(self):
        N.lib().cmtv_batch_reset(self._h)


def new_batch_verifier(ctx: Context | None = None, mode: int = MODE_GO_STDLIB) -> BatchVerifier:
    """ed25519.NewBatchVerifier() (upstream)."""
    return BatchVerifier(ctx, mode)
