"""ctypes binding of libcmtverify.so (include/cmtverify.h).

The shared library is built in-tree (`cometbft_amd/libcmtverify.so`, see
`__graft_entry__.build()`); there is no fallback: if it is missing or the device
cannot be opened, calls raise.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CMTV_LIBRARY") or os.path.join(_HERE, "libcmtverify.so")

CMTV_OK = 0
CMTV_EINVAL = -1
CMTV_ENODEV = -2
CMTV_ENOMEM = -3
CMTV_EHIP = -4
CMTV_ERCCL = -5
CMTV_ECOMMIT = -6

MODE_GO_STDLIB = 0
MODE_ZIP215 = 1

VERIFY_COMMIT = 0
VERIFY_COMMIT_LIGHT = 1
VERIFY_COMMIT_LIGHT_TRUSTING = 2

COMMIT_OK = 0
COMMIT_ERR_SET_SIZE = 1
COMMIT_ERR_HEIGHT = 2
COMMIT_ERR_BLOCK_ID = 3
COMMIT_ERR_WRONG_SIGNATURE = 4
COMMIT_ERR_NOT_ENOUGH_POWER = 5
COMMIT_ERR_DOUBLE_VOTE = 6
CMTV_KEYS_WIDE = 1
COMMIT_ERR_TRUST_LEVEL = 7
COMMIT_PANIC_BAD_PUBKEY = 8
COMMIT_PANIC_UNKNOWN_FLAG = 9

# every symbol include/cmtverify.h declares (checked by tests/test_abi.py)
EXPORTS = (
    "cmtv_open", "cmtv_open_devices", "cmtv_device_count", "cmtv_device_ordinal", "cmtv_device_stream", "cmtv_sync",
    "cmtv_verify_ed25519_sharded_device", "cmtv_verify_ed25519_indexed_sharded_device", "cmtv_verify_ed25519_multi_device", "cmtv_close", "cmtv_strerror", "cmtv_abi_version", "cmtv_stats_get", "cmtv_device_stats_get", "cmtv_stream",
    "cmtv_verify_ed25519", "cmtv_verify_ed25519_device", "cmtv_verify_sr25519", "cmtv_verify_sr25519_device",
    "cmtv_register_keys", "cmtv_register_keys_ex", "cmtv_keyset_free", "cmtv_keyset_len", "cmtv_verify_ed25519_indexed",
    "cmtv_verify_ed25519_indexed_device",
    "cmtv_batch_new", "cmtv_batch_add", "cmtv_batch_len", "cmtv_batch_verify", "cmtv_batch_reset",
    "cmtv_batch_free", "cmtv_verify_commit", "cmtv_verify_commits", "cmtv_verdict_cache", "cmtv_keyset_cache", "cmtv_vote_sign_bytes", "cmtv_pubkeys_ed25519", "cmtv_sign_ed25519",
    "cmtv_alloc_pinned", "cmtv_free_pinned",
)


class CmtvError(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        self.code = code
        msg = lib().cmtv_strerror(code).decode() if _lib is not None else str(code)
        super().__init__(f"{what}: {msg} ({code})" if what else f"{msg} ({code})")


class cmtv_config(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("default_mode", ctypes.c_uint32),
                ("flags", ctypes.c_uint32), ("reserved", ctypes.c_uint32)]


class cmtv_stats(ctypes.Structure):
    _fields_ = [("calls", ctypes.c_uint64), ("signatures", ctypes.c_uint64), ("invalid", ctypes.c_uint64),
                ("kernel_launches", ctypes.c_uint64), ("device_ms", ctypes.c_double),
                ("last_kernel_ms", ctypes.c_double), ("cache_hits", ctypes.c_uint64),
                ("cache_entries", ctypes.c_uint64), ("keyed_launches", ctypes.c_uint64),
                ("sharded_calls", ctypes.c_uint64), ("gathers", ctypes.c_uint64),
                ("faults_injected", ctypes.c_uint64), ("n_devices", ctypes.c_uint32), ("rccl", ctypes.c_uint32),
                ("fused_sign_bytes", ctypes.c_uint64), ("device_failures", ctypes.c_uint64),
                ("reshards", ctypes.c_uint64), ("late_k_waves", ctypes.c_uint64),
                ("live_devices", ctypes.c_uint32), ("reserved", ctypes.c_uint32),
                ("timed_calls", ctypes.c_uint64), ("rccl_failures", ctypes.c_uint64),
                ("polled_calls", ctypes.c_uint64), ("direct_chunks", ctypes.c_uint64),
                ("masked_chunks", ctypes.c_uint64), ("isolated_calls", ctypes.c_uint64)]


class cmtv_device_stats(ctypes.Structure):
    _fields_ = [("ordinal", ctypes.c_int32), ("failed", ctypes.c_uint32), ("calls", ctypes.c_uint64),
                ("signatures", ctypes.c_uint64), ("kernel_launches", ctypes.c_uint64),
                ("device_ms", ctypes.c_double), ("timed_calls", ctypes.c_uint64)]


_u8p = ctypes.POINTER(ctypes.c_uint8)


class cmtv_block_id(ctypes.Structure):
    _fields_ = [("hash", _u8p), ("hash_len", ctypes.c_uint32), ("psh_total", ctypes.c_uint32),
                ("psh_hash", _u8p), ("psh_hash_len", ctypes.c_uint32)]


class cmtv_commit(ctypes.Structure):
    _fields_ = [("height", ctypes.c_int64), ("round", ctypes.c_int32), ("block_id", cmtv_block_id),
                ("n_sigs", ctypes.c_uint32), ("flags", _u8p), ("ts_seconds", ctypes.POINTER(ctypes.c_int64)),
                ("ts_nanos", ctypes.POINTER(ctypes.c_int32)), ("sigs", _u8p),
                ("sig_off", ctypes.POINTER(ctypes.c_uint32)), ("val_addrs", _u8p)]


class cmtv_valset(ctypes.Structure):
    _fields_ = [("n_vals", ctypes.c_uint32), ("pubkeys", _u8p), ("pk_off", ctypes.POINTER(ctypes.c_uint32)),
                ("voting_power", ctypes.POINTER(ctypes.c_int64)), ("addrs", _u8p),
                ("proposer_priority", ctypes.POINTER(ctypes.c_int64))]


class cmtv_commit_result(ctypes.Structure):
    _fields_ = [("code", ctypes.c_int32), ("sig_index", ctypes.c_int32), ("got", ctypes.c_int64),
                ("needed", ctypes.c_int64), ("n_verified", ctypes.c_uint32), ("reserved", ctypes.c_uint32)]


_lib = None


def lib() -> ctypes.CDLL:
    """Load libcmtverify.so; raises if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    L = ctypes.CDLL(LIB_PATH)
    vp, sz, u32, i32, u64, i64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_int32, ctypes.c_uint64, ctypes.c_int64
    u32p = ctypes.POINTER(ctypes.c_uint32)
    L.cmtv_open.argtypes = [ctypes.POINTER(cmtv_config), ctypes.POINTER(vp)]
    L.cmtv_open.restype = ctypes.c_int
    vpp = ctypes.POINTER(vp)
    szp = ctypes.POINTER(sz)
    L.cmtv_open_devices.argtypes = [ctypes.POINTER(cmtv_config), ctypes.POINTER(i32), sz, ctypes.POINTER(vp)]
    L.cmtv_open_devices.restype = ctypes.c_int
    L.cmtv_device_count.argtypes = [vp]
    L.cmtv_device_count.restype = ctypes.c_int
    L.cmtv_device_ordinal.argtypes = [vp, ctypes.c_int]
    L.cmtv_device_ordinal.restype = ctypes.c_int
    L.cmtv_device_stream.argtypes = [vp, ctypes.c_int]
    L.cmtv_device_stream.restype = vp
    L.cmtv_sync.argtypes = [vp]
    L.cmtv_sync.restype = ctypes.c_int
    L.cmtv_verify_ed25519_sharded_device.argtypes = [vp, szp, vpp, vpp, vpp, vpp, u32, vpp, vpp, szp]
    L.cmtv_verify_ed25519_sharded_device.restype = ctypes.c_int
    L.cmtv_verify_ed25519_multi_device.argtypes = [vp, szp, vpp, vpp, vpp, vpp, u32, vpp, vpp]
    L.cmtv_verify_ed25519_multi_device.restype = ctypes.c_int
    L.cmtv_verify_ed25519_indexed_sharded_device.argtypes = [vp, vp, szp, vpp, vpp, vpp, vpp, u32, vpp, vpp, szp]
    L.cmtv_verify_ed25519_indexed_sharded_device.restype = ctypes.c_int
    L.cmtv_close.argtypes = [vp]
    L.cmtv_close.restype = None
    L.cmtv_strerror.argtypes = [ctypes.c_int]
    L.cmtv_strerror.restype = ctypes.c_char_p
    L.cmtv_abi_version.argtypes = []
    L.cmtv_abi_version.restype = ctypes.c_int
    L.cmtv_stats_get.argtypes = [vp, ctypes.POINTER(cmtv_stats)]
    L.cmtv_stats_get.restype = ctypes.c_int
    L.cmtv_device_stats_get.argtypes = [vp, ctypes.c_int, ctypes.POINTER(cmtv_device_stats)]
    L.cmtv_device_stats_get.restype = ctypes.c_int
    L.cmtv_stream.argtypes = [vp]
    L.cmtv_stream.restype = vp
    L.cmtv_verify_ed25519.argtypes = [vp, sz, _u8p, _u8p, _u8p, u32p, u32, _u8p, ctypes.POINTER(u64)]
    L.cmtv_verify_ed25519.restype = ctypes.c_int
    L.cmtv_verify_ed25519_device.argtypes = [vp, sz, vp, vp, vp, vp, u32, vp, vp, vp]
    L.cmtv_verify_ed25519_device.restype = ctypes.c_int
    L.cmtv_verify_sr25519.argtypes = [vp, sz, _u8p, _u8p, _u8p, u32p, _u8p, ctypes.POINTER(u64)]
    L.cmtv_verify_sr25519.restype = ctypes.c_int
    L.cmtv_verify_sr25519_device.argtypes = [vp, sz, vp, vp, vp, vp, vp, vp, vp]
    L.cmtv_verify_sr25519_device.restype = ctypes.c_int
    L.cmtv_register_keys.argtypes = [vp, sz, _u8p, ctypes.POINTER(vp)]
    L.cmtv_register_keys.restype = ctypes.c_int
    L.cmtv_register_keys_ex.argtypes = [vp, sz, _u8p, ctypes.c_uint32, ctypes.POINTER(vp)]
    L.cmtv_register_keys_ex.restype = ctypes.c_int
    L.cmtv_keyset_free.argtypes = [vp]
    L.cmtv_keyset_free.restype = None
    L.cmtv_keyset_len.argtypes = [vp]
    L.cmtv_keyset_len.restype = sz
    L.cmtv_verify_ed25519_indexed.argtypes = [vp, vp, sz, u32p, _u8p, _u8p, u32p, u32, _u8p, ctypes.POINTER(u64)]
    L.cmtv_verify_ed25519_indexed.restype = ctypes.c_int
    L.cmtv_verify_ed25519_indexed_device.argtypes = [vp, vp, sz, vp, vp, vp, vp, u32, vp, vp, vp]
    L.cmtv_verify_ed25519_indexed_device.restype = ctypes.c_int
    L.cmtv_batch_new.argtypes = [vp, u32, ctypes.POINTER(vp)]
    L.cmtv_batch_new.restype = ctypes.c_int
    L.cmtv_batch_add.argtypes = [vp, _u8p, sz, _u8p, sz, _u8p, sz]
    L.cmtv_batch_add.restype = ctypes.c_int
    L.cmtv_batch_len.argtypes = [vp]
    L.cmtv_batch_len.restype = sz
    L.cmtv_batch_verify.argtypes = [vp, _u8p, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(i64)]
    L.cmtv_batch_verify.restype = ctypes.c_int
    L.cmtv_batch_reset.argtypes = [vp]
    L.cmtv_batch_reset.restype = None
    L.cmtv_batch_free.argtypes = [vp]
    L.cmtv_batch_free.restype = None
    L.cmtv_verify_commit.argtypes = [vp, u32, u32, ctypes.c_char_p, sz, ctypes.POINTER(cmtv_valset),
                                     ctypes.POINTER(cmtv_block_id), i64, ctypes.POINTER(cmtv_commit), u64, u64,
                                     ctypes.POINTER(cmtv_commit_result), ctypes.c_char_p, sz]
    L.cmtv_verify_commit.restype = ctypes.c_int
    L.cmtv_verify_commits.argtypes = [vp, u32, u32, ctypes.c_char_p, sz, sz, ctypes.POINTER(cmtv_valset),
                                      ctypes.POINTER(cmtv_block_id), ctypes.POINTER(i64), ctypes.POINTER(cmtv_commit),
                                      u64, u64, ctypes.POINTER(cmtv_commit_result), ctypes.POINTER(ctypes.c_int),
                                      ctypes.c_char_p, sz]
    L.cmtv_verify_commits.restype = ctypes.c_int
    L.cmtv_keyset_cache.argtypes = [vp, sz]
    L.cmtv_keyset_cache.restype = ctypes.c_int
    L.cmtv_verdict_cache.argtypes = [vp, sz]
    L.cmtv_verdict_cache.restype = ctypes.c_int
    L.cmtv_vote_sign_bytes.argtypes = [ctypes.c_char_p, sz, i32, i64, i32, ctypes.POINTER(cmtv_block_id), i64, i32,
                                       _u8p, sz]
    L.cmtv_vote_sign_bytes.restype = i64
    L.cmtv_pubkeys_ed25519.argtypes = [vp, sz, _u8p, _u8p]
    L.cmtv_pubkeys_ed25519.restype = ctypes.c_int
    L.cmtv_sign_ed25519.argtypes = [vp, sz, _u8p, u32p, _u8p, u32p, _u8p]
    L.cmtv_sign_ed25519.restype = ctypes.c_int
    L.cmtv_alloc_pinned.argtypes = [vp, sz, ctypes.POINTER(vp)]
    L.cmtv_alloc_pinned.restype = ctypes.c_int
    L.cmtv_free_pinned.argtypes = [vp, vp]
    L.cmtv_free_pinned.restype = ctypes.c_int
    _lib = L
    return L


def check(rc: int, what: str = "") -> int:
    if rc < 0 and rc != CMTV_ECOMMIT:
        raise CmtvError(rc, what)
    return rc
