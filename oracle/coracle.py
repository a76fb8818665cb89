"""ctypes loader for the C oracle (oracle/liboracle.so) -- TEST INFRASTRUCTURE ONLY.

Used by tests/, __graft_entry__.smoke() (as the checker) and bench.py's
cpu_baseline leg. Never imported by the product package.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "liboracle.so")
_lib = None


def build() -> str:
    subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build()
        L = ctypes.CDLL(_LIB)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        u32p = ctypes.POINTER(ctypes.c_uint32)
        L.oracle_verify_batch.argtypes = [ctypes.c_size_t, u8p, u8p, u8p, u32p, ctypes.c_int, u8p, ctypes.c_int]
        L.oracle_verify_batch.restype = None
        L.oracle_sign_batch.argtypes = [ctypes.c_size_t, u8p, u32p, u8p, u32p, u8p, ctypes.c_int]
        L.oracle_sign_batch.restype = None
        L.oracle_pubkey_from_seed.argtypes = [u8p, u8p]
        L.oracle_pubkey_from_seed.restype = None
        L.oracle_sr25519_verify_batch.argtypes = [ctypes.c_size_t, u8p, u8p, u8p, u32p, u8p, ctypes.c_int]
        L.oracle_sr25519_verify_batch.restype = None
        L.oracle_sr25519_pubkey.argtypes = [u8p, u8p]
        L.oracle_sr25519_pubkey.restype = None
        L.oracle_sr25519_sign_batch.argtypes = [ctypes.c_size_t, u8p, u32p, u8p, u32p, u8p]
        L.oracle_sr25519_sign_batch.restype = None
        L.oracle_sr25519_challenge_batch.argtypes = [ctypes.c_size_t, u8p, u8p, u8p, u32p, u8p]
        L.oracle_sr25519_challenge_batch.restype = None
        _lib = L
    return _lib


def _p(a: np.ndarray, t=ctypes.c_uint8):
    return a.ctypes.data_as(ctypes.POINTER(t))


def pack_msgs(msgs):
    off = np.zeros(len(msgs) + 1, dtype=np.uint32)
    off[1:] = np.cumsum([len(m) for m in msgs], dtype=np.uint64).astype(np.uint32)
    buf = np.frombuffer(b"".join(msgs) + b"\0", dtype=np.uint8).copy()
    return buf, off


def verify_batch(pk: np.ndarray, sig: np.ndarray, msg: np.ndarray, off: np.ndarray, mode: int,
                 nthreads: int = 1) -> np.ndarray:
    n = len(off) - 1
    pk = np.ascontiguousarray(pk, dtype=np.uint8)
    sig = np.ascontiguousarray(sig, dtype=np.uint8)
    msg = np.ascontiguousarray(msg, dtype=np.uint8)
    if msg.size == 0:
        msg = np.zeros(1, np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint32)
    out = np.zeros(max(n, 1), dtype=np.uint8)
    lib().oracle_verify_batch(n, _p(pk), _p(sig), _p(msg), _p(off, ctypes.c_uint32), mode, _p(out), nthreads)
    return out[:n]


def pubkeys_from_seeds(seeds: np.ndarray) -> np.ndarray:
    seeds = np.ascontiguousarray(seeds, dtype=np.uint8).reshape(-1, 32)
    out = np.zeros_like(seeds)
    for i in range(len(seeds)):
        lib().oracle_pubkey_from_seed(_p(seeds[i]), _p(out[i]))
    return out


def sign_batch(seeds: np.ndarray, msg: np.ndarray, off: np.ndarray, key_idx=None, nthreads: int = 1) -> np.ndarray:
    n = len(off) - 1
    seeds = np.ascontiguousarray(seeds, dtype=np.uint8)
    msg = np.ascontiguousarray(msg, dtype=np.uint8)
    if msg.size == 0:
        msg = np.zeros(1, np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint32)
    out = np.zeros((max(n, 1), 64), dtype=np.uint8)
    kp = None
    if key_idx is not None:
        key_idx = np.ascontiguousarray(key_idx, dtype=np.uint32)
        kp = _p(key_idx, ctypes.c_uint32)
    lib().oracle_sign_batch(n, _p(seeds), kp, _p(msg), _p(off, ctypes.c_uint32), _p(out), nthreads)
    return out[:n]


# ---- sr25519 (schnorrkel / ristretto255): crypto/sr25519/pubkey.go:34-60

def sr25519_verify_batch(pk: np.ndarray, sig: np.ndarray, msg: np.ndarray, off: np.ndarray,
                         nthreads: int = 1) -> np.ndarray:
    n = len(off) - 1
    pk = np.ascontiguousarray(pk, dtype=np.uint8)
    sig = np.ascontiguousarray(sig, dtype=np.uint8)
    msg = np.ascontiguousarray(msg, dtype=np.uint8)
    if msg.size == 0:
        msg = np.zeros(1, np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint32)
    out = np.zeros(max(n, 1), dtype=np.uint8)
    lib().oracle_sr25519_verify_batch(n, _p(pk), _p(sig), _p(msg), _p(off, ctypes.c_uint32), _p(out), nthreads)
    return out[:n]


def sr25519_pubkeys(minis: np.ndarray) -> np.ndarray:
    minis = np.ascontiguousarray(minis, dtype=np.uint8).reshape(-1, 32)
    out = np.zeros_like(minis)
    for i in range(len(minis)):
        lib().oracle_sr25519_pubkey(_p(minis[i]), _p(out[i]))
    return out


def sr25519_sign_batch(minis: np.ndarray, msg: np.ndarray, off: np.ndarray, key_idx=None) -> np.ndarray:
    n = len(off) - 1
    minis = np.ascontiguousarray(minis, dtype=np.uint8)
    msg = np.ascontiguousarray(msg, dtype=np.uint8)
    if msg.size == 0:
        msg = np.zeros(1, np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint32)
    out = np.zeros((max(n, 1), 64), dtype=np.uint8)
    kp = None
    if key_idx is not None:
        key_idx = np.ascontiguousarray(key_idx, dtype=np.uint32)
        kp = _p(key_idx, ctypes.c_uint32)
    lib().oracle_sr25519_sign_batch(n, _p(minis), kp, _p(msg), _p(off, ctypes.c_uint32), _p(out))
    return out[:n]


def sr25519_challenges(pk: np.ndarray, R: np.ndarray, msg: np.ndarray, off: np.ndarray) -> np.ndarray:
    """The merlin challenge k (32-byte little-endian, reduced mod L) of each
    (pk, R, msg) triple, as sr25519 verification computes it."""
    n = len(off) - 1
    pk = np.ascontiguousarray(pk, dtype=np.uint8)
    R = np.ascontiguousarray(R, dtype=np.uint8)
    msg = np.ascontiguousarray(msg, dtype=np.uint8)
    if msg.size == 0:
        msg = np.zeros(1, np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint32)
    out = np.zeros((max(n, 1), 32), dtype=np.uint8)
    lib().oracle_sr25519_challenge_batch(n, _p(pk), _p(R), _p(msg), _p(off, ctypes.c_uint32), _p(out))
    return out[:n]
