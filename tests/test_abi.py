"""CPU tests of the C-ABI library (no GPU compute): it loads, exports every
symbol include/cmtverify.h declares, fails loudly without a device, and its
host-side pieces (sign-bytes encoder, argument checks) behave."""
import ctypes
import os
import re

import numpy as np
import pytest

from cometbft_amd import _native as N
from cometbft_amd import types as T
from oracle import signbytes as SB

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    with open(os.path.join(ROOT, "include", "cmtverify.h")) as f:
        src = f.read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(cmtv_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    lib = N.lib()
    declared = _declared_symbols()
    assert len(declared) >= 18
    missing = [s for s in declared if not hasattr(lib, s)]
    assert not missing, missing
    assert set(declared) == set(N.EXPORTS)


def test_abi_version_and_strerror():
    lib = N.lib()
    assert lib.cmtv_abi_version() == 11
    for code in (N.CMTV_OK, N.CMTV_EINVAL, N.CMTV_ENODEV, N.CMTV_ENOMEM, N.CMTV_EHIP, N.CMTV_ERCCL, N.CMTV_ECOMMIT):
        assert lib.cmtv_strerror(code)


def test_open_without_gpu_fails_loudly():
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from cometbft_amd import Context

    with pytest.raises(N.CmtvError) as ei:
        Context()
    assert ei.value.code == N.CMTV_ENODEV


def test_null_context_is_einval():
    lib = N.lib()
    assert lib.cmtv_verify_ed25519(None, 1, None, None, None, None, 0, None, None) == N.CMTV_EINVAL
    assert lib.cmtv_batch_new(None, 0, ctypes.byref(ctypes.c_void_p())) == N.CMTV_EINVAL
    assert lib.cmtv_open(None, None) == N.CMTV_EINVAL


def test_sign_bytes_encoder_matches_oracle_randomized():
    rng = np.random.default_rng(11)
    for _ in range(300):
        chain = "".join(chr(int(c)) for c in rng.integers(97, 123, int(rng.integers(0, 51))))
        vtype = int(rng.choice([0, 1, 2, 32]))
        height = int(rng.integers(-2**40, 2**40))
        round_ = int(rng.integers(-5, 2**20))
        if rng.random() < 0.3:
            bid = None
        else:
            bid = (rng.integers(0, 256, int(rng.choice([0, 32])), dtype=np.uint8).tobytes(),
                   int(rng.integers(0, 2**32)), rng.integers(0, 256, int(rng.choice([0, 32])), dtype=np.uint8).tobytes())
        sec = int(rng.choice([0, SB.GO_ZERO_TIME_SECONDS, int(rng.integers(0, 2**34))]))
        nanos = int(rng.choice([0, int(rng.integers(0, 10**9))]))
        want = SB.vote_sign_bytes(chain, vtype, height, round_, bid, sec, nanos)
        b = T.BlockID(bid[0], T.PartSetHeader(bid[1], bid[2])) if bid else None
        got = T.vote_sign_bytes(chain, vtype, height, round_, b, sec, nanos)
        assert got == want


def test_sign_bytes_kat_through_library():
    import json

    with open(os.path.join(ROOT, "tests", "golden", "signbytes_kat.json")) as f:
        kat = json.load(f)
    for c in kat["cases"]:
        got = T.vote_sign_bytes(c["chain_id"], c["type"], c["height"], c["round"], None,
                                kat["go_zero_time_seconds"], 0)
        assert got.hex() == c["want"].replace(" ", "")


def test_commit_vote_sign_bytes_lengths():
    """commit vote = 109..161 B, nil vote 41..42 B with this template."""
    from cometbft_amd import testutil as TU

    msgs = TU.commit_messages(64, 1000)
    assert all(100 <= len(m) <= 161 for m in msgs)
    nil = TU.commit_messages(4, 1000, flags=[T.BLOCK_ID_FLAG_NIL] * 4)
    assert all(len(m) < 50 for m in nil)


def test_keyset_entry_points_reject_bad_arguments_without_gpu():
    lib = N.lib()
    ks = ctypes.c_void_p()
    assert lib.cmtv_register_keys(None, 1, None, ctypes.byref(ks)) == N.CMTV_EINVAL
    assert lib.cmtv_register_keys(None, 1, None, None) == N.CMTV_EINVAL
    assert lib.cmtv_register_keys_ex(None, 1, None, N.CMTV_KEYS_WIDE, ctypes.byref(ks)) == N.CMTV_EINVAL
    assert lib.cmtv_keyset_len(None) == 0
    lib.cmtv_keyset_free(None)
    assert lib.cmtv_verify_ed25519_indexed(None, None, 1, None, None, None, None, 0, None, None) == N.CMTV_EINVAL
    assert lib.cmtv_verify_ed25519_indexed_device(None, None, 1, None, None, None, None, 0, None, None,
                                                  None) == N.CMTV_EINVAL


def test_multi_device_entry_points_reject_bad_arguments_without_gpu():
    lib = N.lib()
    h = ctypes.c_void_p()
    assert lib.cmtv_open_devices(None, None, 0, None) == N.CMTV_EINVAL
    assert lib.cmtv_open_devices(None, None, 3, ctypes.byref(h)) == N.CMTV_EINVAL  # n > 0 needs a list
    assert lib.cmtv_device_count(None) == 0
    assert lib.cmtv_device_ordinal(None, 0) == N.CMTV_EINVAL
    assert lib.cmtv_device_stream(None, 0) is None
    assert lib.cmtv_sync(None) == N.CMTV_EINVAL
    assert lib.cmtv_verify_ed25519_sharded_device(None, None, None, None, None, None, 0, None, None,
                                                  None) == N.CMTV_EINVAL
    assert lib.cmtv_verify_ed25519_indexed_sharded_device(None, None, None, None, None, None, None, 0, None, None,
                                                          None) == N.CMTV_EINVAL
    assert lib.cmtv_verify_ed25519_multi_device(None, None, None, None, None, None, 0, None, None) == N.CMTV_EINVAL


def test_open_devices_without_gpu_is_enodev():
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    arr = (ctypes.c_int32 * 2)(0, 1)
    h = ctypes.c_void_p()
    assert N.lib().cmtv_open_devices(None, arr, 2, ctypes.byref(h)) == N.CMTV_ENODEV


def test_rccl_stub_exports_what_the_library_binds():
    """tests/host/librccl_stub.so (the multi-rank rehearsal's RCCL double,
    selected by CMTV_RCCL_LIB) exports the five entry points runtime.cpp
    load_rccl resolves, and rejects bad arguments like RCCL (no device
    work: a NULL communicator list is ncclInvalidArgument)."""
    path = os.path.join(ROOT, "tests", "host", "librccl_stub.so")
    if not os.path.exists(path):
        pytest.skip("librccl_stub.so not built (make -C cometbft_amd/csrc stub)")
    stub = ctypes.CDLL(path)
    syms = {"ncclCommInitAll", "ncclCommDestroy", "ncclAllGather", "ncclGroupStart", "ncclGroupEnd", "ncclCommAbort"}
    for sym in syms:
        assert hasattr(stub, sym), sym
    src = open(os.path.join(ROOT, "cometbft_amd", "csrc", "runtime.cpp")).read()
    bound = set(re.findall(r'dlsym\(h, "(nccl[A-Za-z]+)"\)', src))
    assert bound == syms
    assert stub.ncclCommInitAll(None, 2, None) == 4  # ncclInvalidArgument
    assert stub.ncclGroupEnd() == 5                  # unbalanced: ncclInvalidUsage
    assert stub.ncclGroupStart() == 0 and stub.ncclGroupEnd() == 0
