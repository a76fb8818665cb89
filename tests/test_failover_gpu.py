"""GPU tests of the runtime's failure handling:

  * k_verify_keyed_quad_split's bounded wait for its hash helper never decides
    a verdict: with CMTV_FORCE_K_LATE=1 every quad wave stops waiting at once
    and hashes its own signatures; host, device-resident and VerifyCommit
    (keyset cache) calls stay oracle-exact and cmtv_stats.late_k_waves counts
    the waves that did so (0 without the knob);
  * a device that fails (CMTV_FAULT_DEV=g, the libs/fail/fail.go:9-39
    analogue, SURVEY.md 5 "per-GPU failure -> re-shard onto the remaining
    GPUs") is retired: the batch is re-planned over the other devices inside
    the same call and returns the oracle's verdicts, device_failures and
    reshards count it, later batches avoid it, and device-resident calls that
    need it return CMTV_ENODEV;
  * partial-device shard plans: a batch uses as many devices as get
    CMTV_SHARD_MIN signatures each (cmtv_device_stats shows which ran).
Multi-device contexts here are over a repeated ordinal (one-GPU box)."""
import numpy as np
import pytest

from oracle import coracle
from cometbft_amd import MODE_GO_STDLIB, MODE_ZIP215, Context
from cometbft_amd import _native as N
from cometbft_amd import testutil as TU
from test_runtime_gpu import _batch, _env

pytestmark = pytest.mark.gpu


def _err(fn):
    try:
        fn()
    except Exception as e:  # noqa: BLE001 -- the reference's error value
        return e
    return None


@pytest.mark.parametrize("n", [48, 1000, 12_289])
def test_keyed_split_late_hash_is_exact(n):
    import torch

    # the keyed quad kernel at every size (n <= 512 would take the keyed row
    # kernel, whose helper hands k over at a barrier, no bounded wait)
    with _env(CMTV_FORCE_K_LATE=1, CMTV_FORM="kquad"):
        late = Context(device=0)
    pk, kidx, sig, m, off = _batch(n, 300 + n, nkeys=150)
    ks = late.register_keys(pk)
    for mode in (MODE_GO_STDLIB, MODE_ZIP215):
        exp = coracle.verify_batch(pk[kidx], sig, m, off, mode, nthreads=16)
        got, words = late.verify_indexed(ks, kidx, sig, m, off, mode, bitmap=True)
        assert np.array_equal(got, exp), np.nonzero(got != exp)[0][:10]
        assert np.array_equal(np.unpackbits(words.view(np.uint8), bitorder="little")[:n], exp)
    waves = 3 * ((4 * ((n + 63) // 64) + 2) // 3)  # the kernel's quad waves per launch
    assert late.stats()["late_k_waves"] >= 2 * waves
    # the device-resident entry point, on its own stream
    dev = torch.device("cuda:0")
    t = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in
         {"idx": kidx, "sig": sig, "m": m, "off": off.view(np.int32)}.items()}
    v = torch.zeros(n, dtype=torch.uint8, device=dev)
    s = torch.cuda.Stream(device=dev)
    late.verify_indexed_device(ks, n, t["idx"].data_ptr(), t["sig"].data_ptr(), t["m"].data_ptr(),
                               t["off"].data_ptr(), MODE_GO_STDLIB, v.data_ptr(), 0, stream=s.cuda_stream)
    s.synchronize()
    assert np.array_equal(v.cpu().numpy(), coracle.verify_batch(pk[kidx], sig, m, off, MODE_GO_STDLIB, nthreads=16))
    ks.free()


def test_keyed_split_waits_without_the_knob(gpu_ctx):
    pk, kidx, sig, m, off = _batch(2000, 31, nkeys=150)
    ctx = Context(device=0)
    ks = ctx.register_keys(pk)
    exp = coracle.verify_batch(pk[kidx], sig, m, off, MODE_GO_STDLIB, nthreads=16)
    assert np.array_equal(ctx.verify_indexed(ks, kidx, sig, m, off, MODE_GO_STDLIB), exp)
    assert ctx.stats()["late_k_waves"] == 0
    ks.free()


def test_verify_commit_keyset_cache_late_hash():
    """VerifyCommit with the keyset cache (the keyed split kernel) under
    CMTV_FORCE_K_LATE: a valid commit verifies, a flipped signature gives the
    reference's 'wrong signature (#i)' at the right index, never another."""
    # the keyed quad kernel at every size (n <= 512 would take the keyed row
    # kernel, whose helper hands k over at a barrier, no bounded wait)
    with _env(CMTV_FORCE_K_LATE=1, CMTV_FORM="kquad"):
        late = Context(device=0)
    late.keyset_cache(2)
    plain = Context(device=0)
    sv = TU.make_validator_set(plain, 150)
    bid = TU.block_id_for_height(500)
    commit, _, _ = TU.make_commit(plain, sv, 500)
    for _ in range(2):  # first call registers the set, second verifies by key index
        assert sv.valset.verify_commit(TU.CHAIN_ID, bid, 500, commit, ctx=late) is None
    s = bytearray(commit.signatures[101].signature)
    s[40] ^= 2
    commit.signatures[101].signature = bytes(s)
    e_late = _err(lambda: sv.valset.verify_commit(TU.CHAIN_ID, bid, 500, commit, ctx=late))
    e_ref = _err(lambda: sv.valset.verify_commit(TU.CHAIN_ID, bid, 500, commit, ctx=plain))
    assert e_late is not None and str(e_late) == str(e_ref) and "#101" in str(e_late)
    st = late.stats()
    assert st["keyed_launches"] >= 2 and st["late_k_waves"] > 0


@pytest.mark.parametrize("bad", [0, 1, 2])
def test_device_failure_reshards(bad):
    with _env(CMTV_SHARD_MIN=64, CMTV_FAULT_DEV=bad):
        ctx = Context(devices=[0, 0, 0])
    n = 3001
    pk, kidx, sig, m, off = _batch(n, 90 + bad)
    for mode in (MODE_GO_STDLIB, MODE_ZIP215):
        exp = coracle.verify_batch(pk[kidx], sig, m, off, mode, nthreads=16)
        got, words = ctx.verify(pk[kidx], sig, m, off, mode, bitmap=True)
        assert np.array_equal(got, exp), np.nonzero(got != exp)[0][:10]
        assert np.array_equal(np.unpackbits(words.view(np.uint8), bitorder="little")[:n], exp)
    st = ctx.stats()
    assert st["device_failures"] == 1 and st["reshards"] == 1 and st["live_devices"] == 2
    ds = ctx.device_stats()
    assert [d["failed"] for d in ds] == [int(g == bad) for g in range(3)]
    assert ds[bad]["calls"] == 0 and all(ds[g]["calls"] >= 2 for g in range(3) if g != bad)
    # later batches (small, registered keys, commits) run on the survivors
    small = ctx.verify(pk[kidx][:100], sig[:100], m, off[:101])
    assert np.array_equal(small, coracle.verify_batch(pk[kidx][:100], sig[:100], m, off[:101], 0, nthreads=4))
    ks = ctx.register_keys(pk)
    assert np.array_equal(ctx.verify_indexed(ks, kidx, sig, m, off, MODE_GO_STDLIB),
                          coracle.verify_batch(pk[kidx], sig, m, off, MODE_GO_STDLIB, nthreads=16))
    ks.free()
    sv = TU.make_validator_set(ctx, 20)
    commit, _, _ = TU.make_commit(ctx, sv, 9)
    assert sv.valset.verify_commit(TU.CHAIN_ID, TU.block_id_for_height(9), 9, commit, ctx=ctx) is None
    assert ctx.stats()["device_failures"] == 1
    # a device-resident multi-device call needs every device: refused
    with pytest.raises(N.CmtvError) as ei:
        ctx.verify_multi_device([1, 1, 1], [0, 0, 0], [0, 0, 0], [0, 0, 0], [0, 0, 0], MODE_GO_STDLIB, [0, 0, 0])
    assert ei.value.code in (N.CMTV_ENODEV, N.CMTV_EINVAL)


def test_single_device_failure_is_an_error():
    """With nowhere to re-shard, the device's error reaches the caller (the Go
    shim then runs the reference body)."""
    with _env(CMTV_FAULT_DEV=0):
        ctx = Context(devices=[0])
    pk, kidx, sig, m, off = _batch(200, 5)
    with pytest.raises(N.CmtvError) as ei:
        ctx.verify(pk[kidx], sig, m, off)
    assert ei.value.code == N.CMTV_EHIP
    assert ctx.stats()["device_failures"] == 0


def test_partial_device_plan_uses_enough_devices():
    ctx = Context(devices=[0, 0, 0, 0])  # default CMTV_SHARD_MIN = 8192
    n = 20_000
    pk, kidx, sig, m, off = _batch(n, 111, flip=0.02)
    exp = coracle.verify_batch(pk[kidx], sig, m, off, MODE_GO_STDLIB, nthreads=16)
    assert np.array_equal(ctx.verify(pk[kidx], sig, m, off), exp)
    ds = ctx.device_stats()
    assert [d["calls"] > 0 for d in ds] == [True, True, False, False]
    assert ds[0]["signatures"] + ds[1]["signatures"] == n
    st = ctx.stats()
    assert st["sharded_calls"] == 1 and st["gathers"] == 1
