"""GPU tests of the host runtime (cometbft_amd/csrc/runtime.cpp):

  * multi-device contexts (cmtv_open_devices): a one-device
    context equals the single-device path; a context over a REPEATED
    ordinal ([0, 0]) drives the whole sharding machinery on one GPU --
    64-aligned shards, per-device staging and keysets, the bitmap gather (peer
    copies; RCCL needs distinct devices) -- and must return the oracle's
    verdicts, for host batches, registered keys, commits and the sharded
    device-resident entry point;
  * the CMTV_FAULT_AT knob (libs/fail/fail.go:10-25 analogue): the N-th launch
    fails with CMTV_EHIP and the context keeps working;
  * concurrent callers (consensus/state.go:715, light/client.go:474,
    blockchain/v0/reactor.go:255 call VerifyCommit* from several
    goroutines): host-buffer and device-resident calls on different streams,
    lane-kernel sized (shared A-table scratch), from 4 threads at once;
  * the keyset cache takes the registered-key kernel for cross-height
    batches (each commit carries its own copy of the validator set);
  * batches whose sign-bytes exceed the device batch limit are split;
  * safeMul's edge cases (types/validator_set.go:1086-1105).
"""
import os
import threading

import numpy as np
import pytest

from oracle import coracle
from cometbft_amd import MODE_GO_STDLIB, MODE_ZIP215, Context, pack_messages
from cometbft_amd import _native as N
from cometbft_amd import testutil as TU
from cometbft_amd import types as T

pytestmark = pytest.mark.gpu


def _batch(n, seed, nkeys=64, flip=0.1, msg_len=116):
    rng = np.random.default_rng(seed)
    seeds = rng.integers(0, 256, (nkeys, 32), dtype=np.uint8)
    kidx = rng.integers(0, nkeys, n).astype(np.uint32)
    msgs = [rng.integers(0, 256, msg_len, dtype=np.uint8).tobytes() for _ in range(n)]
    m, off = coracle.pack_msgs(msgs)
    sig = coracle.sign_batch(seeds, m, off, key_idx=kidx, nthreads=16).copy()
    rows = np.nonzero(rng.random(n) < flip)[0]
    sig[rows, rng.integers(0, 64, rows.size)] ^= (1 << rng.integers(0, 8, rows.size)).astype(np.uint8)
    pk = coracle.pubkeys_from_seeds(seeds)
    return pk, kidx, sig, m, off


class _env:
    def __init__(self, **kv):
        self.kv = kv

    def __enter__(self):
        self.old = {k: os.environ.get(k) for k in self.kv}
        os.environ.update({k: str(v) for k, v in self.kv.items()})

    def __exit__(self, *a):
        for k, v in self.old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


def test_one_device_context_equals_single_device_path(gpu_ctx, corpus):
    multi = Context(devices=[0])
    assert multi.n_devices == 1 and multi.device_ordinal(0) == 0
    msg, off = pack_messages(corpus["msgs"])
    for mode, key in ((MODE_GO_STDLIB, "go"), (MODE_ZIP215, "zip215")):
        got, words = multi.verify(corpus["pk"], corpus["sig"], msg, off, mode, bitmap=True)
        assert np.array_equal(got, corpus[key])
        assert np.array_equal(words, gpu_ctx.verify(corpus["pk"], corpus["sig"], msg, off, mode, bitmap=True)[1])
    st = multi.stats()
    assert st["n_devices"] == 1 and st["sharded_calls"] == 0


@pytest.mark.parametrize("n", [400, 3001, 50_000])
def test_sharding_over_a_repeated_device(n):
    with _env(CMTV_SHARD_MIN=64):
        ctx = Context(devices=[0, 0, 0])
    assert ctx.n_devices == 3
    pk, kidx, sig, m, off = _batch(n, 20 + n)
    for mode in (MODE_GO_STDLIB, MODE_ZIP215):
        exp = coracle.verify_batch(pk[kidx], sig, m, off, mode, nthreads=16)
        got, words = ctx.verify(pk[kidx], sig, m, off, mode, bitmap=True)
        assert np.array_equal(got, exp), np.nonzero(got != exp)[0][:10]
        assert np.array_equal(np.unpackbits(words.view(np.uint8), bitorder="little")[:n], exp)
        ks = ctx.register_keys(pk)
        assert np.array_equal(ctx.verify_indexed(ks, kidx, sig, m, off, mode), exp)
        ks.free()
    st = ctx.stats()
    assert st["sharded_calls"] >= 4 and st["gathers"] >= 4 and st["rccl"] == 0


def test_sharded_commit_replay_over_a_repeated_device():
    with _env(CMTV_SHARD_MIN=64):
        ctx = Context(devices=[0, 0])
    plain = Context(device=0)
    sv = TU.make_validator_set(plain, 100)
    items = []
    for h in range(300, 306):
        commit, _, _ = TU.make_commit(plain, sv, h)
        if h == 303:
            s = bytearray(commit.signatures[77].signature)
            s[5] ^= 1
            commit.signatures[77].signature = bytes(s)
        items.append((sv.valset, TU.block_id_for_height(h), h, commit))
    for kc in (0, 2):
        ctx.keyset_cache(kc)
        for kind in (N.VERIFY_COMMIT, N.VERIFY_COMMIT_LIGHT):
            a = [None if e is None else str(e) for e in T.verify_commits(kind, TU.CHAIN_ID, items, ctx=ctx)]
            b = [None if e is None else str(e) for e in T.verify_commits(kind, TU.CHAIN_ID, items, ctx=plain)]
            assert a == b
    assert ctx.stats()["sharded_calls"] >= 2


def test_sharded_device_api_over_a_repeated_device():
    import torch

    ctx = Context(devices=[0, 0])
    dev = torch.device("cuda:0")
    shards, exp, d = [], [], []
    for g, n in enumerate((1000, 777)):
        pk, kidx, sig, m, off = _batch(n, 40 + g)
        exp.append(coracle.verify_batch(pk[kidx], sig, m, off, MODE_GO_STDLIB, nthreads=16))
        t = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in
             {"pk": pk[kidx], "sig": sig, "m": m, "off": off.view(np.int32)}.items()}
        d.append(t)
        shards.append(n)
    W = max((n + 63) // 64 for n in shards)
    out = [torch.full((2 * W,), -1, dtype=torch.int64, device=dev) for _ in range(2)]
    valid = [torch.zeros(n, dtype=torch.uint8, device=dev) for n in shards]
    w = ctx.verify_sharded_device(shards, [t["pk"].data_ptr() for t in d], [t["sig"].data_ptr() for t in d],
                                  [t["m"].data_ptr() for t in d], [t["off"].data_ptr() for t in d], MODE_GO_STDLIB,
                                  [o.data_ptr() for o in out], [v.data_ptr() for v in valid])
    ctx.sync()
    assert w == W
    for g in range(2):
        assert np.array_equal(valid[g].cpu().numpy(), exp[g])
        words = out[g].cpu().numpy().view(np.uint64)  # every device holds every shard
        for h, n in enumerate(shards):
            bits = np.unpackbits(words[h * W:(h + 1) * W].view(np.uint8), bitorder="little")
            assert np.array_equal(bits[:n], exp[h]) and not bits[n:].any()


def test_multi_device_api_independent_batches():
    """cmtv_verify_ed25519_multi_device over a repeated ordinal: each device
    verifies its own batch into its own bitmap words (no exchange)."""
    import torch

    ctx = Context(devices=[0, 0])
    dev = torch.device("cuda:0")
    shards, exp, d = (10_000, 333), [], []
    for g, n in enumerate(shards):
        pk, kidx, sig, m, off = _batch(n, 60 + g)
        sig = sig.copy()
        sig[g::101, 9] ^= 4
        exp.append(coracle.verify_batch(pk[kidx], sig, m, off, MODE_GO_STDLIB, nthreads=16))
        d.append({k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in
                  {"pk": pk[kidx], "sig": sig, "m": m, "off": off.view(np.int32)}.items()})
    out = [torch.full(((n + 63) // 64 + 1,), -1, dtype=torch.int64, device=dev) for n in shards]
    valid = [torch.zeros(n, dtype=torch.uint8, device=dev) for n in shards]
    g0 = ctx.stats()["gathers"]
    ctx.verify_multi_device(list(shards), [t["pk"].data_ptr() for t in d], [t["sig"].data_ptr() for t in d],
                            [t["m"].data_ptr() for t in d], [t["off"].data_ptr() for t in d], MODE_GO_STDLIB,
                            [o.data_ptr() for o in out], [v.data_ptr() for v in valid])
    ctx.sync()
    assert ctx.stats()["gathers"] == g0
    for g, n in enumerate(shards):
        assert np.array_equal(valid[g].cpu().numpy(), exp[g])
        words = out[g].cpu().numpy().view(np.uint64)
        bits = np.unpackbits(words[:(n + 63) // 64].view(np.uint8), bitorder="little")
        assert np.array_equal(bits[:n], exp[g])
        assert words[-1] == np.uint64((1 << 64) - 1)  # nothing written past its own words


def test_rccl_path_on_one_device():
    """CMTV_FORCE_RCCL: a one-rank RCCL communicator over device 0, so the
    library's RCCL init (ncclCommInitAll) and its in-place grouped all-gather
    of the bitmap run on a one-GPU box; verdicts and bitmap vs the oracle."""
    import torch

    with _env(CMTV_FORCE_RCCL=1):
        ctx = Context(devices=[0])
    assert ctx.stats()["rccl"] == 1
    dev = torch.device("cuda:0")
    n = 1500
    pk, kidx, sig, m, off = _batch(n, 77)
    sig = sig.copy()
    sig[::17, 5] ^= 1
    exp = coracle.verify_batch(pk[kidx], sig, m, off, MODE_GO_STDLIB, nthreads=16)
    t = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in
         {"pk": pk[kidx], "sig": sig, "m": m, "off": off.view(np.int32)}.items()}
    W = (n + 63) // 64
    out = torch.full((W,), -1, dtype=torch.int64, device=dev)
    valid = torch.zeros(n, dtype=torch.uint8, device=dev)
    w = ctx.verify_sharded_device([n], [t["pk"].data_ptr()], [t["sig"].data_ptr()], [t["m"].data_ptr()],
                                  [t["off"].data_ptr()], MODE_GO_STDLIB, [out.data_ptr()], [valid.data_ptr()])
    ctx.sync()
    assert w == W and ctx.stats()["gathers"] >= 1
    assert np.array_equal(valid.cpu().numpy(), exp)
    bits = np.unpackbits(out.cpu().numpy().view(np.uint64).view(np.uint8), bitorder="little")
    assert np.array_equal(bits[:n], exp) and not bits[n:].any()
    got = ctx.verify(pk[kidx], sig, m, off, MODE_GO_STDLIB)
    assert np.array_equal(got, exp)


def test_fault_injection_knob():
    with _env(CMTV_FAULT_AT=3):
        ctx = Context(device=0)
    pk, kidx, sig, m, off = _batch(200, 5)
    exp = coracle.verify_batch(pk[kidx], sig, m, off, MODE_GO_STDLIB, nthreads=16)
    for _ in range(2):
        assert np.array_equal(ctx.verify(pk[kidx], sig, m, off), exp)
    with pytest.raises(N.CmtvError) as ei:
        ctx.verify(pk[kidx], sig, m, off)
    assert ei.value.code == N.CMTV_EHIP
    # the context recovers: later calls (host, commit, device) are exact
    assert np.array_equal(ctx.verify(pk[kidx], sig, m, off), exp)
    sv = TU.make_validator_set(ctx, 20)
    commit, _, _ = TU.make_commit(ctx, sv, 9)
    assert sv.valset.verify_commit(TU.CHAIN_ID, TU.block_id_for_height(9), 9, commit, ctx=ctx) is None
    st = ctx.stats()
    assert st["faults_injected"] == 1


def test_concurrent_callers_share_a_context():
    """4 threads on one context: two host-buffer callers and two
    device-resident callers on their own streams, all above the quad
    crossover (lane kernel, shared A-table scratch), each checking its
    verdicts every iteration; plus the null-stream device call immediately
    followed by a host call."""
    import torch

    ctx = Context(device=0)
    dev = torch.device("cuda:0")
    n = 45_000
    jobs = []
    for j in range(4):
        pk, kidx, sig, m, off = _batch(n, 70 + j, flip=0.05)
        exp = coracle.verify_batch(pk[kidx], sig, m, off, MODE_GO_STDLIB, nthreads=16)
        jobs.append((pk[kidx], sig, m, off, exp))
    errors = []

    def host(j):
        pk, sig, m, off, exp = jobs[j]
        try:
            for _ in range(3):
                got = ctx.verify(pk, sig, m, off)
                if not np.array_equal(got, exp):
                    errors.append(("host", j, int((got != exp).sum())))
        except Exception as e:  # noqa: BLE001
            errors.append(("host", j, repr(e)))

    def device(j):
        pk, sig, m, off, exp = jobs[j]
        try:
            s = torch.cuda.Stream(device=dev)
            t = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in
                 {"pk": pk, "sig": sig, "m": m, "off": off.view(np.int32)}.items()}
            v = torch.zeros(n, dtype=torch.uint8, device=dev)
            for _ in range(3):
                v.zero_()
                torch.cuda.synchronize(dev)
                ctx.verify_device(n, t["pk"].data_ptr(), t["sig"].data_ptr(), t["m"].data_ptr(),
                                  t["off"].data_ptr(), MODE_GO_STDLIB, v.data_ptr(), 0, s.cuda_stream)
                s.synchronize()
                got = v.cpu().numpy()
                if not np.array_equal(got, exp):
                    errors.append(("device", j, int((got != exp).sum())))
        except Exception as e:  # noqa: BLE001
            errors.append(("device", j, repr(e)))

    ths = [threading.Thread(target=host, args=(0,)), threading.Thread(target=host, args=(1,)),
           threading.Thread(target=device, args=(2,)), threading.Thread(target=device, args=(3,))]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=110)
    assert not any(t.is_alive() for t in ths)
    assert not errors, errors[:5]
    # a null-stream device call, then at once a host call
    pk, sig, m, off, exp = jobs[2]
    t = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in
         {"pk": pk, "sig": sig, "m": m, "off": off.view(np.int32)}.items()}
    v = torch.zeros(n, dtype=torch.uint8, device=dev)
    ctx.verify_device(n, t["pk"].data_ptr(), t["sig"].data_ptr(), t["m"].data_ptr(), t["off"].data_ptr(),
                      MODE_GO_STDLIB, v.data_ptr(), 0, 0)
    pk1, sig1, m1, off1, exp1 = jobs[1]
    assert np.array_equal(ctx.verify(pk1, sig1, m1, off1), exp1)
    torch.cuda.synchronize(dev)
    assert np.array_equal(v.cpu().numpy(), exp)


def test_keyset_cache_cross_height_uses_keyed_kernel(gpu_ctx):
    """cmtv_verify_commits gives each commit its own valset
    struct; sets with the same keys must still take the registered-key
    kernel (and agree with the generic path)."""
    sv = TU.make_validator_set(gpu_ctx, 30)
    items = []
    for h in range(40, 46):
        commit, _, _ = TU.make_commit(gpu_ctx, sv, h)
        vs = T.ValidatorSet([T.Validator(v.pub_key, v.voting_power) for v in sv.valset.validators])  # a copy
        items.append((vs, TU.block_id_for_height(h), h, commit))
    keyed = Context(device=0)
    keyed.keyset_cache(2)
    before = keyed.stats()["keyed_launches"]
    out = T.verify_commits(0, TU.CHAIN_ID, items, ctx=keyed)
    assert all(e is None for e in out)
    assert keyed.stats()["keyed_launches"] > before
    # a set with different keys at one height turns it off (generic path)
    other = TU.make_validator_set(gpu_ctx, 30, offset=1000)
    c2, _, _ = TU.make_commit(gpu_ctx, other, 46)
    items2 = items + [(other.valset, TU.block_id_for_height(46), 46, c2)]
    k0 = keyed.stats()["keyed_launches"]
    assert all(e is None for e in T.verify_commits(0, TU.CHAIN_ID, items2, ctx=keyed))
    assert keyed.stats()["keyed_launches"] == k0


def test_batch_split_by_sign_bytes_size(gpu_ctx):
    sv = TU.make_validator_set(gpu_ctx, 50)
    items = []
    for h in range(60, 70):
        commit, _, _ = TU.make_commit(gpu_ctx, sv, h)
        if h == 64:
            s = bytearray(commit.signatures[9].signature)
            s[0] ^= 1
            commit.signatures[9].signature = bytes(s)
        items.append((sv.valset, TU.block_id_for_height(h), h, commit))
    want = [None if e is None else str(e) for e in T.verify_commits(0, TU.CHAIN_ID, items, ctx=gpu_ctx)]
    with _env(CMTV_MAX_BATCH_MSG_BYTES=4000):
        before = gpu_ctx.stats()["calls"]
        got = [None if e is None else str(e) for e in T.verify_commits(0, TU.CHAIN_ID, items, ctx=gpu_ctx)]
        calls = gpu_ctx.stats()["calls"] - before
    assert got == want and want[4] is not None
    assert calls >= 10  # 500 signatures x ~116 B in < 4000-byte device batches


def test_safe_mul_edge_cases(gpu_ctx):
    """types/validator_set.go:1086-1105 safeMul with Go's int64 wrap:
    numerator 2^63 is MinInt64 after the cast -> overflow; denominator
    2^64 - 1 is -1 -> votingPowerNeeded = -total, so the first signature
    already passes (no SIGFPE on MinInt64 / -1)."""
    vals = TU.make_validator_set(gpu_ctx, 4)
    commit, _, _ = TU.make_commit(gpu_ctx, vals, 12)
    e = None
    try:
        vals.valset.verify_commit_light_trusting(TU.CHAIN_ID, commit, (2**63, 3), ctx=gpu_ctx)
    except T.ErrTrustLevel as x:
        e = x
    assert e is not None and "int64 overflow" in str(e)
    assert vals.valset.verify_commit_light_trusting(TU.CHAIN_ID, commit, (1, 2**64 - 1), ctx=gpu_ctx) is None
