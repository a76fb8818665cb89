"""The library's multi-rank RCCL code, executed on one GPU.

libcmtverify resolves RCCL with dlopen (runtime.cpp load_rccl). With
CMTV_RCCL_LIB pointing at tests/host/librccl_stub.so -- a test double of
ncclCommInitAll / ncclGroupStart / ncclGroupEnd / ncclAllGather /
ncclCommDestroy that gathers with ordered device copies and logs every call
-- and CMTV_FORCE_RCCL=1, a context over a repeated ordinal builds a G-rank
communicator and takes the RCCL branch of gather_bitmaps, exactly as on an
8-GPU node, instead of the peer-copy branch the other one-GPU tests take.

Checked here, against the oracle (oracle/liboracle.so):
  * G = 2, 4, 8: host batches, device-resident sharded batches (generic and
    registered keys) and commits give the oracle's verdicts; the stub saw one
    G-rank communicator and in-place all-gathers of W words from every rank;
    cmtv_stats.rccl = 1;
  * device failure (CMTV_FAULT_DEV=g before the launch, CMTV_FAULT_SYNC_DEV=g
    after it): the communicator is destroyed and rebuilt over the survivors
    with ranks renumbered by live position, and the retried batch gathers
    over G - 1 ranks;
  * a node whose RCCL refuses a gather at run time (the stub's
    CMTV_RCCL_STUB_FAIL_GROUP): that gather and every later one fall back to
    peer copies, verdicts stay exact, cmtv_stats.rccl_failures counts it;
  * after device 0 is retired, the single-device device-resident
    entry points return CMTV_ENODEV instead of launching on it (key
    generation, which takes host buffers, moves to a live device).
Hardware RCCL over xGMI across distinct GPUs stays unmeasured here: the
driver's 8-GPU bench is the only place it runs."""
import os
import re

import numpy as np
import pytest

from oracle import coracle
from cometbft_amd import MODE_GO_STDLIB, MODE_ZIP215, Context
from cometbft_amd import _native as N
from cometbft_amd import testutil as TU
from test_runtime_gpu import _batch, _env

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STUB = os.path.join(ROOT, "tests", "host", "librccl_stub.so")


@pytest.fixture(autouse=True)
def _stub_log_env(monkeypatch, tmp_path):
    """The stub reads CMTV_RCCL_STUB_LOG at every ncclCommInitAll, including
    the rebuilds after a device failure, so it stays set for the whole test."""
    monkeypatch.setenv("CMTV_RCCL_STUB_LOG", str(tmp_path / "rccl.log"))


def _stub_ctx(G, log, **env):
    if not os.path.exists(STUB):
        pytest.fail("tests/host/librccl_stub.so missing: run __graft_entry__.build() (make -C cometbft_amd/csrc stub)")
    assert os.environ["CMTV_RCCL_STUB_LOG"] == str(log)
    with _env(CMTV_RCCL_LIB=STUB, CMTV_FORCE_RCCL=1, CMTV_SHARD_MIN=64, **env):
        return Context(devices=[0] * G)


def _log(log):
    return open(log).read().splitlines() if os.path.exists(log) else []


def _inits(lines):
    return [(int(m.group(1)), int(m.group(2))) for m in
            (re.match(r"init n=(\d+) devs=[\d,]+ comm=(\d+)", x) for x in lines) if m]


def _gathers(lines):
    out = []
    for x in lines:
        m = re.match(r"allgather comm=(\d+) rank=(\d+) nranks=(\d+) count=(\d+) dtype=(\d+) inplace=(\d)", x)
        if m:
            out.append(tuple(int(v) for v in m.groups()))
    return out


@pytest.mark.parametrize("G", [2, 4, 8])
def test_rccl_branch_host_batches(tmp_path, G):
    log = tmp_path / "rccl.log"
    ctx = _stub_ctx(G, log)
    assert ctx.stats()["rccl"] == 1
    inits = _inits(_log(log))
    assert len(inits) == 1 and inits[0][0] == G
    comm = inits[0][1]
    n = 64 * 37 * G + 5  # G shards, the last one ragged
    pk, kidx, sig, m, off = _batch(n, 1000 + G, flip=0.05)
    for mode in (MODE_GO_STDLIB, MODE_ZIP215):
        exp = coracle.verify_batch(pk[kidx], sig, m, off, mode, nthreads=16)
        got, words = ctx.verify(pk[kidx], sig, m, off, mode, bitmap=True)
        assert np.array_equal(got, exp), np.nonzero(got != exp)[0][:10]
        assert np.array_equal(np.unpackbits(words.view(np.uint8), bitorder="little")[:n], exp)
    st = ctx.stats()
    assert st["gathers"] == 2 and st["sharded_calls"] == 2
    ds = ctx.device_stats()
    assert all(d["calls"] == 2 for d in ds)
    g = _gathers(_log(log))
    # every rank of the one communicator, in place, uint64 words, per call
    assert len(g) == 2 * G
    W = (-(-n // G) + 63) // 64
    for call in range(2):
        rows = g[call * G:(call + 1) * G]
        assert sorted(r[1] for r in rows) == list(range(G))
        assert all(r[0] == comm and r[2] == G and r[4] == 5 and r[5] == 1 for r in rows)
        assert all(r[3] == rows[0][3] for r in rows) and rows[0][3] >= W - 1
    # registered keys and a commit through the same communicator
    ks = ctx.register_keys(pk)
    exp = coracle.verify_batch(pk[kidx], sig, m, off, MODE_GO_STDLIB, nthreads=16)
    assert np.array_equal(ctx.verify_indexed(ks, kidx, sig, m, off, MODE_GO_STDLIB), exp)
    ks.free()
    sv = TU.make_validator_set(ctx, 64 * G + 7)
    commit, _, _ = TU.make_commit(ctx, sv, 11)
    assert sv.valset.verify_commit(TU.CHAIN_ID, TU.block_id_for_height(11), 11, commit, ctx=ctx) is None
    assert ctx.stats()["gathers"] >= 4
    ctx.close()
    assert sum(1 for x in _log(log) if x.startswith("destroy")) == G


@pytest.mark.parametrize("keyed", [False, True])
def test_rccl_branch_sharded_device(tmp_path, keyed):
    import torch

    G = 4
    log = tmp_path / "rccl.log"
    ctx = _stub_ctx(G, log)
    dev = torch.device("cuda:0")
    shards = (3000, 64, 1, 2500)
    exp, d = [], []
    pk, kidx, sig, m, off = _batch(sum(shards), 77, flip=0.1, nkeys=150)
    ks = ctx.register_keys(pk) if keyed else None
    a = 0
    for n in shards:
        sl = slice(a, a + n)
        mm = m[off[a]:off[a + n]]
        oo = (off[a:a + n + 1] - off[a]).astype(np.uint32)
        exp.append(coracle.verify_batch(pk[kidx[sl]], sig[sl], mm, oo, MODE_ZIP215, nthreads=16))
        keys = kidx[sl].astype(np.int32) if keyed else pk[kidx[sl]]
        d.append([torch.from_numpy(np.ascontiguousarray(v)).to(dev) for v in (keys, sig[sl], mm, oo.view(np.int32))])
        a += n
    W = max((n + 63) // 64 for n in shards)
    out = [torch.full((G * W,), -1, dtype=torch.int64, device=dev) for _ in range(G)]
    w = ctx.verify_sharded_device(shards, [t[0].data_ptr() for t in d], [t[1].data_ptr() for t in d],
                                  [t[2].data_ptr() for t in d], [t[3].data_ptr() for t in d], MODE_ZIP215,
                                  [o.data_ptr() for o in out], keys=ks)
    ctx.sync()
    assert w == W
    for g in range(G):  # every device holds every shard
        words = out[g].cpu().numpy().view(np.uint64)
        for h, n in enumerate(shards):
            bits = np.unpackbits(words[h * W:(h + 1) * W].view(np.uint8), bitorder="little")
            assert np.array_equal(bits[:n], exp[h]) and not bits[n:].any(), (g, h)
    gl = _gathers(_log(log))
    assert len(gl) == G and all(r[2] == G and r[3] == W and r[5] == 1 for r in gl)
    if ks is not None:
        ks.free()


@pytest.mark.parametrize("knob,bad", [("CMTV_FAULT_DEV", 2), ("CMTV_FAULT_SYNC_DEV", 1), ("CMTV_FAULT_SYNC_DEV", 0)])
def test_rccl_rebuild_after_device_failure(tmp_path, knob, bad):
    G = 4
    log = tmp_path / "rccl.log"
    ctx = _stub_ctx(G, log, **{knob: bad})
    n = 64 * 40 * G
    pk, kidx, sig, m, off = _batch(n, 500 + bad, flip=0.05)
    exp = coracle.verify_batch(pk[kidx], sig, m, off, MODE_GO_STDLIB, nthreads=16)
    got, words = ctx.verify(pk[kidx], sig, m, off, MODE_GO_STDLIB, bitmap=True)
    assert np.array_equal(got, exp), np.nonzero(got != exp)[0][:10]
    assert np.array_equal(np.unpackbits(words.view(np.uint8), bitorder="little")[:n], exp)
    st = ctx.stats()
    assert st["device_failures"] == 1 and st["reshards"] == 1 and st["live_devices"] == G - 1
    assert st["rccl"] == 1
    lines = _log(log)
    inits = _inits(lines)
    assert [i[0] for i in inits] == [G, G - 1]
    old, new = inits[0][1], inits[1][1]
    # the old communicator was destroyed (every rank) before the new one
    destroyed = [x for x in lines if x.startswith(f"destroy comm={old} ")]
    assert len(destroyed) == G
    assert lines.index(destroyed[-1]) < lines.index(next(x for x in lines if x.startswith(f"init n={G - 1}")))
    # the retried batch gathered over the survivors, ranks 0 .. G-2
    g_new = [r for r in _gathers(lines) if r[0] == new]
    assert sorted(r[1] for r in g_new) == list(range(G - 1)) and all(r[2] == G - 1 for r in g_new)
    ds = ctx.device_stats()
    assert [d["failed"] for d in ds] == [int(g == bad) for g in range(G)]
    # a later batch stays on the survivors and the same communicator
    got2 = ctx.verify(pk[kidx], sig, m, off, MODE_ZIP215)
    assert np.array_equal(got2, coracle.verify_batch(pk[kidx], sig, m, off, MODE_ZIP215, nthreads=16))
    assert len(_inits(_log(log))) == 2
    if bad == 0:
        _assert_dev0_calls_refused(ctx, pk, kidx, sig, m, off)


@pytest.mark.parametrize("G", [2, 8])
def test_rccl_gather_failure_falls_back_to_peer_copies(tmp_path, monkeypatch, G):
    """The first grouped all-gather fails: the batch still gives the oracle's
    verdicts (peer copies), rccl drops to 0, rccl_failures = 1, and later
    batches never call RCCL again; CMTV_NO_RCCL_FALLBACK=1 reports CMTV_ERCCL
    instead."""
    log = tmp_path / "rccl.log"
    monkeypatch.setenv("CMTV_RCCL_STUB_FAIL_GROUP", "1")
    ctx = _stub_ctx(G, log)
    assert ctx.stats()["rccl"] == 1
    n = 64 * 21 * G + 3
    pk, kidx, sig, m, off = _batch(n, 2000 + G, flip=0.05)
    for mode in (MODE_GO_STDLIB, MODE_ZIP215):
        exp = coracle.verify_batch(pk[kidx], sig, m, off, mode, nthreads=16)
        got, words = ctx.verify(pk[kidx], sig, m, off, mode, bitmap=True)
        assert np.array_equal(got, exp), np.nonzero(got != exp)[0][:10]
        assert np.array_equal(np.unpackbits(words.view(np.uint8), bitorder="little")[:n], exp)
    st = ctx.stats()
    assert st["rccl"] == 0 and st["rccl_failures"] == 1 and st["gathers"] == 2
    lines = _log(log)
    assert sum(1 for x in lines if x.startswith("groupend failed")) == 1
    assert not _gathers(lines)  # nothing went through the stub's copies
    ctx.close()
    log2 = tmp_path / "rccl2.log"
    monkeypatch.setenv("CMTV_RCCL_STUB_LOG", str(log2))
    ctx = _stub_ctx(G, log2, CMTV_NO_RCCL_FALLBACK=1)
    with pytest.raises(RuntimeError):
        ctx.verify(pk[kidx], sig, m, off, MODE_GO_STDLIB)
    assert ctx.stats()["rccl_failures"] == 1
    ctx.close()


def test_rccl_partial_group_failure_reports_erccl(tmp_path, monkeypatch):
    """the failed group had already enqueued rank 0's collective
    (the stub holds that stream, as a collective waiting for peers that never
    come). The library does not queue peer copies behind it: the bounded
    drain (CMTV_RCCL_DRAIN_MS) times out, the communicators are aborted --
    which ends the stuck collective -- and the call returns CMTV_ERCCL
    instead of hanging. The next call gathers by peer copies with exact
    verdicts, and no communicator is ever built again."""
    log = tmp_path / "rccl.log"
    monkeypatch.setenv("CMTV_RCCL_STUB_FAIL_GROUP", "1")
    monkeypatch.setenv("CMTV_RCCL_STUB_PARTIAL", "1")
    G = 4
    ctx = _stub_ctx(G, log, CMTV_RCCL_DRAIN_MS=300)
    n = 64 * 19 * G + 9
    pk, kidx, sig, m, off = _batch(n, 3100, flip=0.05)
    with pytest.raises(RuntimeError):
        ctx.verify(pk[kidx], sig, m, off, MODE_GO_STDLIB)
    lines = _log(log)
    assert any(x.startswith("partial rank=0") for x in lines)
    assert sum(1 for x in lines if x.startswith("abort")) == G
    st = ctx.stats()
    assert st["rccl"] == 0 and st["rccl_failures"] == 1
    exp = coracle.verify_batch(pk[kidx], sig, m, off, MODE_ZIP215, nthreads=16)
    assert np.array_equal(ctx.verify(pk[kidx], sig, m, off, MODE_ZIP215), exp)
    assert len(_inits(_log(log))) == 1 and not _gathers(_log(log))
    ctx.close()


def test_rccl_failure_survives_device_retirement(tmp_path, monkeypatch):
    """after a gather failed in RCCL, a device retirement
    (CMTV_FAULT_SYNC_DEV: device 1 fails after the gather) rebuilds nothing:
    the retried batch and later ones keep using peer copies."""
    log = tmp_path / "rccl.log"
    monkeypatch.setenv("CMTV_RCCL_STUB_FAIL_GROUP", "1")
    G = 4
    ctx = _stub_ctx(G, log, CMTV_FAULT_SYNC_DEV=1)
    n = 64 * 23 * G + 1
    pk, kidx, sig, m, off = _batch(n, 3200, flip=0.05)
    exp = coracle.verify_batch(pk[kidx], sig, m, off, MODE_GO_STDLIB, nthreads=16)
    assert np.array_equal(ctx.verify(pk[kidx], sig, m, off, MODE_GO_STDLIB), exp)
    st = ctx.stats()
    assert st["device_failures"] == 1 and st["rccl"] == 0 and st["rccl_failures"] == 1
    assert np.array_equal(ctx.verify(pk[kidx], sig, m, off, MODE_GO_STDLIB), exp)
    assert len(_inits(_log(log))) == 1 and not _gathers(_log(log))
    ctx.close()


def _assert_dev0_calls_refused(ctx, pk, kidx, sig, m, off):
    """ADVICE r3 (runtime.cpp:1730): device 0 retired -> the single-device
    entry points return CMTV_ENODEV; a key set registered afterwards has no
    tables on device 0 and is refused by the device-resident indexed call."""
    import torch

    dev = torch.device("cuda:0")
    n = 100
    t = [torch.from_numpy(np.ascontiguousarray(v)).to(dev) for v in
         (pk[kidx[:n]], kidx[:n].astype(np.int32), sig[:n], m, off[:n + 1].view(np.int32))]
    bm = torch.zeros(2, dtype=torch.int64, device=dev)
    with pytest.raises(N.CmtvError) as ei:
        ctx.verify_device(n, t[0].data_ptr(), t[2].data_ptr(), t[3].data_ptr(), t[4].data_ptr(), MODE_GO_STDLIB,
                          0, bm.data_ptr())
    assert ei.value.code == N.CMTV_ENODEV
    ks = ctx.register_keys(pk)
    with pytest.raises(N.CmtvError) as ei:
        ctx.verify_indexed_device(ks, n, t[1].data_ptr(), t[2].data_ptr(), t[3].data_ptr(), t[4].data_ptr(),
                                  MODE_GO_STDLIB, 0, bm.data_ptr())
    assert ei.value.code == N.CMTV_ENODEV
    # the host path still runs on the survivors
    exp = coracle.verify_batch(pk[kidx[:n]], sig[:n], m, off[:n + 1], MODE_GO_STDLIB, nthreads=4)
    assert np.array_equal(ctx.verify_indexed(ks, kidx[:n], sig[:n], m, off[:n + 1], MODE_GO_STDLIB), exp)
    ks.free()
    # host-buffer key generation moves to the first live device
    seeds = np.arange(128, dtype=np.uint8).reshape(4, 32)
    assert np.array_equal(ctx.pubkeys(seeds), coracle.pubkeys_from_seeds(seeds))


def test_peer_copy_context_dev0_retired_refuses_device_calls():
    """The same refusal on a peer-copy context (no RCCL), CMTV_FAULT_DEV=0."""
    with _env(CMTV_SHARD_MIN=64, CMTV_FAULT_DEV=0):
        ctx = Context(devices=[0, 0, 0])
    n = 3001
    pk, kidx, sig, m, off = _batch(n, 4)
    exp = coracle.verify_batch(pk[kidx], sig, m, off, MODE_GO_STDLIB, nthreads=16)
    assert np.array_equal(ctx.verify(pk[kidx], sig, m, off), exp)
    assert ctx.stats()["device_failures"] == 1
    _assert_dev0_calls_refused(ctx, pk, kidx, sig, m, off)


def test_fault_at_in_device_call_does_not_stick():
    """ADVICE r3 (runtime.cpp:456): CMTV_FAULT_AT firing inside a
    single-device _device call is that call's failure only; a later host
    batch's genuine device fault (CMTV_FAULT_SYNC_DEV) still retires the
    device and re-shards."""
    import torch

    with _env(CMTV_SHARD_MIN=64, CMTV_FAULT_AT=1, CMTV_FAULT_SYNC_DEV=1):
        ctx = Context(devices=[0, 0])
    dev = torch.device("cuda:0")
    pk, kidx, sig, m, off = _batch(200, 8)
    t = [torch.from_numpy(np.ascontiguousarray(v)).to(dev) for v in (pk[kidx], sig, m, off.view(np.int32))]
    bm = torch.zeros(4, dtype=torch.int64, device=dev)
    with pytest.raises(N.CmtvError) as ei:
        ctx.verify_device(200, t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(), t[3].data_ptr(), MODE_GO_STDLIB,
                          0, bm.data_ptr())
    assert ei.value.code == N.CMTV_EHIP
    n = 3001
    pk, kidx, sig, m, off = _batch(n, 9)
    exp = coracle.verify_batch(pk[kidx], sig, m, off, MODE_GO_STDLIB, nthreads=16)
    assert np.array_equal(ctx.verify(pk[kidx], sig, m, off), exp)
    st = ctx.stats()
    assert st["device_failures"] == 1 and st["reshards"] == 1 and st["live_devices"] == 1
