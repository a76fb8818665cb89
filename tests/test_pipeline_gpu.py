"""The chunked cross-height pipeline (cometbft_amd/csrc/pipeline.cpp) on the GPU.

Large cmtv_verify_commits calls (blocksync / light-client replay:
blockchain/v0/reactor.go:349-400, light/client.go:613-689) are cut into
commit-aligned chunks that are planned, packed and replayed on host worker
threads while earlier chunks verify on the bulk lanes. Parity is against the
one-batch path of the same library (CMTV_PIPELINE=0), whose per-commit
outcomes tests/test_replay_gpu.py and tests/test_commit_gpu.py pin to
types/validator_set_test.go: every commit's return code, result struct and
error string must be byte-identical, over a chain with assorted faults, three
validator sets (two of them sharing no keys, one with a bad key length), all
three kinds, both modes, with and without registered keys, one and several
(repeated-ordinal) devices, and a device retired in the middle of a call.

configs[2] scale: 7,000 heights x 150 validators (1.05M
signatures, 1% flipped, seed 42) through cmtv_verify_commits from host
memory, full and light, each height's outcome checked against the reference
loop over the known flips (ReplayChain.expected); the flips themselves are
checked on a 2,000-signature sample by the C restatement of Go's
ed25519.Verify (oracle/liboracle.so)."""
import ctypes

import numpy as np
import pytest

from oracle import coracle
from cometbft_amd import MODE_GO_STDLIB, MODE_ZIP215, Context
from cometbft_amd import _native as N
from cometbft_amd import testutil as TU
from cometbft_amd import types as T
from test_runtime_gpu import _env

pytestmark = pytest.mark.gpu

N_VALS = 150


def _flip(cs, byte, bit):
    if len(cs.signature) == 64:
        s = bytearray(cs.signature)
        s[byte] ^= bit
        cs.signature = bytes(s)


def _mutate(commit, h):
    """Faults by height (every kind meets each of them somewhere)."""
    sigs = commit.signatures
    if h % 13 == 0:  # a bad signature early
        _flip(sigs[2], 10, 1)
    if h % 17 == 0:  # ... and late (only VerifyCommit reaches it)
        _flip(sigs[-1], 40, 4)
    if h % 19 == 0 and sigs[5].signature:  # a signature of the wrong length
        sigs[5].signature = sigs[5].signature[:63]
    if h % 29 == 0:  # an unknown BlockIDFlag (the reference panics in VerifyCommit)
        sigs[10].block_id_flag = 7
    if h % 31 == 0:  # a double vote for LightTrusting (same validator address twice)
        sigs[6].validator_address = sigs[4].validator_address
    if h % 37 == 0:  # an address the trusted set does not know
        sigs[7].validator_address = bytes(20)


@pytest.fixture(scope="module")
def faulty_chain(gpu_ctx):
    """300 heights: set A (150), set B (150 other keys), set C (120 keys), a
    set with one 31-byte key, then A again; flags, faults, wrong heights and
    BlockIDs by height."""
    A = TU.make_validator_set(gpu_ctx, N_VALS)
    B = TU.make_validator_set(gpu_ctx, N_VALS, offset=10_000)
    C = TU.make_validator_set(gpu_ctx, 120, offset=20_000)
    bad = TU.make_validator_set(gpu_ctx, N_VALS, offset=30_000)
    vbad = T.ValidatorSet([T.Validator(v.pub_key[:31] if i == 40 else v.pub_key, v.voting_power)
                           for i, v in enumerate(bad.valset.validators)])
    items = []
    for h in range(1, 301):
        sv = A if h <= 100 or h > 260 else (B if h <= 200 else (C if h <= 250 else bad))
        n = len(sv.valset.validators)
        flags = [T.BLOCK_ID_FLAG_COMMIT] * n
        if h % 7 == 0:
            flags = [T.BLOCK_ID_FLAG_NIL if i % 4 == 0 else f for i, f in enumerate(flags)]
        if h % 11 == 0:
            flags = [T.BLOCK_ID_FLAG_ABSENT if i < 30 else f for i, f in enumerate(flags)]
        if h % 43 == 0:  # too few signatures: not enough voting power
            flags = [T.BLOCK_ID_FLAG_ABSENT if i < n // 2 else f for i, f in enumerate(flags)]
        commit, _, _ = TU.make_commit(gpu_ctx, sv, h, flags=flags)
        _mutate(commit, h)
        vals = vbad if sv is bad else sv.valset
        height = h + 1 if h % 23 == 0 else h
        bid = TU.block_id_for_height(h + 5000) if h % 41 == 0 else TU.block_id_for_height(h)
        items.append((vals, bid, height, commit))
    return items


def _raw(pc):
    return list(pc.rcs), bytes(pc.res), pc.bufs.raw


def _ctx(devices=None, keyset=False, **env):
    with _env(**env):
        c = Context(devices=devices) if devices else Context(device=0)
    if keyset:
        c.keyset_cache(8)
    return c


@pytest.mark.parametrize("kind", [N.VERIFY_COMMIT, N.VERIFY_COMMIT_LIGHT, N.VERIFY_COMMIT_LIGHT_TRUSTING])
def test_pipeline_matches_one_batch(faulty_chain, kind):
    one = _ctx(CMTV_PIPELINE=0)
    one_k = _ctx(keyset=True, CMTV_PIPELINE=0)
    pipes = [_ctx(CMTV_PIPE_MIN=1, CMTV_PIPE_CHUNK=1000, CMTV_PIPE_SLOTS=2, CMTV_HOST_THREADS=4),
             _ctx(keyset=True, CMTV_PIPE_MIN=1, CMTV_PIPE_CHUNK=3000, CMTV_HOST_THREADS=3),
             _ctx(devices=[0, 0, 0], keyset=True, CMTV_PIPE_MIN=1, CMTV_PIPE_CHUNK=700, CMTV_PIPE_SLOTS=4)]
    modes = (MODE_GO_STDLIB, MODE_ZIP215) if kind == N.VERIFY_COMMIT else (MODE_GO_STDLIB,)
    for mode in modes:
        pc = T.PackedCommits(kind, TU.CHAIN_ID, faulty_chain, mode=mode, trust_level=(1, 3))
        pc.call(one)
        want = _raw(pc)
        outcomes = {type(e).__name__ if e is not None else None for e in pc.verify(one)}
        assert len(outcomes) >= 3, outcomes  # the chain exercises errors and successes
        pc.call(one_k)
        assert _raw(pc) == want
        for c in pipes:
            st0 = c.stats()
            pc.call(c)
            got = _raw(pc)
            assert got[0] == want[0]
            assert got[1] == want[1], np.nonzero(np.frombuffer(got[1], np.uint8) != np.frombuffer(want[1], np.uint8))
            assert got[2] == want[2]
            assert c.stats()["calls"] > st0["calls"]
    for c in [one, one_k] + pipes:
        c.close()


def test_pipeline_small_chunks_and_keyset_switches(faulty_chain):
    """Chunks of a few commits each, two slots, key classes switching between
    the sets (a chunk never mixes sets): every chunk boundary case at once."""
    one = _ctx(CMTV_PIPELINE=0)
    c = _ctx(keyset=True, CMTV_PIPE_MIN=1, CMTV_PIPE_CHUNK=64, CMTV_PIPE_SLOTS=2, CMTV_HOST_THREADS=2)
    pc = T.PackedCommits(N.VERIFY_COMMIT_LIGHT, TU.CHAIN_ID, faulty_chain)
    pc.call(one)
    want = _raw(pc)
    pc.call(c)
    assert _raw(pc) == want
    st = c.stats()
    assert st["keyed_launches"] > 0
    one.close()
    c.close()


def test_pipeline_device_retired_mid_call(faulty_chain):
    """Four lanes over one GPU; device 1's chunk fails after its launch
    (CMTV_FAULT_SYNC_DEV): the device is retired, the chunks not yet replayed
    run on the other three, and every outcome is still the one-batch path's."""
    one = _ctx(CMTV_PIPELINE=0)
    pc = T.PackedCommits(N.VERIFY_COMMIT, TU.CHAIN_ID, faulty_chain)
    pc.call(one)
    want = _raw(pc)
    c = _ctx(devices=[0, 0, 0, 0], keyset=True, CMTV_PIPE_MIN=1, CMTV_PIPE_CHUNK=1500, CMTV_FAULT_SYNC_DEV=1)
    pc.call(c)
    assert _raw(pc) == want
    st = c.stats()
    assert st["device_failures"] == 1 and st["live_devices"] == 3
    pc.call(c)  # later calls stay on the survivors
    assert _raw(pc) == want
    one.close()
    c.close()


@pytest.fixture(scope="module")
def c3_chain(gpu_ctx):
    sv = TU.make_validator_set(gpu_ctx, N_VALS)
    return sv, TU.ReplayChain(gpu_ctx, sv, 1, 7000)


def _check_chain(chain, kind):
    rcs, code, si = chain.outcome()
    first = chain.expected(kind)
    bad = first >= 0
    assert bad.sum() > 0 and (~bad).sum() > 0
    assert np.all(rcs[~bad] == 0)
    assert np.all(rcs[bad] == N.CMTV_ECOMMIT)
    assert np.all(code[bad] == N.COMMIT_ERR_WRONG_SIGNATURE)
    assert np.array_equal(si[bad], first[bad])


def test_configs2_scale_flips_are_what_the_oracle_says(c3_chain):
    """The chain's data: a 2,000-signature sample verified by the C
    restatement of Go 1.19 ed25519.Verify is invalid exactly where a bit was
    flipped."""
    sv, chain = c3_chain
    rng = np.random.default_rng(7)
    total = chain.n_heights * N_VALS
    sample = np.unique(np.concatenate([rng.choice(total, 1900, replace=False), chain.flipped[:100]]))
    m_all, off_all = TU.replay_messages(1, chain.n_heights, N_VALS)
    m, off = coracle.pack_msgs([m_all[off_all[g]:off_all[g + 1]].tobytes() for g in sample])
    pk = np.ascontiguousarray(sv.pubkeys[sample % N_VALS])
    got = coracle.verify_batch(pk, chain.sig[sample], m, off, MODE_GO_STDLIB, nthreads=16)
    assert np.array_equal(got == 0, np.isin(sample, chain.flipped))


@pytest.mark.parametrize("devices", [None, [0, 0, 0, 0]])
@pytest.mark.parametrize("kind", [N.VERIFY_COMMIT, N.VERIFY_COMMIT_LIGHT])
def test_configs2_scale_through_verify_commits(c3_chain, kind, devices):
    """7,000 heights x 150 through cmtv_verify_commits with the keyset cache
    (a node's steady state), on one lane set and on four (the sharded node
    path); per height nil or ErrWrongSignature at the first flipped index the
    reference loop reaches."""
    sv, chain = c3_chain
    c = _ctx(devices=devices, keyset=True)
    st0 = c.stats()
    chain.call(c, kind)
    _check_chain(chain, kind)
    st = c.stats()
    reach = N_VALS if kind == N.VERIFY_COMMIT else (N_VALS * 10 * 2 // 3) // 10 + 1
    assert st["signatures"] - st0["signatures"] == chain.n_heights * reach
    assert st["keyed_launches"] > 0
    if devices:
        assert all(d["signatures"] > 0 for d in c.device_stats())
    c.close()


def test_configs2_scale_generic_and_zip215(c3_chain):
    """The same chain without registered keys (each key decoded per
    signature: the generic lane kernel) and in ZIP-215 mode."""
    sv, chain = c3_chain
    c = _ctx()
    chain.call(c, N.VERIFY_COMMIT_LIGHT)
    _check_chain(chain, N.VERIFY_COMMIT_LIGHT)
    assert c.stats()["keyed_launches"] == 0
    k = _ctx(keyset=True)
    chain.call(k, N.VERIFY_COMMIT, mode=MODE_ZIP215)
    _check_chain(chain, N.VERIFY_COMMIT)
    c.close()
    k.close()


@pytest.mark.parametrize("kind", [N.VERIFY_COMMIT, N.VERIFY_COMMIT_LIGHT, N.VERIFY_COMMIT_LIGHT_TRUSTING])
def test_direct_chunks_match_one_batch(faulty_chain, kind):
    """The commits' arrays in the context's cmtv_alloc_pinned memory (the Go
    shim's arena): commits whose plan is a prefix go to the
    device by DMA and k_bulk_gather lays them out (direct chunks), the others
    are packed as before; every outcome is byte-identical to the one-batch
    path. LightTrusting maps through addresses and never goes direct."""
    one = _ctx(CMTV_PIPELINE=0)
    pc = T.PackedCommits(kind, TU.CHAIN_ID, faulty_chain, trust_level=(1, 3))
    pc.call(one)
    want = _raw(pc)
    for devices, chunk in ((None, 3000), ([0, 0, 0], 700), (None, 64)):
        c = _ctx(devices=devices, keyset=True, CMTV_PIPE_MIN=1, CMTV_PIPE_CHUNK=chunk, CMTV_HOST_THREADS=4)
        pp = T.PackedCommits(kind, TU.CHAIN_ID, faulty_chain, trust_level=(1, 3), pinned=c)
        pp.call(c)
        assert _raw(pp) == want
        direct = c.stats()["direct_chunks"]
        assert (direct > 0) == (kind != N.VERIFY_COMMIT_LIGHT_TRUSTING), direct
        c.close()
    one.close()


@pytest.mark.parametrize("devices", [None, [0, 0, 0, 0]])
def test_configs2_scale_direct_from_pinned(gpu_ctx, devices):
    """configs[2]'s chain (7,000 heights x 150, 1% flipped) built in the
    context's pinned memory: every chunk is direct (no host pack), verified
    by the same keyed kernels, and each height's outcome is the reference
    loop's over the known flips, both kinds."""
    c = _ctx(devices=devices, keyset=True)
    sv = TU.make_validator_set(c, N_VALS)
    chain = TU.ReplayChain(c, sv, 1, 7000, pinned=c)
    for kind in (N.VERIFY_COMMIT, N.VERIFY_COMMIT_LIGHT):
        st0 = c.stats()
        chain.call(c, kind)
        _check_chain(chain, kind)
        st = c.stats()
        reach = N_VALS if kind == N.VERIFY_COMMIT else (N_VALS * 10 * 2 // 3) // 10 + 1
        assert st["signatures"] - st0["signatures"] == chain.n_heights * reach
        assert st["direct_chunks"] > st0["direct_chunks"]
    # the same bytes packed (CMTV_PIPE_DIRECT=0) give the same outcomes
    p = _ctx(devices=devices, keyset=True, CMTV_PIPE_DIRECT=0)
    chain.call(p, N.VERIFY_COMMIT)
    _check_chain(chain, N.VERIFY_COMMIT)
    assert p.stats()["direct_chunks"] == 0
    p.close()
    del chain
    c.close()


@pytest.mark.parametrize("n_vals,devices", [(150, None), (4096, None), (150, [0, 0])])
def test_latency_calls_beside_a_pipeline(n_vals, devices):
    """VerifyCommit while another thread runs a pipelined cmtv_verify_commits
    on the same context (consensus beside blocksync, round 6): the call runs
    on the device's latency stream -- the CUs the pipeline's masked chunks
    leave free (runtime.cpp LatencyStreams) -- in its under-load form (the
    registered-key quad kernel, polled through its tagged slices). Every
    outcome equals the same call's on the idle context (clean, a flipped
    signature, a wrong height), every load pass's outcomes are the reference
    loop's over the known flips, and the calls did run isolated."""
    import threading
    import time

    c = _ctx(devices=devices, keyset=True)
    lat = TU.make_validator_set(c, n_vals, offset=50_000)
    chain = TU.ReplayChain(c, TU.make_validator_set(c, N_VALS), 1, 3000, pinned=c)
    h = 77
    b, keep_b = TU.block_id_for_height(h)._c()
    cid = TU.CHAIN_ID.encode()
    vs, keep_v = lat.valset._pack()
    clean, _, _ = TU.make_commit(c, lat, height=h)
    flipped, _, _ = TU.make_commit(c, lat, height=h)
    s = bytearray(flipped.signatures[n_vals - 2].signature)
    s[9] ^= 2
    flipped.signatures[n_vals - 2].signature = bytes(s)
    packed = [(T._pack_commit(cm), hh) for cm, hh in ((clean, h), (flipped, h), (clean, h + 1))]

    def outcomes():
        out = []
        for (cm, _keep), hh in packed:
            res = N.cmtv_commit_result()
            rc = N.lib().cmtv_verify_commit(c.handle, N.VERIFY_COMMIT, 0, cid, len(cid), ctypes.byref(vs),
                                            ctypes.byref(b), hh, ctypes.byref(cm), 0, 0, ctypes.byref(res), None, 0)
            out.append((rc, res.code, res.sig_index))
        return out

    idle = outcomes()
    assert idle[0][0] == N.CMTV_OK
    assert idle[1][1] == N.COMMIT_ERR_WRONG_SIGNATURE and idle[1][2] == n_vals - 2
    assert idle[2][1] == N.COMMIT_ERR_HEIGHT
    stop = threading.Event()
    errors = []

    def load():
        try:
            while not stop.is_set():
                chain.call(c, N.VERIFY_COMMIT)
                _check_chain(chain, N.VERIFY_COMMIT)
        except Exception as e:  # reported by the main thread
            errors.append(e)

    st0 = c.stats()
    th = threading.Thread(target=load)
    th.start()
    try:
        time.sleep(0.2)
        for _ in range(50):
            assert outcomes() == idle
            time.sleep(0.001)
    finally:
        stop.set()
        th.join()
    assert not errors, errors
    st = c.stats()
    assert st["isolated_calls"] > st0["isolated_calls"]
    assert st["masked_chunks"] > st0["masked_chunks"]
    del chain, keep_b, keep_v
    c.close()
