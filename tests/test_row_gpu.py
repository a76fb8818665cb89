"""The one-signature-per-wave row kernel (cometbft_amd/csrc/row.h,
k_verify_row_split) and its four-wave form (k_verify_row4_split): the
production kernels for Ed25519 batches up to 1,536 signatures (runtime.cpp
kRowMax; 256 and below on the four-wave form), i.e. the 150-validator
VerifyCommit.

Its corpus, ragged-size, wide-schedule and forced-wide parity runs live with
the other kernels' (test_gpu_parity.py, test_wide_gpu.py: kernels "row4", "row");
here: the bitmap assembly (the last wave of a launch packs the words from a
ring slot of verdict bytes) under concurrent launches on several streams,
and the default dispatch at the commit sizes. Oracle: oracle/liboracle.so
(the C restatement of Go 1.19 ed25519.Verify, crypto/ed25519/ed25519.go:148).
"""
import threading

import numpy as np
import pytest

from oracle import coracle
from cometbft_amd import MODE_GO_STDLIB, MODE_ZIP215, Context

pytestmark = pytest.mark.gpu


def _batch(n, seed, flip=0.1):
    rng = np.random.default_rng(seed)
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    msgs = [rng.integers(0, 256, 116, dtype=np.uint8).tobytes() for _ in range(n)]
    m, off = coracle.pack_msgs(msgs)
    sig = coracle.sign_batch(seeds, m, off, nthreads=8).copy()
    for i in np.nonzero(rng.random(n) < flip)[0]:
        sig[i, rng.integers(0, 64)] ^= 1 << rng.integers(0, 8)
    return coracle.pubkeys_from_seeds(seeds), sig, m, off


@pytest.mark.parametrize("n", [150, 255, 256, 257, 767, 768, 769, 1024, 1535, 1536, 1537])
def test_default_dispatch_commit_sizes(gpu_ctx, n):
    """The default context at and around the row crossover, both modes,
    verdict bytes and bitmap words (no bit past n set)."""
    pk, sig, m, off = _batch(n, 500 + n)
    for mode in (MODE_GO_STDLIB, MODE_ZIP215):
        exp = coracle.verify_batch(pk, sig, m, off, mode, nthreads=8)
        got, words = gpu_ctx.verify(pk, sig, m, off, mode, bitmap=True)
        assert np.array_equal(got, exp)
        bits = np.unpackbits(words.view(np.uint8), bitorder="little")
        assert np.array_equal(bits[:n], exp) and not bits[n:].any()



@pytest.mark.parametrize("n", [256, 257, 400, 512, 513])
def test_default_keyed_dispatch_around_the_keyed_row_crossover(gpu_ctx, n):
    """Registered keys on the default context at and around kKeyedRowMax
    (512: the keyed row kernel, two workgroups per CU above 256; the keyed
    quad kernel past it), both modes, verdict bytes against the oracle."""
    pk, sig, m, off = _batch(n, 1700 + n, flip=0.15)
    ks = gpu_ctx.register_keys(pk)
    try:
        for mode in (MODE_GO_STDLIB, MODE_ZIP215):
            exp = coracle.verify_batch(pk, sig, m, off, mode, nthreads=8)
            got = gpu_ctx.verify_indexed(ks, np.arange(n, dtype=np.uint32), sig, m, off, mode)
            assert np.array_equal(got, exp), np.nonzero(got != exp)[0][:10]
    finally:
        ks.free()

def test_concurrent_row_launches_pack_their_own_bitmaps():
    """5 threads, each on its own stream, 25 device-resident row launches of
    different sizes with bitmaps (1,200: two row workgroups per CU): every
    launch takes its own ring slot, so each bitmap holds exactly its own
    verdicts."""
    import torch

    ctx = Context(device=0)
    dev = torch.device("cuda:0")
    jobs = []
    for j, n in enumerate((150, 64, 333, 700, 1200)):
        pk, sig, m, off = _batch(n, 900 + j, flip=0.2)
        exp = coracle.verify_batch(pk, sig, m, off, MODE_GO_STDLIB, nthreads=8)
        jobs.append((n, pk, sig, m, off, exp))
    errors = []

    def run(j):
        n, pk, sig, m, off, exp = jobs[j]
        try:
            s = torch.cuda.Stream(device=dev)
            t = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in
                 {"pk": pk, "sig": sig, "m": m, "off": off.view(np.int32)}.items()}
            words = (n + 63) // 64
            bm = torch.zeros(words, dtype=torch.int64, device=dev)
            want = np.packbits(exp, bitorder="little")
            want = np.pad(want, (0, 8 * words - want.size)).view(np.int64)
            for _ in range(25):
                bm.fill_(-1)
                torch.cuda.synchronize(dev)
                ctx.verify_device(n, t["pk"].data_ptr(), t["sig"].data_ptr(), t["m"].data_ptr(),
                                  t["off"].data_ptr(), MODE_GO_STDLIB, 0, bm.data_ptr(), s.cuda_stream)
                s.synchronize()
                got = bm.cpu().numpy()
                if not np.array_equal(got, want):
                    errors.append((j, np.nonzero(got != want)[0][:4].tolist()))
        except Exception as e:  # noqa: BLE001
            errors.append((j, repr(e)))

    ths = [threading.Thread(target=run, args=(j,)) for j in range(len(jobs))]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=110)
    assert not any(t.is_alive() for t in ths)
    assert not errors, errors[:5]


def test_concurrent_keyed_row_launches():
    """The keyed row kernel takes ring slots too: 3 threads on their own
    streams, registered keys, 20 device-resident launches each with bitmaps,
    sizes inside the keyed row range."""
    import torch

    ctx = Context(device=0)
    dev = torch.device("cuda:0")
    jobs = []
    for j, n in enumerate((150, 40, 256)):
        pk, sig, m, off = _batch(n, 1300 + j, flip=0.2)
        ks = ctx.register_keys(pk)
        exp = coracle.verify_batch(pk, sig, m, off, MODE_ZIP215, nthreads=8)
        jobs.append((n, ks, sig, m, off, exp))
    errors = []

    def run(j):
        n, ks, sig, m, off, exp = jobs[j]
        try:
            s = torch.cuda.Stream(device=dev)
            t = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in
                 {"idx": np.arange(n, dtype=np.int32), "sig": sig, "m": m, "off": off.view(np.int32)}.items()}
            words = (n + 63) // 64
            bm = torch.zeros(words, dtype=torch.int64, device=dev)
            want = np.packbits(exp, bitorder="little")
            want = np.pad(want, (0, 8 * words - want.size)).view(np.int64)
            for _ in range(20):
                bm.fill_(-1)
                torch.cuda.synchronize(dev)
                ctx.verify_indexed_device(ks, n, t["idx"].data_ptr(), t["sig"].data_ptr(), t["m"].data_ptr(),
                                          t["off"].data_ptr(), MODE_ZIP215, 0, bm.data_ptr(), s.cuda_stream)
                s.synchronize()
                got = bm.cpu().numpy()
                if not np.array_equal(got, want):
                    errors.append((j, np.nonzero(got != want)[0][:4].tolist()))
        except Exception as e:  # noqa: BLE001
            errors.append((j, repr(e)))

    ths = [threading.Thread(target=run, args=(j,)) for j in range(3)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=110)
    assert not any(t.is_alive() for t in ths)
    assert not errors, errors[:5]
    for job in jobs:
        job[1].free()


@pytest.mark.parametrize("mode", [MODE_GO_STDLIB, MODE_ZIP215])
def test_row_kernels_on_random_malformed_inputs(form_ctx, mode):
    """Random bytes where the corpus has crafted ones: 240 signatures whose A,
    R and s are random (mostly off-curve points, s >= L, set high bits), mixed
    with honest ones and with honest R / A paired with a wrong s, through every
    row form and the keyed row kernel, against the C oracle bit for bit."""
    rng = np.random.default_rng(4242 + mode)
    n = 240
    pk, sig, m, off = _batch(n, 77, flip=0.0)
    pk, sig = pk.copy(), sig.copy()
    kind = rng.integers(0, 6, n)
    for i in range(n):
        if kind[i] == 0:
            pk[i] = rng.integers(0, 256, 32, dtype=np.uint8)          # random A
        elif kind[i] == 1:
            sig[i, :32] = rng.integers(0, 256, 32, dtype=np.uint8)    # random R
        elif kind[i] == 2:
            sig[i, 32:] = rng.integers(0, 256, 32, dtype=np.uint8)    # random s (often >= L)
        elif kind[i] == 3:
            sig[i, 63] |= 0x80 >> int(rng.integers(0, 3))              # s's high bits
        elif kind[i] == 4:
            pk[i, 31] ^= 0x80                                          # A's sign bit
    exp = coracle.verify_batch(pk, sig, m, off, mode, nthreads=8)
    assert 0 < exp.sum() < n
    for ctx in (form_ctx("row4"), form_ctx("row")):
        got = ctx.verify(pk, sig, m, off, mode)
        assert np.array_equal(got, exp), np.nonzero(got != exp)[0][:10]
    krow = form_ctx("krow")
    ks = krow.register_keys(pk)
    got = krow.verify_indexed(ks, np.arange(n, dtype=np.uint32), sig, m, off, mode)
    assert np.array_equal(got, exp), np.nonzero(got != exp)[0][:10]
    ks.free()


def test_host_batches_read_the_completion_flag():
    """Small single-device host batches on a row kernel return when the
    kernel's completion flag arrives (kernels.h RowSlot, runtime.cpp
    wait_row_done), not when the stream drains: back-to-back calls of ragged
    sizes (word and half-word edges) and both modes, plain and registered-key,
    each against the oracle bit for bit, and each counted in polled_calls; a
    batch past the row range synchronises instead. CMTV_HOST_POLL=0 polls
    nothing and gives the same verdicts."""
    from conftest import _env_ctx

    cases = []
    for j, n in enumerate((1, 31, 32, 33, 63, 64, 65, 150, 256, 257, 700)):
        pk, sig, m, off = _batch(n, 2100 + j, flip=0.25)
        cases.append((n, pk, sig, m, off, [coracle.verify_batch(pk, sig, m, off, md, nthreads=8)
                                           for md in (MODE_GO_STDLIB, MODE_ZIP215)]))
    for poll in (1, 0):
        ctx = _env_ctx(CMTV_HOST_POLL=poll)
        before = ctx.stats()["polled_calls"]
        calls = 0
        for rep in range(3):
            for n, pk, sig, m, off, exps in cases:
                for md, exp in zip((MODE_GO_STDLIB, MODE_ZIP215), exps):
                    got, words = ctx.verify(pk, sig, m, off, md, bitmap=True)
                    bits = np.unpackbits(words.view(np.uint8), bitorder="little")
                    assert np.array_equal(got, exp) and np.array_equal(bits[:n], exp) and not bits[n:].any()
                    calls += 1
        n, pk, sig, m, off, exps = cases[7]
        ks = ctx.register_keys(pk)
        for md, exp in zip((MODE_GO_STDLIB, MODE_ZIP215), exps):
            assert np.array_equal(ctx.verify_indexed(ks, np.arange(n, dtype=np.uint32), sig, m, off, md), exp)
            calls += 1
        ks.free()
        assert ctx.stats()["polled_calls"] - before == (calls if poll else 0)
        # past the row kernels (kRowMax 1,536; the oct kernel): the stream is synchronised
        pk, sig, m, off = _batch(2000, 2200)
        exp = coracle.verify_batch(pk, sig, m, off, MODE_GO_STDLIB, nthreads=8)
        assert np.array_equal(ctx.verify(pk, sig, m, off, MODE_GO_STDLIB), exp)
        assert ctx.stats()["polled_calls"] - before == (calls if poll else 0)
        ctx.close()
