"""Multi-rank path on CPU: world_size-2 gloo group. Exercises the sharding,
bitmap packing and the all-gather that bench.py / parallel.verify_sharded use
on RCCL; the per-rank verdicts come from the oracle standing in for the
device (no GPU here)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from cometbft_amd import parallel as P


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_ranges_cover_and_align():
    for n in (0, 1, 63, 64, 65, 1000, 10_000, 15_000_000):
        for world in (1, 2, 3, 4, 8):
            spans = [P.shard_range(n, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            for (a, b), (c, d) in zip(spans, spans[1:]):
                assert b == c
            assert all(a % 64 == 0 for a, b in spans if b > a)


def test_pack_unpack_roundtrip():
    rng = np.random.default_rng(3)
    for n in (1, 63, 64, 65, 500):
        v = (rng.random(n) < 0.7).astype(np.uint8)
        w = P.pack_bitmap(v)
        assert w.size == -(-n // 64)
        assert np.array_equal(P.unpack_bitmap(w, n), v)


def _worker(rank, world, port, data, q):
    import torch
    import torch.distributed as dist

    from oracle import coracle

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pk, sig, m, off, mode = data
    n = len(off) - 1
    lo, hi = P.shard_range(n, world, rank)
    per = P.shard_size(n, world)
    # device stand-in: verdicts for this rank's shard
    local = coracle.verify_batch(pk[lo:hi], sig[lo:hi], m, off[lo:hi + 1], mode) if hi > lo else np.zeros(0, np.uint8)
    words = torch.from_numpy(P.pack_bitmap(local, per // 64).view(np.int64).copy())
    out = P.gather_bitmaps(words, n, world)
    q.put((rank, out.numpy().view(np.uint64).copy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n", [130, 257])
def test_gloo_world2_gathers_global_bitmap(n):
    from oracle import coracle

    rng = np.random.default_rng(n)
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    msgs = [rng.integers(0, 256, int(rng.integers(0, 150)), dtype=np.uint8).tobytes() for _ in range(n)]
    m, off = coracle.pack_msgs(msgs)
    sig = coracle.sign_batch(seeds, m, off, nthreads=4)
    pk = coracle.pubkeys_from_seeds(seeds)
    sig[rng.random(n) < 0.25, 40] ^= 1
    expect = coracle.verify_batch(pk, sig, m, off, 0, nthreads=4)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, (pk, sig, m, off, 0), q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(2):
        assert np.array_equal(P.unpack_bitmap(res[r], n), expect)
