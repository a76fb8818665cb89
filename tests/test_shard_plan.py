"""CPU test of the multi-device shard planner (cometbft_amd/csrc/shard.h,
host-compiled by tests/host/shardcheck.cpp): for every batch size and
device count the shards are contiguous, cover [0, n) exactly once, start on
64-signature (bitmap-word) boundaries so their bitmaps concatenate in place,
and a batch uses as many devices as give each at least shard_min signatures
(partial-G plans: a 40k batch runs on 4 of 8 GPUs)."""
import os
import struct
import subprocess

import numpy as np

from test_host_math import _build

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "host", "shardcheck.cpp")
BIN = os.path.join(ROOT, "build", "shardcheck")


def test_shard_plan_invariants():
    binary = _build(SRC, BIN, ["-std=c++17"])
    rng = np.random.default_rng(8)
    cases = [(n, g, m) for n in (0, 1, 63, 64, 65, 1000, 8191, 8192, 65536, 15_000_000)
             for g in (1, 2, 3, 4, 7, 8) for m in (0, 64, 8192)]
    cases += [(int(rng.integers(0, 2**26)), int(rng.integers(1, 9)), int(rng.choice([0, 1, 64, 8192])))
              for _ in range(2000)]
    buf = b"".join(struct.pack("<3Q", *c) for c in cases)
    out = subprocess.run([binary], input=buf, capture_output=True, check=True).stdout
    plans = np.frombuffer(out, np.uint64).reshape(-1, 3)
    for (n, g, m), (G, S, W) in zip(cases, plans.tolist()):
        per = max(m, 64)
        assert 1 <= G <= g
        # as many devices as get shard_min signatures each, at least one
        assert G == min(g, max(1, n // per)), (n, g, m, G)
        if G == 1:
            assert S == n
            continue
        assert S % 64 == 0 and W == S // 64
        # every used device has at least shard_min signatures but the last
        # (ceil(n / G) >= per, rounded up to whole words)
        assert S >= per
        los = [min(n, k * S) for k in range(G)]
        his = [min(n, (k + 1) * S) for k in range(G)]
        assert los[0] == 0 and his[-1] == n, (n, g, m)
        assert all(his[k] == los[k + 1] for k in range(G - 1))
        # every shard but the tail is full; the gathered bitmap (G x W words)
        # holds the batch's ceil(n / 64) words
        assert all(his[k] - los[k] == S for k in range(G) if his[k] < n)
        assert G * W >= (n + 63) // 64
        # balanced: no device gets more than one 64-signature word over n / G
        assert S - (n + G - 1) // G < 64


def test_partial_device_plans():
    """The VERDICT r2 case: 40k signatures on 8 GPUs at the default
    shard_min (8192) run on 4 devices, each a whole-word shard."""
    binary = _build(SRC, BIN, ["-std=c++17"])
    cases = [(40_000, 8, 8192), (16_384, 8, 8192), (16_383, 8, 8192), (8192 * 8, 8, 8192), (10**6, 8, 8192),
             (24_576, 3, 8192), (100, 8, 0)]
    buf = b"".join(struct.pack("<3Q", *c) for c in cases)
    out = subprocess.run([binary], input=buf, capture_output=True, check=True).stdout
    got = [tuple(r) for r in np.frombuffer(out, np.uint64).reshape(-1, 3).tolist()]
    assert got[0] == (4, 10_048, 157)
    assert got[1] == (2, 8192, 128)
    assert got[2][0] == 1
    assert got[3] == (8, 8192, 128)
    assert got[4][0] == 8
    assert got[5] == (3, 8192, 128)
    assert got[6][0] == 1
