"""CPU test of the multi-device shard planner (cometbft_amd/csrc/shard.h,
host-compiled by tests/host/shardcheck.cpp): for every batch size and
device count the shards are contiguous, cover [0, n) exactly once, start on
64-signature (bitmap-word) boundaries so their bitmaps concatenate in place,
and small batches stay on one device."""
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
        assert 1 <= G <= g
        if g > 1 and n < g * max(m, 64):
            assert G == 1, (n, g, m)
        if G == 1:
            assert S == n
            continue
        assert G == g and S % 64 == 0 and W == S // 64
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
