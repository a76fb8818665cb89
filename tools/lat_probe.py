"""Latency probe (dev tool): p50 of cmtv_verify_commit on a 150-validator
commit through the C ABI, plus the kernel-only time from the context's
launch-stream events. Run under `rocprofv3 --runtime-trace` to see the
per-call API / copy / kernel timeline (tools/lat_timeline.py reads it)."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

from cometbft_amd import Context
from cometbft_amd import _native as N
from cometbft_amd import testutil as TU
from cometbft_amd import types as T

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 200
ctx = Context(device=0)
sv = TU.make_validator_set(ctx, 150)
commit, msgs, sigs = TU.make_commit(ctx, sv, height=1000)
bid = TU.block_id_for_height(1000)
vs, kv = sv.valset._pack()
cm, kc = T._pack_commit(commit)
bcb, kb = bid._c()
res = N.cmtv_commit_result()
cid = TU.CHAIN_ID.encode()
L = N.lib()


def call():
    rc = L.cmtv_verify_commit(ctx.handle, N.VERIFY_COMMIT, 0, cid, len(cid), ctypes.byref(vs), ctypes.byref(bcb),
                              1000, ctypes.byref(cm), 0, 0, ctypes.byref(res), None, 0)
    assert rc == 0, rc


for _ in range(20):
    call()
ts = []
k0 = ctx.stats()["device_ms"]
for _ in range(iters):
    t = time.perf_counter()
    call()
    ts.append(time.perf_counter() - t)
k1 = ctx.stats()["device_ms"]
ts = np.array(ts) * 1e3
print(f"verify_commit 150: p50 {np.percentile(ts, 50):.4f} ms p99 {np.percentile(ts, 99):.4f} ms "
      f"kernel mean {(k1 - k0) / iters:.4f} ms", flush=True)
