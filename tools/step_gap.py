"""Back-to-back configs[1] steps (one 10k commit, device-resident inputs,
cmtv_verify_ed25519_multi_device as bench.py) with and without the library's
kernel-timing event pair (CMTV_TIMING): how much of ms_per_step beyond the
kernel is the event markers between consecutive launches. One JSON line.

    python tools/step_gap.py [--steps 400]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--n", type=int, default=10_000)
    a = ap.parse_args()
    import torch

    torch.cuda.init()
    from cometbft_amd import Context, pack_messages
    from cometbft_amd import testutil as TU

    dev = torch.device("cuda:0")
    kctx = Context(device=0)
    sv = TU.make_validator_set(kctx, a.n)
    m, off = pack_messages(TU.commit_messages(a.n, 1000))
    sig = kctx.sign(sv.seeds, m, off)
    t = [torch.from_numpy(np.ascontiguousarray(v)).to(dev) for v in (sv.pubkeys, sig, m, off.view(np.int32))]
    bm = torch.zeros((a.n + 63) // 64, dtype=torch.int64, device=dev)
    out = {"n": a.n, "steps": a.steps}
    for timing in ("1", "0", "16", "1", "0", "16"):
        os.environ["CMTV_TIMING"] = timing
        ctx = Context(devices=[0])
        del os.environ["CMTV_TIMING"]

        def step():
            ctx.verify_multi_device([a.n], [t[0].data_ptr()], [t[1].data_ptr()], [t[2].data_ptr()],
                                    [t[3].data_ptr()], 0, [bm.data_ptr()])
        for _ in range(200):
            step()
        ctx.sync()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        ctx.sync()
        el = time.perf_counter() - t0
        st = ctx.stats()
        key = f"timing{timing}"
        out.setdefault(key, []).append({"ms_per_step": round(el / a.steps * 1e3, 4),
                                        "kernel_ms": round(st["device_ms"] / max(1, st["timed_calls"]), 4)})
        ctx.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
