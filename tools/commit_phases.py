"""VerifyCommit at configs[1] scale, phase by phase.

For each n: the host-API batch (cmtv_verify_ed25519) and one n-validator
VerifyCommit through the C ABI with its arguments packed once
(cmtv_verify_commits, as a cgo shim holds them), p50 / p99 wall, the mean
kernel time, and -- from a context opened with CMTV_HOST_PHASES=1 -- the mean
host time per call in each phase (prepare: the plan and the signature batch;
stage: copies into pinned staging; launch: H2D + kernel enqueue; wait: stream
sync; post: bitmap -> verdicts; replay: the reference loop). One JSON line per
n on stdout (the library prints its phase line on stderr at close; both are
merged here).

    python tools/commit_phases.py [--n 4096,8192,10000,16384] [--iters 200]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _pct(fn, iters):
    ts = []
    for _ in range(iters):
        t = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t)
    ts = np.array(ts) * 1e3
    return round(float(np.percentile(ts, 50)), 4), round(float(np.percentile(ts, 99)), 4)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", default="4096,8192,10000,16384")
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--mode", type=int, default=0)
    ap.add_argument("--zc-max", type=int, default=0, help="CMTV_ZC_MAX for the commit context (0: default; the knob was retired in round 5)")
    ap.add_argument("--ctx-env", default="", help="KEY=VAL,... set while the commit context opens")
    a = ap.parse_args()
    import torch

    torch.cuda.init()
    from cometbft_amd import Context
    from cometbft_amd import testutil as TU
    from cometbft_amd import types as T

    for n in [int(x) for x in a.n.split(",")]:
        keyctx = Context(device=0)
        sv = TU.make_validator_set(keyctx, n)
        commit, _, _ = TU.make_commit(keyctx, sv, 1000)
        msgs = TU.commit_messages(n, 1000)
        from cometbft_amd import pack_messages

        m, off = pack_messages(msgs)
        sig = keyctx.sign(sv.seeds, m, off)
        row = {"n": n, "zc_max": a.zc_max or None, "ctx_env": a.ctx_env or None}
        for _ in range(5):
            keyctx.verify(sv.pubkeys, sig, m, off, a.mode)
        row["host_api_p50_ms"], row["host_api_p99_ms"] = _pct(lambda: keyctx.verify(sv.pubkeys, sig, m, off, a.mode),
                                                              a.iters)
        os.environ["CMTV_HOST_PHASES"] = "1"
        extra = dict(kv.split("=", 1) for kv in a.ctx_env.split(",") if kv)
        if a.zc_max:
            extra["CMTV_ZC_MAX"] = str(a.zc_max)
        os.environ.update(extra)
        ctx = Context(device=0)
        del os.environ["CMTV_HOST_PHASES"]
        for k in extra:
            os.environ.pop(k, None)
        packed = T.PackedCommits(0, TU.CHAIN_ID, [(sv.valset, TU.block_id_for_height(1000), 1000, commit)],
                                 mode=a.mode)
        for _ in range(5):
            packed.call(ctx)
        assert packed.rcs[0] == 0
        st0 = ctx.stats()
        row["commit_p50_ms"], row["commit_p99_ms"] = _pct(lambda: packed.call(ctx), a.iters)
        st1 = ctx.stats()
        row["kernel_ms"] = round((st1["device_ms"] - st0["device_ms"]) / max(1, st1["timed_calls"] - st0["timed_calls"]), 4)
        row["cpu_p50_1core_ms"] = None
        row["commit_over_host"] = round(row["commit_p50_ms"] / row["host_api_p50_ms"], 3)
        print(json.dumps(row), flush=True)
        sys.stderr.flush()
        ctx.close()  # prints the phase line (stderr)
        sys.stderr.flush()
        keyctx.close()


if __name__ == "__main__":
    main()
