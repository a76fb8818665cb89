"""CPU/GPU crossover sweep: for
n = 1, 2, 4, ..., 65536 signatures, the end-to-end GPU time of

  * one host-API batch (cmtv_verify_ed25519: staging + H2D + kernel + D2H), and
  * one VerifyCommit of an n-validator commit through the C ABI with the
    arguments packed once, as a cgo shim holds them (cmtv_verify_commits with
    one commit: sign-bytes templated on the device, replay on the host),

against the CPU oracle (oracle/liboracle.so, the C restatement of Go 1.19
ed25519.Verify) on ONE core -- the shape of the reference's VerifyCommit loop,
a single goroutine (types/validator_set.go:685) -- and on 16 threads (the GPU
box's CPU share per GPU). The smallest n from which the commit path beats the
one-core loop at every larger n sets CMTVERIFY_MIN_BATCH.

    python tools/crossover.py [--max 65536] > profiles/r03_crossover.json
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _median_ms(fn, reps):
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t)
    return float(np.median(ts)) * 1e3


def _first_stable(rows, key):
    """smallest n from which the GPU leg wins at every larger n"""
    cross = None
    for r in reversed(rows):
        if r[key]:
            cross = r["n"]
        else:
            break
    return cross


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--max", type=int, default=65536)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--mode", type=int, default=0)
    args = ap.parse_args()

    from cometbft_amd import Context, pack_messages
    from cometbft_amd import testutil as TU
    from cometbft_amd import types as T
    from oracle import coracle

    ctx = Context(device=0)
    nmax = args.max
    sv = TU.make_validator_set(ctx, nmax)
    msgs = TU.commit_messages(nmax, 1000)
    m_all, off_all = pack_messages(msgs)
    sig_all = ctx.sign(sv.seeds, m_all, off_all)
    rows = []
    n = 1
    while n <= nmax:
        pk, sig = sv.pubkeys[:n], sig_all[:n]
        m, off = m_all[: off_all[n]], off_all[: n + 1]
        reps = max(5, min(300, 40000 // n))
        for _ in range(5):
            ctx.verify(pk, sig, m, off, args.mode)
        g_host = _median_ms(lambda: ctx.verify(pk, sig, m, off, args.mode), reps)
        # the same n validators as a commit (types/validator_set.go:667)
        svn = TU.make_validator_set(ctx, n)
        commit, _, _ = TU.make_commit(ctx, svn, 1000)
        packed = T.PackedCommits(0, TU.CHAIN_ID, [(svn.valset, TU.block_id_for_height(1000), 1000, commit)],
                                 mode=args.mode)
        for _ in range(5):
            packed.call(ctx)
        assert packed.rcs[0] == 0
        g_commit = _median_ms(lambda: packed.call(ctx), reps)
        creps = max(3, min(50, 2000 // n))
        c1 = _median_ms(lambda: coracle.verify_batch(pk, sig, m, off, args.mode, nthreads=1), creps)
        cT = _median_ms(lambda: coracle.verify_batch(pk, sig, m, off, args.mode, nthreads=min(args.threads, n)),
                        creps)
        rows.append({"n": n, "gpu_host_ms": round(g_host, 4), "gpu_commit_ms": round(g_commit, 4),
                     "cpu_1core_ms": round(c1, 4), f"cpu_{args.threads}thr_ms": round(cT, 4),
                     "commit_beats_1core": bool(g_commit < c1), "commit_beats_threads": bool(g_commit < cT),
                     "host_beats_1core": bool(g_host < c1), "host_beats_threads": bool(g_host < cT)})
        print(json.dumps(rows[-1]), file=sys.stderr, flush=True)
        n *= 2
    out = {"mode": args.mode, "cpu_threads": args.threads,
           "cpu": "oracle/liboracle.so (C restatement of Go 1.19 ed25519.Verify)",
           "crossover_commit_vs_1core": _first_stable(rows, "commit_beats_1core"),
           "crossover_commit_vs_threads": _first_stable(rows, "commit_beats_threads"),
           "crossover_host_vs_1core": _first_stable(rows, "host_beats_1core"),
           "crossover_host_vs_threads": _first_stable(rows, "host_beats_threads"),
           "rows": rows}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
