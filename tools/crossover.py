"""CPU/GPU crossover sweep: for n = 1, 2, 4, ..., 65536
signatures, the end-to-end GPU time of one host-API batch (H2D + kernel + D2H)
against the all-core CPU oracle (C restatement of the Go 1.19 verify). The
smallest n where the GPU wins sets CMTVERIFY_MIN_BATCH.

    python tools/crossover.py [--max 65536] [--threads 16] > profiles/crossover.json
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--max", type=int, default=65536)
    ap.add_argument("--threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "16")))
    ap.add_argument("--mode", type=int, default=0)
    args = ap.parse_args()

    from cometbft_amd import Context, pack_messages
    from cometbft_amd import testutil as TU
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
        reps = max(3, min(200, 20000 // n))
        for _ in range(3):
            ctx.verify(pk, sig, m, off, args.mode)
        t = time.perf_counter()
        for _ in range(reps):
            ctx.verify(pk, sig, m, off, args.mode)
        g = (time.perf_counter() - t) / reps
        creps = max(1, min(50, 4000 // n))
        t = time.perf_counter()
        for _ in range(creps):
            coracle.verify_batch(pk, sig, m, off, args.mode, nthreads=min(args.threads, n))
        c = (time.perf_counter() - t) / creps
        rows.append({"n": n, "gpu_e2e_ms": round(g * 1e3, 4), "cpu_ms": round(c * 1e3, 4),
                     "gpu_faster": bool(g < c)})
        print(json.dumps(rows[-1]), file=sys.stderr, flush=True)
        n *= 2
    cross = next((r["n"] for r in rows if r["gpu_faster"]), None)
    print(json.dumps({"cpu_threads": args.threads, "mode": args.mode, "crossover_n": cross, "rows": rows}))


if __name__ == "__main__":
    main()
