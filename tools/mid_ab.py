"""Host-API batch and VerifyCommit (C ABI, packed once) medians at the
row/oct crossover sizes, for an A/B of the forms (dev tool):

    CMTV_FORM=oct2 python tools/mid_ab.py 768 1024 1536
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def med_ms(fn, reps):
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t)
    return float(np.median(ts)) * 1e3


def main():
    from cometbft_amd import Context, pack_messages
    from cometbft_amd import testutil as TU
    from cometbft_amd import types as T

    sizes = [int(x) for x in sys.argv[1:]] or [768, 1024, 1536]
    ctx = Context(device=0)
    tag = os.environ.get("TAG") or os.environ.get("CMTV_FORM", "default")
    for n in sizes:
        sv = TU.make_validator_set(ctx, n)
        msgs = TU.commit_messages(n, 1000)
        m, off = pack_messages(msgs)
        sig = ctx.sign(sv.seeds, m, off)
        for _ in range(10):
            ctx.verify(sv.pubkeys, sig, m, off, 0)
        host = med_ms(lambda: ctx.verify(sv.pubkeys, sig, m, off, 0), 300)
        commit, _, _ = TU.make_commit(ctx, sv, 1000)
        packed = T.PackedCommits(0, TU.CHAIN_ID, [(sv.valset, TU.block_id_for_height(1000), 1000, commit)])
        for _ in range(10):
            packed.call(ctx)
        assert packed.rcs[0] == 0
        cm = med_ms(lambda: packed.call(ctx), 300)
        print(f"ROW_MAX={tag} n={n} host_ms={host:.4f} commit_ms={cm:.4f}", flush=True)


if __name__ == "__main__":
    main()
