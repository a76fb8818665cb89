"""bench.py -- headline benchmark: Ed25519 commit-signature verification on MI355X.

Metric (BASELINE.json): "Ed25519 verifs/sec at 1/2/4/8 GPUs + p50 VerifyCommit
latency, 150 vals".

Step = verify one synthetic 10,000-validator commit (BASELINE.json configs[1])
per GPU: its (pk, sig, sign-bytes) already resident in HBM, the gfx950 verify
kernel writes the per-signature verdict bytes and the packed verdict bitmap;
for N > 1 each rank verifies its own commit (weak scaling, no data-path
collective) and the bitmaps are all-gathered over RCCL so every rank holds the
job's full verdict vector (the exchange the caller needs).

Extra fields on the JSON line:
  roofline       -- VALU integer-MAC roofline of the verify kernel: algorithmic
                    work = 300,000 32x32->64 MACs per verification
                    per launch / the kernel's mean duration (HIP events on the
                    launch stream); peak = measured v_mad_u64_u32 rate
                    (tools/microbench, profiles/r01_int_rates.txt)
  cpu_baseline   -- oracle/liboracle.so (C restatement of the Go-1.19 verify) on
                    the host cores, bounded sample, rank 0 only
  latency_150    -- p50/p99 of cmtv_verify_commit (VerifyCommit, 150 validators:
                    sign-bytes + H2D + kernel + D2H + reference-loop replay),
                    beside the oracle's single-core sequential VerifyCommit time
  replay_150     -- blocksync replay per height (light + 2 x full VerifyCommit of
                    a 150-validator commit): plain, with the verdict cache, and
                    with cross-height batching (N=1 only)
  replay_c3      -- configs[2]: 100k commits x 150 validators (15M signatures)
                    sharded by height across the N ranks (strong scaling),
                    registered-key kernel + RCCL bitmap all-gather, 1% flipped
                    signatures checked exactly; the generic kernel beside it
  sr25519        -- configs[4]: 10k sr25519 verifications per step (N=1 only),
                    with the C restatement on the host cores as its CPU baseline
Run: python bench.py [--gpus N --steps K --warmup W]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Ed25519 verifs/sec at 1/2/4/8 GPUs + p50 VerifyCommit latency, 150 vals"
MACS_PER_VERIFY = 300_000          # 3,000 field mults x 100 limb MACs
INT_MAC_PEAK_T = 33.0              # measured v_mad_u64_u32 lane-ops/s, 1e12 (profiles/r01_int_rates.txt)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--n", type=int, default=10_000, help="signatures per GPU per step")
    ap.add_argument("--mode", choices=["go", "zip215"], default="go")
    ap.add_argument("--cpu-seconds", type=float, default=20.0, help="CPU-seconds of oracle work for cpu_baseline")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--latency-iters", type=int, default=200)
    ap.add_argument("--no-latency", action="store_true")
    ap.add_argument("--no-c3", action="store_true", help="skip the configs[2] 15M-signature replay side line")
    ap.add_argument("--c3-heights", type=int, default=100_000, help="configs[2] commits (150 validators each)")
    ap.add_argument("--no-sr25519", action="store_true", help="skip the configs[4] sr25519 side measurement")
    return ap.parse_args()


def cpu_threads() -> int:
    for k in ("OMP_NUM_THREADS", "CMTV_CPU_THREADS"):
        v = os.environ.get(k)
        if v and v.isdigit() and int(v) > 0:
            return min(int(v), os.cpu_count() or 1)
    return min(16, os.cpu_count() or 1)


def cpu_baseline(pk, sig, m, off, mode, cpu_seconds):
    """The oracle (C restatement of Go 1.19 crypto/ed25519.Verify) on the host
    cores over the same commit, repeated to a bounded amount of CPU work."""
    from oracle import coracle  # the checker / CPU baseline only

    threads = cpu_threads()
    n = len(off) - 1
    t = time.perf_counter()
    out = coracle.verify_batch(pk, sig, m, off, mode, nthreads=threads)
    first = time.perf_counter() - t
    assert out.all(), "oracle rejected an honest synthetic signature"
    reps = max(1, int(cpu_seconds / max(first * threads, 1e-3)))
    t = time.perf_counter()
    for _ in range(reps):
        coracle.verify_batch(pk, sig, m, off, mode, nthreads=threads)
    dt = time.perf_counter() - t
    # single-core figure on a short slice
    sl = min(n, 400)
    t = time.perf_counter()
    coracle.verify_batch(pk[:sl], sig[:sl], m, off[: sl + 1], mode, nthreads=1)
    one = sl / (time.perf_counter() - t)
    return {"value": round(reps * n / dt, 1), "unit": "verifs/s", "cores": threads, "kind": "port",
            "sample": f"{n}-signature synthetic commit x {reps} passes, {threads} threads, oracle/liboracle.so "
                      f"(C restatement of Go 1.19 ed25519.Verify)",
            "single_core_verifs_per_s": round(one, 1), "seconds": round(dt, 2),
            "host_cpu": _cpu_model()}


def sr25519_line(ctx, dev, n, steps, cpu_seconds, with_cpu):
    """configs[4]: sr25519 batch verification of a 10k-signature batch (150
    keys, 116-byte messages), inputs resident in HBM, timed with HIP events on
    the launch stream; the C restatement (oracle/liboracle.so) on the host
    cores as its CPU baseline."""
    import torch
    from oracle import coracle  # synthetic data + CPU baseline only

    rng = np.random.default_rng(4)
    minis = rng.integers(0, 256, (150, 32), dtype=np.uint8)
    kidx = (np.arange(n) % 150).astype(np.uint32)
    msgs = [rng.integers(0, 256, 116, dtype=np.uint8).tobytes() for _ in range(n)]
    m, off = coracle.pack_msgs(msgs)
    sig = coracle.sr25519_sign_batch(minis, m, off, key_idx=kidx)
    pk = coracle.sr25519_pubkeys(minis)[kidx]
    d_pk = torch.from_numpy(np.ascontiguousarray(pk)).to(dev)
    d_sig = torch.from_numpy(sig).to(dev)
    d_m = torch.from_numpy(m).to(dev)
    d_off = torch.from_numpy(off.view(np.int32)).to(dev)
    d_valid = torch.zeros(n, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)

    def run():
        ctx.verify_sr25519_device(n, d_pk.data_ptr(), d_sig.data_ptr(), d_m.data_ptr(), d_off.data_ptr(),
                                  d_valid.data_ptr(), 0, stream.cuda_stream)

    for _ in range(3):
        run()
    torch.cuda.synchronize(dev)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    t0 = time.perf_counter()
    for a, b in evs:
        a.record(stream)
        run()
        b.record(stream)
    torch.cuda.synchronize(dev)
    wall = (time.perf_counter() - t0) / steps
    kms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    res = {"workload": f"configs[4]: {n} sr25519 signatures over 150 keys, 116-byte messages, inputs in HBM",
           "value": round(n / wall, 1), "unit": "verifs/s", "ms_per_step": round(wall * 1e3, 4),
           "kernel_ms": round(kms, 4), "verdicts_ok": bool(int(d_valid.sum().item()) == n)}
    if with_cpu:
        threads = cpu_threads()
        t = time.perf_counter()
        out = coracle.sr25519_verify_batch(pk, sig, m, off, nthreads=threads)
        first = time.perf_counter() - t
        assert out.all()
        reps = max(1, int(cpu_seconds / max(first * threads, 1e-3)))
        t = time.perf_counter()
        for _ in range(reps):
            coracle.sr25519_verify_batch(pk, sig, m, off, nthreads=threads)
        dt = time.perf_counter() - t
        res["cpu_baseline"] = {"value": round(reps * n / dt, 1), "unit": "verifs/s", "cores": threads, "kind": "port",
                               "sample": f"{n}-signature batch x {reps} passes, {threads} threads, oracle/liboracle.so "
                                         f"(C restatement of go-schnorrkel verify)", "seconds": round(dt, 2)}
        res["cpu_baseline"]["gpu_over_cpu"] = round(res["value"] / res["cpu_baseline"]["value"], 1)
    return res


def replay_line(dev_index, heights=60, n_vals=150):
    """SURVEY 8f ranks 2-3 on the blocksync pattern: per height
    VerifyCommitLight + VerifyCommit + VerifyCommit of one 150-validator
    commit (blockchain/v0/reactor.go:366-400), end to end through the host API
    (sign-bytes, H2D, kernel, D2H, replay), plain vs with the verdict cache;
    and cross-height batching (cmtv_verify_commits) of the same commits."""
    from cometbft_amd import Context
    from cometbft_amd import testutil as TU
    from cometbft_amd import types as T

    plain = Context(device=dev_index)
    cached = Context(device=dev_index)
    cached.verdict_cache(1 << 20)
    sv = TU.make_validator_set(plain, n_vals)
    chain = []
    for h in range(2000, 2000 + heights):
        commit, _, _ = TU.make_commit(plain, sv, h)
        chain.append((sv.valset, TU.block_id_for_height(h), h, commit))

    def blocksync(ctx):
        for vals, bid, h, c in chain:
            vals.verify_commit_light(TU.CHAIN_ID, bid, h, c, ctx=ctx)
            vals.verify_commit(TU.CHAIN_ID, bid, h, c, ctx=ctx)
            vals.verify_commit(TU.CHAIN_ID, bid, h, c, ctx=ctx)

    blocksync(plain)  # warm-up
    t = time.perf_counter()
    blocksync(plain)
    t_plain = (time.perf_counter() - t) / heights
    t = time.perf_counter()
    blocksync(cached)  # cold cache: one device call per height
    t_cached = (time.perf_counter() - t) / heights
    T.verify_commits(0, TU.CHAIN_ID, chain, ctx=plain)
    t = time.perf_counter()
    errs = T.verify_commits(0, TU.CHAIN_ID, chain, ctx=plain)
    t_batch = (time.perf_counter() - t) / heights
    assert all(e is None for e in errs)
    return {"workload": f"{heights} heights x {n_vals}-validator commits, blocksync pattern (light + 2 x full)",
            "ms_per_height_plain": round(t_plain * 1e3, 4), "ms_per_height_verdict_cache": round(t_cached * 1e3, 4),
            "ms_per_height_cross_height_batch": round(t_batch * 1e3, 4),
            "note": "host API end to end; cross-height = one cmtv_verify_commits (VerifyCommit) over all heights"}


def c3_line(ctx, dev, world, rank, mode, steps=3, n_heights=100_000, n_vals=150):
    """configs[2]: blocksync / light-client replay of 100k commits x 150
    validators (15M signatures, every message and signature distinct).
    Contiguous height ranges are sharded across the ranks (strong scaling: the
    total is fixed); each rank registers the 150 keys once (cmtv_register_keys)
    and verifies its shard by key index (cmtv_verify_ed25519_indexed_device,
    inputs resident in HBM); the per-rank verdict bitmaps are all-gathered over
    RCCL. 1% of the signatures (seed 42, global indices) carry one flipped bit
    and must be rejected: the gathered verdicts are checked exactly. The
    generic kernel (A decoded per signature) is timed on the same shard."""
    import torch
    import torch.distributed as dist
    from cometbft_amd import parallel as P
    from cometbft_amd import testutil as TU

    per_h = -(-n_heights // world)
    lo, hi = min(n_heights, rank * per_h), min(n_heights, (rank + 1) * per_h)
    nh, n, total = hi - lo, (hi - lo) * n_vals, n_heights * n_vals
    t_gen = time.perf_counter()
    sv = TU.make_validator_set(ctx, n_vals)
    ks = ctx.register_keys(sv.pubkeys)
    m, off = TU.replay_messages(1 + lo, nh, n_vals)
    kidx = np.tile(np.arange(n_vals, dtype=np.uint32), nh)
    sig = ctx.sign(sv.seeds, m, off, kidx)
    rng = np.random.default_rng(42)
    flip = rng.choice(total, total // 100, replace=False)
    bit = rng.integers(0, 512, flip.size)
    g0 = lo * n_vals

    def expected(r):
        a = min(n_heights, r * per_h) * n_vals
        b = min(n_heights, (r + 1) * per_h) * n_vals
        e = np.ones(b - a, np.uint8)
        e[flip[(flip >= a) & (flip < b)] - a] = 0
        return e

    sel = (flip >= g0) & (flip < g0 + n)
    li, lb = flip[sel] - g0, bit[sel]
    sig[li, lb // 8] ^= (1 << (lb % 8)).astype(np.uint8)
    t_gen = time.perf_counter() - t_gen

    words = -(-per_h * n_vals // 64)
    d_idx = torch.from_numpy(kidx).to(dev)
    d_sig = torch.from_numpy(sig).to(dev)
    d_msg = torch.from_numpy(m).to(dev)
    d_off = torch.from_numpy(off.view(np.int32)).to(dev)
    d_valid = torch.zeros(max(n, 1), dtype=torch.uint8, device=dev)
    d_bm = torch.zeros(words, dtype=torch.int64, device=dev)
    d_all = torch.zeros(world * words, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream
    del m, sig

    def timed(fn, k):
        fn()  # warm-up
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        for _ in range(k):
            fn()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t
        if world > 1:
            x = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(x, op=dist.ReduceOp.MAX)
            el = float(x.item())
        return el / k

    def keyed():
        ctx.verify_indexed_device(ks, n, d_idx.data_ptr(), d_sig.data_ptr(), d_msg.data_ptr(), d_off.data_ptr(),
                                  mode, d_valid.data_ptr(), d_bm.data_ptr(), sptr)
        if world > 1:
            dist.all_gather_into_tensor(d_all, d_bm)
        else:
            d_all.copy_(d_bm)

    t_keyed = timed(keyed, steps)
    ok = np.array_equal(d_valid[:n].cpu().numpy(), expected(rank))
    allw = d_all.cpu().numpy().view(np.uint64).reshape(world, words)
    for r in range(world):
        e = expected(r)
        ok = ok and np.array_equal(P.unpack_bitmap(allw[r], e.size), e)
    del d_idx
    d_pk = torch.from_numpy(np.ascontiguousarray(sv.pubkeys[kidx])).to(dev)

    def generic():
        ctx.verify_device(n, d_pk.data_ptr(), d_sig.data_ptr(), d_msg.data_ptr(), d_off.data_ptr(), mode,
                          d_valid.data_ptr(), d_bm.data_ptr(), sptr)

    t_generic = timed(generic, 1)
    ok = ok and np.array_equal(d_valid[:n].cpu().numpy(), expected(rank))
    if world > 1:
        x = torch.tensor([0.0 if ok else 1.0], dtype=torch.float64, device=dev)
        dist.all_reduce(x, op=dist.ReduceOp.MAX)
        ok = float(x.item()) == 0.0
    del d_pk, d_sig, d_msg, d_off, d_valid
    torch.cuda.empty_cache()
    return {"workload": f"configs[2]: {n_heights} commits x {n_vals} validators = {total} signatures, "
                        f"sharded by height over {world} GPU(s), 1% bit-flipped (seed 42)",
            "scaling": "strong", "sigs_per_gpu": n, "value": round(total / t_keyed, 1), "unit": "verifs/s",
            "ms_per_pass": round(t_keyed * 1e3, 3), "steps": steps,
            "path": "registered keys (cmtv_verify_ed25519_indexed_device) + RCCL all-gather of bitmaps",
            "generic_value": round(total / t_generic, 1), "generic_ms_per_pass": round(t_generic * 1e3, 3),
            "verdicts_ok": bool(ok), "setup_s": round(t_gen, 2)}


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def ctx_device(ctx) -> int:
    import torch

    return torch.cuda.current_device()


def latency_150(ctx, mode, iters):
    """p50/p99 VerifyCommit latency for a 150-validator commit (host API, end to end)."""
    from cometbft_amd import testutil as TU

    sv = TU.make_validator_set(ctx, 150)
    commit, msgs, sigs = TU.make_commit(ctx, sv, height=1000)
    bid = TU.block_id_for_height(1000)
    for _ in range(20):
        sv.valset.verify_commit(TU.CHAIN_ID, bid, 1000, commit, ctx=ctx, mode=mode)
    ts = []
    for _ in range(iters):
        t = time.perf_counter()
        sv.valset.verify_commit(TU.CHAIN_ID, bid, 1000, commit, ctx=ctx, mode=mode)
        ts.append(time.perf_counter() - t)
    ts = np.array(ts) * 1e3
    res = {"n_validators": 150, "iters": iters, "p50_ms": round(float(np.percentile(ts, 50)), 4),
           "p99_ms": round(float(np.percentile(ts, 99)), 4),
           "path": "cmtv_verify_commit: sign-bytes + H2D + kernel + D2H + VerifyCommit replay"}
    # the same commit on a context that keeps the validator set's registered
    # keys (cmtv_keyset_cache; the set is registered by the first call)
    from cometbft_amd import Context

    kctx = Context(device=ctx_device(ctx))
    kctx.keyset_cache(4)
    for _ in range(20):
        sv.valset.verify_commit(TU.CHAIN_ID, bid, 1000, commit, ctx=kctx, mode=mode)
    kts = []
    for _ in range(iters):
        t = time.perf_counter()
        sv.valset.verify_commit(TU.CHAIN_ID, bid, 1000, commit, ctx=kctx, mode=mode)
        kts.append(time.perf_counter() - t)
    kts = np.array(kts) * 1e3
    res["keyset_cache"] = {"p50_ms": round(float(np.percentile(kts, 50)), 4),
                           "p99_ms": round(float(np.percentile(kts, 99)), 4),
                           "path": "same, validator set registered once (cmtv_keyset_cache): keyed quad kernel"}
    # the reference's shape: one core verifying 150 signatures sequentially
    from oracle import coracle

    m, off = coracle.pack_msgs(msgs)
    pks = np.array([np.frombuffer(v.pub_key, np.uint8) for v in sv.valset.validators])
    cts = []
    for _ in range(5):
        t = time.perf_counter()
        coracle.verify_batch(pks, sigs, m, off, mode, nthreads=1)
        cts.append(time.perf_counter() - t)
    res["cpu_single_core_p50_ms"] = round(float(np.median(cts)) * 1e3, 3)
    return res


def load_traffic():
    p = os.path.join(ROOT, "profiles", "r01_traffic.json")
    try:
        with open(p) as f:
            d = json.load(f)
        return d.get("bytes_per_launch")
    except (OSError, ValueError):
        return None


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"# note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    from cometbft_amd import Context, pack_messages
    from cometbft_amd import testutil as TU

    mode = 0 if args.mode == "go" else 1
    ctx = Context(device=local)
    n = args.n
    height = 1000 + rank
    sv = TU.make_validator_set(ctx, n)
    msgs = TU.commit_messages(n, height)
    m, off = pack_messages(msgs)
    sigs = ctx.sign(sv.seeds, m, off)
    pk = np.ascontiguousarray(sv.pubkeys)

    d_pk = torch.from_numpy(pk.copy()).to(dev)
    d_sig = torch.from_numpy(sigs.copy()).to(dev)
    d_msg = torch.from_numpy(np.concatenate([m, np.zeros(16, np.uint8)])).to(dev)
    d_off = torch.from_numpy(off.view(np.int32).copy()).to(dev)
    d_valid = torch.zeros(n, dtype=torch.uint8, device=dev)
    words = (n + 63) // 64
    d_bm = torch.zeros(words, dtype=torch.int64, device=dev)
    d_all = torch.zeros(world * words, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]

    def step(i=None):
        if i is not None:
            ev[i][0].record(stream)
        ctx.verify_device(n, d_pk.data_ptr(), d_sig.data_ptr(), d_msg.data_ptr(), d_off.data_ptr(), mode,
                          d_valid.data_ptr(), d_bm.data_ptr(), sptr)
        if i is not None:
            ev[i][1].record(stream)
        if world > 1:
            dist.all_gather_into_tensor(d_all, d_bm)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kernel_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))

    # correctness of the timed work: every honest signature accepted, bitmap full
    ok_local = int(d_valid.sum().item()) == n
    full = (1 << 64) - 1
    bm = d_bm.cpu().numpy().view(np.uint64)
    tail = n % 64
    exp_words = np.full(words, full, dtype=np.uint64)
    if tail:
        exp_words[-1] = np.uint64((1 << tail) - 1)
    ok_local = ok_local and np.array_equal(bm, exp_words)
    if world > 1:
        t = torch.tensor([elapsed, 0.0 if ok_local else 1.0], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, bad = float(t[0].item()), float(t[1].item())
        ok = bad == 0.0
        allw = d_all.cpu().numpy().view(np.uint64).reshape(world, words)
        ok = ok and all(np.array_equal(allw[r], exp_words) for r in range(world))
    else:
        ok = ok_local

    c3 = None if args.no_c3 else c3_line(ctx, dev, world, rank, mode, n_heights=args.c3_heights)

    if rank == 0:
        total = world * n * args.steps
        value = total / elapsed
        achieved = n * MACS_PER_VERIFY / (kernel_ms * 1e-3) / 1e12
        line = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "verifs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic",
            "config": {"workload": "configs[1]: one synthetic 10,000-validator commit per GPU per step "
                                   "(inputs resident in HBM; RCCL all-gather of verdict bitmaps when N>1)",
                       "sigs_per_gpu": n, "mode": args.mode, "msg_bytes_mean": round(float(m.size) / n, 1),
                       "parallelism": f"dp{world}", "verdicts_ok": bool(ok)},
            "roofline": {"bound": "valu_int", "achieved": round(achieved, 3), "peak": INT_MAC_PEAK_T,
                         "unit": "TMAC/s", "frac": round(achieved / INT_MAC_PEAK_T, 4),
                         "traffic": load_traffic(), "kernel_ms": round(kernel_ms, 4),
                         "work": f"{MACS_PER_VERIFY} int32 MACs/verify x {n} verifies per launch"},
        }
        if not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(pk, sigs, m, off, mode, args.cpu_seconds)
            line["cpu_baseline"]["gpu_over_cpu"] = round(value / world / line["cpu_baseline"]["value"], 1)
        if not args.no_latency:
            line["latency_150"] = latency_150(ctx, mode, args.latency_iters)
        if not args.no_latency and world == 1:
            line["replay_150"] = replay_line(local)
        if not args.no_sr25519 and world == 1:
            line["sr25519"] = sr25519_line(ctx, dev, 10_000, 20, args.cpu_seconds / 4, not args.no_cpu_baseline)
        if c3 is not None:
            line["replay_c3"] = c3
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if not ok or (c3 is not None and not c3["verdicts_ok"]):
        sys.exit(3)


if __name__ == "__main__":
    main()
