"""bench.py -- headline benchmark: Ed25519 commit-signature verification on MI355X.

Metric (BASELINE.json): "Ed25519 verifs/sec at 1/2/4/8 GPUs + p50 VerifyCommit
latency, 150 vals".

Step = verify one synthetic 10,000-validator commit (BASELINE.json configs[1])
per GPU: its (pk, sig, sign-bytes) already resident in HBM, the gfx950 verify
kernel writes the packed verdict bitmap. With N GPUs ONE process drives all of
them through one multi-device context (cmtv_open_devices -- a node is one Go
process): every device verifies its own commit and keeps its
own verdict bitmap (cmtv_verify_ed25519_multi_device: independent units, weak
scaling, no data-path collective). The RCCL bitmap all-gather inside
libcmtverify belongs to the sharded configs[2] replay (replay_c3), where the
host replay needs every shard's verdicts. Under torchrun (the driver's N > 1 launch) rank 0
is that process; the other ranks only join the barriers (gloo, on the CPU).
--process-per-gpu keeps the earlier harness instead (one process per GPU,
torch.distributed over RCCL).

Extra fields on the JSON line:
  roofline       -- VALU integer-MAC roofline of the verify kernel: algorithmic
                    work = 300,000 32x32->64 MACs per verification
                    per launch / the kernel's mean duration (HIP events recorded
                    by libcmtverify on the launch stream); peak = measured
                    v_mad_u64_u32 rate (tools/microbench, profiles/r01_int_rates.txt);
                    traffic = raw FETCH_SIZE + WRITE_SIZE bytes per launch
  zip215         -- the same step in ZIP-215 mode (the north-star semantics)
  e2e_10k        -- the 10k commit through the host-buffer API (pinned staging,
                    H2D + kernel + D2H): the PCIe-inclusive rate
  cpu_baseline   -- oracle/liboracle.so (C restatement of the Go-1.19 verify) on
                    the host cores (16 threads = the box's share, and nproc),
                    bounded sample, rank 0 only
  latency_150    -- p50/p99 of VerifyCommit on 150 validators (cmtv_verify_commit:
                    sign-bytes + H2D + kernel + D2H + replay), C-call-only and
                    through the Python mirror, plus the keyset-cache variant
  replay_150     -- blocksync replay per height (light + 2 x full VerifyCommit)
  light_client   -- light/client_benchmark_test.go:25-110 shapes: 1000 heights x
                    100 validators, sequential (VerifyCommitLight per header) and
                    bisection (LightTrusting + Light to the tip)
  replay_c3_host -- configs[2] the way a node calls it: cmtv_verify_commits over
                    100k commits x 150 validators from host memory (plan,
                    pinned staging, H2D, kernels, replay; the chunked
                    pipeline), VerifyCommit and VerifyCommitLight, every
                    height's outcome checked
  replay_c3      -- configs[2]: 100k commits x 150 validators (15M signatures)
                    sharded by height over the N devices (strong scaling),
                    registered-key kernel (radix-256 key combs, [s]B over B's
                    radix-2^16 comb) + RCCL bitmap all-gather, 1% flipped
                    signatures checked exactly; own roofline; the radix-2^16 key
                    combs and the generic kernel beside it
  sr25519        -- configs[4]: 10k sr25519 verifications per step (N=1 only)
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
# registered-key verification by the keyed quad kernel (keyed_quad.h,
# q_verify_keyed_split<MODE, true>): 32 key-comb + 16 B-comb additions (7 field
# mults each in the one-lane form) + decode R (~265) + final check (~8) = 609
# field mults (721 before round 4, with B over its radix-256 comb: 64 additions)
MACS_PER_KEYED_VERIFY = 60_900
# the same over the radix-2^16 key combs (CMTV_KEYS_WIDE) in GO_STDLIB with 8
# signatures per lane sharing one inversion (k_verify_keyed_batch<0, 8, 2>):
# 32 additions x 7 + 265 / 8 + 3 (batch products) + 2 (x, y) = 262 field mults
MACS_PER_KEYED_WIDE_GO_VERIFY = 26_200
# ZIP-215 on the same batches checks R by coset instead of decoding it
# (verify_core.h zip_coset): 32 additions x 7 + R' + T8 (6) + y_R Z, iX, iY on
# two bases (6) + 265 / 8 + 3 (batch products) + 1 (x) = 273 field mults
MACS_PER_KEYED_WIDE_ZIP_VERIFY = 27_300
# configs[2]'s primary path (round 4): the keys' radix-256 combs (32 additions)
# with [s]B over the B table's radix-2^16 comb (16), batched inversion as above:
# 48 x 7 + 265 / 8 + 5 = 374 field mults (Go); ZIP-215 48 x 7 + 12 + 265 / 8 + 4 = 385
MACS_PER_KEYED_MIXED_GO_VERIFY = 37_400
MACS_PER_KEYED_MIXED_ZIP_VERIFY = 38_500
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
    ap.add_argument("--latency-iters", type=int, default=1000)
    ap.add_argument("--no-latency", action="store_true")
    ap.add_argument("--no-c3", action="store_true", help="skip the configs[2] 15M-signature replay side line")
    ap.add_argument("--c3-heights", type=int, default=100_000, help="configs[2] commits (150 validators each)")
    ap.add_argument("--no-c3-host", action="store_true",
                    help="skip configs[2] through cmtv_verify_commits from host memory")
    ap.add_argument("--no-sr25519", action="store_true", help="skip the configs[4] sr25519 side measurement")
    ap.add_argument("--no-light", action="store_true", help="skip the light-client replay line")
    ap.add_argument("--no-keyset", action="store_true", help="skip the registered-keys 10k side line")
    ap.add_argument("--process-per-gpu", action="store_true",
                    help="one process per GPU over torch.distributed (the round-1 harness)")
    return ap.parse_args()


def cpu_threads() -> int:
    for k in ("OMP_NUM_THREADS", "CMTV_CPU_THREADS"):
        v = os.environ.get(k)
        if v and v.isdigit() and int(v) > 0:
            return min(int(v), os.cpu_count() or 1)
    return min(16, os.cpu_count() or 1)


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _sockets():
    try:
        ids = set()
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("physical id"):
                    ids.add(line.split(":", 1)[1].strip())
        return len(ids) or None
    except OSError:
        return None


def _physical_cores():
    """Physical cores of the host: distinct (physical id, core id) pairs of
    /proc/cpuinfo (SMT siblings counted once)."""
    try:
        pairs, phys = set(), None
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("physical id"):
                    phys = line.split(":", 1)[1].strip()
                elif line.startswith("core id"):
                    pairs.add((phys, line.split(":", 1)[1].strip()))
        return len(pairs) or None
    except OSError:
        return None


def _cpu_share():
    """CPUs this process may actually use: the affinity mask and the cgroup
    v2 quota (cpu.max; the GPU box gives one GPU's job a 16-CPU share while
    nproc shows the whole machine)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
            if q != "max":
                quota = round(int(q) / int(p), 2)
    except (OSError, ValueError):
        pass
    return {"affinity_cpus": aff, "cgroup_quota_cpus": quota}


def _oracle_rate(fn, n, threads, cpu_seconds):
    t = time.perf_counter()
    fn(threads)
    first = time.perf_counter() - t
    reps = max(1, int(cpu_seconds / max(first * threads, 1e-3)))
    t = time.perf_counter()
    for _ in range(reps):
        fn(threads)
    dt = time.perf_counter() - t
    return reps * n / dt, reps, dt


def _single_core(pk, sig, m, off, mode, n_max=2000):
    """verifs/s of the oracle on one core over the first n_max signatures of
    the commit: the shape of the reference, whose VerifyCommit loop is one
    goroutine (types/validator_set.go:685)"""
    from oracle import coracle

    sl = min(len(off) - 1, n_max)
    coracle.verify_batch(pk[:64], sig[:64], m, off[:65], mode, nthreads=1)
    t = time.perf_counter()
    coracle.verify_batch(pk[:sl], sig[:sl], m, off[: sl + 1], mode, nthreads=1)
    return sl / (time.perf_counter() - t), sl


def cpu_baseline(pk, sig, m, off, mode, cpu_seconds):
    """The oracle (C restatement of Go 1.19 crypto/ed25519.Verify) on the host
    cores over the same commit, repeated to a bounded amount of CPU work:
      value          -- 16 threads (the GPU box's CPU share per GPU);
      single_core    -- one core, the reference's own shape (its VerifyCommit
                        loop is one goroutine), in both verdict modes;
      extrapolated_all_cores -- single_core x the host's physical cores, the
                        honest all-core figure (no SMT credit);
      quota_bound_all_threads -- nproc threads as measured; on the GPU box the
                        job's cgroup quota (~16 CPUs) caps this, so it is NOT
                        an all-core figure."""
    from oracle import coracle  # the checker / CPU baseline only

    n = len(off) - 1
    out = coracle.verify_batch(pk, sig, m, off, mode, nthreads=cpu_threads())
    assert out.all(), "oracle rejected an honest synthetic signature"
    run = lambda th: coracle.verify_batch(pk, sig, m, off, mode, nthreads=th)  # noqa: E731
    threads = cpu_threads()
    v16, reps, dt = _oracle_rate(run, n, threads, cpu_seconds)
    nproc = os.cpu_count() or 1
    # nproc threads: the commit tiled so every thread gets >= 400 signatures
    # per pass (a 10k commit over 256 threads is ~40 each: spawn-bound)
    tile = max(1, -(-400 * nproc // n))
    body = int(off[-1])
    mt = np.concatenate([np.tile(m[:body], tile), np.zeros(1, np.uint8)])
    offt = np.concatenate([off[:-1].astype(np.uint64) + j * body for j in range(tile)]
                          + [[tile * body]]).astype(off.dtype)
    pkt, sigt = np.tile(pk, (tile, 1)), np.tile(sig, (tile, 1))
    run_all = lambda th: coracle.verify_batch(pkt, sigt, mt, offt, mode, nthreads=th)  # noqa: E731
    assert run_all(nproc).all(), "tiled commit"
    vall, reps_all, dt_all = _oracle_rate(run_all, n * tile, nproc, cpu_seconds * max(1, nproc // threads) / 4)
    one, sl = _single_core(pk, sig, m, off, mode)
    one_z, _ = _single_core(pk, sig, m, off, 1 - mode)
    phys = _physical_cores()
    share = _cpu_share()
    return {"value": round(v16, 1), "unit": "verifs/s", "cores": threads, "kind": "port",
            "sample": f"{n}-signature synthetic commit x {reps} passes, {threads} threads, oracle/liboracle.so "
                      f"(C restatement of Go 1.19 ed25519.Verify)",
            "seconds": round(dt, 2),
            "single_core": {"value": round(one, 1), "mode": "zip215" if mode else "go",
                            "value_other_mode": round(one_z, 1), "sample": f"first {sl} signatures, 1 thread",
                            "note": "the reference's shape: VerifyCommit is one goroutine "
                                    "(types/validator_set.go:685)"},
            "single_core_verifs_per_s": round(one, 1),
            "extrapolated_all_cores": {"value": round(one * phys, 1) if phys else None,
                                       "value_other_mode": round(one_z * phys, 1) if phys else None,
                                       "physical_cores": phys,
                                       "how": "single_core x physical cores (distinct physical id/core id of "
                                              "/proc/cpuinfo); not measured: the job's quota forbids it"},
            "quota_bound_all_threads": {"value": round(vall, 1), "threads": nproc, "passes": reps_all,
                                        "seconds": round(dt_all, 2),
                                        "sample": f"the commit tiled x{tile} ({n * tile} signatures per pass)",
                                        "note": f"{nproc} threads under a cgroup quota of "
                                                f"{share.get('cgroup_quota_cpus')} CPUs: quota-bound, "
                                                "not an all-core figure"},
            "host_cpu": _cpu_model(), "nproc": nproc, "sockets": _sockets(), **share}


class Devices:
    """Per-device synthetic inputs of one 10k commit each (heights 1000+g),
    resident in HBM, for the multi-device context."""

    def __init__(self, ctx, n_dev, n):
        import torch

        from cometbft_amd import Context, pack_messages
        from cometbft_amd import testutil as TU

        self.n_dev, self.n = n_dev, n
        self.words = (n + 63) // 64
        self.t = []
        self.host = []
        for g in range(n_dev):
            dev = torch.device("cuda", ctx.device_ordinal(g))
            gen = ctx if g == 0 else Context(device=ctx.device_ordinal(g))
            sv = TU.make_validator_set(gen, n)
            msgs = TU.commit_messages(n, 1000 + g)
            m, off = pack_messages(msgs)
            sigs = gen.sign(sv.seeds, m, off)
            pk = np.ascontiguousarray(sv.pubkeys)
            self.host.append((pk, sigs, m, off))
            self.t.append({"pk": torch.from_numpy(pk.copy()).to(dev), "sig": torch.from_numpy(sigs.copy()).to(dev),
                           "m": torch.from_numpy(np.concatenate([m, np.zeros(16, np.uint8)])).to(dev),
                           "off": torch.from_numpy(off.view(np.int32).copy()).to(dev),
                           "bm": torch.zeros(self.words, dtype=torch.int64, device=dev)})
            if g:
                del gen
        self.msg_bytes_mean = float(self.host[0][2].size) / n

    def step(self, ctx, mode):
        # each device verifies its own commit: independent units, no exchange
        ts = self.t
        ctx.verify_multi_device([self.n] * self.n_dev, [t["pk"].data_ptr() for t in ts],
                                [t["sig"].data_ptr() for t in ts], [t["m"].data_ptr() for t in ts],
                                [t["off"].data_ptr() for t in ts], mode, [t["bm"].data_ptr() for t in ts])

    def verdicts_ok(self):
        full = np.full(self.words, np.uint64((1 << 64) - 1), np.uint64)
        mask = np.full(self.words, np.uint64((1 << 64) - 1), np.uint64)
        if self.n % 64:  # bits past n in the last word are not specified
            full[-1] = mask[-1] = np.uint64((1 << (self.n % 64)) - 1)
        return all(np.array_equal(self.t[g]["bm"].cpu().numpy().view(np.uint64) & mask, full)
                   for g in range(self.n_dev))


# The GPU leaves its idle clock state only after some milliseconds of load: the
# first 50 configs[1] steps after a 1 s pause average 0.2637 ms of kernel time,
# every later block 0.2545 ms (tools/clock_probe.py, profiles/r02_clock_probe.txt).
# The warm-up therefore runs back-to-back steps for at least CLOCK_SETTLE_S
# before its W counted steps; the timed region itself is unchanged.
CLOCK_SETTLE_S = 0.1


def _device_streams(ctx):
    """Each device's launch stream (the context's own; cmtv_device_stream)
    as a torch stream, for HIP events on the stream the kernels run on."""
    import torch

    return [torch.cuda.ExternalStream(ctx.device_stream(g), device=torch.device(f"cuda:{ctx.device_ordinal(g)}"))
            for g in range(ctx.n_devices)]


def timed_steps(ctx, fn, steps, warmup, barrier, settle_s=CLOCK_SETTLE_S):
    """Runs W warm-up steps, then times exactly `steps` back-to-back steps.
    Returns the wall time and the mean launch duration: HIP events recorded on
    every device's launch stream at both ends of the timed region (one pair per
    device, so no marker packets between the launches), region / steps, the
    largest over the devices. The library's own sampled per-call timing
    (cmtv_stats device_ms / timed_calls) is kept beside it in LAST_RUN."""
    import torch

    t_settle = time.perf_counter() + settle_s
    while time.perf_counter() < t_settle:
        fn()
        ctx.sync()
    for _ in range(warmup):
        fn()
    ctx.sync()
    barrier()
    ctx.sync()
    streams = _device_streams(ctx)
    ev0 = [torch.cuda.Event(enable_timing=True) for _ in streams]
    ev1 = [torch.cuda.Event(enable_timing=True) for _ in streams]
    s0 = ctx.stats()
    d0 = ctx.device_stats()
    for e, st in zip(ev0, streams):
        e.record(st)
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    for e, st in zip(ev1, streams):
        e.record(st)
    ctx.sync()
    barrier()
    elapsed = time.perf_counter() - t0
    s1 = ctx.stats()
    d1 = ctx.device_stats()
    region = [a.elapsed_time(b) / steps for a, b in zip(ev0, ev1)]
    kernel_ms = max(region)
    timed = s1["timed_calls"] - s0["timed_calls"]
    global LAST_RUN
    LAST_RUN = {"per_device": [{"ordinal": b["ordinal"], "calls": b["calls"] - a["calls"],
                                "signatures": b["signatures"] - a["signatures"],
                                "kernel_ms": round(r, 4),
                                "sampled_kernel_ms": round((b["device_ms"] - a["device_ms"])
                                                           / max(b["timed_calls"] - a["timed_calls"], 1), 4)}
                               for a, b, r in zip(d0, d1, region)],
                "context": {k: s1[k] - s0[k] for k in ("sharded_calls", "gathers", "calls", "timed_calls")} |
                           {k: s1[k] for k in ("n_devices", "live_devices", "rccl", "device_failures")},
                "sampled_kernel_ms": round((s1["device_ms"] - s0["device_ms"]) / timed, 4) if timed else None}
    return elapsed, kernel_ms


# per-device work of the last timed_steps region (bench line evidence that
# every device of the context ran and whether RCCL carried the gathers)
LAST_RUN: dict = {}


def e2e_10k(ctx, host, mode, iters=20):
    """The 10k commit through the host-buffer API: pinned staging + H2D +
    kernel + D2H + verdict bytes (PCIe-inclusive)."""
    pk, sig, m, off = host
    for _ in range(3):
        ctx.verify(pk, sig, m, off, mode)
    ts = []
    for _ in range(iters):
        t = time.perf_counter()
        v = ctx.verify(pk, sig, m, off, mode)
        ts.append(time.perf_counter() - t)
    ms = float(np.median(ts)) * 1e3
    return {"ms": round(ms, 4), "value": round((len(off) - 1) / ms * 1e3, 1), "unit": "verifs/s",
            "verdicts_ok": bool(v.all()), "path": "cmtv_verify_ed25519 (host buffers, pinned staging)"}


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
    sptr = ctx.stream()

    def run():
        ctx.verify_sr25519_device(n, d_pk.data_ptr(), d_sig.data_ptr(), d_m.data_ptr(), d_off.data_ptr(),
                                  d_valid.data_ptr(), 0, sptr)

    wall, kms = timed_steps(ctx, run, steps, 3, lambda: None)
    wall /= steps
    res = {"workload": f"configs[4]: {n} sr25519 signatures over 150 keys, 116-byte messages, inputs in HBM",
           "value": round(n / wall, 1), "unit": "verifs/s", "ms_per_step": round(wall * 1e3, 4),
           "kernel_ms": round(kms, 4), "verdicts_ok": bool(int(d_valid.sum().item()) == n)}
    if with_cpu:
        threads = cpu_threads()
        v, reps, dt = _oracle_rate(lambda th: coracle.sr25519_verify_batch(pk, sig, m, off, nthreads=th), n, threads,
                                   cpu_seconds)
        res["cpu_baseline"] = {"value": round(v, 1), "unit": "verifs/s", "cores": threads, "kind": "port",
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
    # the same through the C ABI with the arguments packed once, as a cgo
    # shim holds them (the Python mirror above re-packs every call)
    per_height = [(T.PackedCommits(1, TU.CHAIN_ID, [it]), T.PackedCommits(0, TU.CHAIN_ID, [it])) for it in chain]

    def blocksync_c(ctx):
        for light, full in per_height:
            light.call(ctx)
            full.call(ctx)
            full.call(ctx)

    blocksync_c(plain)
    t = time.perf_counter()
    blocksync_c(plain)
    t_plain_c = (time.perf_counter() - t) / heights
    whole = T.PackedCommits(0, TU.CHAIN_ID, chain)
    whole.call(plain)
    ts = []
    for _ in range(21):  # one call is ~0.5 ms: the median of 21
        t = time.perf_counter()
        whole.call(plain)
        ts.append(time.perf_counter() - t)
    t_batch_c = float(np.median(ts)) / heights
    assert all(r == 0 for r in whole.rcs)
    return {"workload": f"{heights} heights x {n_vals}-validator commits, blocksync pattern (light + 2 x full)",
            "ms_per_height_plain": round(t_plain * 1e3, 4), "ms_per_height_verdict_cache": round(t_cached * 1e3, 4),
            "ms_per_height_cross_height_batch": round(t_batch * 1e3, 4),
            "c_call": {"ms_per_height_plain": round(t_plain_c * 1e3, 4),
                       "ms_per_height_cross_height_batch": round(t_batch_c * 1e3, 4)},
            "note": "host API end to end through the Python mirror (re-packs each call); c_call: the C ABI with "
                    "arguments packed once; cross-height = one cmtv_verify_commits (VerifyCommit) over all heights"}


def light_line(dev_index, heights=1000, n_vals=100):
    """light/client_benchmark_test.go:25-110 (genMockNode(chainID, 1000, 100,
    ...)): a light client syncing 1 -> 1000 over a 100-validator chain.
    Sequential = VerifyAdjacent per header (light/verifier.go:93-126 ->
    untrustedVals.VerifyCommitLight), per call and as one cross-height
    cmtv_verify_commits batch (with and without the keyset cache);
    bisection = VerifyNonAdjacent 1 -> 1000 (verifier.go:32-73:
    trustedVals.VerifyCommitLightTrusting(1/3) + untrustedVals.VerifyCommitLight).
    The validator set is static here, so bisection needs one hop."""
    from cometbft_amd import Context
    from cometbft_amd import testutil as TU
    from cometbft_amd import types as T
    from oracle import coracle

    ctx = Context(device=dev_index)
    kctx = Context(device=dev_index)
    kctx.keyset_cache(2)
    sv = TU.make_validator_set(ctx, n_vals, offset=50_000)
    chain = []
    for h in range(1, heights + 1):
        commit, _, _ = TU.make_commit(ctx, sv, h)
        chain.append((sv.valset, TU.block_id_for_height(h), h, commit))
    seq = chain[1:]
    for vals, bid, h, c in seq[:20]:
        vals.verify_commit_light(TU.CHAIN_ID, bid, h, c, ctx=ctx)
    t = time.perf_counter()
    for vals, bid, h, c in seq:
        vals.verify_commit_light(TU.CHAIN_ID, bid, h, c, ctx=ctx)
    t_seq = time.perf_counter() - t
    def median3(fn):
        fn()
        ts = []
        for _ in range(3):
            t = time.perf_counter()
            out = fn()
            ts.append(time.perf_counter() - t)
        return float(np.median(ts)), out

    # the Python mirror re-packs 999 commits per call: median of 3
    t_batch, errs = median3(lambda: T.verify_commits(1, TU.CHAIN_ID, seq, ctx=ctx))
    assert all(e is None for e in errs)
    t_kbatch, errs = median3(lambda: T.verify_commits(1, TU.CHAIN_ID, seq, ctx=kctx))
    assert all(e is None for e in errs)
    # the C calls alone, arguments packed once (what the cgo shim passes)
    per_call = [T.PackedCommits(1, TU.CHAIN_ID, [it]) for it in seq]
    for p in per_call[:20]:
        p.call(ctx)
    t = time.perf_counter()
    for p in per_call:
        p.call(ctx)
    t_seq_c = time.perf_counter() - t
    # the same per-call loop with the keyset cache (the Go binding's default)
    for p in per_call[:20]:
        p.call(kctx)
    t = time.perf_counter()
    for p in per_call:
        p.call(kctx)
    t_kseq_c = time.perf_counter() - t
    assert all(p.rcs[0] == 0 for p in per_call)
    whole = T.PackedCommits(1, TU.CHAIN_ID, seq)
    whole.call(ctx)
    ts = []
    for _ in range(5):
        t = time.perf_counter()
        whole.call(ctx)
        ts.append(time.perf_counter() - t)
    t_batch_c = float(np.median(ts))
    whole.call(kctx)
    ts = []
    for _ in range(5):
        t = time.perf_counter()
        whole.call(kctx)
        ts.append(time.perf_counter() - t)
    t_kbatch_c = float(np.median(ts))
    assert all(r == 0 for r in whole.rcs)
    vals, bid, h, c = chain[-1]
    ts = []
    for _ in range(50):
        t = time.perf_counter()
        sv.valset.verify_commit_light_trusting(TU.CHAIN_ID, c, (1, 3), ctx=ctx)
        vals.verify_commit_light(TU.CHAIN_ID, bid, h, c, ctx=ctx)
        ts.append(time.perf_counter() - t)
    # the reference's shape on one core: every signature the sequential
    # light calls verify (2/3 + 1 of each commit), oracle single-threaded
    need = n_vals * 2 // 3 + 1
    pk = np.ascontiguousarray(sv.pubkeys)
    msgs, sigs = [], []
    for _, _, hh, cc in seq[:100]:
        mm = TU.commit_messages(n_vals, hh)
        for i in range(need):
            msgs.append(mm[i])
            sigs.append(np.frombuffer(cc.signatures[i].signature, np.uint8))
    m, off = coracle.pack_msgs(msgs)
    t = time.perf_counter()
    coracle.verify_batch(np.tile(pk[:need], (100, 1)), np.array(sigs), m, off, 0, nthreads=1)
    cpu_seq_s = (time.perf_counter() - t) * len(seq) / 100
    return {"workload": f"light client 1 -> {heights}, {n_vals} validators (light/client_benchmark_test.go:25-110)",
            "sequential_ms_per_call_loop": round(t_seq * 1e3, 2),
            "sequential_ms_cross_height_batch": round(t_batch * 1e3, 2),
            "sequential_ms_cross_height_batch_keyset": round(t_kbatch * 1e3, 2),
            "c_call": {"sequential_ms_per_call_loop": round(t_seq_c * 1e3, 2),
                       "sequential_ms_per_call_loop_keyset": round(t_kseq_c * 1e3, 2),
                       "sequential_ms_cross_height_batch": round(t_batch_c * 1e3, 2),
                       "sequential_ms_cross_height_batch_keyset": round(t_kbatch_c * 1e3, 2)},
            "bisection_p50_ms": round(float(np.median(ts)) * 1e3, 4),
            "cpu_single_core_sequential_ms": round(cpu_seq_s * 1e3, 1),
            "note": f"{len(seq)} VerifyCommitLight calls; CPU = oracle verifying the same "
                    f"{need} signatures per header on one core (extrapolated from 100 headers)"}


def c3_line(ctx, n_dev, mode, steps=3, n_heights=100_000, n_vals=150):
    """configs[2]: blocksync / light-client replay of 100k commits x 150
    validators (15M signatures, every message and signature distinct).
    Contiguous height ranges are sharded across the context's devices (strong
    scaling: the total is fixed); the 150 keys are registered once
    (cmtv_register_keys, on every device) and each device verifies its shard
    by key index (cmtv_verify_ed25519_indexed_sharded_device, inputs resident
    in HBM); the shard bitmaps are all-gathered over RCCL inside the library.
    1% of the signatures (seed 42, global indices) carry one flipped bit and
    must be rejected: the gathered verdicts are checked exactly. The generic
    kernel (A decoded per signature) is timed on the same shards."""
    import torch

    from cometbft_amd import Context
    from cometbft_amd import parallel as P
    from cometbft_amd import testutil as TU

    per_h = -(-n_heights // n_dev)
    total = n_heights * n_vals
    t_gen = time.perf_counter()
    sv = TU.make_validator_set(ctx, n_vals)
    t_reg = time.perf_counter()
    ks = ctx.register_keys(sv.pubkeys, wide=True)  # 64 MiB of radix-2^16 comb per key and device
    t_reg = time.perf_counter() - t_reg
    ks256 = ctx.register_keys(sv.pubkeys)
    rng = np.random.default_rng(42)
    flip = rng.choice(total, total // 100, replace=False)
    bit = rng.integers(0, 512, flip.size)
    shards, exp = [], []
    for g in range(n_dev):
        lo, hi = min(n_heights, g * per_h), min(n_heights, (g + 1) * per_h)
        n = (hi - lo) * n_vals
        dev = torch.device("cuda", ctx.device_ordinal(g))
        m, off = TU.replay_messages(1 + lo, max(hi - lo, 1), n_vals)
        kidx = np.tile(np.arange(n_vals, dtype=np.uint32), max(hi - lo, 1))
        gen = ctx if g == 0 else Context(device=ctx.device_ordinal(g))
        sig = gen.sign(sv.seeds, m, off, kidx)
        g0 = lo * n_vals
        sel = (flip >= g0) & (flip < g0 + n)
        li, lb = flip[sel] - g0, bit[sel]
        sig[li, lb // 8] ^= (1 << (lb % 8)).astype(np.uint8)
        e = np.ones(n, np.uint8)
        e[li] = 0
        exp.append(e)
        shards.append({"n": n, "idx": torch.from_numpy(kidx).to(dev), "sig": torch.from_numpy(sig).to(dev),
                       "m": torch.from_numpy(m).to(dev), "off": torch.from_numpy(off.view(np.int32)).to(dev),
                       "pk": None, "dev": dev})
        del m, sig, gen
    t_gen = time.perf_counter() - t_gen
    W = max((s["n"] + 63) // 64 for s in shards)
    for s in shards:
        s["bm"] = torch.zeros(n_dev * W, dtype=torch.int64, device=s["dev"])
    ns = [s["n"] for s in shards]

    def keyed(keys):
        ctx.verify_sharded_device(ns, [s["idx"].data_ptr() for s in shards], [s["sig"].data_ptr() for s in shards],
                                  [s["m"].data_ptr() for s in shards], [s["off"].data_ptr() for s in shards], mode,
                                  [s["bm"].data_ptr() for s in shards], keys=keys)

    def check():
        ok = True
        for g in range(n_dev):
            allw = shards[g]["bm"].cpu().numpy().view(np.uint64).reshape(n_dev, W)
            for h in range(n_dev):
                ok = ok and np.array_equal(P.unpack_bitmap(allw[h], ns[h]), exp[h])
        return ok

    # the primary path: the keys' radix-256 combs (512 KiB per key, the keyset
    # cache's form) with [s]B over the B table's radix-2^16 comb (kCombMixed)
    el, kms_keyed = timed_steps(ctx, lambda: keyed(ks256), steps, 1, lambda: None)
    t_keyed = el / steps
    run_keyed = dict(LAST_RUN)
    ok = check()
    ks256.free()
    for s in shards:
        s["bm"].zero_()
    # the radix-2^16 key combs beside it (64 MiB per key)
    el, kms_wide = timed_steps(ctx, lambda: keyed(ks), steps, 1, lambda: None)
    t_wide = el / steps
    ok = ok and check()
    for s in shards:
        s["bm"].zero_()
        s["pk"] = torch.from_numpy(np.ascontiguousarray(sv.pubkeys[s["idx"].cpu().numpy()])).to(s["dev"])
        s["idx"] = None
    torch.cuda.empty_cache()

    def generic():
        ctx.verify_sharded_device(ns, [s["pk"].data_ptr() for s in shards], [s["sig"].data_ptr() for s in shards],
                                  [s["m"].data_ptr() for s in shards], [s["off"].data_ptr() for s in shards], mode,
                                  [s["bm"].data_ptr() for s in shards])

    el, kms_generic = timed_steps(ctx, generic, 1, 1, lambda: None)
    t_generic = el
    ok = ok and check()
    ks.free()
    shards.clear()
    torch.cuda.empty_cache()
    per_dev = total / n_dev
    # algorithmic work of the path that ran (ZIP-215 decodes R instead of the
    # batched inversion: the radix-256 figure's decode term, with 32 additions)
    macs = MACS_PER_KEYED_MIXED_GO_VERIFY if mode == 0 else MACS_PER_KEYED_MIXED_ZIP_VERIFY
    work = ("48 comb additions (32 key, 16 B) x 7 + inversion / 8 + 5, x 100" if mode == 0
            else "48 comb additions (32 key, 16 B) x 7 + coset check 12 + inversion / 8 + 4, x 100")
    macs_wide = MACS_PER_KEYED_WIDE_GO_VERIFY if mode == 0 else MACS_PER_KEYED_WIDE_ZIP_VERIFY
    ach = per_dev / (kms_keyed * 1e-3) * macs / 1e12 if kms_keyed > 0 else None
    return {"workload": f"configs[2]: {n_heights} commits x {n_vals} validators = {total} signatures, "
                        f"sharded by height over {n_dev} GPU(s), 1% bit-flipped (seed 42)",
            "scaling": "strong", "sigs_per_gpu": int(per_dev), "value": round(total / t_keyed, 1), "unit": "verifs/s",
            "ms_per_pass": round(t_keyed * 1e3, 3), "steps": steps,
            "path": "registered keys: radix-256 key combs (512 KiB per key, cmtv_register_keys) with [s]B over "
                    "the B table's radix-2^16 comb (keyed_lane.hip kCombMixed, 8 signatures per lane sharing one "
                    "inversion), cmtv_verify_ed25519_indexed_sharded_device + RCCL all-gather of bitmaps",
            "kernel_ms_per_device": round(kms_keyed, 3),
            "roofline": {"bound": "valu_int", "work": f"{macs} int32 MACs/keyed verify ({work}); a path-specific "
                                                      "count (the headline's 300k is the generic path's); SHA-512 "
                                                      "and table loads not counted",
                         "achieved": round(ach, 3) if ach else None, "peak": INT_MAC_PEAK_T, "unit": "TMAC/s",
                         "frac": round(ach / INT_MAC_PEAK_T, 4) if ach else None},
            "wide_value": round(total / t_wide, 1), "wide_kernel_ms_per_device": round(kms_wide, 3),
            "wide_frac": round(per_dev / (kms_wide * 1e-3) * macs_wide / 1e12 / INT_MAC_PEAK_T, 4)
            if kms_wide > 0 else None,
            "wide_path": "radix-2^16 key combs (64 MiB per key, cmtv_register_keys_ex CMTV_KEYS_WIDE: 32 additions, "
                         "rows from HBM staged by LDS-DMA)", "register_wide_s": round(t_reg, 3),
            "generic_value": round(total / t_generic, 1), "generic_ms_per_pass": round(t_generic * 1e3, 3),
            "generic_frac": round(per_dev / (kms_generic * 1e-3) * MACS_PER_VERIFY / 1e12 / INT_MAC_PEAK_T, 4)
            if kms_generic > 0 else None,
            "verdicts_ok": bool(ok), "setup_s": round(t_gen, 2),
            "devices": run_keyed}


def c3_host_line(ctx, mode, n_heights=100_000, n_vals=150, steps=3, kinds=(0, 1), packed_ctx=None):
    """configs[2] through the entry point a node calls:
    cmtv_verify_commits over n_heights commits x n_vals validators from HOST
    memory, arguments packed once as a cgo shim holds them (ReplayChain: the
    Go slices' pointers), the validator set's keys registered on first use by
    the keyset cache (a node keeps its set across heights). One call per pass
    = commit plan, sign-bytes templates, H2D, sign-bytes + registered-key
    kernels, verdicts back, and the reference loop replayed per commit
    (types/validator_set.go:685-713 VerifyCommit, :740-764 VerifyCommitLight).
    The shim's arena is in the context's cmtv_alloc_pinned memory (round 6,
    VERDICT r5 item 1: the direct chunks -- DMA'd from it, laid out on the
    device, no host pack per signature); `packed` times the same chain
    through a context that does not own the memory (every chunk packed on the
    host workers, the round-5 path). 1% of the signatures (seed 42) carry a
    flipped bit; every height's outcome (nil, or ErrWrongSignature at the
    first flipped index the loop reaches) is checked exactly. value =
    signatures the call verified / wall time of the call (VerifyCommit
    verifies all 15M; the light kind stops each commit past 2/3: its
    chain_signatures_per_s divides the whole chain's 15M instead)."""
    from cometbft_amd import _native as N
    from cometbft_amd import testutil as TU

    t_gen = time.perf_counter()
    sv = TU.make_validator_set(ctx, n_vals)
    chain = TU.ReplayChain(ctx, sv, 1, n_heights, pinned=ctx)
    t_gen = time.perf_counter() - t_gen
    total = n_heights * n_vals
    out = {"workload": f"configs[2] from host memory: {n_heights} commits x {n_vals} validators = {total} "
                       "signatures, one cmtv_verify_commits call per pass, 1% bit-flipped (seed 42), the "
                       "arguments in a cmtv_alloc_pinned arena",
           "unit": "verifs/s", "setup_s": round(t_gen, 2), "steps": steps}
    names = {N.VERIFY_COMMIT: "verify_commit", N.VERIFY_COMMIT_LIGHT: "verify_commit_light",
             N.VERIFY_COMMIT_LIGHT_TRUSTING: "verify_commit_light_trusting"}

    def run(c, kind):
        chain.call(c, kind, mode)  # warm-up: registers the key set, grows the staging
        st0 = c.stats()
        ts = []
        for _ in range(steps):
            t = time.perf_counter()
            chain.call(c, kind, mode)
            ts.append(time.perf_counter() - t)
        st1 = c.stats()
        rcs, code, si = chain.outcome()
        first = chain.expected(kind)
        bad = first >= 0
        ok = bool(np.all(rcs[~bad] == 0) and np.all(rcs[bad] == N.CMTV_ECOMMIT)
                  and np.all(code[bad] == N.COMMIT_ERR_WRONG_SIGNATURE) and np.all(si[bad] == first[bad]))
        t = float(np.median(ts))
        verified = (st1["signatures"] - st0["signatures"]) / steps
        return {"value": round(verified / t, 1), "ms_per_pass": round(t * 1e3, 2), "ms_min": round(min(ts) * 1e3, 2),
                "signatures_verified_per_pass": int(verified), "chain_signatures_per_s": round(total / t, 1),
                "direct_chunks_per_pass": (st1["direct_chunks"] - st0["direct_chunks"]) / steps,
                "verdicts_ok": ok, "heights_with_error": int(bad.sum())}

    for kind in kinds:
        out[names[kind]] = run(ctx, kind)
    if packed_ctx is not None:
        out["packed"] = {"path": "the same chain through a context that does not own its memory: every chunk "
                                 "packed into pinned staging by the host workers (round 5)"}
        for kind in kinds:
            out["packed"][names[kind]] = run(packed_ctx, kind)
    del chain
    return out


def keyset_10k(ctx, D, mode, steps):
    """configs[1] with the validator set registered once (cmtv_register_keys,
    outside the timed region, as a node keeps it across heights): the same
    10k commit, inputs in HBM, verified by key index
    (cmtv_verify_ed25519_indexed_device: no decompression of A, the key's
    comb instead of its doublings). A side line: the headline step decodes
    every key, as the reference's VerifyCommit does."""
    import torch

    pk, sigs, m, off = D.host[0]
    t = D.t[0]
    dev = t["pk"].device
    t_reg = time.perf_counter()
    ks = ctx.register_keys(pk)
    ctx.sync()
    t_reg = time.perf_counter() - t_reg
    idx = torch.arange(D.n, dtype=torch.int32, device=dev)
    bm = torch.zeros(D.words, dtype=torch.int64, device=dev)

    stream = torch.cuda.current_stream(dev)

    def step():
        # the device entry point enqueues on the caller's stream: torch's
        ctx.verify_indexed_device(ks, D.n, idx.data_ptr(), t["sig"].data_ptr(), t["m"].data_ptr(),
                                  t["off"].data_ptr(), mode, 0, bm.data_ptr(), stream=stream.cuda_stream)

    def sync():
        stream.synchronize()
        ctx.sync()

    for _ in range(5):
        step()
    sync()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    e1.record(stream)
    sync()
    el = time.perf_counter() - t0
    kms = e0.elapsed_time(e1) / steps  # HIP events on the launch stream around the region
    ok = bool(np.array_equal(bm.cpu().numpy().view(np.uint64), t["bm"].cpu().numpy().view(np.uint64)))
    ks.free()
    ach = D.n / (kms * 1e-3) * MACS_PER_KEYED_VERIFY / 1e12 if kms > 0 else None
    return {"value": round(D.n * steps / el, 1), "unit": "verifs/s", "ms_per_step": round(el / steps * 1e3, 4),
            "kernel_ms": round(kms, 4), "register_keys_s": round(t_reg, 2),
            "frac": round(ach / INT_MAC_PEAK_T, 4) if ach else None,
            "work": f"{MACS_PER_KEYED_VERIFY} int32 MACs/keyed verify",
            "verdicts_match_headline": ok,
            "path": "cmtv_verify_ed25519_indexed_device over 10,000 registered keys (keyed quad kernel)"}


def _commit_c_call(c, sv, commit, bid, height, mode, pinned=False):
    """cmtv_verify_commit on a commit packed once (what a cgo binding holds):
    returns the call and the objects that keep the packed buffers alive.
    pinned: the commit's arrays and the set's keys in the context's
    cmtv_alloc_pinned memory (the binding's arena there: the signatures and
    keys go to the device by DMA, no host copy)."""
    import ctypes

    import numpy as np

    from cometbft_amd import _native as N
    from cometbft_amd import testutil as TU
    from cometbft_amd import types as T

    vs, kv = sv.valset._pack()
    arena = None
    if pinned:
        nsig = len(commit.signatures)
        arena = T._Arena(c.alloc_pinned(4096 + 100 * (nsig + 1) + 32 * len(sv.valset.validators)))
        pk = arena.put(kv[0])  # the set's keys (+ pad byte), as ValidatorSet._pack lays them out
        vs = N.cmtv_valset.from_buffer_copy(vs)
        vs.pubkeys = pk.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
        kv = (kv, pk, arena)
    cm, kc = T._pack_commit(commit, arena)
    bcb, kb = bid._c()
    res = N.cmtv_commit_result()
    cid = TU.CHAIN_ID.encode()
    L = N.lib()

    def call():
        rc = L.cmtv_verify_commit(c.handle, N.VERIFY_COMMIT, mode, cid, len(cid), ctypes.byref(vs),
                                  ctypes.byref(bcb), height, ctypes.byref(cm), 0, 0, ctypes.byref(res), None, 0)
        assert rc == 0, rc
    return call, (kv, kc, kb, res)


def _p50_p99_inner(fn, between, iters, warm=20):
    """p50 / p99 of fn() alone, each call followed by between() (untimed)."""
    for _ in range(warm):
        fn()
        between()
    ts = []
    for _ in range(iters):
        t = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t)
        between()
    ts = np.array(ts) * 1e3
    return round(float(np.percentile(ts, 50)), 4), round(float(np.percentile(ts, 99)), 4)


def _p50_p99(fn, iters, warm=50):
    for _ in range(warm):
        fn()
    ts = []
    for _ in range(iters):
        t = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t)
    ts = np.array(ts) * 1e3
    return round(float(np.percentile(ts, 50)), 4), round(float(np.percentile(ts, 99)), 4)


def crossover(ctx, mode, sizes=(1, 2, 4, 8, 16, 32), iters=100):
    """The small-batch crossover (tools/crossover.py is the
    full sweep, profiles/r04_crossover.json): the smallest n from which one
    n-validator VerifyCommit through cmtv_verify_commit (packed once, as a cgo
    shim holds it) beats the CPU oracle on ONE core over the same n signatures
    -- the reference's loop is one goroutine (types/validator_set.go:685) --
    at every larger n measured. Below it the Go binding keeps the CPU path
    (INTEGRATION.md CMTVERIFY_MIN_BATCH)."""
    from cometbft_amd import testutil as TU
    from oracle import coracle  # the CPU baseline only

    rows = []
    for n in sizes:
        sv = TU.make_validator_set(ctx, n)
        commit, msgs, sig = TU.make_commit(ctx, sv, height=1000)
        call, keep = _commit_c_call(ctx, sv, commit, TU.block_id_for_height(1000), 1000, mode)
        g50, _ = _p50_p99(call, iters, warm=10)
        m, off = coracle.pack_msgs(msgs)  # the commit's sign-bytes and signatures
        pk = np.ascontiguousarray(sv.pubkeys)
        c50, _ = _p50_p99(lambda: coracle.verify_batch(pk, sig, m, off, mode, nthreads=1), max(20, iters // 4), warm=3)
        rows.append({"n": n, "gpu_commit_ms": g50, "cpu_1core_ms": c50, "gpu_wins": bool(g50 < c50)})
        del keep
    cross = None
    for r in reversed(rows):
        if not r["gpu_wins"]:
            break
        cross = r["n"]
    return {"n": cross, "rows": rows,
            "how": "smallest n from which cmtv_verify_commit (p50, one n-validator commit) beats the oracle on one "
                   "core (p50, the same n signatures) at every larger n measured"}


def verify_commit_10k(ctx, mode, iters, host_api_ms=None):
    """VerifyCommit at configs[1] scale: one 10,000-
    validator commit through cmtv_verify_commit, packed once, p50 / p99 wall
    (plan + staging + sign-bytes templated on the device + kernel + replay of
    types/validator_set.go:667-714), beside the host-API batch of the same
    signatures (e2e_10k)."""
    from cometbft_amd import testutil as TU

    sv = TU.make_validator_set(ctx, 10_000)
    commit, _, _ = TU.make_commit(ctx, sv, height=1000)
    call, keep = _commit_c_call(ctx, sv, commit, TU.block_id_for_height(1000), 1000, mode)
    st0 = ctx.stats()
    p50, p99 = _p50_p99(call, iters, warm=10)
    st1 = ctx.stats()
    kms = (st1["device_ms"] - st0["device_ms"]) / max(1, st1["timed_calls"] - st0["timed_calls"])
    res = {"n_validators": 10_000, "iters": iters, "p50_ms": p50, "p99_ms": p99, "kernel_ms": round(kms, 4),
           "value": round(10_000 / p50 * 1e3, 1), "unit": "verifs/s",
           "path": "cmtv_verify_commit (C ABI, commit packed once): plan + pinned staging + device sign-bytes + "
                   "k_verify_quad_hs + VerifyCommit replay"}
    if host_api_ms:
        res["over_host_api"] = round(p50 / host_api_ms, 3)
    # the same commit in the context's pinned memory (signatures and keys DMA'd from it)
    callp, keepp = _commit_c_call(ctx, sv, commit, TU.block_id_for_height(1000), 1000, mode, pinned=True)
    p50p, p99p = _p50_p99(callp, iters, warm=10)
    res["pinned"] = {"p50_ms": p50p, "p99_ms": p99p, "value": round(10_000 / p50p * 1e3, 1)}
    del keep, keepp
    return res


def latency_150(ctx, mode, iters):
    """p50/p99 VerifyCommit latency for a 150-validator commit (host API, end
    to end): the C call alone (cmtv_verify_commit on a pre-packed commit, what
    a cgo binding pays) and through the Python mirror (which re-packs the
    commit's Python objects every call), plus the keyset-cache variant."""
    from cometbft_amd import Context
    from cometbft_amd import testutil as TU

    sv = TU.make_validator_set(ctx, 150)
    commit, msgs, sigs = TU.make_commit(ctx, sv, height=1000)
    bid = TU.block_id_for_height(1000)

    def c_call(c):
        return _commit_c_call(c, sv, commit, bid, 1000, mode)

    def measure(fn):
        return _p50_p99(fn, iters, warm=50)  # 1000 iterations, 50 warm-up

    call, keep = c_call(ctx)
    p50c, p99c = measure(call)
    p50, p99 = measure(lambda: sv.valset.verify_commit(TU.CHAIN_ID, bid, 1000, commit, ctx=ctx, mode=mode))
    res = {"n_validators": 150, "iters": iters, "p50_ms": p50c, "p99_ms": p99c,
           "path": "cmtv_verify_commit (C ABI, commit packed once as a cgo shim would hold it): sign-bytes + H2D "
                   "+ kernel + D2H + VerifyCommit replay",
           "kernel": "k_verify_row4_split: one signature per CU in the row layout (DESIGN.md 4.9)",
           "python_mirror": {"p50_ms": p50, "p99_ms": p99, "path": "ValidatorSet.verify_commit (re-packs per call)"}}
    kctx = Context(device=ctx.device_ordinal(0))
    kctx.keyset_cache(4)
    kcall, kkeep = c_call(kctx)
    kp50, kp99 = measure(kcall)
    res["keyset_cache"] = {"p50_ms": kp50, "p99_ms": kp99,
                           "path": "same C call, validator set registered once (cmtv_keyset_cache): keyed row kernel, one signature per CU"}
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


def latency_150_under_load(mode, iters, load_heights=30_000, gap_ms=1.0, windows=None):
    """p50 / p99 of a 150-validator
    VerifyCommit (cmtv_verify_commit, packed once, keyset cache on) while
    another thread keeps running cmtv_verify_commits over load_heights x
    150-validator commits on the SAME context (blocksync / light-client replay
    beside consensus: consensus/state.go:1661 -> state/execution.go:135 while
    blockchain/v0/reactor.go:349-400 runs). 30,000 heights = 4.5M signatures
    per call: configs[2]'s long-call chunking (2^20-signature keyed batch
    launches that hold every SIMD for ~2.7 ms each). The bulk call holds the
    context lock only while it enqueues a chunk; near a latency call its
    chunks run on a CU-masked stream that leaves 8 CUs to the 150-validator
    call's kernel (runtime.cpp lat_window_ns); idle numbers from the same
    context beside it. The 150-validator calls are gap_ms apart (a node's
    consensus commits come a block time apart; back to back, they hold the
    context lock nearly all the time and starve the load's submissions, so
    the "loaded" numbers would be of an idle GPU); the load's own rate over
    the window is reported beside them. windows: a list that gets each
    loaded call's (start, end) CLOCK_MONOTONIC ns (tools/lat_trace.py)."""
    import threading

    from cometbft_amd import Context
    from cometbft_amd import _native as N
    from cometbft_amd import testutil as TU

    ctx = Context(device=0)
    ctx.keyset_cache(4)
    sv = TU.make_validator_set(ctx, 150)
    commit, _, _ = TU.make_commit(ctx, sv, height=1000)
    call, keep = _commit_c_call(ctx, sv, commit, TU.block_id_for_height(1000), 1000, mode)
    chain = TU.ReplayChain(ctx, sv, 2000, load_heights, flip=0.0)
    idle = _p50_p99(call, iters, warm=50)
    # the same calls 1 ms apart with no load (the loaded pattern without the load)
    idle_spaced = _p50_p99_inner(call, lambda: time.sleep(gap_ms * 1e-3), iters, warm=20)
    stop = threading.Event()
    passes = [0]
    t_bulk = []

    def load():
        while not stop.is_set():
            t = time.perf_counter()
            chain.call(ctx, N.VERIFY_COMMIT, mode)
            t_bulk.append(time.perf_counter() - t)
            passes[0] += 1

    th = threading.Thread(target=load, daemon=True)
    st0 = ctx.stats()
    th.start()
    time.sleep(0.2)

    def gap():
        time.sleep(gap_ms * 1e-3)  # releases the GIL: the load thread's Python runs here

    timed = call
    if windows is not None:
        def timed():
            t0 = time.monotonic_ns()
            call()
            windows.append((t0, time.monotonic_ns()))

    s_load0 = ctx.stats()["signatures"]
    t_win = time.perf_counter()
    loaded = _p50_p99_inner(timed, gap, iters, warm=20)
    t_win = time.perf_counter() - t_win
    s_load = ctx.stats()["signatures"] - s_load0 - 150 * iters
    stop.set()
    th.join()
    st1 = ctx.stats()
    rcs, _, _ = chain.outcome()
    del keep
    ctx.close()
    return {"idle_p50_ms": idle[0], "idle_p99_ms": idle[1], "p50_ms": loaded[0], "p99_ms": loaded[1],
            "p99_over_idle_p99": round(loaded[1] / idle[1], 2), "iters": iters,
            "idle_spaced_p50_ms": idle_spaced[0], "idle_spaced_p99_ms": idle_spaced[1],
            "p99_over_idle_spaced_p99": round(loaded[1] / idle_spaced[1], 2),
            "load": f"cmtv_verify_commits over {load_heights} x 150 commits in a loop on the same context "
                    f"({passes[0]} passes, median {round(float(np.median(t_bulk)) * 1e3, 2) if t_bulk else None} "
                    "ms each)", "load_ok": bool(np.all(rcs == 0)),
            "masked_chunks": st1["masked_chunks"] - st0["masked_chunks"], "gap_ms": gap_ms,
            "load_verifs_per_s_during_window": round(s_load / t_win, 1),
            "path": "cmtv_verify_commit (150 validators, keyset cache) from the main thread; the load from a second "
                    "thread"}


def verify_commit_10k_keyset(mode, iters):
    """configs[1] as a node runs it in steady state --
    cmtv_verify_commit on the 10,000-validator commit, the validator set's
    keys registered once by the keyset cache (the first call), p50 / p99."""
    from cometbft_amd import Context
    from cometbft_amd import testutil as TU

    ctx = Context(device=0)
    ctx.keyset_cache(4)
    sv = TU.make_validator_set(ctx, 10_000)
    commit, _, _ = TU.make_commit(ctx, sv, height=1000)
    call, keep = _commit_c_call(ctx, sv, commit, TU.block_id_for_height(1000), 1000, mode)
    st0 = ctx.stats()
    p50, p99 = _p50_p99(call, iters, warm=10)
    st1 = ctx.stats()
    kms = (st1["device_ms"] - st0["device_ms"]) / max(1, st1["timed_calls"] - st0["timed_calls"])
    callp, keepp = _commit_c_call(ctx, sv, commit, TU.block_id_for_height(1000), 1000, mode, pinned=True)
    p50p, p99p = _p50_p99(callp, iters, warm=10)
    del keep, keepp
    ctx.close()
    return {"p50_ms": p50, "p99_ms": p99, "kernel_ms": round(kms, 4), "value": round(10_000 / p50 * 1e3, 1),
            "pinned": {"p50_ms": p50p, "p99_ms": p99p, "value": round(10_000 / p50p * 1e3, 1),
                       "path": "the commit's arrays in the context's cmtv_alloc_pinned memory: the keyed kernel "
                               "reads its signatures in place from there over PCIe (no host copy, no DMA; "
                               "CMTV_KEYED_ZC)"},
            "unit": "verifs/s", "iters": iters,
            "path": "cmtv_verify_commit with cmtv_keyset_cache: plan + staging + device sign-bytes + keyed kernel "
                    "+ VerifyCommit replay"}


# The PMC summaries of THIS round's tree (TAG=r05 tools/gpu_prof_r04.sh: rocprofv3
# --pmc passes over the quick form of this bench command)
PMC_SQ = "r06_pmc_sq.json"
PMC_TRAFFIC = "r06_traffic.json"


def load_valu_busy(n=10_000, kernel="k_verify_quad_hs<0u>"):
    """VALUBusy (SQ_ACTIVE_INST_VALU-based, chip-wide) of the bench's verify
    kernel at the step's size, from the committed PMC summary of the bench
    command (profiles/PMC_SQ, tools/pmc_summary.py)."""
    try:
        with open(os.path.join(ROOT, "profiles", PMC_SQ)) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    waves = 4 * ((4 * ((n + 63) // 64) + 2) // 3)  # the split kernel's grid for n signatures
    for k, v in d.items():
        if kernel in k and f"grid={waves} waves" in k and "valu_busy_pct" in v:
            return {"valu_busy_pct": v["valu_busy_pct"], "valu_insts_per_wave": v.get("valu_insts_per_wave"),
                    "wave_cycles_per_wave": v.get("wave_cycles_per_wave"),
                    "source": f"profiles/{PMC_SQ}", "kernel": k}
    return None


def load_traffic(mode_key="go"):
    """Raw FETCH_SIZE + WRITE_SIZE bytes per launch of the step's kernel
    (profiles/PMC_TRAFFIC; 'go' / 'zip215' instantiation)."""
    p = os.path.join(ROOT, "profiles", PMC_TRAFFIC)
    try:
        with open(p) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, None
    d = d.get(mode_key, d)
    return d.get("bytes_per_launch"), f"profiles/{PMC_TRAFFIC}"


def process_per_gpu_main(args):
    """The round-1 harness: one process per GPU over torch.distributed."""
    import torch
    import torch.distributed as dist

    from cometbft_amd import Context

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    mode = 0 if args.mode == "go" else 1
    ctx = Context(devices=[local])
    D = Devices(ctx, 1, args.n)
    d_all = torch.zeros(world * D.words, dtype=torch.int64, device=dev)

    def step():
        D.step(ctx, mode)
        if world > 1:
            with torch.cuda.stream(torch.cuda.ExternalStream(ctx.device_stream(0))):
                dist.all_gather_into_tensor(d_all, D.t[0]["bm"][: D.words])

    barrier = (lambda: dist.barrier()) if world > 1 else (lambda: None)
    elapsed, kms = timed_steps(ctx, step, args.steps, args.warmup, barrier)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if rank == 0:
        value = world * args.n * args.steps / elapsed
        print(json.dumps({"metric": METRIC, "value": round(value, 1), "unit": "verifs/s", "n_gpus": world,
                          "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
                          "scaling": "weak", "vs_baseline": None, "dtype": "u32", "data": "synthetic",
                          "config": {"workload": "configs[1] per GPU, process per GPU", "sigs_per_gpu": args.n,
                                     "parallelism": f"dp{world}", "kernel_ms": round(kms, 4),
                                     "verdicts_ok": bool(D.verdicts_ok())}}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def main():
    args = parse()
    if args.process_per_gpu:
        return process_per_gpu_main(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    n_dev = world if world > 1 else max(1, args.gpus)
    import torch.distributed as dist

    if world > 1:
        # ranks only meet at barriers: gloo on the CPU; rank 0 drives every GPU
        dist.init_process_group("gloo")

    def barrier():
        if world > 1:
            dist.barrier()

    def max_over_ranks(x):
        if world == 1:
            return x
        import torch

        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    if rank != 0:
        # the timed region's two barriers, the max-over-ranks reduction and
        # the final barrier, in rank 0's order
        for _ in range(2):
            barrier()
        max_over_ranks(0.0)
        barrier()
        dist.destroy_process_group()
        return

    import torch

    from cometbft_amd import Context

    torch.cuda.set_device(0)
    mode = 0 if args.mode == "go" else 1
    # CMTV_BENCH_DEVICES="0,0" rehearses the N-device flow on fewer GPUs
    # (a repeated ordinal: peer-copy gathers instead of RCCL)
    env_devs = os.environ.get("CMTV_BENCH_DEVICES")
    ordinals = [int(x) for x in env_devs.split(",")] if env_devs else list(range(n_dev))
    assert len(ordinals) == n_dev, (ordinals, n_dev)
    ctx = Context(devices=ordinals)
    D = Devices(ctx, n_dev, args.n)
    elapsed, kernel_ms = timed_steps(ctx, lambda: D.step(ctx, mode), args.steps, args.warmup, barrier)
    run_head = dict(LAST_RUN)
    ok = D.verdicts_ok()
    elapsed = max_over_ranks(elapsed)
    total = n_dev * args.n * args.steps
    value = total / elapsed
    achieved = args.n * MACS_PER_VERIFY / (kernel_ms * 1e-3) / 1e12
    traffic, tfile = load_traffic("go" if mode == 0 else "zip215")
    # algorithmic HBM bytes per launch: key, signature, offset and message in,
    # one verdict bit out
    alg_bytes = round(args.n * (32 + 64 + 4 + D.msg_bytes_mean) + args.n / 8)
    line = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "verifs/s",
        "n_gpus": n_dev,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic",
        "config": {"workload": "configs[1]: one synthetic 10,000-validator commit per GPU per step "
                               "(inputs resident in HBM; one process drives every GPU through "
                               "cmtv_verify_ed25519_multi_device: independent commits, no data-path collective; "
                               "the RCCL bitmap all-gather is measured in replay_c3)",
                   "sigs_per_gpu": args.n, "mode": args.mode, "msg_bytes_mean": round(D.msg_bytes_mean, 1),
                   "parallelism": f"dp{n_dev} (single process, cmtv_open_devices)",
                   "warmup_clock_settle_s": CLOCK_SETTLE_S,
                   "collective": "none",
                   "verdicts_ok": bool(ok),
                   "devices": run_head},
        "roofline": {"bound": "valu_int", "achieved": round(achieved, 3), "peak": INT_MAC_PEAK_T,
                     "unit": "TMAC/s", "frac": round(achieved / INT_MAC_PEAK_T, 4),
                     "traffic": traffic, "traffic_source": tfile, "algorithmic_bytes": alg_bytes,
                     "traffic_over_algorithmic": round(traffic / alg_bytes, 2) if traffic else None,
                     "kernel_ms": round(kernel_ms, 4),
                     "valu_utilisation": load_valu_busy(args.n),
                     "work": f"{MACS_PER_VERIFY} int32 MACs/verify x {args.n} verifies per launch",
                     "timing": "HIP events on each device's launch stream at both ends of the timed region "
                               "(back-to-back launches): region / steps; the library's sampled per-call "
                               "events are config.devices.sampled_kernel_ms"},
    }
    # ZIP-215 mode on the same inputs (the north-star semantics)
    el_z, kms_z = timed_steps(ctx, lambda: D.step(ctx, 1 - mode), args.steps, 2, lambda: None)
    line["zip215" if mode == 0 else "go_stdlib"] = {
        "value": round(n_dev * args.n * args.steps / el_z, 1), "unit": "verifs/s",
        "ms_per_step": round(el_z / args.steps * 1e3, 4), "kernel_ms": round(kms_z, 4),
        "frac": round(args.n * MACS_PER_VERIFY / (kms_z * 1e-3) / 1e12 / INT_MAC_PEAK_T, 4)}
    # the side lines below never cost the headline: a failure (say, a
    # collective that a multi-GPU node refuses) is recorded in its own key
    def aux(key, fn):
        try:
            line[key] = fn()
        except Exception as e:  # noqa: BLE001 -- reported in the line, not swallowed
            line[key] = {"error": f"{type(e).__name__}: {e}"[:400]}
            print(f"bench: {key} failed: {e!r}", file=sys.stderr, flush=True)

    aux("e2e_10k", lambda: e2e_10k(Context(device=0), D.host[0], mode))
    if not args.no_latency and n_dev == 1:
        aux("verify_commit_10k",
            lambda: verify_commit_10k(Context(device=0), mode, 200, line["e2e_10k"].get("ms") or 0.0))
    if n_dev == 1 and not args.no_keyset:
        aux("keyset_10k", lambda: keyset_10k(ctx, D, mode, args.steps))
    if not args.no_cpu_baseline and n_dev == 1:  # rank 0 at N=1 only (bench contract)
        pk, sigs, m, off = D.host[0]
        line["cpu_baseline"] = cpu_baseline(pk, sigs, m, off, mode, args.cpu_seconds)
        cb = line["cpu_baseline"]
        z = line.get("zip215") or line.get("go_stdlib")
        cb["gpu_over_cpu"] = round(value / n_dev / cb["value"], 1)
        cb["single_core"]["gpu_over_cpu"] = round(value / n_dev / cb["single_core"]["value"], 1)
        cb["quota_bound_all_threads"]["gpu_over_cpu"] = round(value / n_dev / cb["quota_bound_all_threads"]["value"],
                                                              1)
        ex = cb["extrapolated_all_cores"]
        if ex["value"]:
            ex["gpu_over_cpu"] = round(value / n_dev / ex["value"], 1)
            ex["gpu_over_cpu_other_mode"] = round(z["value"] / n_dev / ex["value_other_mode"], 1)
        try:
            cb["crossover"] = crossover(Context(device=0), mode)
        except Exception as e:  # noqa: BLE001 -- an aux figure never sinks the bench line
            cb["crossover"] = {"error": f"{type(e).__name__}: {e}"[:400]}
    if not args.no_latency and n_dev == 1:
        aux("verify_commit_10k_keyset", lambda: verify_commit_10k_keyset(mode, 200))
    if not args.no_latency:
        aux("latency_150", lambda: latency_150(ctx, mode, args.latency_iters))
        if n_dev == 1:
            aux("latency_150_under_load", lambda: latency_150_under_load(mode, args.latency_iters))
        if n_dev == 1:
            aux("replay_150", lambda: replay_line(0))
    if not args.no_light and n_dev == 1:
        aux("light_client", lambda: light_line(0))
    if not args.no_sr25519 and n_dev == 1:
        aux("sr25519", lambda: sr25519_line(ctx, torch.device("cuda", 0), 10_000, 20, args.cpu_seconds / 4,
                                            not args.no_cpu_baseline))
    if not args.no_c3_host:
        def c3h():
            hctx = Context(devices=ordinals)
            hctx.keyset_cache(4)  # a node registers its validator set once
            pctx = Context(devices=ordinals)
            pctx.keyset_cache(4)
            try:
                return c3_host_line(hctx, mode, n_heights=args.c3_heights, packed_ctx=pctx)
            finally:
                pctx.close()
                hctx.close()
        aux("replay_c3_host", c3h)
    c3 = None
    if not args.no_c3:
        del D
        torch.cuda.empty_cache()
        aux("replay_c3", lambda: c3_line(ctx, n_dev, mode, n_heights=args.c3_heights))
        c3 = line["replay_c3"]
    print(json.dumps(line), flush=True)
    barrier()
    if world > 1:
        dist.destroy_process_group()
    # a wrong verdict anywhere fails the run (an aux line's error does not)
    if not ok or (c3 is not None and c3.get("verdicts_ok") is False):
        sys.exit(3)


if __name__ == "__main__":
    main()
