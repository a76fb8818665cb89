"""Runs each verify kernel a few times on device-resident synthetic batches,
for rocprofv3 --pmc passes (tools/gpu_prof.sh): the default forms at 150
(k_verify_row4_split), 8192 and the 10k commit (k_verify_quad_hs), the oct2
form at 150 (CMTV_FORM=oct2), k_verify (100k, lane kernel),
k_verify_keyed_quad_split (10k over 150 keys) and the keyed lane kernels (262k
/ 1M over 150 keys).
Every batch is checked (all valid) so a counter pass never profiles a
broken kernel."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from cometbft_amd import Context, pack_messages

REPS = int(os.environ.get("PMC_REPS", "3"))
# PMC_ONLY=name,name,... runs only those batches (e.g. keyed_lane1m,lane262k)
ONLY = set(filter(None, os.environ.get("PMC_ONLY", "").split(",")))
dev = torch.device("cuda:0")
ctx = Context(device=0)
rng = np.random.default_rng(7)
NK = 150
seeds = rng.integers(0, 256, (NK, 32), dtype=np.uint8)
pks = ctx.pubkeys(seeds)


def batch(n):
    msgs = [rng.integers(0, 256, 116, dtype=np.uint8).tobytes() for _ in range(min(n, 20000))]
    reps = -(-n // len(msgs))
    msgs = (msgs * reps)[:n]
    m, off = pack_messages(msgs)
    kidx = (np.arange(n) % NK).astype(np.uint32)
    sig = ctx.sign(seeds, m, off, key_idx=kidx)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    return dict(n=n, kidx=t(kidx), pk=t(pks[kidx]), sig=t(sig), m=t(np.concatenate([m, np.zeros(16, np.uint8)])),
                off=t(off.view(np.int32)), valid=torch.zeros(n, dtype=torch.uint8, device=dev),
                bm=torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev))


def run(name, c, b, keyed=None):
    if ONLY and name not in ONLY:
        return
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(REPS):
        b["valid"].zero_()
        if keyed is None:
            c.verify_device(b["n"], b["pk"].data_ptr(), b["sig"].data_ptr(), b["m"].data_ptr(), b["off"].data_ptr(),
                            0, b["valid"].data_ptr(), b["bm"].data_ptr(), s)
        else:
            c.verify_indexed_device(keyed, b["n"], b["kidx"].data_ptr(), b["sig"].data_ptr(), b["m"].data_ptr(),
                                    b["off"].data_ptr(), 0, b["valid"].data_ptr(), b["bm"].data_ptr(), s)
    torch.cuda.synchronize()
    ok = int(b["valid"].sum().item())
    assert ok == b["n"], (name, ok, b["n"])
    print(f"{name}: n={b['n']} x{REPS} ok", flush=True)


def env_ctx(**env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update({k: str(v) for k, v in env.items()})
    try:
        return Context(device=0)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


def lane_ctx():
    return env_ctx(CMTV_FORM="lane,klane")


def want(*names):
    return not ONLY or any(n in ONLY for n in names)


if want("row4_150", "quad8192", "quad10k", "oct2_150", "keyed_quad10k"):
    b150, b8k, b10k = batch(150), batch(8192), batch(10000)
    run("row4_150", ctx, b150)
    run("quad8192", ctx, b8k)
    run("quad10k", ctx, b10k)
    run("oct2_150", env_ctx(CMTV_FORM="oct2"), b150)
lctx = lane_ctx()
if want("lane100k"):
    b100k = batch(100_000)
    run("lane100k", lctx, b100k)
    del b100k
if want("keyed_quad10k"):
    ks = ctx.register_keys(pks)
    run("keyed_quad10k", ctx, b10k, keyed=ks)
# configs[2]'s launch shape: 262,144 signatures per launch (kChunk), the 150
# keys cycling as in consecutive 150-validator commits
if want("lane262k", "keyed_lane262k", "keyed_lane1m", "keyed_wide1m"):
    b262k = batch(262_144)
    run("lane262k", lctx, b262k)
    lks = lctx.register_keys(pks)
    run("keyed_lane262k", lctx, b262k, keyed=lks)
    if want("keyed_lane1m", "keyed_wide1m"):
        del b262k
        b1m = batch(1 << 20)
        if want("keyed_lane1m"):
            run("keyed_lane1m", lctx, b1m, keyed=lks)
        if want("keyed_wide1m"):
            # radix-2^16 key combs (CMTV_KEYS_WIDE): configs[2]'s 2^20-signature launches
            wks = lctx.register_keys(pks, wide=True)
            run("keyed_wide1m", lctx, b1m, keyed=wks)
