"""Quad-kernel time vs batch size (dev tool): device-resident inputs, HIP-event
timing on the launch stream. Env CMTV_FORM forces the kernel."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from cometbft_amd import Context, pack_messages

ctx = Context(device=0)
dev = torch.device("cuda:0")
for n in [int(x) for x in (sys.argv[1:] or ["10000"])]:
    rng = np.random.default_rng(0)
    nk = min(n, 4096)
    seeds = rng.integers(0, 256, (nk, 32), dtype=np.uint8)
    msgs = [rng.integers(0, 256, 116, dtype=np.uint8).tobytes() for _ in range(n)]
    m, off = pack_messages(msgs)
    kidx = (np.arange(n) % nk).astype(np.uint32)
    sig = ctx.sign(seeds, m, off, key_idx=kidx)
    pk = ctx.pubkeys(seeds)[kidx]
    d_pk = torch.from_numpy(pk.copy()).to(dev)
    d_sig = torch.from_numpy(sig.copy()).to(dev)
    d_m = torch.from_numpy(np.concatenate([m, np.zeros(16, np.uint8)])).to(dev)
    d_off = torch.from_numpy(off.view(np.int32)).to(dev)
    d_valid = torch.zeros(n, dtype=torch.uint8, device=dev)
    d_bm = torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev)
    st = torch.cuda.current_stream()
    s = st.cuda_stream
    for mode in (0,):
        for _ in range(3):
            ctx.verify_device(n, d_pk.data_ptr(), d_sig.data_ptr(), d_m.data_ptr(), d_off.data_ptr(), mode,
                              d_valid.data_ptr(), d_bm.data_ptr(), s)
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
        for a, b in evs:
            a.record(st)
            ctx.verify_device(n, d_pk.data_ptr(), d_sig.data_ptr(), d_m.data_ptr(), d_off.data_ptr(), mode,
                              d_valid.data_ptr(), d_bm.data_ptr(), s)
            b.record(st)
        torch.cuda.synchronize()
        ms = float(np.median([a.elapsed_time(b) for a, b in evs]))
        ok = int(d_valid.sum().item())
        print(f"n={n} mode={mode} kernel_ms={ms:.4f} verifs/s={n / ms * 1e3:.4e} valid={ok}/{n} "
              f"waves={(n * 4 + 63) // 64}", flush=True)
