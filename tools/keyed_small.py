"""Registered-key verification at commit sizes (dev tool): mean wall time per
device-resident call (cmtv_verify_ed25519_indexed_device) and the context's
kernel time, for n in argv (default 150). CMTV_FORM=kquad selects the
keyed quad kernel instead of the keyed row kernel."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from cometbft_amd import Context
from cometbft_amd import testutil as TU
from cometbft_amd import pack_messages

ctx = Context(device=0)
for n in [int(a) for a in (sys.argv[1:] or ["150"])]:
    sv = TU.make_validator_set(ctx, n)
    m, off = pack_messages(TU.commit_messages(n, 1000))
    sig = ctx.sign(sv.seeds, m, off)
    ks = ctx.register_keys(np.ascontiguousarray(sv.pubkeys))
    dev = torch.device("cuda:0")
    d_idx = torch.arange(n, dtype=torch.int32, device=dev)
    d_sig = torch.from_numpy(sig.copy()).to(dev)
    d_m = torch.from_numpy(m).to(dev)
    d_off = torch.from_numpy(off.view(np.int32)).to(dev)
    d_v = torch.zeros(n, dtype=torch.uint8, device=dev)
    d_bm = torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    for mode in (0, 1):
        def call():
            ctx.verify_indexed_device(ks, n, d_idx.data_ptr(), d_sig.data_ptr(), d_m.data_ptr(), d_off.data_ptr(),
                                      mode, d_v.data_ptr(), d_bm.data_ptr(), s)
        for _ in range(5):
            call()
        torch.cuda.synchronize()
        k0 = ctx.stats()["device_ms"]
        c0 = ctx.stats()["timed_calls"]
        reps = 50
        t = time.time()
        for _ in range(reps):
            call()
            torch.cuda.synchronize()
        dt = (time.time() - t) / reps
        st = ctx.stats()
        kms = (st["device_ms"] - k0) / max(1, st["timed_calls"] - c0)
        print(f"n={n} mode={mode} wall_ms={dt * 1e3:.3f} kernel_ms={kms:.4f} valid={int(d_v.sum())}/{n}", flush=True)
    ks.free()
