"""Quick GPU timing of the verify kernel on device-resident inputs (dev tool)."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from cometbft_amd import Context, pack_messages
from oracle import coracle

ctx = Context(device=0)
for n in [int(x) for x in (sys.argv[1:] or ["10000"])]:
    rng = np.random.default_rng(0)
    nk = min(n, int(os.environ.get("NKEYS", "4096")))
    seeds = rng.integers(0, 256, (nk, 32), dtype=np.uint8)
    msgs = [rng.integers(0, 256, 116, dtype=np.uint8).tobytes() for _ in range(n)]
    m, off = pack_messages(msgs)
    kidx = (np.arange(n) % nk).astype(np.uint32)
    t = time.time()
    sig = ctx.sign(seeds, m, off, key_idx=kidx)
    pk = ctx.pubkeys(seeds)[kidx]
    ts = time.time() - t
    dev = torch.device("cuda:0")
    d_pk = torch.from_numpy(pk.copy()).to(dev)
    d_sig = torch.from_numpy(sig.copy()).to(dev)
    d_m = torch.from_numpy(m).to(dev)
    d_off = torch.from_numpy(off.view(np.int32)).to(dev)
    d_valid = torch.zeros(n, dtype=torch.uint8, device=dev)
    d_bm = torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    for mode in (0, 1):
        for _ in range(2):
            ctx.verify_device(n, d_pk.data_ptr(), d_sig.data_ptr(), d_m.data_ptr(), d_off.data_ptr(), mode,
                              d_valid.data_ptr(), d_bm.data_ptr(), s)
        torch.cuda.synchronize()
        reps = 5
        t = time.time()
        for _ in range(reps):
            ctx.verify_device(n, d_pk.data_ptr(), d_sig.data_ptr(), d_m.data_ptr(), d_off.data_ptr(), mode,
                              d_valid.data_ptr(), d_bm.data_ptr(), s)
        torch.cuda.synchronize()
        dt = (time.time() - t) / reps
        ok = int(d_valid.sum().item())
        print(f"n={n} mode={mode} ms={dt*1e3:.3f} verifs/s={n/dt:.4e} valid={ok}/{n} sign_s={ts:.2f}", flush=True)
    if os.environ.get("KEYED"):
        t = time.time()
        ks = ctx.register_keys(ctx.pubkeys(seeds))
        treg = time.time() - t
        d_idx = torch.from_numpy(kidx.view(np.int32)).to(dev)
        for mode in (0, 1):
            for _ in range(2):
                ctx.verify_indexed_device(ks, n, d_idx.data_ptr(), d_sig.data_ptr(), d_m.data_ptr(), d_off.data_ptr(),
                                          mode, d_valid.data_ptr(), d_bm.data_ptr(), s)
            torch.cuda.synchronize()
            reps = 5
            t = time.time()
            for _ in range(reps):
                ctx.verify_indexed_device(ks, n, d_idx.data_ptr(), d_sig.data_ptr(), d_m.data_ptr(), d_off.data_ptr(),
                                          mode, d_valid.data_ptr(), d_bm.data_ptr(), s)
            torch.cuda.synchronize()
            dt = (time.time() - t) / reps
            ok = int(d_valid.sum().item())
            print(f"KEYED n={n} keys={nk} mode={mode} ms={dt*1e3:.3f} verifs/s={n/dt:.4e} valid={ok}/{n} "
                  f"register_ms={treg*1e3:.1f}", flush=True)
        ks.free()
