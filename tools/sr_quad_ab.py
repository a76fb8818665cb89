"""sr25519 quad/lane crossover (dev tool): device-resident
cmtv_verify_sr25519_device wall time per call at the sizes in argv, for an
A/B of the forms:  CMTV_FORM=quad python tools/sr_quad_ab.py 40960 49152 (and lane)"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from cometbft_amd import Context
from oracle import coracle  # synthetic signatures only

torch.zeros(1, device="cuda:0")  # torch's HIP init before the library's
ctx = Context(device=0)
rng = np.random.default_rng(4)
minis = rng.integers(0, 256, (150, 32), dtype=np.uint8)
for n in [int(a) for a in (sys.argv[1:] or ["49152"])]:
    kidx = (np.arange(n) % 150).astype(np.uint32)
    msgs = [rng.integers(0, 256, 116, dtype=np.uint8).tobytes() for _ in range(n)]
    m, off = coracle.pack_msgs(msgs)
    sig = coracle.sr25519_sign_batch(minis, m, off, key_idx=kidx)
    pk = coracle.sr25519_pubkeys(minis)[kidx]
    dev = torch.device("cuda:0")
    t = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in
         {"pk": pk, "sig": sig, "m": m, "off": off.view(np.int32)}.items()}
    d_v = torch.zeros(n, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    call = lambda: ctx.verify_sr25519_device(n, t["pk"].data_ptr(), t["sig"].data_ptr(), t["m"].data_ptr(),
                                             t["off"].data_ptr(), d_v.data_ptr(), 0, s)
    for _ in range(3):
        call()
    torch.cuda.synchronize()
    reps = 10
    t0 = time.perf_counter()
    for _ in range(reps):
        call()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    print(f"FORM={os.environ.get('CMTV_FORM', 'default')} n={n} ms={dt * 1e3:.3f} "
          f"valid={int(d_v.sum())}/{n}", flush=True)
