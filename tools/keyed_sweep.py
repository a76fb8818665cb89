"""Kernel time of registered-key verification vs batch size for the keyed quad
(two-helper) and keyed lane kernels, to place the keyed quad/lane band
(runtime.cpp kKeyedQuadMax), each forced with CMTV_FORM.

    python tools/keyed_sweep.py 4096 8192 12288 16384 24576 32768
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from cometbft_amd import Context, pack_messages
    from cometbft_amd import testutil as TU

    sizes = [int(x) for x in sys.argv[1:]] or [4096, 8192, 12288, 16384, 24576, 32768]
    nmax = max(sizes)
    gen = Context(device=0)
    sv = TU.make_validator_set(gen, 150)
    msgs = TU.commit_messages(nmax, 1000)
    m, off = pack_messages(msgs)
    kidx = (np.arange(nmax) % 150).astype(np.uint32)
    sig = gen.sign(sv.seeds, m, off, kidx)
    dev = torch.device("cuda", 0)
    res = {}
    for kind, env in (("quad2", "kquad"), ("lane", "klane")):
        os.environ["CMTV_FORM"] = env
        ctx = Context(device=0)
        ks = ctx.register_keys(sv.pubkeys)
        for n in sizes:
            ki = torch.from_numpy(kidx[:n].copy()).to(dev)
            sg = torch.from_numpy(sig[:n].copy()).to(dev)
            mm = torch.from_numpy(np.concatenate([m[: off[n]], np.zeros(16, np.uint8)])).to(dev)
            oo = torch.from_numpy(off[: n + 1].view(np.int32).copy()).to(dev)
            bm = torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev)
            st = torch.cuda.current_stream(dev)

            def step():
                ctx.verify_indexed_device(ks, n, ki.data_ptr(), sg.data_ptr(), mm.data_ptr(), oo.data_ptr(), 0, 0,
                                          bm.data_ptr(), stream=st.cuda_stream)

            for _ in range(5):
                step()
            st.synchronize()
            s0 = ctx.stats()
            for _ in range(20):
                step()
            st.synchronize()
            s1 = ctx.stats()
            kms = (s1["device_ms"] - s0["device_ms"]) / max(s1["timed_calls"] - s0["timed_calls"], 1)
            ok = bool((bm.cpu().numpy().view(np.uint64)[: n // 64] == np.uint64((1 << 64) - 1)).all())
            res.setdefault(str(n), {})[kind] = {"kernel_ms": round(kms, 4), "ok": ok}
            print(kind, n, round(kms, 4), ok, flush=True)
        ks.free()
        del ctx
    print(json.dumps(res))


if __name__ == "__main__":
    main()
