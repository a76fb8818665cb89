"""Phase timeline of the helper-wave quad kernel (k_verify_quad_split) on one
10k commit, per workgroup, from the probe build of the library.

  make -C cometbft_amd/csrc OUT=../../abtest/libprobe.so BUILD=../../build/probe KFLAGS=-DCMTV_PHASE_PROBE
  CMTV_LIBRARY=$PWD/abtest/libprobe.so python tools/phase_probe.py [n]
  CMTV_LIBRARY=$PWD/abtest/libprobe.so python tools/phase_probe.py --sr [n]   (k_verify_sr25519_quad_hs)
  (inputs resident in HBM as in bench.py; --host: host arrays through the staging / zero-copy path)

Lane 0 of every wave records the shader clock at kernel entry (0), before /
after barrier 1 (1, 2: the helper's scalars), before / after barrier 2 (3, 4:
the helper's [u]B) and, for the quad waves, at exit (5); in the helper-summed
kernel (k_verify_quad_hs) slot 6 holds the cycles each wave waited at the
per-window barriers. Printed per mode:
the spread of workgroup starts, and for the workgroup that ends last and the
median workgroup, when the helper and the quad waves reach each barrier --
which of them waits, and for how long.
"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SLOTS = 8


def main():
    sr = "--sr" in sys.argv
    host = "--host" in sys.argv  # host arrays (zero-copy / staged inputs) instead of HBM-resident ones
    argv = [a for a in sys.argv[1:] if a not in ("--sr", "--host")]
    n = int(argv[0]) if len(argv) > 0 else 10_000
    # signatures per 4-wave workgroup: 48 (k_verify_quad_split) or 3 (the row
    # kernel, k_verify_row_split, which the library picks up to kRowMax)
    per_wg = int(argv[1]) if len(argv) > 1 else 48
    from cometbft_amd import Context, pack_messages
    from cometbft_amd import _native as N
    from cometbft_amd import testutil as TU

    if not host:  # torch first (as bench.py): its HIP init before the library's
        import torch

        dev = torch.device("cuda", 0)
        torch.zeros(1, device=dev)
    L = N.lib()
    fn = L.cmtv_debug_phase_times_sr if sr else L.cmtv_debug_phase_times
    fn.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_size_t]
    ctx = Context(device=0)
    m, off = pack_messages(TU.commit_messages(n, 1000))
    if sr:
        from oracle import coracle  # synthetic sr25519 signatures only

        rng = np.random.default_rng(4)
        minis = rng.integers(0, 256, (150, 32), dtype=np.uint8)
        kidx = (np.arange(n) % 150).astype(np.uint32)
        sig = coracle.sr25519_sign_batch(minis, m, off, key_idx=kidx)
        pk = np.ascontiguousarray(coracle.sr25519_pubkeys(minis)[kidx])
    else:
        sv = TU.make_validator_set(ctx, n)
        sig = ctx.sign(sv.seeds, m, off)
        pk = np.ascontiguousarray(sv.pubkeys)
    wgs = -(-n // per_wg)
    out = {}
    if not host:
        # the bench's form: inputs resident in HBM (bench.py configs[1] / [4] lines)
        d_pk = torch.from_numpy(np.ascontiguousarray(pk)).to(dev)
        d_sig = torch.from_numpy(np.ascontiguousarray(sig)).to(dev)
        d_m = torch.from_numpy(np.ascontiguousarray(m)).to(dev)
        d_off = torch.from_numpy(np.ascontiguousarray(off).view(np.int32)).to(dev)
        d_valid = torch.zeros(n, dtype=torch.uint8, device=dev)
    for mode, name in (((0, "sr25519"),) if sr else ((0, "go"), (1, "zip215"))):
        for _ in range(20):
            if host:
                v = ctx.verify_sr25519(pk, sig, m, off) if sr else ctx.verify(pk, sig, m, off, mode)
            else:
                args = (n, d_pk.data_ptr(), d_sig.data_ptr(), d_m.data_ptr(), d_off.data_ptr())
                if sr:
                    ctx.verify_sr25519_device(*args, d_valid.data_ptr())
                else:
                    ctx.verify_device(*args, mode, d_valid.data_ptr())
                torch.cuda.synchronize()
                v = d_valid.cpu().numpy()
        assert v.all()
        buf = np.zeros(wgs * 4 * SLOTS, np.uint64)
        assert fn(buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), buf.size) == 0
        st = buf.reshape(wgs, 4, SLOTS).astype(np.int64)
        waits = st[:, :, 6].copy()  # k_verify_quad_hs: cycle counts, not stamps
        # each workgroup against its own first entry: s_memtime counters of
        # different XCDs are not synchronised, so cross-workgroup offsets of
        # the shader clock mean nothing
        t0 = st[:, :, 0].min(axis=1)
        st = st - t0[:, None, None]
        q, h = st[:, :3, :], st[:, 3, :]
        end = q[:, :, 5].max(axis=1)
        start = st[:, :, 0].min(axis=1)

        def wg(b):
            return {"start": int(start[b]), "helper_at_b1": int(h[b, 1]), "quads_at_b1": [int(x) for x in q[b, :, 1]],
                    "b1_release": int(q[b, :, 2].max()), "helper_at_b2": int(h[b, 3]),
                    "quads_at_b2": [int(x) for x in q[b, :, 3]], "b2_release": int(q[b, :, 4].max()),
                    "quads_end": [int(x) for x in q[b, :, 5]]}

        last = int(np.argmax(end))
        med = int(np.argsort(end)[len(end) // 2])
        # waits: at barrier 1 the quads wait for the helper if it arrives last
        w1 = np.maximum(h[:, 1] - q[:, :, 1].max(axis=1), 0)
        w2 = np.maximum(h[:, 3] - q[:, :, 3].max(axis=1), 0)
        out[name] = {
            "span": int(end.max()), "start_spread": int(start.max()),
            "end_median": int(np.median(end)), "end_max": int(end.max()),
            "quads_wait_at_b1_for_helper": {"wgs": int((w1 > 0).sum()), "median": float(np.median(w1)),
                                            "max": int(w1.max())},
            "quads_wait_at_b2_for_helper": {"wgs": int((w2 > 0).sum()), "median": float(np.median(w2)),
                                            "max": int(w2.max())},
            "helper_b1_median": float(np.median(h[:, 1] - start)),
            # slot 7 of the helper: the end of its merlin transcripts / SHA-512s
            ("helper_transcript_end_median" if sr else "helper_hash_end_median"): float(np.median(h[:, 7] - start)),
            **({} if sr else {"helper_message_start_median": float(np.median(h[:, 5] - start)),
                              "helper_message_ready_median": float(np.median(h[:, 4] - start))}),
            "helper_b2_minus_b1_release_median": float(np.median(h[:, 3] - q[:, :, 2].max(axis=1))),
            "quad_b1_median": float(np.median(q[:, :, 1] - start[:, None])),
            "quad_b2_median": float(np.median(q[:, :, 3] - start[:, None])),
            "quad_end_median": float(np.median(q[:, :, 5] - start[:, None])),
            # k_verify_quad_hs (slot 6): cycles waited at the per-window barriers
            "hs_helper_window_wait_median": float(np.median(waits[:, 3])),
            "hs_quad_window_wait_median": float(np.median(waits[:, :3])),
            "hs_quad_window_wait_last_wg": [int(x) for x in waits[last, :3]],
            "last_wg": dict(wg(last), index=last), "median_wg": dict(wg(med), index=med),
        }
        print(name, json.dumps(out[name]), flush=True)
    with open(os.path.join(ROOT, "gpurun_out", "phase_probe_sr.json" if sr else "phase_probe.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
