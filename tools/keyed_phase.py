"""Phase timeline of the registered-key quad kernel (k_verify_keyed_quad_split,
keyset_10k / the keyset-cache VerifyCommit of configs[1]) from the probe build
of the library (where its 71 us go).

  make -C cometbft_amd/csrc OUT=../../tools/probe/libprobe.so BUILD=../../build/probe KFLAGS=-DCMTV_PHASE_PROBE
  CMTV_LIBRARY=$PWD/tools/probe/libprobe.so python tools/keyed_phase.py [n]

Five waves per workgroup (kernels.hip CMTV_STAMP5): 0 entry; the hash
helper (wave 4) slot 3 = k published; the decode helper (wave 3) slot 3 = R
decoded; the quads (waves 0-2) slot 4 = k taken, 1 = their 48 comb additions
done (before the barrier), 2 = after it, 5 = exit. Cycles of the shader clock
against each workgroup's first entry (XCD clocks are not synchronised).
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
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000
    import torch

    dev = torch.device("cuda", 0)
    torch.zeros(1, device=dev)
    from cometbft_amd import Context, pack_messages
    from cometbft_amd import _native as N
    from cometbft_amd import testutil as TU

    L = N.lib()
    L.cmtv_debug_phase_times.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_size_t]
    ctx = Context(device=0)
    m, off = pack_messages(TU.commit_messages(n, 1000))
    sv = TU.make_validator_set(ctx, n)
    sig = ctx.sign(sv.seeds, m, off)
    ks = ctx.register_keys(np.ascontiguousarray(sv.pubkeys))
    d_idx = torch.arange(n, dtype=torch.int32, device=dev)
    d_sig = torch.from_numpy(np.ascontiguousarray(sig)).to(dev)
    d_m = torch.from_numpy(np.ascontiguousarray(m)).to(dev)
    d_off = torch.from_numpy(np.ascontiguousarray(off).view(np.int32)).to(dev)
    d_valid = torch.zeros(n, dtype=torch.uint8, device=dev)
    wgs = -(-(4 * ((n + 63) // 64)) // 3)
    out = {}
    for mode, name in ((0, "go"), (1, "zip215")):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        for it in range(20):
            if it == 10:
                ev[0].record()
            ctx.verify_indexed_device(ks, n, d_idx.data_ptr(), d_sig.data_ptr(), d_m.data_ptr(), d_off.data_ptr(),
                                      mode, d_valid.data_ptr(), stream=torch.cuda.current_stream().cuda_stream)
        ev[1].record()
        torch.cuda.synchronize()
        assert d_valid.cpu().numpy().all()
        buf = np.zeros(wgs * 5 * SLOTS, np.uint64)
        assert L.cmtv_debug_phase_times(buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), buf.size) == 0
        st = buf.reshape(wgs, 5, SLOTS).astype(np.int64)
        simd = (st[:, :, 6] >> 4) & 3  # HW_ID of each wave: its SIMD
        shares = {f"wave{w}": int((simd[:, w][:, None] == np.delete(simd, w, axis=1)).any(axis=1).sum())
                  for w in range(5)}
        t0 = st[:, :, 0].min(axis=1)
        st = st - t0[:, None, None]
        q, dec, hsh = st[:, :3, :], st[:, 3, :], st[:, 4, :]
        end = q[:, :, 5].max(axis=1)
        med = lambda x: float(np.median(x))  # noqa: E731
        out[name] = {
            "ms_per_launch_events": round(ev[0].elapsed_time(ev[1]) / 10, 4),
            "workgroups": int(wgs), "end_median": med(end), "end_max": int(end.max()),
            "hash_helper_k_published_median": med(hsh[:, 3]),
            "decode_helper_R_done_median": med(dec[:, 3]),
            "quads_k_taken_median": med(q[:, :, 4]),
            "quads_combs_done_median": med(q[:, :, 1]),
            "barrier_release_median": med(q[:, :, 2].max(axis=1)),
            "quads_wait_for_R_median": med(np.maximum(q[:, :, 2].max(axis=1) - q[:, :, 1].max(axis=1), 0)),
            "after_barrier_to_exit_median": med(end - q[:, :, 2].max(axis=1)),
            "simd_of_wave_first_wg": [int(x) for x in simd[0]],
            "workgroups_where_wave_shares_its_simd": shares,
        }
        print(name, json.dumps(out[name]), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "keyed_phase.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
