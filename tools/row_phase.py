"""Phase timeline of the four-wave row kernel (k_verify_row4_split) or the
keyed row kernel on one 150-validator batch, from the probe build of the
library.

  make -C cometbft_amd/csrc OUT=../../abtest/libprobe.so BUILD=../../build/probe KFLAGS=-DCMTV_PHASE_PROBE
  CMTV_LIBRARY=$PWD/abtest/libprobe.so python tools/row_phase.py [n] [row4|krow]

Shader-clock stamps per wave (kernels.hip CMTV_STAMP), relative to the
workgroup's first entry: row4's lo wave (0): 1/2 at/after barrier 1, 3/4
at/after barrier 2, 5 verdict; A-hi and R-hi (1, 2): 6 decoded, 1-3 as lo;
helper (3): 1 scalars ready, 3 [u]B ready. Medians over workgroups, per mode, into gpurun_out/row_phase.json.
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
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 150
    form = sys.argv[2] if len(sys.argv) > 2 else "row4"
    from cometbft_amd import Context, pack_messages
    from cometbft_amd import _native as N
    from cometbft_amd import testutil as TU

    fn = N.lib().cmtv_debug_phase_times
    fn.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_size_t]
    ctx = Context(device=0)
    sv = TU.make_validator_set(ctx, n)
    m, off = pack_messages(TU.commit_messages(n, 1000))
    sig = ctx.sign(sv.seeds, m, off)
    pk = np.ascontiguousarray(sv.pubkeys)
    out = {}
    ks = ctx.register_keys(pk) if form == "krow" else None
    kidx = np.arange(n, dtype=np.uint32)
    if form == "krow":  # keyed row: R decode (meets barrier 1 mid-chain), A comb, B comb, hash helper
        names = {"R": (0, [1, 2, 3, 4, 5]), "A": (1, [1, 2, 3]), "B": (2, [1, 2]), "helper": (3, [1])}
    else:  # row4: lo (decodes A and R), A-hi, R-hi, helper
        names = {"lo": (0, [1, 2, 3, 4, 5]), "A_hi": (1, [6, 1, 2, 3]), "R_hi": (2, [6, 1, 2, 3]),
                 "helper": (3, [1, 3])}
    nw = len(names)
    for mode, name in ((0, "go"), (1, "zip215")):
        for _ in range(10):
            v = ctx.verify_indexed(ks, kidx, sig, m, off, mode) if ks is not None else ctx.verify(pk, sig, m, off, mode)
        assert v.all()
        buf = np.zeros(n * 4 * SLOTS, np.uint64)
        assert fn(buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), buf.size) == 0
        st = buf.reshape(n, 4, SLOTS).astype(np.int64)
        t0 = st[:, :nw, 0].min(axis=1)
        rel = st - t0[:, None, None]
        res = {}
        for w, (wi, slots) in names.items():
            res[w] = {str(k): float(np.median(rel[:, wi, k])) for k in slots}
        res["end_max"] = float((st[:, 0, 5] - t0).max())
        # across workgroups (absolute shader clock): dispatch spread and the
        # first-start-to-last-verdict span of the whole launch
        res["start_spread"] = float(t0.max() - t0.min())
        res["launch_span"] = float(st[:, 0, 5].max() - t0.min())
        res["end_median"] = float(np.median(st[:, 0, 5] - t0))
        if form == "row4":
            # the 100 MHz constant clock (kernels.hip CMTV_STAMP_RT): entry of
            # every wave (slot 7) and the lo wave's verdict (slot 6)
            rt0 = st[:, :nw, 7].min(axis=1)
            cyc = (st[:, 0, 5] - t0).astype(np.float64)
            ns = (st[:, 0, 6] - rt0).astype(np.float64) * 10.0
            res["shader_clock_ghz_median"] = round(float(np.median(cyc / ns)), 3)
            res["wall_us_median"] = round(float(np.median(ns)) / 1e3, 2)
            res["launch_wall_us"] = round(float((st[:, 0, 6].max() - rt0.min()) * 10.0) / 1e3, 2)
            res["start_spread_us"] = round(float((rt0.max() - rt0.min()) * 10.0) / 1e3, 2)
        out[name] = res
        print(name, json.dumps(res), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "row_phase.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
