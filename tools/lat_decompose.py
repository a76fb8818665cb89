"""Decomposes each loaded 150-validator call of tools/lat_trace.py (run under
rocprofv3 --hip-runtime-trace --kernel-trace) into: call start -> its
hipLaunchKernel returning (host: lock wait, plan, staging), launch -> kernel
start (queue / dispatch), the kernel, kernel end -> call end (completion
wake-up, replay, release).  python tools/lat_decompose.py <trace dir> <windows.json>"""
import csv
import glob
import json
import sys

import numpy as np


def rows(tdir, pat):
    out = []
    for f in glob.glob(f"{tdir}/**/*{pat}", recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def main():
    tdir, wfile = sys.argv[1:3]
    K = rows(tdir, "kernel_trace.csv")
    A = rows(tdir, "hip_api_trace.csv")
    W = json.load(open(wfile))
    print(json.dumps(W.get("result", {}))[:400])
    lat_k = [r for r in K if "keyed_quad_split" in r["Kernel_Name"] or "keyed_row_split" in r["Kernel_Name"]]
    me = lat_k[0]["Thread_Id"]
    lat = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in lat_k)
    launch = sorted(int(r["End_Timestamp"]) for r in A if r["Function"] == "hipLaunchKernel" and r["Thread_Id"] == me)
    out = []
    for t0, t1 in W["windows"]:
        ks = [k for k in lat if t0 <= k[0] <= t1]
        ls = [x for x in launch if t0 <= x <= t1]
        if not ks or not ls:
            continue
        k, l = ks[-1], ls[-1]
        out.append(((t1 - t0) / 1e3, (l - t0) / 1e3, (k[0] - l) / 1e3, (k[1] - k[0]) / 1e3, (t1 - k[1]) / 1e3))
    r = np.array(out)
    print(f"{len(r)} calls (us)")
    for name, i in [("call", 0), ("start -> launch", 1), ("launch -> kernel start", 2), ("kernel", 3),
                    ("kernel end -> call end", 4)]:
        print(f"  {name:24s} p50 {np.percentile(r[:, i], 50):8.1f}  p90 {np.percentile(r[:, i], 90):8.1f}  "
              f"p99 {np.percentile(r[:, i], 99):8.1f}")
    print("  slowest calls [call, pre-launch, dispatch, kernel, post]:")
    for row in r[np.argsort(r[:, 0])[-8:]]:
        print("   ", row.round(1))


if __name__ == "__main__":
    main()
