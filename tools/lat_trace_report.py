"""Where a 150-validator call waits under load: matches tools/lat_trace.py's
call windows with the rocprofv3 kernel / memory-copy trace of the same run.
Ops issued from the calling thread (Thread_Id of the main thread) are the
call's own; the others are the load's.
  python tools/lat_trace_report.py <trace dir> <windows.json>"""
import csv
import glob
import json
import sys

import numpy as np


def load(pattern):
    rows = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    return rows


def main():
    tdir, wfile = sys.argv[1:3]
    W = json.load(open(wfile))
    win = W["windows"]
    kern = load(f"{tdir}/**/*kernel_trace.csv")
    copy = load(f"{tdir}/**/*memory_copy_trace.csv")
    ops = []
    for r in kern:
        ops.append(("K", r.get("Kernel_Name", "?")[:40], int(r["Thread_Id"]), int(r["Start_Timestamp"]),
                    int(r["End_Timestamp"])))
    for r in copy:
        ops.append(("C", r.get("Direction", "?"), int(r.get("Thread_Id", 0) or 0), int(r["Start_Timestamp"]),
                    int(r["End_Timestamp"])))
    for r in load(f"{tdir}/**/*hip_api_trace.csv"):
        ops.append(("A", r.get("Function", "?")[:40], int(r["Thread_Id"]), int(r["Start_Timestamp"]),
                    int(r["End_Timestamp"])))
    ops.sort(key=lambda o: o[3])
    # the calling thread: the thread whose ops fall inside most windows
    starts = np.array([o[3] for o in ops])
    votes = {}
    for t0, t1 in win[:50]:
        i, j = np.searchsorted(starts, t0), np.searchsorted(starts, t1)
        for o in ops[i:j]:
            if o[0] == "K" and ("quad_split" in o[1] or "row_split" in o[1]):
                votes[o[2]] = votes.get(o[2], 0) + 1
    me = max(votes, key=votes.get) if votes else None
    print(f"{len(kern)} kernels, {len(copy)} copies, {len(win)} windows, calling thread {me}")
    lat = np.array([(t1 - t0) / 1e3 for t0, t1 in win])
    order = np.argsort(lat)
    bulk = [o for o in ops if o[2] != me and o[0] != "A"]
    bk = [o for o in bulk if o[0] == "K"]
    bc = [o for o in bulk if o[0] == "C"]

    def active(lst, t):
        return sum(1 for o in lst if o[3] <= t < o[4])

    def show(k):
        t0, t1 = win[k]
        i, j = np.searchsorted(starts, t0 - 1000), np.searchsorted(starts, t1)
        mine = [o for o in ops[i:j] if o[2] == me]
        print(f"call {k}: {lat[k]:.1f} us; load kernels active at start {active(bk, t0)}, copies {active(bc, t0)}")
        for o in mine:
            print(f"   {o[0]} {o[1]:<40} +{(o[3] - t0) / 1e3:8.1f} .. +{(o[4] - t0) / 1e3:8.1f} us "
                  f"(load kernels {active(bk, o[3])}, load copies {active(bc, o[3])})")

    print("p50 / p90 / p99 / max us:", [round(float(np.percentile(lat, q)), 1) for q in (50, 90, 99, 100)])
    for k in list(order[:2]) + list(order[len(order) // 2:len(order) // 2 + 2]) + list(order[-6:]):
        show(int(k))


if __name__ == "__main__":
    main()
