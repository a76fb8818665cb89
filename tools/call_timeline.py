"""Mean timeline of a repeated single-thread call from a rocprofv3 trace with
--hip-runtime-trace --kernel-trace --memory-copy-trace (round 6: where
verify_commit_10k_keyset's time between its kernel and its p50 goes).
Calls are cut at each kernel named KERNEL; offsets are from the previous
hipStreamSynchronize's return (the previous call's end, i.e. host time
between calls included) to each API call / copy / kernel edge.
  python tools/call_timeline.py <trace dir> [kernel substring] [last N calls]"""
import csv
import glob
import sys

import numpy as np


def rows(tdir, pat):
    out = []
    for f in glob.glob(f"{tdir}/**/*{pat}", recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def main():
    tdir = sys.argv[1]
    kname = sys.argv[2] if len(sys.argv) > 2 else "keyed_quad_split"
    last = int(sys.argv[3]) if len(sys.argv) > 3 else 150
    api = rows(tdir, "hip_api_trace.csv")
    kern = rows(tdir, "kernel_trace.csv")
    copy = rows(tdir, "memory_copy_trace.csv")
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in kern if kname in r["Kernel_Name"])
    ks = ks[-last:]
    ev = []
    for r in api:
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "api " + r["Function"]))
    for r in copy:
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy " + r["Direction"][12:]))
    for r in kern:
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "kernel " + r["Kernel_Name"][:40]))
    ev.sort()
    starts = np.array([e[0] for e in ev])
    table = {}
    for i in range(1, len(ks)):
        k0, k1 = ks[i]
        # the previous call's end: its last hipStreamSynchronize returning after its kernel
        lo = np.searchsorted(starts, ks[i - 1][0])
        hi = np.searchsorted(starts, k1 + 200_000)
        prev_sync = [e for e in ev[lo:hi] if e[2] == "api hipStreamSynchronize" and e[1] >= ks[i - 1][1] and e[0] < k0]
        if not prev_sync:
            continue
        t0 = prev_sync[0][1]
        seen = {}
        for s, e, name in ev[lo:hi]:
            if s < t0 or s > k1 + 100_000:
                continue
            if name == "api hipStreamSynchronize" and s > k1:
                seen.setdefault(name + " (this call)", (s, e))
                break
            seen.setdefault(name, (s, e))
        for name, (s, e) in seen.items():
            table.setdefault(name, []).append(((s - t0) / 1e3, (e - t0) / 1e3))
    print(f"{len(ks) - 1} calls; offsets in us from the previous call's sync return (median start .. end)")
    order = sorted(table.items(), key=lambda kv: np.median([a for a, _ in kv[1]]))
    for name, v in order:
        if len(v) < len(ks) // 3:
            continue
        a = np.median([x for x, _ in v])
        b = np.median([y for _, y in v])
        print(f"  {a:8.1f} .. {b:8.1f}  {name}  (n={len(v)})")


if __name__ == "__main__":
    main()
