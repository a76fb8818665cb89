"""Per-call timeline of a small-batch verify (dev tool) from a rocprofv3
--runtime-trace directory (tools/lat_probe.py under the profiler).

  python tools/lat_timeline.py <trace_dir> [calls]

A call = the HIP API calls after one hipStreamSynchronize up to the next
one's return. Prints, for the median call, every API call,
copy and kernel as offsets (us) from the call's first API entry, and the
medians of: API time on the host, the first GPU op's start, kernel time,
and the sync's wake-up after the last GPU op ends."""
import csv
import os
import sys

import numpy as np


def rows(d, name):
    p = os.path.join(d, f"run_{name}.csv")
    with open(p) as f:
        return list(csv.DictReader(f))


def main():
    d = sys.argv[1]
    ncalls = int(sys.argv[2]) if len(sys.argv) > 2 else 60
    api = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"], int(r["Correlation_Id"]))
                  for r in rows(d, "hip_api_trace")))
    gpu = []
    for r in rows(d, "kernel_trace"):
        gpu.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K:" + r["Kernel_Name"].split("(")[0][-40:],
                    int(r["Correlation_Id"])))
    for r in rows(d, "memory_copy_trace"):
        gpu.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C:" + r["Direction"].split("_")[-1] + "_" +
                    r["Direction"].split("_")[-3], int(r["Correlation_Id"])))
    gpu.sort()
    # calls: from the API call after one hipStreamSynchronize to the next one's return
    syncs = [i for i, a in enumerate(api) if a[2] == "hipStreamSynchronize"]
    calls = [(a + 1, b) for a, b in zip(syncs, syncs[1:]) if b > a + 1]
    calls = calls[-ncalls:]
    stats = []
    for a, b in calls:
        t0, t1 = api[a][0], api[b][1]
        g = [x for x in gpu if x[0] >= t0 and x[1] <= t1 + 1000]
        if not g:
            continue
        kern = [x for x in g if x[2].startswith("K:")]
        stats.append(dict(total=(t1 - t0) / 1e3, api_host=sum(x[1] - x[0] for x in api[a:b]) / 1e3,
                          first_gpu=(g[0][0] - t0) / 1e3, kernels=sum(x[1] - x[0] for x in kern) / 1e3,
                          wake=(t1 - g[-1][1]) / 1e3, gpu_span=(g[-1][1] - g[0][0]) / 1e3, ab=(a, b)))
    if not stats:
        sys.exit("no calls found")
    tot = np.array([s["total"] for s in stats])
    med = stats[int(np.argsort(tot)[len(tot) // 2])]
    for k in ("total", "api_host", "first_gpu", "gpu_span", "kernels", "wake"):
        print(f"median {k:10s} {np.median([s[k] for s in stats]):9.1f} us")
    a, b = med["ab"]
    t0, t1 = api[a][0], api[b][1]
    print(f"\nmedian call ({med['total']:.1f} us):")
    ev = [(x[0], x[1], "api " + x[2]) for x in api[a:b + 1]]
    ev += [(x[0], x[1], "gpu " + x[2]) for x in gpu if x[0] >= t0 and x[1] <= t1 + 1000]
    for s, e, nm in sorted(ev):
        print(f"  {(s - t0) / 1e3:8.1f} .. {(e - t0) / 1e3:8.1f}  ({(e - s) / 1e3:7.1f})  {nm}")


if __name__ == "__main__":
    main()
