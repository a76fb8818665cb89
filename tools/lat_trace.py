"""latency_150_under_load under rocprofv3 --kernel-trace --memory-copy-trace:
each loaded 150-validator call's host window (CLOCK_MONOTONIC ns) written to
argv[1], to be matched with the trace's kernels and copies offline
(tools/lat_trace_report.py).  python tools/lat_trace.py out.json [iters]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

iters = int(sys.argv[2]) if len(sys.argv) > 2 else 300
win = []
r = bench.latency_150_under_load(0, iters, windows=win)
clk = {"monotonic_ns": time.monotonic_ns(), "boottime_ns": time.clock_gettime_ns(time.CLOCK_BOOTTIME)}
json.dump({"result": r, "windows": win, "clocks": clk}, open(sys.argv[1], "w"))
print(json.dumps(r), flush=True)
