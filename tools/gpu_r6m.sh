#!/bin/bash
# round 6: latency under load, isolated, with the HIP API trace (what the
# call waits for before its kernel starts); then the 10k keyset timeline
set -o pipefail
OUT=gpurun_out/r6m
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --hip-runtime-trace --kernel-trace --memory-copy-trace --output-format csv -d "$OUT/trace" -o run -- python3 tools/lat_trace.py "$OUT/trace_windows.json" 300 > "$OUT/trace.log" 2>&1 || { tail -20 "$OUT/trace.log"; exit 1; }
tail -1 "$OUT/trace.log"
python3 tools/lat_trace_report.py "$OUT/trace" "$OUT/trace_windows.json" > "$OUT/report.txt" 2>&1 || { cat "$OUT/report.txt"; exit 1; }
head -c 20000 "$OUT/report.txt" | tail -c 6000
bash tools/gpu_r6l.sh
