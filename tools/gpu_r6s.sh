#!/bin/bash
# round 6: where the isolated, unpolled 150-validator call's tail goes (trace
# with the HIP API), and the host ceiling with the cut phase
set -o pipefail
OUT=gpurun_out/r6s
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --hip-runtime-trace --kernel-trace --memory-copy-trace --output-format csv -d "$OUT/trace" -o run -- python3 tools/lat_trace.py "$OUT/trace_windows.json" 1000 > "$OUT/trace.log" 2>&1 || { tail -20 "$OUT/trace.log"; exit 1; }
tail -1 "$OUT/trace.log"
for R in 1 2; do for K in 0 1; do timeout -k 10 120 ./tests/host/pipebench 100000 16 $K 1048576 150 1 0 8 1; done; done > "$OUT/pipebench.txt" 2>&1 || { cat "$OUT/pipebench.txt"; exit 1; }
cat "$OUT/pipebench.txt"
