#!/bin/bash
# round 6: latency under a configs[2] load (masked lane, dedicated queues) + host ceiling
set -o pipefail
OUT=gpurun_out/r6c
mkdir -p "$OUT"
export TMPDIR=/tmp
for T in 16; do for K in 0 1; do timeout -k 10 120 ./tests/host/pipebench 100000 $T $K 1048576 150 1 0 8 1; done; done > "$OUT/pipebench.txt" 2>&1 || exit 1
cat "$OUT/pipebench.txt"
timeout -k 10 300 python -u tools/lat_load.py 1000 > "$OUT/lat_default.json" 2> "$OUT/lat_default.err" || exit 1
cat "$OUT/lat_default.json"
CMTV_LAT_WINDOW_MS=0 timeout -k 10 300 python -u tools/lat_load.py 1000 > "$OUT/lat_nomask.json" 2> "$OUT/lat_nomask.err" || exit 1
cat "$OUT/lat_nomask.json"
CMTV_LIBRARY=$PWD/tools/probe/libprobe.so timeout -k 10 300 python -u tools/keyed_phase.py > "$OUT/keyed_phase.txt" 2>&1 || exit 1
cat "$OUT/keyed_phase.txt"
