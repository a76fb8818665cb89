#!/bin/bash
# round 6: latency under load -- where the 150-validator call waits (trace), and
# the A/B of its in-place staging beside a pipeline (CMTV_LOAD_ZC) x masking
set -o pipefail
OUT=gpurun_out/r6f
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # run <name> [env...]
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u tools/lat_load.py 1000 > "$OUT/$name.json" 2> "$OUT/$name.err" || { tail "$OUT/$name.err"; exit 1; }
  echo "$name $(tail -1 "$OUT/$name.json")"
}
run zc_mask
run zc_nomask CMTV_LAT_WINDOW_MS=0
run zc_mask_idleform CMTV_LOAD_FORM=0
run copy_nomask CMTV_LOAD_ZC=0 CMTV_LAT_WINDOW_MS=0
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$OUT/trace" -o run -- python3 tools/lat_trace.py "$OUT/trace_windows.json" 300 > "$OUT/trace.log" 2>&1 || { tail -20 "$OUT/trace.log"; exit 1; }
tail -2 "$OUT/trace.log"
find "$OUT/trace" -name '*.csv' | head
