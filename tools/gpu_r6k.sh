#!/bin/bash
# round 6: latency calls isolated on the reserved CU pairs beside a pipeline
# (LatencyStreams) -- GPU tests of the commit / pipeline paths, then the A/B
set -o pipefail
OUT=gpurun_out/r6k
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_commit_gpu.py tests/test_pipeline_gpu.py > "$OUT/tests.txt" 2>&1 || { tail -30 "$OUT/tests.txt"; exit 1; }
tail -2 "$OUT/tests.txt"
run() {  # run <name> [env...]
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u tools/lat_load.py 1000 > "$OUT/$name.json" 2> "$OUT/$name.err" || { tail "$OUT/$name.err"; exit 1; }
  echo "$name $(tail -1 "$OUT/$name.json")"
}
run iso16_kquad
run iso16_krow CMTV_LOAD_FORM=0
run iso8_kquad CMTV_LAT_RESERVE_CUS=8
run noiso CMTV_LAT_ISOLATE=0
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$OUT/trace" -o run -- python3 tools/lat_trace.py "$OUT/trace_windows.json" 300 > "$OUT/trace.log" 2>&1 || { tail -20 "$OUT/trace.log"; exit 1; }
tail -1 "$OUT/trace.log"
