#!/bin/bash
# round 6: latency stream without the idle cross-queue wait; tagged keyed quad
# slices (polled completion) -- GPU tests, latency under load, 10k keyset
set -o pipefail
OUT=gpurun_out/r6o
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_commit_gpu.py tests/test_pipeline_gpu.py tests/test_keyed_gpu.py > "$OUT/tests.txt" 2>&1 || { tail -30 "$OUT/tests.txt"; exit 1; }
tail -2 "$OUT/tests.txt"
run() {  # run <name> [env...]
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u tools/lat_load.py 1000 > "$OUT/$name.json" 2> "$OUT/$name.err" || { tail "$OUT/$name.err"; exit 1; }
  echo "$name $(cat "$OUT/$name.json" | tr '\n' ' ')"
}
run iso16_kquad
run iso16_krow CMTV_LOAD_FORM=0
run nopoll CMTV_HOST_POLL=0
timeout -k 10 300 rocprofv3 --hip-runtime-trace --kernel-trace --memory-copy-trace --output-format csv -d "$OUT/trace" -o run -- python3 tools/lat_trace.py "$OUT/trace_windows.json" 300 > "$OUT/trace.log" 2>&1 || { tail -20 "$OUT/trace.log"; exit 1; }
tail -1 "$OUT/trace.log"
