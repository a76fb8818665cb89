#!/bin/bash
# Row kernel bring-up: DPP/permlane probe + product timing, the row GPU tests,
# kernel timing (row vs oct2) and a short bench (latency_150 included).
set -o pipefail
OUT=gpurun_out/row
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 60 tools/microbench/row_lat > "$OUT/row_lat.txt" 2>&1; cat "$OUT/row_lat.txt"
timeout -k 10 600 python -u -m pytest tests/test_row_gpu.py tests/test_gpu_parity.py tests/test_wide_gpu.py -k "row" -x -v \
  -m gpu --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?
tail -25 "$OUT/pytest.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/quick_time.py 150 300 768 > "$OUT/time_row.txt" 2>&1 && cat "$OUT/time_row.txt" || exit 1
CMTV_ROW_MAX=0 timeout -k 10 120 python tools/quick_time.py 150 768 > "$OUT/time_oct2.txt" 2>&1 && cat "$OUT/time_oct2.txt" || exit 1
timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline --no-c3 --no-sr25519 --no-light --no-keyset > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
