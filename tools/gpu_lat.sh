#!/bin/bash
# GPU tests, then the 150-validator latency probe plain and under a runtime trace
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-lat2}
mkdir -p "$OUT"
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
  rc=$?; tail -3 "$OUT/pytest.log"
  [ $rc -eq 0 ] || { grep -B5 -A30 "FAIL\|Error" "$OUT/pytest.log" | head -80; exit $rc; }
fi
timeout -k 10 200 python3 tools/lat_probe.py 300 > "$OUT/plain.log" 2>&1 || { cat "$OUT/plain.log"; exit 1; }
grep verify_commit "$OUT/plain.log"
timeout -k 10 300 rocprofv3 --runtime-trace --output-format csv -d "$OUT/tr" -o run -- python3 tools/lat_probe.py 100 > "$OUT/trace.log" 2>&1 || { tail -20 "$OUT/trace.log"; exit 1; }
echo done
