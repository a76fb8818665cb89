#!/bin/bash
# Row kernel iteration: row GPU tests (all forms), timing A/B of the forms at 150/256.
set -o pipefail
OUT=gpurun_out/row2
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_row_gpu.py tests/test_gpu_parity.py tests/test_wide_gpu.py tests/test_commit_gpu.py -k "row or commit" -x -q \
  -m gpu --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?
tail -5 "$OUT/pytest.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/quick_time.py 150 256 > "$OUT/time_row4.txt" 2>&1 && cat "$OUT/time_row4.txt" || exit 1
CMTV_ROW_WAVES=2 timeout -k 10 120 python tools/quick_time.py 150 256 > "$OUT/time_row2.txt" 2>&1 && cat "$OUT/time_row2.txt" || exit 1
CMTV_LIBRARY=$PWD/abtest/libprobe.so timeout -k 10 180 python tools/row_phase.py 150 row4 > "$OUT/phase.txt" 2>&1; cat "$OUT/phase.txt"
