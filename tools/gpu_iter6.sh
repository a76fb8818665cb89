#!/bin/bash
# GPU tests, then the A/B of abtest/libold.so vs the in-tree library
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${ITER:-iter6}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || { grep -B5 -A40 "FAIL\|Error" "$OUT/pytest.log" | head -100; exit $rc; }
ITER=${ITER:-iter6}/ab bash tools/gpu_ab.sh
