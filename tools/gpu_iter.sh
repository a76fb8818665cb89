#!/bin/bash
# iteration loop: parity tests on the default build, then timing (default dispatch, lane-only, quad-only)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/quick_time.py ${SIZES:-150 1000 10000 30000 100000 1000000} > gpurun_out/qt_default.log 2>&1 || exit 1
cat gpurun_out/qt_default.log
echo "== quad kernel only"
CMTV_QUAD_MAX=100000000 timeout -k 10 300 python tools/quick_time.py ${QSIZES:-10000 65536 300000} > gpurun_out/qt_quad.log 2>&1 || exit 1
cat gpurun_out/qt_quad.log
