#!/bin/bash
# iteration loop: parity tests on the default build, then timing (quad vs lane kernels)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/quick_time.py ${SIZES:-1000 10000 30000 65536 100000 1000000} > gpurun_out/qt_default.log 2>&1 || exit 1
cat gpurun_out/qt_default.log
echo "== lane kernel only"
CMTV_QUAD_MAX=0 timeout -k 10 300 python tools/quick_time.py ${SIZES:-1000 10000 30000 65536} > gpurun_out/qt_lane.log 2>&1 || exit 1
cat gpurun_out/qt_lane.log
echo "== quad kernel only"
CMTV_QUAD_MAX=100000000 timeout -k 10 300 python tools/quick_time.py ${SIZES:-100000 300000} > gpurun_out/qt_quad.log 2>&1 || exit 1
cat gpurun_out/qt_quad.log
