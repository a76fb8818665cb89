#!/bin/bash
# iteration loop: parity tests on the default build, then timing of variants
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/quick_time.py ${SIZES:-10000 100000 1000000} > gpurun_out/qt_default.log 2>&1 || exit 1
cat gpurun_out/qt_default.log
for v in tools/variants/*.so; do
  [ -f "$v" ] || continue
  CMTV_LIBRARY=$v timeout -k 10 300 python tools/quick_time.py ${SIZES:-10000 100000 1000000} > gpurun_out/qt_$(basename $v).log 2>&1 || exit 1
  echo "== $v"; cat gpurun_out/qt_$(basename $v).log
done
