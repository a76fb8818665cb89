#!/bin/bash
# keyed path: parity tests, then timing of generic vs registered-key verification
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
KEYED=1 NKEYS=150 timeout -k 10 400 python tools/quick_time.py ${SIZES:-10000 100000 1000000 4000000} > gpurun_out/qt_keyed.log 2>&1
rc=$?; cat gpurun_out/qt_keyed.log; exit $rc
