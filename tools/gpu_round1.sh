#!/bin/bash
# First GPU session: parity tests + quick timing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/quick_time.py 10000 100000 > gpurun_out/quick_time.log 2>&1
rc=$?
cat gpurun_out/quick_time.log
exit $rc
