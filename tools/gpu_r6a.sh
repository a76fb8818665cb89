#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r6a
export TMPDIR=/tmp
nproc > gpurun_out/r6a/host.txt; lscpu | head -20 >> gpurun_out/r6a/host.txt
# host ceiling of the pipeline on the box's CPU share (no device)
for T in 8 16; do for P in 0 1; do timeout -k 10 120 ./tests/host/pipebench 100000 $T 0 1048576 150 1 0 8 $P; done; done > gpurun_out/r6a/pipebench.txt 2>&1
timeout -k 10 120 ./tests/host/pipebench 100000 16 1 1048576 150 1 0 8 1 >> gpurun_out/r6a/pipebench.txt 2>&1
timeout -k 10 900 python -u -m pytest tests/test_pipeline_gpu.py tests/test_commit_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r6a/pytest.log 2>&1
rc=$?
tail -15 gpurun_out/r6a/pytest.log
exit $rc
